"""Host-side mirror of the reference's pyramid interface, on top of the libgdp C ABI.

`GaussPyramid` keeps the reference class's names, argument meaning and call semantics
(GuassDePyramid.h:11-29):

    g = GaussPyramid(img, len, S)   # ctor copies img[0:len][0:len] and runs GaussPyInit (:36-58)
    g.GaussPyInit()                 # refill every level with the decimated input (:60-87)
    g.GaussFilter(o)                # window-multiply every scale of octave o in place (:106-134)
    g.GenerateDoG()                 # GaussFilter + DoG for every octave, in place (:136-149)
    g.output()                      # print scale 0 of every octave (:89-104)
    g.GaussPy[o][s][r][c]           # the pyramid (downloaded lazily from the device)

GaussPy is two-way state, as the reference's float**** is (:16; GaussFilter / GenerateDoG work
on whatever the caller left in it, :122-131, :140-146): a level the caller touched through
GaussPy[o][s] is ONE host array for the object's lifetime (like a reference row, it stays live:
a handle taken before a call reads the new contents after it, and writes through it are seen),
and it may be written any way (g.GaussPy[o][s][r][c] = v, row slices, views, ufuncs with out=).
Every mutating call first uploads each touched level whose bits differ from what the device last
gave it (an exact comparison against a snapshot; levels only read are not uploaded, so reading
GaussPy — output() included — never costs the fused GaussPyInit+GenerateDoG path), then runs,
then refreshes every touched level in place — the touched levels are views into ONE host buffer in
the device's raw layout, so when they hold at least half of the pyramid's bytes (e.g. a caller
that walks every level) the refresh is one gdp_download_image_raw instead of one blocking copy per
level; levels touched once stay in the refresh for the object's lifetime (like
reference rows, a dropped handle may still have been written).  GaussPyInit re-reads the CURRENT `data` (:80) and
overwrites host edits, as the reference's refill does.  Levels never touched cost nothing.
SyncDevice() uploads the edited levels on demand.
GaussPyramid(img, len, S, defer=True) (round 6, as the C++ classes' DeferDownload): the levels are
views of ONE write-tracked host mirror in the device layout; after a call its pages are fetched
from the device only when first touched (sequential readers get the next block ahead), and the
pages the caller writes are found by page faults — no snapshot comparison, no copy of levels the
caller does not read.  Writing such an array to a file or socket straight from its memory (tofile,
np.save, file.write) may fail with EFAULT on a page not fetched yet: copy it first (np.array(a)).

Calling GenerateDoG() twice without GaussPyInit() re-filters the pyramid exactly like the
reference's timing loop does (main.cpp:66-73).  The one behavioural difference is error
handling: the reference never reports errors (all methods return void); here a failing call
raises GdpError instead of continuing on bad state.

`PyramidContext` is the batched, stream-ordered interface (one context = `batch` images or one
row band), used by bench.py and the multi-GPU driver.
"""
import ctypes
import sys

import numpy as np

from ._lib import check, lib

_i = ctypes.c_int


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data)


GDP_STREAM_NULL = 1  # include/gdp.h: selects HIP's default (null) stream


def _stream_handle(stream):
    """None -> the context's own stream; a torch.cuda.Stream or raw int handle -> that stream
    (handle 0, torch's default stream, is passed as GDP_STREAM_NULL so it is not mistaken for
    "the context's stream")."""
    if stream is None:
        return None
    handle = stream if isinstance(stream, int) else getattr(stream, "cuda_stream", None)
    if handle is None:
        raise TypeError(f"unsupported stream object {stream!r}")
    return ctypes.c_void_p(handle if handle != 0 else GDP_STREAM_NULL)


def octaves_for(n):
    """floor(log2 n) + 1 — the reference's `layer` (GuassDePyramid.h:48-53)."""
    return lib().gdp_octaves_for(int(n))


def conv_taps(S, scale):
    """(taps[0:2R+1], R) of the convolution-mode Gaussian of `scale` (gdp_conv_taps)."""
    t = np.zeros(13, np.float32)
    r = _i()
    check(lib().gdp_conv_taps(int(S), int(scale), _ptr(t), ctypes.byref(r)))
    return t[:2 * r.value + 1].copy(), r.value


class PyramidContext:
    """`batch` images of H x W int32 (or the row band [row_begin, row_end)) on one GPU.

    Level (o, s) of image b is a rows_o x cols_o float32 array; rows_o covers the band's rows.
    All compute calls are asynchronous on `stream` (None = the context's own stream).
    """

    def __init__(self, height, width, S=2, octaves=0, batch=1, device=0, row_begin=0, row_end=None,
                 input_format="i32", centre="serial"):
        L = lib()
        self._ctx = ctypes.c_void_p()
        row_end = height if row_end is None else row_end
        check(L.gdp_create_band(ctypes.byref(self._ctx), int(height), int(width), int(S), int(octaves), int(batch),
                                int(row_begin), int(row_end), int(device)))
        H, W, S_, O, B = (_i() for _ in range(5))
        check(L.gdp_get_geometry(self._ctx, *(ctypes.byref(v) for v in (H, W, S_, O, B))), self._ctx)
        self.H, self.W, self.S, self.O, self.batch = H.value, W.value, S_.value, O.value, B.value
        self.device = device
        self.row_begin, self.row_end = int(row_begin), int(row_end)
        self._dims = []
        for o in range(self.O):
            r, c, f = _i(), _i(), _i()
            check(L.gdp_level_dims(self._ctx, o, ctypes.byref(r), ctypes.byref(c), ctypes.byref(f)), self._ctx)
            self._dims.append((r.value, c.value, f.value))
        self._bound = None  # keeps a caller's device input alive
        self.input_format = "i32"
        if input_format != "i32":
            self.set_input_format(input_format)
        self.centre = "serial"
        if centre != "serial":
            self.set_window_centre(centre)

    def set_window_centre(self, mode):
        """'serial' (GuassDePyramid.h:107-115: the float length halved o times) or 'intlen'
        (the multi-process variants' integer length, GaussDePyramid-MPI.h:273, mpitest.cpp:44)."""
        from ._lib import GDP_CENTRE_INTLEN, GDP_CENTRE_SERIAL

        code = {"serial": GDP_CENTRE_SERIAL, "intlen": GDP_CENTRE_INTLEN}[mode]
        check(lib().gdp_set_window_centre(self._ctx, code), self._ctx)
        self.centre = mode

    def copy_band_from(self, full, b=0, full_image=0, stream=None):
        """Load this band context's rows of `full`'s current pyramid (gdp_copy_band)."""
        check(lib().gdp_copy_band(self._ctx, int(b), full._ctx, int(full_image), _stream_handle(stream)), self._ctx)

    def set_input_format(self, fmt):
        """'i32' (the reference's int pixels) or 'u8' (8-bit images, 4x fewer input bytes)."""
        from ._lib import GDP_INPUT_I32, GDP_INPUT_U8

        code = {"i32": GDP_INPUT_I32, "u8": GDP_INPUT_U8}[fmt]
        check(lib().gdp_set_input_format(self._ctx, code), self._ctx)
        self.input_format = fmt

    # ------------------------------------------------------------------ geometry
    @property
    def levels_per_octave(self):
        return self.S + 3

    def level_dims(self, o):
        """(rows held, cols, first global row) of octave o."""
        return self._dims[o]

    def packed_floats(self):
        return lib().gdp_packed_floats(self._ctx)

    def pyramid_bytes(self):
        return lib().gdp_pyramid_bytes(self._ctx)

    # ------------------------------------------------------------------ input
    def set_input(self, img, b=0, stream=None):
        """Upload one H x W (band: band-rows x W) image from host memory, in the context's input
        format (int32, or uint8 for an input_format='u8' context)."""
        u8 = self.input_format == "u8"
        img = np.asarray(img)
        if u8 and img.dtype != np.uint8:
            raise TypeError("a u8 context takes uint8 images")
        img = np.ascontiguousarray(img, dtype=np.uint8 if u8 else np.int32)
        rows = self.row_end - self.row_begin
        if img.ndim != 2 or img.shape[1] != self.W or img.shape[0] != rows:
            raise ValueError(f"expected a ({rows}, {self.W}) image, got {img.shape}")
        fn = lib().gdp_set_input_host_u8 if u8 else lib().gdp_set_input_host
        check(fn(self._ctx, int(b), _ptr(img), self.W, _stream_handle(stream)), self._ctx)

    def set_input_rows(self, rows, b=0, stream=None):
        """Upload from a list of row arrays — the reference ctor's `int** img` (GuassDePyramid.h:38-46)."""
        arrs = [np.ascontiguousarray(r, dtype=np.int32) for r in rows]
        ptrs = (ctypes.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])
        check(lib().gdp_set_input_rows(self._ctx, int(b), ptrs, _stream_handle(stream)), self._ctx)

    def bind_device_input(self, ptr, pitch, image_stride, keepalive=None):
        """Read images straight from caller device memory (pitch/stride in elements of the
        context's input format)."""
        fn = lib().gdp_set_input_device_u8 if self.input_format == "u8" else lib().gdp_set_input_device
        check(fn(self._ctx, ctypes.c_void_p(ptr), int(pitch), int(image_stride)), self._ctx)
        self._bound = keepalive

    def unbind_device_input(self):
        check(lib().gdp_set_input_device(self._ctx, None, 0, 0), self._ctx)
        self._bound = None

    # ------------------------------------------------------------------ row-band halos (conv extension)
    def conv_halo_rows(self):
        """(above, below): input rows a band's build_gaussian reads beyond its own rows."""
        a, b = _i(), _i()
        check(lib().gdp_conv_halo_rows(self._ctx, ctypes.byref(a), ctypes.byref(b)), self._ctx)
        return a.value, b.value

    def bind_input_halo(self, above=None, below=None, pitch=None, image_stride=None, keepalive=None):
        """Read the halo rows from caller device memory (device pointers, [batch][rows][pitch] in
        the input format; pitch defaults to the width)."""
        pitch = self.W if pitch is None else int(pitch)
        na, nb = self.conv_halo_rows()
        stride = pitch * max(na, nb, 1) if image_stride is None else int(image_stride)
        check(lib().gdp_bind_input_halo(self._ctx, ctypes.c_void_p(above or 0) if above else None,
                                        ctypes.c_void_p(below or 0) if below else None, pitch, stride), self._ctx)
        self._halo_keepalive = keepalive

    def input_halo(self, side):
        """(device address, pitch) of the context's own halo buffer (side 0 above, 1 below),
        allocated on first call and used by the next band builds; (None, pitch) when none is needed."""
        ptr, pitch = ctypes.c_void_p(), ctypes.c_size_t()
        check(lib().gdp_input_halo(self._ctx, int(side), ctypes.byref(ptr), ctypes.byref(pitch)), self._ctx)
        return ptr.value, pitch.value

    def device_input(self, b=0):
        """(device address, pitch) of image b's input rows (own buffer or the bound one)."""
        ptr, pitch = ctypes.c_void_p(), ctypes.c_size_t()
        check(lib().gdp_device_input(self._ctx, int(b), ctypes.byref(ptr), ctypes.byref(pitch)), self._ctx)
        return ptr.value, pitch.value

    def fill_synthetic(self, seed=0x5EED, first_image=0, stream=None):
        check(lib().gdp_fill_synthetic(self._ctx, int(seed) & 0xFFFFFFFF, int(first_image), _stream_handle(stream)),
              self._ctx)

    # ------------------------------------------------------------------ compute
    def build(self, stream=None):
        """Fused GaussPyInit + GenerateDoG of every image (one launch)."""
        check(lib().gdp_build(self._ctx, _stream_handle(stream)), self._ctx)

    def build_gaussian(self, stream=None):
        """Extension (no reference counterpart): true separable Gaussian convolution pyramid."""
        check(lib().gdp_build_gaussian(self._ctx, _stream_handle(stream)), self._ctx)

    def init(self, stream=None):
        check(lib().gdp_init(self._ctx, _stream_handle(stream)), self._ctx)

    def gauss_octave(self, o, stream=None):
        check(lib().gdp_gauss_octave(self._ctx, int(o), _stream_handle(stream)), self._ctx)

    def gauss_range(self, o_begin=0, o_end=None, stream=None):
        """GaussFilter of octaves [o_begin, o_end) in one launch (in place)."""
        o_end = self.O if o_end is None else o_end
        check(lib().gdp_gauss_range(self._ctx, int(o_begin), int(o_end), _stream_handle(stream)), self._ctx)

    def gauss_scales(self, s_begin, s_end, o_begin=0, o_end=None, stream=None):
        """Window multiply of scales [s_begin, s_end) of octaves [o_begin, o_end) in place (the MPI
        variant's worker step, GaussDePyramid-MPI.h:271-290)."""
        o_end = self.O if o_end is None else o_end
        check(lib().gdp_gauss_scales(self._ctx, int(s_begin), int(s_end), int(o_begin), int(o_end),
                                     _stream_handle(stream)), self._ctx)

    def dog_octave(self, o, stream=None):
        check(lib().gdp_dog_octave(self._ctx, int(o), _stream_handle(stream)), self._ctx)

    def dog_range(self, o_begin=0, o_end=None, stream=None):
        """The DoG pass of octaves [o_begin, o_end) in one launch."""
        o_end = self.O if o_end is None else o_end
        check(lib().gdp_dog_range(self._ctx, int(o_begin), int(o_end), _stream_handle(stream)), self._ctx)

    def generate_dog(self, stream=None):
        check(lib().gdp_generate_dog(self._ctx, _stream_handle(stream)), self._ctx)

    def build_subset(self, stream=None):
        """Fused GaussPyInit + GaussPyramid_a512omp::GenerateDoG_nomp_dynamic (the AVX-512 x OpenMP
        header's subset: scales 0..S-1 windowed, DoG for s < S-1; see gdp.h)."""
        check(lib().gdp_build_subset(self._ctx, _stream_handle(stream)), self._ctx)

    def generate_dog_subset(self, stream=None):
        """GenerateDoG_nomp_dynamic in place on the current contents."""
        check(lib().gdp_generate_dog_subset(self._ctx, _stream_handle(stream)), self._ctx)

    def sync(self):
        check(lib().gdp_sync(self._ctx), self._ctx)

    @property
    def stream(self):
        return lib().gdp_stream(self._ctx)

    _TUNING = ("nontemporal", "blocks_per_cu", "grid", "variant", "tile_order", "inplace_sub", "window_sub",
               "conv_kernel", "conv_rows", "conv_order", "build_lds", "stage_kb", "stage_threads", "conv_waves", "zero_window",
               "store_pace", "conv_pace", "inplace_pace", "pyramid_chunk_kb")  # the last one read-only

    @staticmethod
    def _tuning_key(name):
        from . import _lib

        return getattr(_lib, "GDP_TUNE_" + name.upper())

    def set_tuning(self, nontemporal=None, blocks_per_cu=None, grid=None, variant=None, tile_order=None,
                   inplace_sub=None, window_sub=None, conv_kernel=None, conv_rows=None, conv_order=None,
                   build_lds=None, stage_kb=None, stage_threads=None, conv_waves=None, zero_window=None,
                   store_pace=None, conv_pace=None, inplace_pace=None):
        """Performance knobs of the kernels (outputs are bit-identical for every setting; the
        conv_* knobs select the convolution extension's kernel: 0 register sweep, 1 LDS tiles,
        2 block tiles, and the sweep's rows per wave strip (16 / 32) or the block tiles' rows per
        block with conv_waves waves per block (16 waves: 16 / 32 / 48 rows; 8 waves: 8 / 16 / 24 /
        32 rows — any other pair makes build_gaussian raise GdpError); stage_kb / stage_threads
        size the double-buffered pinned staging of the row-pointer downloads; zero_window = 1 lets the
        build store the input-independent levels of pixels outside every window's support without
        waiting for their input; store_pace / conv_pace / inplace_pace pace the stores of the
        builds / the convolution block tiles / the in-place re-entry, each its own field)."""
        vals = dict(nontemporal=nontemporal, blocks_per_cu=blocks_per_cu, grid=grid, variant=variant,
                    tile_order=tile_order, inplace_sub=inplace_sub, window_sub=window_sub, conv_kernel=conv_kernel,
                    conv_rows=conv_rows, conv_order=conv_order, build_lds=build_lds, stage_kb=stage_kb,
                    stage_threads=stage_threads, conv_waves=conv_waves, zero_window=zero_window,
                    store_pace=store_pace, conv_pace=conv_pace, inplace_pace=inplace_pace)
        for name, val in vals.items():
            if val is not None:
                check(lib().gdp_set_tuning(self._ctx, self._tuning_key(name), int(val)), self._ctx)

    def autotune(self, iters=5, stream=None):
        """Time every build variant x tile order x store mode (zero_window, store_pace) on the
        current input and keep the fastest;
        returns (variant, tile_order, ms per build).  Overwrites the pyramid (bits unchanged)."""
        v, o, ms = _i(), _i(), ctypes.c_float()
        check(lib().gdp_autotune(self._ctx, int(iters), _stream_handle(stream), ctypes.byref(v), ctypes.byref(o),
                                 ctypes.byref(ms)), self._ctx)
        return v.value, o.value, ms.value

    def tuning(self):
        """Current value of every knob of set_tuning()."""
        out = {}
        for name in self._TUNING:
            v = _i()
            check(lib().gdp_get_tuning(self._ctx, self._tuning_key(name), ctypes.byref(v)), self._ctx)
            out[name] = v.value
        return out

    def time_builds(self, iters, stream=None):
        """Total ms of `iters` back-to-back builds, HIP events on the launch stream."""
        ms = ctypes.c_float()
        check(lib().gdp_time_builds(self._ctx, int(iters), _stream_handle(stream), ctypes.byref(ms)), self._ctx)
        return ms.value

    # ------------------------------------------------------------------ output
    def level(self, b, o, s):
        rows, cols, _ = self._dims[o]
        out = np.empty((rows, cols), np.float32)
        if out.size:
            check(lib().gdp_download_level(self._ctx, int(b), int(o), int(s), _ptr(out)), self._ctx)
        return out

    def level_range(self, b, o, s, first_row, nrows):
        """Rows [first_row, first_row + nrows) of level (o, s) of image b, without downloading the
        whole level."""
        cols = self._dims[o][1]
        out = np.empty((int(nrows), cols), np.float32)
        check(lib().gdp_download_level_range(self._ctx, int(b), int(o), int(s), int(first_row), int(nrows),
                                             _ptr(out)), self._ctx)
        return out

    def level_rows(self, b, o, s, rows_out):
        """Download into a list of preallocated float32 row arrays (float**** materialisation)."""
        ptrs = (ctypes.c_void_p * len(rows_out))(*[r.ctypes.data for r in rows_out])
        check(lib().gdp_download_level_rows(self._ctx, int(b), int(o), int(s), ptrs), self._ctx)

    def pyramid(self, b=0):
        """Packed [o][s][rows][cols] float32 copy of image b's pyramid."""
        out = np.empty(self.packed_floats(), np.float32)
        check(lib().gdp_download_pyramid(self._ctx, int(b), _ptr(out)), self._ctx)
        return out

    def upload_level(self, b, o, s, arr):
        """Copy a dense rows x cols float32 host array into level (o, s) of image b."""
        rows, cols, _ = self._dims[o]
        arr = np.ascontiguousarray(arr, dtype=np.float32)
        if arr.shape != (rows, cols):
            raise ValueError(f"level ({o}, {s}) is {rows} x {cols}, got {arr.shape}")
        if arr.size:
            check(lib().gdp_upload_level(self._ctx, int(b), int(o), int(s), _ptr(arr)), self._ctx)

    def upload_pyramid(self, packed, b=0):
        packed = np.ascontiguousarray(packed, dtype=np.float32)
        if packed.size != self.packed_floats():
            raise ValueError("packed pyramid has the wrong size")
        check(lib().gdp_upload_pyramid(self._ctx, int(b), _ptr(packed)), self._ctx)

    def levels(self, b=0):
        """{(o, s): 2-D array} of image b."""
        return {(o, s): self.level(b, o, s) for o in range(self.O) for s in range(self.S + 3)}

    def bind_device_output(self, ptr, nbytes, keepalive=None):
        """Write pyramids into caller device memory (>= pyramid_bytes(), 256-B aligned)."""
        check(lib().gdp_set_output_device(self._ctx, ctypes.c_void_p(ptr), int(nbytes)), self._ctx)
        self._out_bound = keepalive

    def unbind_device_output(self):
        check(lib().gdp_set_output_device(self._ctx, None, 0), self._ctx)
        self._out_bound = None

    def level_offset(self, b, o, s):
        """Float offset of level (o, s) of image b inside the (bound or own) pyramid buffer."""
        return lib().gdp_level_offset(self._ctx, int(b), int(o), int(s))

    def checksum(self, b=0):
        """Order-independent 64-bit checksum of image b's pyramid (see gdp.h)."""
        v = ctypes.c_uint64()
        check(lib().gdp_checksum(self._ctx, int(b), ctypes.byref(v)), self._ctx)
        return v.value

    def device_level_ptr(self, b, o, s):
        return lib().gdp_device_level(self._ctx, int(b), int(o), int(s))

    def taps(self, axis, o, s):
        """Window the device holds: axis 0 = column taps (from W), 1 = row taps (from H)."""
        n = (self.W >> o) if axis == 0 else (self.H >> o)
        out = np.empty(n, np.float32)
        check(lib().gdp_get_taps(self._ctx, int(axis), int(o), int(s), _ptr(out)), self._ctx)
        return out

    # ------------------------------------------------------------------ lifetime
    def close(self):
        if getattr(self, "_ctx", None) and self._ctx.value:
            lib().gdp_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class _TrackedBuffer:
    """gdp_host_alloc_tracked memory seen by numpy (GaussPyramid(defer=True)): arrays made from it
    keep it alive, and it is freed when the last one goes."""

    def __init__(self, nfloats):
        p = ctypes.c_void_p()
        check(lib().gdp_host_alloc_tracked(int(nfloats) * 4, ctypes.byref(p)))
        self.ptr = p.value
        self.__array_interface__ = {"shape": (int(nfloats),), "typestr": "<f4", "data": (self.ptr, False), "version": 3}

    def __del__(self):
        if getattr(self, "ptr", None):
            try:
                lib().gdp_host_free(ctypes.c_void_p(self.ptr))
            except Exception:  # interpreter shutdown: the process unmaps it anyway
                pass
            self.ptr = None


class _LevelView:
    """GaussPy[o] -> list of S+3 level arrays, downloaded on first access after a change."""

    def __init__(self, owner, o):
        self._owner, self._o = owner, o

    def __getitem__(self, s):
        return self._owner._level(self._o, s)

    def __setitem__(self, s, value):  # GaussPy[o][s] = array: the level's new contents
        self._owner._level(self._o, s)[...] = value

    def __len__(self):
        return self._owner.S + 3


class GaussPyramid:
    """GPU mirror of `class GaussPyramid` (GuassDePyramid.h:11-29); see the module docstring."""

    def __init__(self, img=None, len=None, S=2, device=0, defer=False):  # noqa: A002  (reference argument name)
        # GaussPyramid() (GuassDePyramid.h:31-34): empty object
        self.data = None
        self.initialized = False
        self._defer = False
        if img is None:
            return
        length = int(len)
        # :38-46 deep copy of img[0:len][0:len] (img may be larger, as in main.cpp:27-35,61)
        self.data = np.array([np.asarray(img[i][:length], dtype=np.int32) for i in range(length)], dtype=np.int32)
        self.length = length
        self.S = int(S)
        self.layer = octaves_for(length)  # :48-53
        self._ctx = PyramidContext(length, length, self.S, self.layer, batch=1, device=device)
        self._cache = {}  # (o, s) -> the level's host array (live for the object's lifetime)
        self._snap = {}  # (o, s) -> the bits the device last gave that array (edit detection)
        self._raw = None  # one host buffer in the device's raw image layout; the levels are views
        self._fresh = False
        self.uploaded_levels = 0  # levels the last SyncDevice uploaded (0: the host held no edits)
        if defer:
            # deferred download (round 6, the C++ classes' DeferDownload): the levels are views of a
            # write-tracked mirror (gdp_host_alloc_tracked) whose pages are fetched from the device
            # when first touched after a call; edits are found by page faults, not by comparison
            self._raw = np.asarray(_TrackedBuffer(lib().gdp_image_floats(self._ctx._ctx)))
            self._defer = True
            self.uploaded_bytes = 0
        self.GaussPyInit()  # :57

    # reference surface -------------------------------------------------------
    def GaussPyInit(self):
        """:60-87 — refill every level of every octave with the decimated CURRENT `data` (:80)."""
        self._ctx.set_input(self.data)
        self._ctx.init()
        self.initialized = True
        self._fresh = True  # contents == init, so GenerateDoG may take the fused path
        self._refresh()  # every level refilled: host edits are overwritten, as in :76-86

    def GaussFilter(self, theLayer):
        """:106-134 — multiply every scale of octave `theLayer` by its window, in place."""
        self.SyncDevice()
        self._ctx.gauss_octave(int(theLayer))
        self._fresh = False
        self._refresh()

    def GenerateDoG(self):
        """:136-149 — GaussFilter + DoG for every octave, in place on the current contents."""
        self.SyncDevice()
        if self._fresh:
            self._ctx.build()  # fused init+filter+DoG: bit-identical to the in-place sequence
        else:
            self._ctx.generate_dog()
        self._fresh = False
        self._refresh()

    def output(self, file=None):
        """:89-104 — print scale 0 of each octave (space separated) and an `==` separator row."""
        file = sys.stdout if file is None else file
        n = self.length
        for o in range(self.layer):
            lev = self._level(o, 0)
            for row in lev:
                file.write("".join(f"{v:g} " for v in row) + "\n")
            file.write("==" * n + "\n")
            n //= 2

    @property
    def GaussPy(self):
        return [_LevelView(self, o) for o in range(self.layer)]

    def SyncDevice(self):
        """Upload every level the caller obtained through GaussPy AND changed (its bits differ from
        the device's last copy) into the device pyramid; the next call processes the host contents.
        Sets `uploaded_levels`.  With defer=True: the pages written since the last call
        (`uploaded_bytes`; `uploaded_levels` is 0 when nothing was written, else -1)."""
        if self._defer:
            w = ctypes.c_size_t()
            written = w.value if lib().gdp_host_written_bytes(_ptr(self._raw), ctypes.byref(w)) == 0 else None
            check(lib().gdp_upload_image_written(self._ctx._ctx, 0, _ptr(self._raw)), self._ctx._ctx)
            self.uploaded_bytes = written
            self.uploaded_levels = 0 if written == 0 else -1
            if written != 0:
                self._fresh = False
            return
        n = 0
        for key, arr in self._cache.items():
            snap = self._snap[key]
            if not np.array_equal(arr.view(np.uint32), snap.view(np.uint32)):
                self._ctx.upload_level(0, key[0], key[1], arr)
                snap[...] = arr
                n += 1
        self.uploaded_levels = n
        if n:
            self._fresh = False  # the caller's contents, not necessarily GaussPyInit's

    # helpers -----------------------------------------------------------------
    def _level(self, o, s):
        key = (o, s)
        if key not in self._cache and self._defer:  # a view of the deferred mirror: fetched on touch
            rows, cols = self._ctx.level_dims(o)[:2]
            off = self._ctx.level_offset(0, o, s)
            self._cache[key] = self._raw[off:off + rows * cols].reshape(rows, cols)
        if key not in self._cache:
            if self._raw is None:
                self._raw = np.empty(lib().gdp_image_floats(self._ctx._ctx), np.float32)
            rows, cols = self._ctx.level_dims(o)[:2]
            off = self._ctx.level_offset(0, o, s)
            arr = self._raw[off:off + rows * cols].reshape(rows, cols)
            self._ctx.sync()
            if arr.size:
                check(lib().gdp_download_level(self._ctx._ctx, 0, int(o), int(s), _ptr(arr)), self._ctx._ctx)
            self._cache[key] = arr
            self._snap[key] = arr.copy()
        return self._cache[key]

    def _refresh(self):
        """After a device-side change: every touched level re-downloaded INTO its existing array,
        so handles the caller holds stay live (the reference's rows never move) — in one raw copy
        of the image when the touched levels are at least half of its bytes, else level by level.
        With defer=True: nothing is copied — the mirror is deferred (gdp_host_defer)."""
        if self._defer:
            self._ctx.sync()
            check(lib().gdp_host_defer(self._ctx._ctx, 0, _ptr(self._raw)), self._ctx._ctx)
            return
        if not self._cache:
            return
        self._ctx.sync()
        touched = sum(arr.size for arr in self._cache.values())
        if 2 * touched >= self._raw.size:
            check(lib().gdp_download_image_raw(self._ctx._ctx, 0, _ptr(self._raw)), self._ctx._ctx)
        else:
            for (o, s), arr in self._cache.items():
                if arr.size:
                    check(lib().gdp_download_level(self._ctx._ctx, 0, int(o), int(s), _ptr(arr)), self._ctx._ctx)
        for key, arr in self._cache.items():
            self._snap[key][...] = arr

    def pyramid(self):
        """Packed [o][s][r][c] float32 copy (the oracle's layout)."""
        return self._ctx.pyramid(0)

    def close(self):
        if getattr(self, "_ctx", None) is not None:
            self._ctx.close()


class GaussPyramid_a512omp(GaussPyramid):
    """GPU mirror of `class GaussPyramid_a512omp` (GaussDePyramid-AVX512xOpenMP.h:20-48), the
    reference's timed AVX-512 x OpenMP path; same object model as GaussPyramid (include/
    GaussDePyramid-HIP-AVX512.h is the C++ form).  Window centre: that header's integer length."""

    counnt = 2  # GaussDePyramid-AVX512xOpenMP.h:18 (a global there; no effect on the GPU)

    def __init__(self, img=None, len=None, S=2, device=0, defer=False):  # noqa: A002
        super().__init__(img, len, S, device, defer)
        if img is not None:
            self._ctx.set_window_centre("intlen")

    def GaussFilter(self, theLayer):
        """:128-181 — the reference's body is commented out: nothing happens."""

    def GenerateDoG(self):
        """:183-213 — DoG pass only (level j -= level j+1, j = 0..S+1) per octave, twice on octaves
        of side <= 2."""
        self.SyncDevice()
        self._ctx.dog_range(0, self.layer)  # one launch for every octave ...
        tiny = next((o for o in range(self.layer) if self.length >> o <= 2), self.layer)
        if tiny < self.layer:
            self._ctx.dog_range(tiny, self.layer)  # ... and one for the repeat on sides <= 2
        self._fresh = False
        self._refresh()

    def GenerateDoG_nomp_dynamic(self):
        """:240-364 — scales 0..S-1 windowed, DoG for i < S-1: {DoG_0..DoG_{S-2}, G_{S-1}, x, x, x}."""
        self.SyncDevice()
        if self._fresh:
            self._ctx.build_subset()
        else:
            self._ctx.generate_dog_subset()
        self._fresh = False
        self._refresh()

    def GenerateDoG_nomp_static(self):
        """:366-368 — empty in the reference."""


class GaussPyramid_a512xp(GaussPyramid):
    """GPU mirror of `class GaussPyramid_a512xp` (GaussDePyramid-AVX512xPTHREAD.h:21-40): full
    semantics; GenerateDoG with that header's integer-length centre (:193, :218), GaussFilter with
    the serial float-halved one (:113-141)."""

    def __init__(self, img=None, len=None, S=2, device=0, defer=False):  # noqa: A002
        super().__init__(img, len, S, device, defer)
        if img is not None:
            self._ctx.set_window_centre("intlen")

    def GaussFilter(self, theLayer):
        self._ctx.set_window_centre("serial")
        try:
            super().GaussFilter(theLayer)
        finally:
            self._ctx.set_window_centre("intlen")
