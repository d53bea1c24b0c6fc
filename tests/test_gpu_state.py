"""GaussPy as two-way state.

In the reference, `float**** GaussPy` IS the pyramid: GaussFilter / GenerateDoG work on whatever
the caller left in it (GuassDePyramid.h:16, :122-131, :140-146), and GaussPyInit re-reads `data`
(:80).  These tests edit the drop-ins' GaussPy (C++ classes through examples/state_hip, the Python
mirror directly) between calls — a level zeroed, a row scaled, a level negated, single values up
to FLT_MAX, a re-seated row pointer, an edited input pixel — and require the result to be
bit-identical (0 ULP) to the oracle's in-place restatement (gauss_octave / generate_dog /
GenerateDoG_nomp_dynamic's subset) applied to the same edited pyramid.  Runs on an MI355X.
"""
import os
import re
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(REPO, "examples", "state_hip")
EXE_MPITEST = os.path.join(REPO, "examples", "mpitest_hip")


def _bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


def _assert_same(got, want, what):
    g, w = _bits(got), _bits(want)
    assert g.shape == w.shape, (what, g.shape, w.shape)
    bad = np.flatnonzero(g.ravel() != w.ravel())
    assert bad.size == 0, f"{what}: {bad.size} words differ, first at {bad[:5]}"


class _Replay:
    """The oracle side of a state_hip op list: the same edits and calls on a packed pyramid."""

    def __init__(self, oracle, cls, n, S, spec):
        self.o, self.cls, self.n, self.S = oracle, cls, n, S
        self.O = oracle.octaves(n)
        self.img = oracle.image_from_spec(n, spec).astype(np.int32)
        self.pyr = oracle.init_pyramid(self.img, S)
        self.mirror, self.dirty = True, False
        self.host = self.pyr.copy()  # what GaussPy holds on the host

    def _lv(self, pyr, o, s):
        return self.o.levels(pyr, self.n, self.n, self.S, self.O)[(o, s)]

    def _pull(self):  # before a mutating call: GaussPy is uploaded when mirrored or flagged
        if self.mirror or self.dirty:
            self.pyr[:] = self.host
            self.dirty = False

    def _push(self):
        # mpitest.cpp's free functions always leave their result in the global GaussPy
        if self.mirror or self.cls == "mpitest":
            self.host[:] = self.pyr

    def apply(self, op):
        f = op.split(":")
        n, S, O, o = self.n, self.S, self.O, self.o
        intlen = "intlen" if self.cls in ("a512omp", "a512xp", "mpitest") else "serial"
        if f[0] == "init":
            self.pyr[:] = o.init_pyramid(self.img, S)
            self.dirty = False
            self._push()
        elif f[0] in ("dog", "mpi", "omp", "nomp", "filter"):
            self._pull()
            if f[0] == "filter":
                if self.cls != "a512omp":  # that class's GaussFilter is empty (:128-181)
                    o.gauss_octave(self.pyr, n, n, S, int(f[1]))
            elif f[0] in ("mpi", "omp"):
                o.generate_dog(self.pyr, n, n, S, O, centre="intlen")
            elif f[0] == "nomp":
                o.subset_a512omp(self.pyr, n, n, S, O)
            elif self.cls == "a512omp":
                o.generate_dog_a512omp(self.pyr, n, n, S, O)
            else:
                o.generate_dog(self.pyr, n, n, S, O, centre=intlen)
            self._push()
        elif f[0] == "mirror":
            self.mirror = f[1] == "1"
        elif f[0] == "dirty":
            self.dirty = True
        elif f[0] == "syncdev":
            self.pyr[:] = self.host
            self.dirty = False
        elif f[0] == "synchost":
            self.host[:] = self.pyr
        elif f[0] == "data":
            self.img[int(f[1]), int(f[2])] = int(f[3])
        elif f[0] in ("reseat", "track", "written", "defer", "stale", "read", "readmt"):
            pass  # same contents, another address / the upload or download strategy / a report
        else:
            lv = self._lv(self.host, int(f[1]), int(f[2]))
            if f[0] in ("neg", "negmt"):
                lv[:] = -lv
            elif f[0] == "zero":
                lv[:] = 0.0
            elif f[0] == "scale":
                lv[int(f[3])] *= np.float32(float(f[4]))
            elif f[0] == "set":
                lv[int(f[3]), int(f[4])] = np.float32(float(f[5]))
        return self


def _assert_same_nan(got, want, what):
    """Bit-exact except NaN payloads: inf * 0 gives the default NaN of the machine that computes
    it (x86 SSE: 0xFFC00000, gfx950: 0x7FC00000), so NaNs compare by position only."""
    g, w = _bits(got).copy(), _bits(want).copy()
    gn, wn = np.isnan(g.view(np.float32)), np.isnan(w.view(np.float32))
    assert np.array_equal(gn, wn), (what, "NaN positions differ", np.flatnonzero(gn != wn)[:5])
    g[gn] = w[wn] = 0x7FC00000
    _assert_same(g.view(np.float32), w.view(np.float32), what)


def _run(oracle, tmp_path, cls, n, S, spec, ops, want_stale=False):
    if not os.path.exists(EXE):
        subprocess.run(["make", "-s", "-C", os.path.join(REPO, "examples")], check=True)
    out = tmp_path / "state.f32"
    r = subprocess.run([EXE, cls, str(n), str(S), spec, str(out), *ops], check=True, timeout=120, capture_output=True,
                       text=True)
    rp = _Replay(oracle, cls, n, S, spec)
    for op in ops:
        rp.apply(op)
    _assert_same(np.fromfile(out, dtype=np.float32), rp.host, (cls, n, S, ops))
    if want_stale:
        return ([int(x) for x in re.findall(r"written=(-?\d+)", r.stderr)],
                [int(x) for x in re.findall(r"stale=(-?\d+)", r.stderr)])
    return [int(x) for x in re.findall(r"written=(-?\d+)", r.stderr)]


EDITS = ["zero:0:1", "scale:0:2:5:-3.5", "neg:1:0", "set:0:0:3:7:-1e30", "set:2:3:1:1:3.0e38"]


@pytest.mark.parametrize("n,S", [(64, 2), (100, 2), (96, 3)])
def test_cpp_class_processes_host_edits(oracle, tmp_path, n, S):
    """GaussPyramid_hip with the default mirror_host: edits of GaussPy between calls are what
    GaussFilter / GenerateDoG / GenerateDoG_mpi process, and GaussPyInit discards them."""
    _run(oracle, tmp_path, "hip", n, S, "lcg:3", EDITS + ["filter:0", "filter:1", "neg:0:4", "dog"])
    _run(oracle, tmp_path, "hip", n, S, "lcg:4", ["dog"] + EDITS + ["dog", "scale:1:1:0:0.25", "mpi"])
    _run(oracle, tmp_path, "hip", n, S, "lcg:5", EDITS + ["init", "dog"])  # refill overwrites the edits
    _run(oracle, tmp_path, "hip", n, S, "lcg:6", ["data:3:5:-70000", "data:0:0:2147483647", "init", "zero:0:4", "dog"])


def test_cpp_class_write_tracked_mirror_uploads_what_was_written(oracle, tmp_path):
    """the default mirror is write-tracked (gdp_host_track) — after each call
    it is write-protected, a CPU write faults once and is recorded, and the next call uploads only
    the written pages.  A single float written after a call (after SyncHost) is processed; a call
    with nothing written uploads nothing; edits spanning levels, GaussPyInit, GaussFilter, the MPI
    entry, TrackWrites(false / true) and mirror_host toggles all stay bit-identical to the oracle."""
    page = os.sysconf("SC_PAGESIZE")
    n, S = 64, 2
    w = _run(oracle, tmp_path, "hip", n, S, "lcg:13", ["written", "dog", "written", "set:0:0:3:7:-1e30", "written",
                                                        "dog", "written", "dog", "written"])
    assert w == [0, 0, page, 0, 0], w
    w = _run(oracle, tmp_path, "hip", n, S, "lcg:14", ["dog", "synchost", "set:2:4:1:1:5.5", "written", "filter:2",
                                                        "written", "zero:0:1", "neg:1:3", "mpi", "written"])
    assert w[0] == page and w[1] == 0 and w[2] == 0, w
    w = _run(oracle, tmp_path, "hip", 100, S, "lcg:15", ["track:0", "written", "set:0:0:3:7:1e20", "dog", "track:1",
                                                         "written", "neg:0:0", "dog", "written", "scale:1:1:2:-2",
                                                         "written", "dog"])
    assert w[0] == -1 and w[1] == -1 and w[2] == 0 and w[3] > 0, w  # untracked: whole uploads
    w = _run(oracle, tmp_path, "hip", n, S, "lcg:16", ["dog", "mirror:0", "set:0:0:0:0:9", "dog", "mirror:1", "written",
                                                       "neg:0:2", "dog", "written"])
    assert w == [-1, 0], w  # a call without the mirror disarms: the next mirrored call uploads all
    w = _run(oracle, tmp_path, "a512xp", n, S, "lcg:17", ["dog", "set:0:1:2:2:-4", "written", "filter:0", "dog"])
    assert w == [page], w
    w = _run(oracle, tmp_path, "hip", n, S, "lcg:18", EDITS + ["init", "written", "set:0:0:3:7:2", "dog", "dog"])
    assert w == [0], w


def test_cpp_class_without_mirror_uploads_only_when_told(oracle, tmp_path):
    """mirror_host = false: the device pyramid is the state; host edits reach it only through
    host_dirty (next call uploads first) or SyncDevice(), and SyncHost() overwrites the host."""
    n, S = 64, 2
    _run(oracle, tmp_path, "hip", n, S, "lcg:7", ["mirror:0", "zero:0:1", "dog", "synchost"])  # edit never uploaded
    _run(oracle, tmp_path, "hip", n, S, "lcg:7", ["mirror:0", "zero:0:1", "dirty", "dog", "synchost"])
    _run(oracle, tmp_path, "hip", n, S, "lcg:7", ["mirror:0", "neg:0:2", "syncdev", "filter:0", "synchost"])
    _run(oracle, tmp_path, "hip", n, S, "lcg:7", ["mirror:0", "dog", "synchost", "scale:0:0:31:2", "dirty", "dog",
                                                  "synchost"])


def test_cpp_class_honours_reseated_rows(oracle, tmp_path):
    """A caller may point GaussPy[o][s][r] at another array (the reference's rows are separate
    new[] arrays): both directions then go through the staged row copies, not the raw mirror."""
    _run(oracle, tmp_path, "hip", 64, 2, "lcg:8", ["reseat:0:1:7", "scale:0:1:7:-2", "dog", "scale:0:0:7:4", "dog"])
    _run(oracle, tmp_path, "hip", 100, 2, "lcg:9", ["reseat:2:0:0", "reseat:0:4:99", "set:0:4:99:50:1e20", "filter:0",
                                                    "filter:2", "dog"])


def test_cpp_avx512_classes_process_host_edits(oracle, tmp_path):
    """GaussPyramid_a512omp_hip (GenerateDoG_nomp_dynamic's subset; GenerateDoG = DoG only) and
    GaussPyramid_a512xp_hip (integer-length GenerateDoG, serial GaussFilter) on edited state."""
    for n in (64, 8):
        _run(oracle, tmp_path, "a512omp", n, 2, "lcg:10", ["zero:0:0", "neg:0:3", "nomp", "scale:0:1:2:3", "nomp"])
        _run(oracle, tmp_path, "a512omp", n, 2, "lcg:11", ["neg:0:2", "dog", "filter:0", "set:1:4:1:1:-5", "dog"])
        _run(oracle, tmp_path, "a512xp", n, 2, "lcg:12", ["zero:1:1", "scale:0:0:1:-1", "dog", "neg:0:0", "filter:0",
                                                          "dog"])


def _run_mpitest(oracle, tmp_path, n, S, spec, ops):
    if not os.path.exists(EXE_MPITEST):
        subprocess.run(["make", "-s", "-C", os.path.join(REPO, "examples")], check=True)
    out = tmp_path / "mpitest.f32"
    subprocess.run([EXE_MPITEST, str(n), spec, str(out), "mpi", str(S), *ops], check=True, timeout=120,
                   capture_output=True)
    rp = _Replay(oracle, "mpitest", n, S, spec)
    rp.apply("init")  # the driver's own GaussPyInit(p) before the ops
    for op in ops:
        rp.apply(op)
    _assert_same(np.fromfile(out, dtype=np.float32), rp.host, ("mpitest", n, S, ops))


@pytest.mark.parametrize("n,S", [(64, 2), (100, 2), (96, 3)])
def test_cpp_mpitest_free_functions_process_host_edits(oracle, tmp_path, n, S):
    """mpitest.cpp's GenerateDoG_mpi / _omp multiply and subtract the GLOBAL
    GaussPy in place (mpitest.cpp:128-133, :165), so an edit written between GaussPyInit(p) and
    GenerateDoG_mpi is processed.  The drop-in header (include/GaussDePyramid-HIP-mpitest.h) uploads
    GaussPy before each call and runs the in-place pass: a zeroed level, scaled rows, negated
    levels, values near FLT_MAX, re-seated rows -> bit-identical to the oracle's in-place
    generate_dog with the integer-length centre on the same edited pyramid."""
    _run_mpitest(oracle, tmp_path, n, S, "lcg:31", EDITS + ["mpi"])
    _run_mpitest(oracle, tmp_path, n, S, "lcg:32", ["mpi"] + EDITS + ["omp", "neg:0:0", "mpi"])
    _run_mpitest(oracle, tmp_path, n, S, "lcg:33", EDITS + ["init", "mpi"])  # the refill overwrites the edits
    _run_mpitest(oracle, tmp_path, n, S, "lcg:34", ["reseat:0:1:3", "scale:0:1:3:-2", "omp", "reseat:1:0:0",
                                                   "set:1:0:0:1:1e20", "mpi"])


def test_cpp_mpitest_without_mirror_uploads_only_when_told(oracle, tmp_path):
    """gdp_mpitest_mirror_host = false: edits reach the device only with host_dirty / SyncDevice;
    the result is still left in GaussPy after every call (mpitest.cpp's callers read it)."""
    n, S = 64, 2
    _run_mpitest(oracle, tmp_path, n, S, "lcg:35", ["mirror:0", "zero:0:1", "mpi"])  # edit never uploaded
    _run_mpitest(oracle, tmp_path, n, S, "lcg:35", ["mirror:0", "zero:0:1", "dirty", "mpi"])
    _run_mpitest(oracle, tmp_path, n, S, "lcg:35", ["mirror:0", "neg:0:2", "syncdev", "omp", "scale:0:0:5:3",
                                                   "synchost", "mpi"])


def test_cpp_mpitest_deferred_download(oracle, tmp_path):
    """gdp_mpitest_defer_download: GaussPyInit / GenerateDoG_* leave the global GaussPy to be
    fetched on first touch; edits, re-seated rows, the mirror off and the flag toggled in between
    give the eager mirror's bits."""
    n, S = 64, 2
    _run_mpitest(oracle, tmp_path, n, S, "lcg:36", ["defer:1", "init", "mpi"] + EDITS + ["omp", "neg:0:0", "mpi"])
    _run_mpitest(oracle, tmp_path, n, S, "lcg:37", ["defer:1", "mpi", "mirror:0", "zero:0:1", "mpi", "dirty",
                                                   "scale:0:0:5:3", "mpi", "mirror:1", "defer:0", "set:1:2:3:4:5",
                                                   "omp", "defer:1", "reseat:0:1:3", "scale:0:1:3:-2", "mpi"])
    _run_mpitest(oracle, tmp_path, 100, S, "lcg:38", ["defer:1", "init", "syncdev", "mpi", "synchost", "neg:1:1",
                                                     "mpi"])


@pytest.mark.parametrize("defer", [False, True])
def test_python_mirror_processes_host_edits(pkg, oracle, defer):
    """The Python GaussPyramid: writes through GaussPy[o][s] (element, row, whole level) and into
    `data` are processed by the next call, like the reference's float**** and data copy (with
    defer=True: on the deferred, write-tracked mirror)."""
    n, S = 100, 2
    O = oracle.octaves(n)
    img = oracle.lcg_image(n, n, 21)
    g = pkg.GaussPyramid(img, n, S, defer=defer)
    want = oracle.init_pyramid(img, S)
    lv = lambda p, o, s: oracle.levels(p, n, n, S, O)[(o, s)]  # noqa: E731
    g.GaussPy[0][1][5] *= np.float32(-3)
    lv(want, 0, 1)[5] *= np.float32(-3)
    g.GaussPy[1][0] = np.full((n >> 1, n >> 1), 2.5, np.float32)
    lv(want, 1, 0)[:] = 2.5
    g.GaussPy[0][3][10, 20] = np.float32(3e38)
    lv(want, 0, 3)[10, 20] = np.float32(3e38)
    g.GaussFilter(0)
    oracle.gauss_octave(want, n, n, S, 0)
    _assert_same(g.pyramid(), want, "python GaussFilter after edits")
    g.GaussPy[0][0][:] = 0
    lv(want, 0, 0)[:] = 0
    g.GenerateDoG()
    oracle.generate_dog(want, n, n, S, O)
    _assert_same(g.pyramid(), want, "python GenerateDoG after edits")
    g.data[7, 9] = -123456
    img2 = img.copy()
    img2[7, 9] = -123456
    g.GaussPyInit()
    g.GenerateDoG()
    _assert_same(g.pyramid(), oracle.build_pyramid(img2, S), "python GaussPyInit re-reads data")
    g.close()


@pytest.mark.parametrize("defer", [False, True])
def test_python_mirror_handles_stay_live_and_reads_upload_nothing(pkg, oracle, defer):
    """a GaussPy[o][s] array taken before a call is the same live array after it (the
    reference's rows never move): it reads the new contents, and writes through it — including
    ones __setitem__ never sees (a row view, a ufunc with out=) — are processed by the next call.
    Levels only read (output() included) are not uploaded, so GaussPyInit + reads + GenerateDoG
    still takes the fused build; an unchanged pyramid uploads nothing."""
    import io

    n, S = 64, 2
    O = oracle.octaves(n)
    img = oracle.lcg_image(n, n, 41)
    g = pkg.GaussPyramid(img, n, S, defer=defer)
    lv = lambda p, o, s: oracle.levels(p, n, n, S, O)[(o, s)]  # noqa: E731
    a = g.GaussPy[0][0]  # taken before any call
    b = g.GaussPy[1][2]
    g.output(file=io.StringIO())  # reads level (o, 0) of every octave
    g.SyncDevice()
    assert g.uploaded_levels == 0 and g._fresh  # reads uploaded nothing: GenerateDoG takes the fused build
    g.GenerateDoG()
    want = oracle.build_pyramid(img, S)
    _assert_same(a, lv(want, 0, 0), "old handle reads the new level (0, 0)")
    _assert_same(b, lv(want, 1, 2), "old handle reads the new level (1, 2)")
    assert g.GaussPy[0][0] is a
    row = a[3]
    row *= np.float32(-2)  # through a view: no __setitem__ on `a`
    np.multiply(b, np.float32(0.5), out=b)
    lv(want, 0, 0)[3] *= np.float32(-2)
    lv(want, 1, 2)[:] *= np.float32(0.5)
    g.GenerateDoG()
    assert g.uploaded_levels == (-1 if defer else 2)  # deferred mirror: pages, not levels, are tracked
    oracle.generate_dog(want, n, n, S, O)
    _assert_same(g.pyramid(), want, "edits through old handles processed")
    _assert_same(a, lv(want, 0, 0), "handle refreshed after the second call")
    g.GenerateDoG()
    assert g.uploaded_levels == 0  # the host mirror equals the device: nothing to upload
    oracle.generate_dog(want, n, n, S, O)
    _assert_same(g.pyramid(), want, "third call")
    a[:] = 7.0  # edit, then GaussPyInit overwrites it (the refill, :76-86)
    g.GaussPyInit()
    _assert_same(a, lv(oracle.init_pyramid(img, S), 0, 0), "GaussPyInit refreshed the handle")
    g.close()


@pytest.mark.parametrize("H,W,S,B,centre,zw", [(4096, 4096, 2, 1, "serial", 1), (300, 500, 3, 2, "intlen", 0),
                                                (1080, 1920, 2, 2, "serial", 1), (7, 5, 0, 1, "serial", 0)])
def test_generate_dog_mirrored_equals_upload_pass_download(pkg, oracle, H, W, S, B, centre, zw):
    """gdp_generate_dog_mirrored (the drop-ins' GenerateDoG on a mirrored GaussPy: upload, in-place
    pass and download pipelined over row chunks on three streams) == gdp_upload_image_raw +
    gdp_generate_dog + gdp_download_image_raw, bit for bit, on an edited pyramid (values up to 3e38,
    negatives, zeros), for the image it names only; the other images of the batch are untouched."""
    import ctypes

    L = pkg.lib()
    rng = np.random.default_rng(H + W + S)
    with pkg.PyramidContext(H, W, S=S, batch=B) as a, pkg.PyramidContext(H, W, S=S, batch=B) as m:
        n = L.gdp_image_floats(a._ctx)
        raw = []
        for b in range(B):
            img = oracle.lcg_image(H, W, 50 + b)
            for c in (a, m):
                c.set_window_centre(centre)
                c.set_tuning(zero_window=zw)
                c.set_input(img, b)
        for c in (a, m):
            c.build()
            c.sync()
        for b in range(B):
            r = np.empty(n, np.float32)
            assert L.gdp_download_image_raw(a._ctx, b, r.ctypes.data_as(ctypes.c_void_p)) == 0
            r[rng.integers(0, n, 64)] = np.float32(3e38)
            r[rng.integers(0, n, 64)] *= np.float32(-7.5)
            r[rng.integers(0, n, 64)] = 0.0
            raw.append(r)
            for c in (a, m):
                assert L.gdp_upload_image_raw(c._ctx, b, r.ctypes.data_as(ctypes.c_void_p)) == 0
        tgt = B - 1
        a.generate_dog()  # every image of the batch; only image tgt is compared
        a.sync()
        want = np.empty(n, np.float32)
        assert L.gdp_download_image_raw(a._ctx, tgt, want.ctypes.data_as(ctypes.c_void_p)) == 0
        hptr = ctypes.c_void_p()
        assert L.gdp_host_alloc(n * 4, ctypes.byref(hptr)) == 0
        try:
            host = np.ctypeslib.as_array(ctypes.cast(hptr, ctypes.POINTER(ctypes.c_float)), shape=(n,))
            host[:] = raw[tgt]
            assert L.gdp_generate_dog_mirrored(m._ctx, tgt, hptr) == 0
            spans = [(m.level_offset(0, o, s), m.level_dims(o)[0] * m.level_dims(o)[1])
                     for o in range(m.O) for s in range(S + 3)]
            for off, cnt in spans:  # the level extents (the padding between levels is never written)
                _assert_same_nan(host[off:off + cnt], want[off:off + cnt], ("host", H, W, off))
            got = np.empty(n, np.float32)
            assert L.gdp_download_image_raw(m._ctx, tgt, got.ctypes.data_as(ctypes.c_void_p)) == 0
            for off, cnt in spans:
                _assert_same_nan(got[off:off + cnt], want[off:off + cnt], ("device", H, W, off))
            for b in range(B - 1):  # untouched
                assert L.gdp_download_image_raw(m._ctx, b, got.ctypes.data_as(ctypes.c_void_p)) == 0
                for off, cnt in spans:
                    _assert_same_nan(got[off:off + cnt], raw[b][off:off + cnt], ("other image", b))
        finally:
            L.gdp_host_free(hptr)


def test_inplace_zero_window_is_exact_for_caller_values_near_flt_max(pkg, oracle):
    """with S >= 3 some column taps exceed 1, so for a row outside the window support
    (fr = +0) v * fc can overflow to inf and inf * 0 = NaN — the zero-window shortcut of the
    in-place passes must not turn that into a zero.  A caller-written 3e38 at such a pixel, then
    GaussFilter / GenerateDoG re-entry with the knob on == the oracle (bits incl. NaN)."""
    n, S = 255, 3  # odd side: the window centre falls on a pixel, where scale 5's tap is 1.197
    O = oracle.octaves(n)
    img = oracle.lcg_image(n, n, 5)
    base = oracle.build_pyramid(img, S)
    lv = lambda p, o, s: oracle.levels(p, n, n, S, O)[(o, s)]  # noqa: E731
    c = (n - 1) // 2
    assert oracle.taps(n, 0, S + 2)[c] > 1.0
    for s in range(S + 3):
        lv(base, 0, s)[0, c] = np.float32(3.0e38)   # row 0: outside every row window; column: centre
        lv(base, 0, s)[1, c + 1] = np.float32(-3.0e38)
        lv(base, 0, s)[c, 0] = np.float32(3.0e38)   # column 0 outside: exact either way
    with pkg.PyramidContext(n, n, S=S) as ctx:
        for zw in (0, 1):
            ctx.set_tuning(zero_window=zw)
            for sub, wsub in ((1, 4), (0, 1), (16, 16), (-16, 8)):
                ctx.set_tuning(inplace_sub=sub, window_sub=wsub)
                ctx.upload_pyramid(base)
                ctx.gauss_octave(0)
                ctx.sync()
                _assert_same_nan(ctx.pyramid(0), oracle.gauss_octave(base.copy(), n, n, S, 0), ("gauss", zw, sub, wsub))
                ctx.upload_pyramid(base)
                ctx.generate_dog()
                ctx.sync()
                _assert_same_nan(ctx.pyramid(0), oracle.generate_dog(base.copy(), n, n, S, O), ("regen", zw, sub))
    assert np.isnan(lv(oracle.gauss_octave(base.copy(), n, n, S, 0), 0, S + 2)[0, c])  # the case exists


def test_reference_role_map_steps_on_the_gpu(pkg, oracle):
    """The reference's role map (GaussDePyramid-MPI.h:265-335), its two device steps on one GPU:
    each worker's gdp_gauss_scales(i, i+1) of its own pyramid (integer-length centre) == the
    worker state the reference leaves (scale i windowed, the others at GaussPyInit values), and the
    collector's DoG pass over the S+3 workers' scales == the reference collector's pyramid
    (tests/golden/mpi_hashes.json).  The RCCL transport between them (gdp_comm_collect_scales) needs
    >= S+4 GPUs; its schedule is tested on CPU (tests/test_distributed.py)."""
    import importlib
    import json

    import torch

    d = importlib.import_module(pkg.__name__ + ".distributed")
    with open(os.path.join(REPO, "tests", "golden", "mpi_hashes.json")) as f:
        recs = [r for r in json.load(f) if r["variant"] == "GaussDePyramid-MPI.h:GenerateDoG_mpi"]
    for rec in recs:
        n, S, spec = rec["n"], rec["S"], rec["input"]
        O = oracle.octaves(n)
        img = oracle.image_from_spec(n, spec)
        scale_compute, collect = d._gpu_role_compute(n, S, O, 0)
        init = oracle.levels(oracle.init_pyramid(img, S), n, n, S, O)
        scales = []
        for i in range(S + 3):
            lv = scale_compute(img, i)
            for o in range(O):  # the worker's own scale: (x * fc) * fr with the variant's centre
                fc = oracle.taps(n, o, i, centre="intlen")
                want = (init[(o, i)] * fc[None, :]) * fc[:, None]
                _assert_same(lv[o].cpu().numpy(), want.astype(np.float32).ravel(), ("worker", n, i, o))
            scales.append([t.clone() for t in lv])
        got = collect(scales).cpu().numpy()
        lvs = oracle.levels(got, n, n, S, O)
        for o, row in enumerate(rec["octaves"]):
            for s, h in enumerate(row):
                assert oracle.fnv(lvs[(o, s)]) == int(h, 16), ("collector", n, S, spec, o, s)
        torch.cuda.synchronize()


def test_tracked_mirror_uploads_only_written_pages(pkg, oracle):
    """gdp_host_alloc_tracked: a shared-memory object mapped twice — a view
    registered with HIP for the DMA copies and the CPU view returned, the only one ever
    write-protected (protecting hipHostMalloc memory stalls the process's GPU queues, so
    gdp_host_track refuses it).  Downloads through the CPU view land in it; after arming, a
    single-float write is recorded as its page and gdp_generate_dog_mirrored_written == the
    whole-mirror gdp_generate_dog_mirrored on the same edited pyramid, bit for bit; with nothing
    written the next call uploads nothing and still equals the in-place pass on the device copy."""
    import ctypes

    L = pkg.lib()
    page = os.sysconf("SC_PAGESIZE")
    H = W = 512
    S = 2
    with pkg.PyramidContext(H, W, S=S) as a, pkg.PyramidContext(H, W, S=S) as m:
        n = L.gdp_image_floats(a._ctx)
        img = oracle.lcg_image(H, W, 77)
        for c in (a, m):
            c.set_input(img, 0)
            c.build()
            c.sync()
        pinned = ctypes.c_void_p()
        assert L.gdp_host_alloc(n * 4, ctypes.byref(pinned)) == 0
        try:
            assert L.gdp_host_track(pinned, n * 4) == 3  # registered with the GPU: refused
        finally:
            L.gdp_host_free(pinned)
        hptr = ctypes.c_void_p()
        assert L.gdp_host_alloc_tracked(n * 4, ctypes.byref(hptr)) == 0
        try:
            host = np.ctypeslib.as_array(ctypes.cast(hptr, ctypes.POINTER(ctypes.c_float)), shape=(n,))
            assert L.gdp_download_image_raw(m._ctx, 0, hptr) == 0  # DMA through the registered view
            ref = np.empty(n, np.float32)
            assert L.gdp_download_image_raw(a._ctx, 0, ref.ctypes.data_as(ctypes.c_void_p)) == 0
            _assert_same(host, ref, "download through the tracked mirror")
            written = ctypes.c_size_t()
            assert L.gdp_host_written_bytes(hptr, ctypes.byref(written)) == 3  # not armed yet
            assert L.gdp_host_arm(hptr) == 0
            assert L.gdp_host_written_bytes(hptr, ctypes.byref(written)) == 0 and written.value == 0
            off = m.level_offset(0, 0, 2) + 7 * W + 9
            host[off] = np.float32(-1e30)  # one float through the CPU view: faults once, recorded
            ref[off] = np.float32(-1e30)
            assert L.gdp_host_written_bytes(hptr, ctypes.byref(written)) == 0 and written.value == page
            # whole-mirror reference on context a: upload the edited copy, in-place pass, download
            assert L.gdp_generate_dog_mirrored(a._ctx, 0, ref.ctypes.data_as(ctypes.c_void_p)) == 0
            assert L.gdp_generate_dog_mirrored_written(m._ctx, 0, hptr) == 0
            _assert_same(host, ref, "written-page upload == whole upload after a one-float edit")
            assert L.gdp_host_written_bytes(hptr, ctypes.byref(written)) == 0 and written.value == 0  # re-armed
            assert L.gdp_generate_dog_mirrored(a._ctx, 0, ref.ctypes.data_as(ctypes.c_void_p)) == 0
            assert L.gdp_generate_dog_mirrored_written(m._ctx, 0, hptr) == 0  # nothing written: no upload
            _assert_same(host, ref, "no-write call")
            got = np.empty(n, np.float32)
            assert L.gdp_download_image_raw(m._ctx, 0, got.ctypes.data_as(ctypes.c_void_p)) == 0
            _assert_same(got, ref, "device copy")
            host[: W] = np.float32(2.5)  # a row through the CPU view, then gdp_upload_image_written
            ref[: W] = np.float32(2.5)
            assert L.gdp_upload_image_written(m._ctx, 0, hptr) == 0
            assert L.gdp_download_image_raw(m._ctx, 0, got.ctypes.data_as(ctypes.c_void_p)) == 0
            _assert_same(got, ref, "gdp_upload_image_written")
            # single-level copies given an address inside the mirror DMA through its registered view:
            # level (0, 0) of context a (which never saw the 2.5 row) into the mirror, then the mirror's
            # level up into m
            lo, (rows, cols) = a.level_offset(0, 0, 0), a.level_dims(0)[:2]
            want = np.empty(rows * cols, np.float32)
            assert L.gdp_download_level(a._ctx, 0, 0, 0, want.ctypes.data_as(ctypes.c_void_p)) == 0
            assert L.gdp_download_level(a._ctx, 0, 0, 0, ctypes.c_void_p(hptr.value + 4 * lo)) == 0
            _assert_same(host[lo:lo + rows * cols], want, "gdp_download_level into the tracked mirror")
            assert L.gdp_upload_level(m._ctx, 0, 0, 0, ctypes.c_void_p(hptr.value + 4 * lo)) == 0
            lv = np.empty(rows * cols, np.float32)
            assert L.gdp_download_level(m._ctx, 0, 0, 0, lv.ctypes.data_as(ctypes.c_void_p)) == 0
            _assert_same(lv, want, "gdp_upload_level from the tracked mirror")
            ref[lo:lo + rows * cols] = want
            assert L.gdp_host_untrack(hptr) == 0  # writable, not recorded; the DMA view stays
            host[5] = np.float32(1.0)
            assert L.gdp_host_written_bytes(hptr, ctypes.byref(written)) == 3
            assert L.gdp_download_image_raw(m._ctx, 0, hptr) == 0
            _assert_same(host, ref, "download after untrack")
        finally:
            L.gdp_host_free(hptr)


def test_deferred_mirror_fetches_on_first_touch(pkg, oracle):
    """gdp_host_defer: the device pyramid is declared newer than the tracked mirror; every page of
    its CPU view is inaccessible until touched, and a touch fetches a block around it (64 pages,
    doubling while the faults walk forward).  Random reads through numpy equal the device copy
    while only part of the mirror has moved; a write is recorded as one page; a sequential pass
    fetches the rest in few, growing copies; an unrelated download leaves the deferral alone;
    gdp_destroy of the source context completes the mirror; buffers that cannot defer are refused."""
    import ctypes

    L = pkg.lib()
    page = os.sysconf("SC_PAGESIZE")
    H = W = 2048
    S = 2
    size_t = ctypes.c_size_t
    with pkg.PyramidContext(H, W, S=S) as a:
        n = L.gdp_image_floats(a._ctx)
        a.set_input(oracle.lcg_image(H, W, 91), 0)
        a.build()
        a.sync()
        ref = np.empty(n, np.float32)
        assert L.gdp_download_image_raw(a._ctx, 0, ref.ctypes.data_as(ctypes.c_void_p)) == 0
        pinned = ctypes.c_void_p()
        assert L.gdp_host_alloc(n * 4, ctypes.byref(pinned)) == 0
        try:
            assert L.gdp_host_defer(a._ctx, 0, pinned) == 3  # not a tracked alias: refused
        finally:
            L.gdp_host_free(pinned)
        hptr = ctypes.c_void_p()
        assert L.gdp_host_alloc_tracked(n * 4, ctypes.byref(hptr)) == 0
        try:
            host = np.ctypeslib.as_array(ctypes.cast(hptr, ctypes.POINTER(ctypes.c_float)), shape=(n,))
            stale, fetched, fetches = size_t(), size_t(), ctypes.c_uint64()

            def stats():
                assert L.gdp_host_deferred_stats(hptr, ctypes.byref(stale), ctypes.byref(fetched),
                                                 ctypes.byref(fetches)) == 0
                return stale.value, fetched.value, fetches.value

            assert L.gdp_host_defer(a._ctx, 0, hptr) == 0
            full = stats()[0]
            assert full >= n * 4 and full % page == 0, full
            rng = np.random.default_rng(5)
            idx = np.sort(rng.integers(0, n, 40))
            _assert_same(host[idx], ref[idx], "random reads of a deferred mirror")
            st, fb, nf = stats()
            assert 0 < nf <= 40 and 0 < fb < full // 2 and full - page < st + fb <= full, (st, fb, nf)
            # a download into other memory does not touch the deferral
            got = np.empty(n, np.float32)
            assert L.gdp_download_image_raw(a._ctx, 0, got.ctypes.data_as(ctypes.c_void_p)) == 0
            assert stats()[0] == st
            k = int(idx[3]) + 1
            host[k] = np.float32(-7.0)  # a fetched page: one more fault, recorded
            ref[k] = np.float32(-7.0)
            written = size_t()
            assert L.gdp_host_written_bytes(hptr, ctypes.byref(written)) == 0 and written.value == page
            _assert_same(host, ref, "whole deferred mirror after the touches")  # fetches the rest
            st, fb, nf = stats()
            # (a sequential copy stops at each block the random reads fetched and restarts with a
            # block and its read-ahead after it: a few more copies each)
            assert st == 0 and nf <= 4 * 40 + 40, (st, fb, nf)
            # the written page goes up with the next written-page upload; a pass and a new deferral
            assert L.gdp_upload_image_written(a._ctx, 0, hptr) == 0
            assert L.gdp_download_image_raw(a._ctx, 0, got.ctypes.data_as(ctypes.c_void_p)) == 0
            _assert_same(got, ref, "device after the written-page upload")
            assert L.gdp_generate_dog(a._ctx, None) == 0
            assert L.gdp_host_defer(a._ctx, 0, hptr) == 0  # not blocking: fetches queue behind the pass
            assert L.gdp_download_image_raw(a._ctx, 0, got.ctypes.data_as(ctypes.c_void_p)) == 0
            seen = np.empty(n, np.float32)
            for lo in range(0, n, 1 << 20):  # sequential reads: few, growing copies
                seen[lo:lo + (1 << 20)] = host[lo:lo + (1 << 20)]
            _assert_same(seen, got, "sequential reads of the deferred pass result")
            st, fb, nf = stats()
            assert st == 0 and nf <= 32, (st, fb, nf)
            with pkg.PyramidContext(H, W, S=S) as b:  # source context destroyed while deferred
                b.set_input(oracle.lcg_image(H, W, 92), 0)
                b.build()
                b.sync()
                want = np.empty(n, np.float32)
                assert L.gdp_download_image_raw(b._ctx, 0, want.ctypes.data_as(ctypes.c_void_p)) == 0
                assert L.gdp_host_defer(b._ctx, 0, hptr) == 0
            assert stats()[0] == 0
            _assert_same(host, want, "mirror completed by gdp_destroy of its source")
            assert L.gdp_host_defer(a._ctx, 0, hptr) == 0
            assert L.gdp_host_fetch(hptr) == 0 and stats()[0] == 0
            _assert_same(host, got, "gdp_host_fetch")
            assert L.gdp_host_defer(a._ctx, 0, hptr) == 0
            assert L.gdp_download_image_raw(a._ctx, 0, hptr) == 0  # whole download ends the deferral
            assert stats()[0] == 0 and stats()[2] == 0
            _assert_same(host, got, "download over a deferred mirror")
            assert L.gdp_host_defer(a._ctx, 0, hptr) == 0
            assert L.gdp_host_untrack(hptr) == 0  # completes it first
            _assert_same(host, got, "untrack of a deferred mirror")
            assert L.gdp_host_defer(a._ctx, 0, hptr) == 3  # untracked: refused
        finally:
            L.gdp_host_free(hptr)


def test_deferred_mirror_random_sequences(pkg, oracle):
    """Seeded random sequences on the C ABI of the tracked mirror (round 6): CPU reads and writes
    of random spans of a deferred / armed mirror (numpy through the CPU view: faults, fetches,
    read-ahead blocks and their tripwires, written pages), calls that upload the written pages,
    run the in-place pass and defer again (the drop-in's deferred GenerateDoG), mirrored calls that
    upload the written pages and copy everything back, explicit fetches and whole downloads — the
    mirror must always show what a plain host array would, and the device what the same calls on a
    plain array give (computed on a second context)."""
    import ctypes

    L = pkg.lib()
    H = W = 512
    S = 2
    with pkg.PyramidContext(H, W, S=S) as a, pkg.PyramidContext(H, W, S=S) as ref_ctx:
        n = L.gdp_image_floats(a._ctx)
        a.set_input(oracle.lcg_image(H, W, 55), 0)
        a.build()
        a.sync()
        dev = np.empty(n, np.float32)
        assert L.gdp_download_image_raw(a._ctx, 0, dev.ctypes.data_as(ctypes.c_void_p)) == 0

        def generate(x):  # the in-place pass on a plain array, on the second context
            assert L.gdp_upload_image_raw(ref_ctx._ctx, 0, x.ctypes.data_as(ctypes.c_void_p)) == 0
            assert L.gdp_generate_dog(ref_ctx._ctx, None) == 0
            y = np.empty_like(x)
            assert L.gdp_download_image_raw(ref_ctx._ctx, 0, y.ctypes.data_as(ctypes.c_void_p)) == 0
            return y

        hptr = ctypes.c_void_p()
        assert L.gdp_host_alloc_tracked(n * 4, ctypes.byref(hptr)) == 0
        try:
            host = np.ctypeslib.as_array(ctypes.cast(hptr, ctypes.POINTER(ctypes.c_float)), shape=(n,))
            assert L.gdp_download_image_raw(a._ctx, 0, hptr) == 0
            assert L.gdp_host_arm(hptr) == 0
            want = dev.copy()  # what the mirror must show
            rng = np.random.default_rng(2026)
            for case in range(6):
                for step in range(40):
                    k = rng.random()
                    lo = int(rng.integers(0, n))
                    span = int(rng.choice([1, 17, 1024, 40000, 300000]))
                    hi = min(n, lo + span)
                    if k < 0.30:  # a read of a span (sequential: faults, fetches, read-ahead)
                        _assert_same(host[lo:hi], want[lo:hi], (case, step, "read"))
                    elif k < 0.50:  # a write of a span
                        v = rng.standard_normal(hi - lo).astype(np.float32)
                        host[lo:hi] = v
                        want[lo:hi] = v
                    elif k < 0.68:  # the deferred call: written pages up, the pass, deferred again
                        assert L.gdp_upload_image_written(a._ctx, 0, hptr) == 0
                        assert L.gdp_generate_dog(a._ctx, None) == 0
                        assert L.gdp_host_defer(a._ctx, 0, hptr) == 0
                        want = generate(want)
                    elif k < 0.80:  # the eager call: written pages up, the pass, everything back
                        assert L.gdp_generate_dog_mirrored_written(a._ctx, 0, hptr) == 0
                        want = generate(want)
                    elif k < 0.88:
                        assert L.gdp_host_fetch(hptr) == 0
                    elif k < 0.94:  # the device copy back over everything (host edits discarded)
                        assert L.gdp_upload_image_written(a._ctx, 0, hptr) == 0
                        assert L.gdp_download_image_raw(a._ctx, 0, hptr) == 0
                        assert L.gdp_host_arm(hptr) == 0
                    else:  # a span read from several threads at once
                        import threading

                        got = np.empty(hi - lo, np.float32)
                        parts = np.array_split(np.arange(lo, hi), 4)
                        ts = [threading.Thread(target=lambda ix=ix: got.__setitem__(ix - lo, host[ix])) for ix in parts]
                        for t in ts:
                            t.start()
                        for t in ts:
                            t.join()
                        _assert_same(got, want[lo:hi], (case, step, "threads"))
                _assert_same(host, want, (case, "whole mirror"))
                assert L.gdp_upload_image_written(a._ctx, 0, hptr) == 0
                assert L.gdp_download_image_raw(a._ctx, 0, dev.ctypes.data_as(ctypes.c_void_p)) == 0
                _assert_same(dev, want, (case, "device"))
        finally:
            L.gdp_host_free(hptr)


@pytest.mark.parametrize("defer", [False, True])
def test_cpp_class_random_edit_sequences_with_write_tracking(oracle, tmp_path, defer):
    """Seeded random op sequences on GaussPyramid_hip (examples/state_hip): host edits (single
    floats, scaled rows, negated / zeroed levels, the input copy), calls (GenerateDoG, GaussFilter,
    GenerateDoG_mpi, GaussPyInit), mirror on / off with host_dirty / SyncDevice / SyncHost, and the
    write tracking switched off and on in between — the result must not depend on what the tracking
    uploads: bit-identical to the oracle's replay of the same ops in every sequence.  With `defer`,
    the deferred download (DeferDownload) is switched on and off in between as well, starting on,
    and whole-pyramid reads interleave: what GaussPy shows must not depend on when it is fetched."""
    rng = np.random.default_rng(606 if not defer else 616)
    for case in range(16):
        n = int(rng.choice([64, 100, 32]))
        O = oracle.octaves(n)
        ops = []
        for _ in range(int(rng.integers(6, 16))):
            k = rng.random()
            o = int(rng.integers(0, min(O, 4)))
            s_ = int(rng.integers(0, 5))
            ln = n >> o
            if k < 0.22:
                ops.append(str(rng.choice(["dog", "dog", "mpi", f"filter:{o}"])))
            elif k < 0.45:
                ops.append(f"set:{o}:{s_}:{int(rng.integers(0, ln))}:{int(rng.integers(0, ln))}:"
                           f"{float(rng.uniform(-1e3, 1e3)):.6g}")
            elif k < 0.55:
                ops.append(f"scale:{o}:{s_}:{int(rng.integers(0, ln))}:{float(rng.choice([-2.0, 0.5, 3.0]))}")
            elif k < 0.62:
                ops.append(str(rng.choice([f"neg:{o}:{s_}", f"zero:{o}:{s_}"])))
            elif k < 0.70:
                ops.append(str(rng.choice(["track:0", "track:1", "written"] + (["defer:0", "defer:1", "read"] if defer else []))))
            elif k < 0.80:
                ops.append(str(rng.choice(["mirror:0", "mirror:1", "dirty", "syncdev", "synchost"])))
            elif k < 0.87:
                ops.append(f"data:{int(rng.integers(0, n))}:{int(rng.integers(0, n))}:{int(rng.integers(-500, 500))}")
            else:
                ops.append(str(rng.choice(["init", "dog"])))
        if defer:
            ops.insert(0, "defer:1")
        ops += ["mirror:1", "dog"]  # end on a mirrored call so GaussPy holds the final state
        _run(oracle, tmp_path, "hip", n, 2, f"lcg:{(800 if defer else 700) + case}", ops)


def test_cpp_class_deferred_download(oracle, tmp_path):
    """DeferDownload(true): a mutating call leaves GaussPy's pages inaccessible (stale = the whole
    mirror, nothing copied back) and the first access to a page fetches its neighbourhood; values
    read, edited and dumped are bit-identical to the eager mirror's.  A write after a call is
    recorded (one page uploaded by the next call); the mirror off in between fetches first (the
    host keeps the deferred call's state); re-seated rows, SyncHost, GaussPyInit and the MPI entry
    keep the same bits; DeferDownload(false) completes the mirror."""
    page = os.sysconf("SC_PAGESIZE")
    n, S = 64, 2
    (w, st) = _run(oracle, tmp_path, "hip", n, S, "lcg:21", ["defer:1", "dog", "stale", "written", "dog", "stale",
                                                            "set:0:0:3:7:-1e30", "written", "dog", "written", "read",
                                                            "stale"], want_stale=True)
    assert w == [0, page, 0], w
    assert st[0] > 0 and st[1] == st[0] and st[2] == 0, st  # the read fetched every page
    (w, st) = _run(oracle, tmp_path, "hip", 100, S, "lcg:22", ["defer:1", "dog", "mirror:0", "dog", "stale", "mirror:1",
                                                              "neg:0:1", "dog", "filter:1", "mpi", "stale", "defer:0",
                                                              "stale"], want_stale=True)
    assert st[0] == 0 and st[1] > 0 and st[2] == -1, st
    _run(oracle, tmp_path, "hip", n, S, "lcg:23", ["defer:1", "dog", "reseat:0:1:7", "scale:0:1:7:-2", "dog",
                                                   "synchost", "dog", "init", "zero:0:2", "dog"])
    _run(oracle, tmp_path, "hip", n, S, "lcg:24", ["defer:1", "init", "dog", "track:0", "neg:1:0", "dog", "track:1",
                                                   "defer:1", "dog", "scale:1:1:3:0.5", "dog"])
    _run(oracle, tmp_path, "a512xp", n, S, "lcg:25", ["defer:1", "dog", "set:0:1:2:2:-4", "filter:0", "dog"])


def test_cpp_class_deferred_download_concurrent_faults(oracle, tmp_path):
    """Several host threads touching a deferred GaussPy at once (a SIFT detector reading DoG levels
    in parallel): concurrent read faults on stale pages and write faults on fetched ones are served
    one at a time by the handler (fetches on the helper thread) — the values read and the edits
    written from 8 threads give the oracle's bits, with and without deferral."""
    for n in (256, 100):
        for defer in ([], ["defer:1"]):
            _run(oracle, tmp_path, "hip", n, 2, "lcg:26", defer + ["dog", "readmt:8", "negmt:0:1:8", "dog", "negmt:1:3:5",
                                                                   "readmt:3", "dog", "negmt:0:0:8", "mpi"])
