"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes front end of oracle/liboracle.so (the plain-C restatement in oracle/gdp_oracle.c) plus
runners for oracle/_ref/ (the reference's own headers compiled in place).  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg import this module, always as the
checker / CPU baseline — never as the thing measured or shipped.
"""
import ctypes
import json
import os
import subprocess
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
REF_DIR = os.path.join(HERE, "_ref")

_lib = None


def build():
    """Compile liboracle.so (and oracle/_ref when /root/reference is present)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    if os.path.isdir(os.environ.get("GDP_REFERENCE_DIR", "/root/reference")):
        subprocess.run(["make", "-s", "-C", HERE, "ref",
                        "REF_DIR=" + os.environ.get("GDP_REFERENCE_DIR", "/root/reference")], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            subprocess.run(["make", "-s", "-C", HERE], check=True)
        L = ctypes.CDLL(LIB_PATH)
        i, p, sz, u32, u64, lng = ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_long
        L.gdo_octaves.argtypes, L.gdo_octaves.restype = [i], i
        L.gdo_level_offset.argtypes, L.gdo_level_offset.restype = [i, i, i, i, i], sz
        L.gdo_pyramid_floats.argtypes, L.gdo_pyramid_floats.restype = [i, i, i, i], sz
        L.gdo_taps.argtypes, L.gdo_taps.restype = [i, i, i, p], i
        L.gdo_build.argtypes, L.gdo_build.restype = [p, i, i, lng, i, i, p, p], None
        L.gdo_taps_centre.argtypes, L.gdo_taps_centre.restype = [i, i, i, p, i], i
        L.gdo_generate_dog_centre.argtypes, L.gdo_generate_dog_centre.restype = [p, i, i, i, i, p, i], None
        L.gdo_build_centre.argtypes, L.gdo_build_centre.restype = [p, i, i, lng, i, i, p, p, i], None
        L.gdo_init.argtypes, L.gdo_init.restype = [p, i, i, lng, i, i, p], None
        L.gdo_gauss_octave.argtypes, L.gdo_gauss_octave.restype = [p, i, i, i, i, p], None
        L.gdo_dog_octave.argtypes, L.gdo_dog_octave.restype = [p, i, i, i, i], None
        L.gdo_generate_dog.argtypes, L.gdo_generate_dog.restype = [p, i, i, i, i, p], None
        L.gdo_subset_a512omp.argtypes, L.gdo_subset_a512omp.restype = [p, i, i, i, i, p], None
        L.gdo_fnv.argtypes, L.gdo_fnv.restype = [p, sz], u64
        L.gdo_lcg_image.argtypes, L.gdo_lcg_image.restype = [p, i, i, u32], None
        L.gdo_synthetic_image.argtypes, L.gdo_synthetic_image.restype = [p, i, i, u32, lng], None
        L.gdo_synthetic_row.argtypes, L.gdo_synthetic_row.restype = [p, i, i, u32, lng, lng], None
        L.gdo_level_row.argtypes, L.gdo_level_row.restype = [p, i, i, i, i, i, p, p], None
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def octaves(n):
    """floor(log2 n) + 1 (GuassDePyramid.h:48-53); 0 for n == 0."""
    return lib().gdo_octaves(int(n))


def default_octaves(H, W):
    return octaves(min(H, W))


def level_offset(H, W, S, o, s):
    return lib().gdo_level_offset(H, W, S, o, s)


def pyramid_floats(H, W, S, O):
    return lib().gdo_pyramid_floats(H, W, S, O)


def levels(pyr, H, W, S, O):
    """Split a packed pyramid into {(o, s): (H_o, W_o) view}."""
    out = {}
    for o in range(O):
        for s in range(S + 3):
            off = level_offset(H, W, S, o, s)
            out[(o, s)] = pyr[off:off + (H >> o) * (W >> o)].reshape(H >> o, W >> o)
    return out


CENTRES = {"serial": 0, "intlen": 1}  # GuassDePyramid.h:107-115 / GaussDePyramid-MPI.h:273


def taps(length, o, s, centre="serial"):
    out = np.zeros(max(length, 1), np.float32)
    m = lib().gdo_taps_centre(int(length), int(o), int(s), _ptr(out), CENTRES[centre])
    return out[:m].copy()


def _scratch(H, W, S):
    return np.zeros(2 * (S + 3) * max(H, W, 1), np.float32)


def build_pyramid(img, S, O=None, centre="serial"):
    """Closed-form GaussPyInit + GenerateDoG for the first O octaves; packed layout.  centre
    "intlen" restates the multi-process variants (GaussDePyramid-MPI.h:265-335, mpitest.cpp:35-189),
    whose window centre uses the integer octave length."""
    img = np.ascontiguousarray(img, dtype=np.int32)
    H, W = img.shape
    O = default_octaves(H, W) if O is None else O
    out = np.empty(pyramid_floats(H, W, S, O), np.float32)
    lib().gdo_build_centre(_ptr(img), H, W, W, S, O, _ptr(out), _ptr(_scratch(H, W, S)), CENTRES[centre])
    return out


def init_pyramid(img, S, O=None):
    img = np.ascontiguousarray(img, dtype=np.int32)
    H, W = img.shape
    O = default_octaves(H, W) if O is None else O
    out = np.empty(pyramid_floats(H, W, S, O), np.float32)
    lib().gdo_init(_ptr(img), H, W, W, S, O, _ptr(out))
    return out


def generate_dog(pyr, H, W, S, O, centre="serial"):
    """In-place GenerateDoG on the current contents (reference operation order); centre "intlen"
    for the multi-process variants' GenerateDoG_mpi (GaussDePyramid-MPI.h:271-318)."""
    assert pyr.dtype == np.float32 and pyr.flags.c_contiguous
    lib().gdo_generate_dog_centre(_ptr(pyr), H, W, S, O, _ptr(_scratch(H, W, S)), CENTRES[centre])
    return pyr


def gauss_octave(pyr, H, W, S, o):
    lib().gdo_gauss_octave(_ptr(pyr), H, W, S, o, _ptr(_scratch(H, W, S)))
    return pyr


def dog_octave(pyr, H, W, S, o):
    lib().gdo_dog_octave(_ptr(pyr), H, W, S, o)
    return pyr


def subset_a512omp(pyr, H, W, S, O):
    lib().gdo_subset_a512omp(_ptr(pyr), H, W, S, O, _ptr(_scratch(H, W, S)))
    return pyr


def generate_dog_a512omp(pyr, H, W, S, O):
    """GaussPyramid_a512omp::GenerateDoG (GaussDePyramid-AVX512xOpenMP.h:183-213): that class's
    GaussFilter is empty (:128-181, its body commented out), so per octave only the DoG pass
    level j -= level j+1 for j = 0..S+1 runs (:187-193) — and a second time when the octave's
    integer side length is <= 2 (:194-201)."""
    for o in range(O):
        dog_octave(pyr, H, W, S, o)
        if min(H, W) >> o <= 2:
            dog_octave(pyr, H, W, S, o)
    return pyr


def fnv(a):
    a = np.ascontiguousarray(a, dtype=np.float32)
    return lib().gdo_fnv(_ptr(a), a.size)


def lcg_image(H, W, seed=12345):
    img = np.empty((H, W), np.int32)
    lib().gdo_lcg_image(_ptr(img), H, W, seed)
    return img


def synthetic_image(H, W, seed=0x5EED, index=0):
    img = np.empty((H, W), np.int32)
    lib().gdo_synthetic_image(_ptr(img), H, W, seed, index)
    return img


def synthetic_row(H, W, r, seed=0x5EED, index=0):
    """Row r of synthetic_image(H, W, seed, index)."""
    row = np.empty(W, np.int32)
    lib().gdo_synthetic_row(_ptr(row), H, W, seed, index, r)
    return row


def level_row(in_row, H, W, S, o, r):
    """Row r of every level of octave o ([S+3][W >> o] float32) from input row r << o."""
    in_row = np.ascontiguousarray(in_row, dtype=np.int32)
    out = np.empty((S + 3, W >> o), np.float32)
    scratch = np.empty(2 * (S + 3) * max(H, W) + 64, np.float32)
    lib().gdo_level_row(_ptr(in_row), H, W, S, o, r, _ptr(out), _ptr(scratch))
    return out


def image_from_spec(n, spec):
    """The input definitions of oracle/ref_harness.cpp (square n x n)."""
    if spec == "ones":
        return np.ones((n, n), np.int32)
    if spec.startswith("lcg:"):
        return lcg_image(n, n, int(spec[4:], 0))
    if spec.startswith("synth:"):
        parts = spec.split(":")
        return synthetic_image(n, n, int(parts[1], 0), int(parts[2], 0) if len(parts) > 2 else 0)
    raise ValueError(spec)


# ---------------------------------------------------------------- the reference itself (_ref)
def ref_binary(kind="serial"):
    path = os.path.join(REF_DIR, "ref_serial" if kind == "serial" else "ref_avx512")
    return path if os.path.exists(path) else None


def host_has_avx512():
    try:
        with open("/proc/cpuinfo") as f:
            return " avx512f" in f.read()
    except OSError:
        return False


def ref_time(mode, n, S, spec, reps, threads=None):
    """Run a timing mode of oracle/_ref (the reference compiled in place); returns its JSON."""
    binary = ref_binary("serial" if mode == "time-serial" else "avx512")
    if binary is None:
        return None
    args = [binary, mode, str(n), str(S), spec, str(reps)]
    if threads is not None:
        args.append(str(threads))
    env = dict(os.environ)
    if threads is not None:
        env["OMP_NUM_THREADS"] = str(threads)
    out = subprocess.run(args, check=True, capture_output=True, text=True, env=env).stdout
    return json.loads(out.strip().splitlines()[-1])


def ref_dump(mode, n, S, spec, *extra):
    binary = ref_binary("serial" if mode in ("dump", "regen") else "avx512")
    if binary is None:
        return None
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "o.f32")
        subprocess.run([binary, mode, str(n), str(S), spec, *map(str, extra), path], check=True, capture_output=True)
        return np.fromfile(path, dtype=np.float32)


# ---------------------------------------------------------------- checksum (gdp_checksum restated)
_PHI = np.uint64(0x9E3779B97F4A7C15)
_LVL = np.uint64(0xD1B54A32D192ED03)


def _splitmix_fin(x):
    x = x ^ (x >> np.uint64(30))
    x = x * np.uint64(0xBF58476D1CE4E5B9)
    x = x ^ (x >> np.uint64(27))
    x = x * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def level_checksum(lev, o, s, first_row=0):
    """Contribution of one level (rows starting at global row `first_row`) to gdp_checksum."""
    lev = np.ascontiguousarray(lev, dtype=np.float32)
    rows, cols = lev.shape
    with np.errstate(over="ignore"):
        idx = (np.arange(rows, dtype=np.uint64)[:, None] + np.uint64(first_row)) * np.uint64(cols) + \
            np.arange(cols, dtype=np.uint64)[None, :]
        x = idx * _PHI + np.uint64(o * 64 + s) * _LVL + lev.view(np.uint32).astype(np.uint64)
        return int(_splitmix_fin(x).sum(dtype=np.uint64))


def pyramid_checksum(pyr, H, W, S, O):
    """gdp_checksum of a whole-image packed pyramid."""
    total = 0
    for (o, s), lev in levels(pyr, H, W, S, O).items():
        total = (total + level_checksum(lev, o, s)) & 0xFFFFFFFFFFFFFFFF
    return total
