"""Write tracking of host mirrors (gdp_host_track / _arm / _written_bytes / _untrack), on the CPU.

The drop-in classes keep GaussPy two-way (GuassDePyramid.h:16): before a mutating call the host
mirror is the state, but main.cpp's loop (:66-73) never writes it.  libgdp write-protects an armed
mirror; a CPU write faults once, the SIGSEGV handler records the page and makes it writable, and
the next call uploads only the recorded pages.  The mechanism is host code:
these tests drive it on page-aligned anonymous memory with no GPU.  (The uploads themselves are
tested on the GPU: tests/test_gpu_state.py.)"""
import ctypes
import mmap
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "sift-parallel-optimization_amd", "lib", "libgdp.so")
PAGE = os.sysconf("SC_PAGESIZE")


def _buffer(pages):
    buf = mmap.mmap(-1, pages * PAGE)
    return buf, ctypes.addressof(ctypes.c_char.from_buffer(buf))


def _written(L, addr):
    n = ctypes.c_size_t()
    rc = L.gdp_host_written_bytes(ctypes.c_void_p(addr), ctypes.byref(n))
    return rc, n.value


def test_cpu_writes_to_an_armed_mirror_are_recorded_per_page(pkg):
    L = pkg.lib()
    buf, addr = _buffer(64)
    p = ctypes.c_void_p(addr)
    try:
        assert L.gdp_host_track(p, 64 * PAGE) == 0
        assert L.gdp_host_track(p, 64 * PAGE) == 0          # registering twice is a no-op
        assert _written(L, addr)[0] == 3                     # not armed yet: GDP_ERR_STATE
        assert L.gdp_host_arm(p) == 0
        assert _written(L, addr) == (0, 0)
        buf[5 * PAGE + 7] = 1                                # one byte: its page
        assert _written(L, addr) == (0, PAGE)
        buf[5 * PAGE + 100] = 2                              # same page again: no second fault
        buf[10 * PAGE - 1:10 * PAGE + 2 * PAGE + 1] = b"x" * (2 * PAGE + 2)  # pages 9..12
        assert _written(L, addr) == (0, 5 * PAGE)
        assert buf[5 * PAGE + 7] == 1 and buf[10 * PAGE] == ord("x")  # the writes landed
        v = memoryview(buf)
        assert bytes(v[0:16]) == bytes(16)                   # reads never fault
        v.release()
        assert L.gdp_host_arm(p) == 0                        # re-armed: the record restarts
        assert _written(L, addr) == (0, 0)
        buf[63 * PAGE + PAGE - 1] = 3                        # last byte of the buffer
        assert _written(L, addr) == (0, PAGE)
        assert L.gdp_host_untrack(p) == 0
        buf[0] = 9                                           # writable again, nothing recorded
        assert _written(L, addr)[0] == 1                     # unknown buffer: GDP_ERR_ARG
        assert L.gdp_host_untrack(p) == 1
    finally:
        L.gdp_host_untrack(p)
        buf.close()


def test_a_partial_range_tracks_the_pages_it_touches(pkg):
    """A registered range that starts and ends inside pages: written bytes are counted within the
    range only (the upload never leaves the caller's buffer)."""
    L = pkg.lib()
    buf, addr = _buffer(8)
    start, nbytes = addr + 100, 3 * PAGE
    p = ctypes.c_void_p(start)
    try:
        assert L.gdp_host_track(p, nbytes) == 0 and L.gdp_host_arm(p) == 0
        buf[150] = 1                                 # first page of the range: PAGE - 100 bytes of it
        assert _written(L, start) == (0, PAGE - 100)
        buf[3 * PAGE + 50] = 1                       # last (partial) page: 100 bytes of it in range
        assert _written(L, start) == (0, PAGE - 100 + 100)
    finally:
        L.gdp_host_untrack(p)
        buf.close()


_CHAIN = r"""
import ctypes, mmap, sys
L = ctypes.CDLL(sys.argv[1])
buf = mmap.mmap(-1, 4 * 4096)
addr = ctypes.addressof(ctypes.c_char.from_buffer(buf))
assert L.gdp_host_track(ctypes.c_void_p(addr), ctypes.c_size_t(4 * 4096)) == 0
assert L.gdp_host_arm(ctypes.c_void_p(addr)) == 0
buf[1] = 1                     # a tracked page: handled
print("tracked write ok", flush=True)
ctypes.string_at(0x10, 1)      # an unrelated fault: the default action (no handler before ours)
print("unreachable", flush=True)
"""


def test_faults_elsewhere_take_their_default_action(tmp_path):
    """The handler only serves armed mirror pages; any other SIGSEGV goes to the disposition that
    was there before (here the default: the process dies by SIGSEGV, it does not loop or hang)."""
    r = subprocess.run([sys.executable, "-c", _CHAIN, LIB], capture_output=True, text=True, timeout=60,
                       env=dict(os.environ, GDP_NO_TORCH="1"))
    assert "tracked write ok" in r.stdout
    assert "unreachable" not in r.stdout
    assert r.returncode == -11, (r.returncode, r.stderr[-500:])


_CHAIN_PREV = r"""
import ctypes, faulthandler, mmap, sys
faulthandler.enable()          # a SIGSEGV handler installed BEFORE libgdp's
L = ctypes.CDLL(sys.argv[1])
buf = mmap.mmap(-1, 4 * 4096)
addr = ctypes.addressof(ctypes.c_char.from_buffer(buf))
assert L.gdp_host_track(ctypes.c_void_p(addr), ctypes.c_size_t(4 * 4096)) == 0
assert L.gdp_host_arm(ctypes.c_void_p(addr)) == 0
buf[2 * 4096] = 1
print("tracked write ok", flush=True)
ctypes.string_at(0x10, 1)
"""


def test_faults_elsewhere_reach_the_previous_handler(tmp_path):
    """With a handler installed before libgdp's (Python's faulthandler), an unrelated fault reaches
    it: its traceback is printed, then the process dies by SIGSEGV."""
    r = subprocess.run([sys.executable, "-c", _CHAIN_PREV, LIB], capture_output=True, text=True, timeout=60,
                       env=dict(os.environ, GDP_NO_TORCH="1"))
    assert "tracked write ok" in r.stdout
    assert "Fatal Python error: Segmentation fault" in r.stderr, r.stderr[-800:]
    assert r.returncode == -11


def test_bad_arguments(pkg):
    L = pkg.lib()
    n = ctypes.c_size_t()
    assert L.gdp_host_track(None, 4096) == 1
    assert L.gdp_host_track(ctypes.c_void_p(4096), 0) == 1
    assert L.gdp_host_arm(None) == 1
    assert L.gdp_host_untrack(None) == 1
    assert L.gdp_host_written_bytes(None, ctypes.byref(n)) == 1
    assert L.gdp_upload_image_written(None, 0, None) == 1
    assert L.gdp_generate_dog_mirrored_written(None, 0, None) == 1
