"""The reference's OWN drivers build against the drop-in, on CPU.

`make -C oracle dropin` pipes /root/reference/main.cpp (with the two-line include/class switch)
and mpitest.cpp (minus the definitions §3 deletes, oracle/strip_mpitest.py) straight into g++
and links libgdp(_comm); no reference text is written into the repository.  Skipped where the
reference is absent (the GPU box); tests/test_gpu_parity.py runs the binaries there.
"""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.environ.get("GDP_REFERENCE_DIR", "/root/reference")
OUT = os.path.join(REPO, "oracle", "_ref")

pytestmark = pytest.mark.skipif(not os.path.isfile(os.path.join(REF, "main.cpp")), reason="reference sources absent")


def _make(target):
    return subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), target, "REF_DIR=" + REF],
                          capture_output=True, text=True)


def test_main_cpp_two_line_switch_compiles_and_links():
    """main.cpp with `#include "GaussDePyramid-HIP.h"` / `GaussPyramid_hip`."""
    exe = os.path.join(OUT, "dropin_main")
    if os.path.exists(exe):
        os.unlink(exe)
    r = _make("_ref/dropin_main")
    assert r.returncode == 0, r.stderr
    assert os.access(exe, os.X_OK)


@pytest.mark.skipif(not os.path.exists("/opt/conda/include/mpi.h"), reason="no MPI headers")
def test_main_cpp_mpi_switch_compiles_and_links():
    """main.cpp with GaussDePyramid-HIP-mpi.h / GaussPyramid_hip_mpi + MPICH."""
    exe = os.path.join(OUT, "dropin_main_mpi")
    if os.path.exists(exe):
        os.unlink(exe)
    r = _make("_ref/dropin_main_mpi")
    assert r.returncode == 0, r.stderr
    assert os.access(exe, os.X_OK)


def test_mpitest_cpp_with_definitions_stripped_compiles_and_links():
    """mpitest.cpp minus its globals / GenerateDoG_mpi(_omp) / GaussPyInit /
    delete_mpi, plus `#include "GaussDePyramid-HIP-mpitest.h"`; its main() unchanged."""
    exe = os.path.join(OUT, "dropin_mpitest")
    if os.path.exists(exe):
        os.unlink(exe)
    r = _make("_ref/dropin_mpitest")
    assert r.returncode == 0, r.stderr
    assert os.access(exe, os.X_OK)


def test_strip_mpitest_removes_exactly_the_documented_definitions():
    import importlib.util

    spec = importlib.util.spec_from_file_location("strip_mpitest", os.path.join(REPO, "oracle", "strip_mpitest.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    with open(os.path.join(REF, "mpitest.cpp")) as f:
        text = f.read()
    out = mod.strip(text)
    assert out.count('#include "GaussDePyramid-HIP-mpitest.h"') == 1
    code = "\n".join(line.split("//", 1)[0] for line in out.splitlines())
    for name in ("void GenerateDoG_mpi(", "void GenerateDoG_mpi_omp(", "void GaussPyInit(", "void delete_mpi(",
                 "int thread_count", "float **** GaussPy", "bool is_initialized"):
        assert name not in code, name
    assert "int main(int argc,char* argv[])" in code  # the driver itself is untouched
    with pytest.raises(SystemExit):
        mod.strip("int main() { return 0; }\n")  # refuses a file that lacks the definitions
