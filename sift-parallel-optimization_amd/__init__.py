"""sift-parallel-optimization_amd — MI355X-native Gaussian / DoG pyramid (drop-in for the hot
path of ZhangShuui/SIFT-parallel-optimization's GuassDePyramid.h / GaussDePyramid-*.h).

The compute is hand-written HIP for gfx950 in csrc/gdp.hip, exposed through the C ABI of
include/gdp.h (lib/libgdp.so).  This package is the Python host mirror of the reference's
interface (gausspyramid.GaussPyramid) plus the batched / multi-GPU drivers.  The directory name
is not a Python identifier; load it with __graft_entry__.load_package().
"""
from ._lib import GdpError, build_variants, header_functions, lib  # noqa: F401
from .gausspyramid import (GaussPyramid, GaussPyramid_a512omp, GaussPyramid_a512xp, PyramidContext,  # noqa: F401
                           conv_taps, octaves_for)

__all__ = ["GdpError", "GaussPyramid", "GaussPyramid_a512omp", "GaussPyramid_a512xp", "PyramidContext", "conv_taps", "octaves_for", "lib", "header_functions", "build_variants"]
