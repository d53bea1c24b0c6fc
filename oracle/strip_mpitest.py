#!/usr/bin/env python3
"""ORACLE / TEST INFRASTRUCTURE ONLY.

Prints the reference's mpitest.cpp with the definitions INTEGRATION.md §3 says to delete — the
globals (mpitest.cpp:26-34), GenerateDoG_mpi_omp (:35-113), GenerateDoG_mpi (:114-189),
GaussPyInit (:438-473) and delete_mpi (:474-493) — and `#include "GaussDePyramid-HIP-mpitest.h"`
in their place, so the drop-in can be compiled against the UNMODIFIED rest of the file (its
`main`).  Reads the file given on the command line and writes to stdout (oracle/Makefile pipes it
straight into g++): no reference text is stored anywhere.  Definitions are found by name and
brace matching, not by line number, and comment lines are left alone.
"""
import re
import sys

GLOBALS = ("thread_count", "chunk_size", "MAX", "n", "S", "GaussPy", "length", "layer", "is_initialized")
FUNCS = ("GenerateDoG_mpi_omp", "GenerateDoG_mpi", "GaussPyInit", "delete_mpi")


def strip(text):
    lines = text.split("\n")
    out, i, inserted = [], 0, False
    glob_re = re.compile(r"^\s*(const\s+)?(int|bool|float\s*\*\*\*\*)\s*(%s)\b[^(]*;" % "|".join(GLOBALS))
    func_re = re.compile(r"^\s*void\s+(%s)\s*\(" % "|".join(FUNCS))
    removed = set()
    while i < len(lines):
        line = lines[i]
        code = line.split("//", 1)[0]
        g = glob_re.match(code)
        f = func_re.match(code)
        if g or f:
            if not inserted:
                out.append('#include "GaussDePyramid-HIP-mpitest.h"')
                inserted = True
            if g:
                removed.add(g.group(3))
                i += 1
                continue
            removed.add(f.group(1))
            depth, seen = 0, False
            while i < len(lines):
                c = lines[i].split("//", 1)[0]
                depth += c.count("{") - c.count("}")
                seen = seen or "{" in c
                i += 1
                if seen and depth == 0:
                    break
            continue
        out.append(line)
        i += 1
    missing = set(GLOBALS + FUNCS) - removed
    if missing:
        raise SystemExit(f"strip_mpitest: definitions not found: {sorted(missing)}")
    return "\n".join(out)


if __name__ == "__main__":
    with open(sys.argv[1]) as f:
        sys.stdout.write(strip(f.read()))
