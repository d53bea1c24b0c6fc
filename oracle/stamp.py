#!/usr/bin/env python3
"""ORACLE — TEST INFRASTRUCTURE ONLY.

Provenance stamp of a binary built from the reference's own sources (oracle/Makefile): writes
<binary>.stamp.json with the sha256 of every source file the compile read (the reference headers
in place under REF_DIR, this directory's harness), the compiler's version line and the flags, so a
timing or a fixture made with oracle/_ref/<binary> names exactly which reference text it ran.

    python3 stamp.py <binary> <compiler> "<flags>" <source>...
"""
import hashlib
import json
import os
import subprocess
import sys
import time


def main():
    binary, compiler, flags, sources = sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4:]
    try:
        version = subprocess.run([compiler, "--version"], capture_output=True, text=True).stdout.splitlines()[0]
    except (OSError, IndexError):
        version = "unknown"
    commits = {}
    for src in sources:  # the git commit of each source tree that is a checkout (the reference's)
        d = os.path.dirname(os.path.abspath(src))
        if d not in commits:
            r = subprocess.run(["git", "-C", d, "rev-parse", "HEAD"], capture_output=True, text=True)
            commits[d] = r.stdout.strip() if r.returncode == 0 else None
    rec = {
        "binary": os.path.basename(binary),
        "binary_sha256": hashlib.sha256(open(binary, "rb").read()).hexdigest(),
        "sources": {os.path.abspath(s): hashlib.sha256(open(s, "rb").read()).hexdigest() for s in sources},
        "source_tree_commits": commits,
        "compiler": version,
        "flags": flags,
        "built_utc": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime()),
    }
    with open(binary + ".stamp.json", "w") as f:
        json.dump(rec, f, indent=1)


if __name__ == "__main__":
    main()
