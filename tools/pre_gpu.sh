#!/usr/bin/env bash
# Build everything and run the CPU suite; used as `tools/pre_gpu.sh && gpurun ...`.
set -eo pipefail
cd "$(dirname "$0")/.."
python -c "import __graft_entry__ as g; g.build()"
make -s -C tools membench 2>/dev/null || true
python -m pytest tests -q -m "not gpu" -x -p no:cacheprovider 2>&1 | tail -2
