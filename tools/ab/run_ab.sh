#!/usr/bin/env bash
# A/B of library builds on one box: tools/ab/run_ab.sh CONFIG ITERS ROUNDS VARIANTS lib1 lib2 ...
cfg=$1; it=$2; rd=$3; var=$4; shift 4
for lib in "$@"; do
  echo "## $lib"
  GDP_LIBRARY=$lib timeout -k 10 120 python tools/tune.py --config $cfg --iters $it --rounds $rd --no-check --variants "$var" ${TUNE_EXTRA:-} 2>&1 | grep variant || exit 1
done
