#!/usr/bin/env bash
# Runs GPU steps in order on the gpurun box; each step has its own time limit.  A step that
# faults, aborts, segfaults or times out (exit 124/134/137/139 or >128) ends the session: nothing
# else touches the GPU after it.  Ordinary failures (exit 1, e.g. a failing assertion) continue.
# Usage: tools/gpu_session.sh "name|timeout_s|command" ...
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
  name="${spec%%|*}"; rest="${spec#*|}"; limit="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== [$name] (limit ${limit}s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$limit" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] exit $rc after $(( $(date +%s) - start ))s"
  tail -n 15 "gpurun_out/$name.log"
  if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ] || [ $rc -gt 128 ]; then
    echo "=== fatal exit $rc in [$name]: stopping the session"
    exit $rc
  fi
done
exit 0
