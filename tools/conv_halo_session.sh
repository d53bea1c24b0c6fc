#!/usr/bin/env bash
# Round 5, session d: the convolution extension's block-tile halo lanes (GDP_TUNE_CONV_HALO 2 / 4 /
# 8 = 240 / 224 / 192-column tiles) on configs 2 / 4 / 5, alternated, then the PMC traffic of halo
# 8 and 4 on config 2 (FETCH_SIZE and WRITE_SIZE in passes of their own).  Every GPU step under
# its own time limit; a fatal exit ends the session.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name limit cmd...
  local name=$1 limit=$2; shift 2
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== [$name] exit $rc"; tail -n 3 "gpurun_out/$name.log" | cut -c1-300
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "fatal $rc: stopping"; exit $rc; fi
}
for rep in a b; do
  for cfg in c2 c4 c5; do
    for h in 2 4 8; do
      step conv_${cfg}_h${h}${rep}_r05d 200 python3 bench.py --op conv --config $cfg --conv-halo $h --no-cpu
    done
  done
done
for h in 8 4; do
  step pmcf_conv_c2_h${h}_r05d 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcf_conv_c2_h${h} -o run --output-format csv -- python3 bench.py --op conv --conv-halo $h --steps 5 --warmup 2 --no-cpu
  step pmcw_conv_c2_h${h}_r05d 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcw_conv_c2_h${h} -o run --output-format csv -- python3 bench.py --op conv --conv-halo $h --steps 5 --warmup 2 --no-cpu
done
exit 0
