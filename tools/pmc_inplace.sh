#!/usr/bin/env bash
# rocprofv3 evidence for the in-place passes: for each block shape the bench's
# autotune can pick (--op regen: GDP_TUNE_INPLACE_SUB 1 / 4 / 2 / 0; --op gauss: WINDOW_SUB 1 / 4 / 2),
# a kernel trace + stats run and FETCH_SIZE / WRITE_SIZE passes of their own, bench.py forced to that
# shape.  Summarise in the container with profiles/collect_pmc.py --op regen --inplace-sub N.
#   [ZW=1] tools/pmc_inplace.sh c2 [round]   (ZW=1: GDP_TUNE_ZERO_WINDOW on, records tagged _z1)
cfg=$1; rnd=${2:-r03}; zw=${ZW:-0}; zt=$([ "$zw" = 1 ] && echo _z1)
steps=()
for op in regen gauss; do
  subs="${REGEN_SUBS:-1 4 2 0 8 16}"; [ $op = gauss ] && subs="${GAUSS_SUBS:-1 4 2 8 16}"
  for sub in $subs; do
    tag="${cfg}_${op}_s${sub}${zt}_${rnd}"
    force="--op ${op} --inplace-sub ${sub} --zero-window ${zw} --no-cpu"
    steps+=("prof_${tag}_trace|300|rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag}_trace -o run --output-format csv -- python3 bench.py --config ${cfg} --steps 50 --warmup 5 ${force} > gpurun_out/prof_${tag}_trace.json")
    steps+=("prof_${tag}_fetch|180|timeout -s KILL 170 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_${tag}_fetch -o run --output-format csv -- python3 bench.py --config ${cfg} --steps 5 --warmup 1 ${force}")
    steps+=("prof_${tag}_write|180|timeout -s KILL 170 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_${tag}_write -o run --output-format csv -- python3 bench.py --config ${cfg} --steps 5 --warmup 1 ${force}")
  done
done
exec tools/gpu_session.sh "${steps[@]}"
