#!/usr/bin/env bash
# rocprofv3 evidence for one (config, build variant, tile order): a kernel trace + stats run and the
# FETCH_SIZE / WRITE_SIZE counters in passes of their own (never combined with other domains), all
# of bench.py forced to that variant and tile order.  Outputs under gpurun_out/prof_<tag>_*;
# summarise in the container with profiles/collect_pmc.py --variant V --tile-order T.
#   tools/pmc_session.sh c2 15 0 200 [zero_window]
cfg=$1; var=$2; ord=$3; steps=${4:-50}; zw=${5:-0}
tag="${cfg}_v${var}o${ord}$([ "$zw" = 1 ] && echo z1)"
force="--variant ${var} --tile-order ${ord} --zero-window ${zw} --no-cpu"
exec tools/gpu_session.sh \
  "prof_${tag}_trace|300|rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag}_trace -o run --output-format csv -- python3 bench.py --config ${cfg} --steps ${steps} --warmup 5 ${force}" \
  "prof_${tag}_fetch|180|timeout -s KILL 170 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_${tag}_fetch -o run --output-format csv -- python3 bench.py --config ${cfg} --steps 5 --warmup 1 ${force}" \
  "prof_${tag}_write|180|timeout -s KILL 170 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_${tag}_write -o run --output-format csv -- python3 bench.py --config ${cfg} --steps 5 --warmup 1 ${force}"
