#!/usr/bin/env bash
# rocprofv3 evidence for bench.py configs: kernel trace + stats, then FETCH_SIZE and WRITE_SIZE in
# separate --pmc passes (never combined with other trace domains).  Run on the GPU box:
#   tools/profile_session.sh c2 200 && tools/profile_session.sh c4 10
cfg=$1; steps=${2:-50}; extra=${3:-}; tag=${4:-$cfg}
exec tools/gpu_session.sh \
  "prof_${tag}_trace|300|rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag}_trace -o run --output-format csv -- python3 bench.py --config ${cfg} --steps ${steps} --warmup 5 --no-cpu ${extra}" \
  "prof_${tag}_fetch|300|rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_${tag}_fetch -o run --output-format csv -- python3 bench.py --config ${cfg} --steps 5 --warmup 1 --no-cpu ${extra}" \
  "prof_${tag}_write|300|rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_${tag}_write -o run --output-format csv -- python3 bench.py --config ${cfg} --steps 5 --warmup 1 --no-cpu ${extra}"
