# bench.py's gpu_state_after_timed_steps (rocm-smi clocks / power / temperature), default command
set -e
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/bench_default_r05aj.log 2>&1
echo done
