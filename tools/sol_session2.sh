set -e
mkdir -p gpurun_out
timeout -k 10 120 tools/sol_c2 200 > gpurun_out/sol_c2_r05k.log 2>&1
timeout -k 10 300 python bench.py --no-cpu --op regen > gpurun_out/bench_regen_c2_r05k.log 2>&1
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench_default_r05k.log 2>&1
echo done
