# Re-entry (k_levels) on the current tree, configs 2 and 4 (round 5)
set -e
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu --op regen > gpurun_out/bench_regen_c2_r05aa.log 2>&1
timeout -k 10 400 python bench.py --no-cpu --op regen --config c4 > gpurun_out/bench_regen_c4_r05aa.log 2>&1
echo done
