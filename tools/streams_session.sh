# bench.py's informational concurrent_streams figure (round 5)
set -e
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/bench_default_r05p.log 2>&1
echo done
