# Final-tree bench lines of the other configs and ops (round 5)
set -e
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --config c3 --no-cpu > gpurun_out/bench_c3_r05al.log 2>&1
timeout -k 10 500 python bench.py --config c4 --no-cpu > gpurun_out/bench_c4_r05al.log 2>&1
timeout -k 10 400 python bench.py --config c5 --no-cpu > gpurun_out/bench_c5_r05al.log 2>&1
timeout -k 10 300 python bench.py --op subset --no-cpu > gpurun_out/bench_subset_c2_r05al.log 2>&1
timeout -k 10 300 python bench.py --op gauss --no-cpu > gpurun_out/bench_gauss_c2_r05al.log 2>&1
echo done
