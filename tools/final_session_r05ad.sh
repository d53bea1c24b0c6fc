# Final tree (streams figure opt-in): full GPU suite, smoke, conv benches c2/c5, default bench
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gputest_r05ad.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as e; e.smoke(); print('smoke ok')" > gpurun_out/smoke_r05ad.log 2>&1
timeout -k 10 300 python bench.py --no-cpu --op conv > gpurun_out/bench_conv_c2_r05ad.log 2>&1
timeout -k 10 300 python bench.py --no-cpu --op conv --config c5 --steps 10 --warmup 2 > gpurun_out/bench_conv_c5_r05ad.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/bench_default_r05ad.log 2>&1
echo done
