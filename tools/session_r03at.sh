# round-3 session at: pacing in the subset build and the in-place re-entry autotunes — parity, the
# other ops' bench lines, and the driver's default command under rocprofv3 --kernel-trace --stats
exec tools/gpu_session.sh \
  "spt_parity_r03at|500|python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k 'subset or a512 or zero_window or regen or generate_dog or autotune'" \
  "bench_subset_c2_r03at|200|python3 bench.py --op subset --no-cpu" \
  "bench_regen_c2_r03at|200|python3 bench.py --op regen --no-cpu" \
  "bench_gauss_c2_r03at|200|python3 bench.py --op gauss --no-cpu" \
  "bench_regen_c4_r03at|300|python3 bench.py --op regen --config c4 --steps 10 --warmup 2 --no-cpu" \
  "bench_conv_c2_r03at|200|python3 bench.py --op conv --no-cpu" \
  "prof_default_r03at|300|rocprofv3 --kernel-trace --stats -d gpurun_out/prof_default_r03at -o run --output-format csv -- python3 bench.py"
