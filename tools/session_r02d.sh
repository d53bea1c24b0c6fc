# round-2 session: conv tests after the staging-load fix, conv bench lines c2/c4/c5, rocprof
# trace + PMC of the conv default on config 2.
exec tools/gpu_session.sh \
  "gputest_conv_r02d|400|python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k 'convolution or row_bands_with_halo or config5_bands' --timeout 300 --timeout-method thread" \
  "bench_conv_c2_r02|200|python3 bench.py --op conv --no-cpu" \
  "bench_conv_c4_r02|300|python3 bench.py --op conv --config c4 --steps 20 --warmup 3 --no-cpu" \
  "bench_conv_c5_r02|300|python3 bench.py --op conv --config c5 --steps 50 --warmup 5 --no-cpu" \
  "prof_c2_conv_trace|300|rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2_conv_trace -o run --output-format csv -- python3 bench.py --op conv --steps 200 --warmup 5 --no-cpu" \
  "prof_c2_conv_fetch|180|timeout -s KILL 170 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_c2_conv_fetch -o run --output-format csv -- python3 bench.py --op conv --steps 5 --warmup 1 --no-cpu" \
  "prof_c2_conv_write|180|timeout -s KILL 170 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_c2_conv_write -o run --output-format csv -- python3 bench.py --op conv --steps 5 --warmup 1 --no-cpu"
