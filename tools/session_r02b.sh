# round-2 session: GPU suite with the block-tile convolution default, conv bench lines, PMC of every
# build-kernel instance on config 2, rocprof trace + PMC of the conv default on config 2.
exec tools/gpu_session.sh \
  "gputest_r02b|600|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "bench_conv_c2_r02|200|python3 bench.py --op conv --no-cpu" \
  "bench_conv_c4_r02|300|python3 bench.py --op conv --config c4 --steps 20 --warmup 3 --no-cpu" \
  "pmcv_fetch|300|timeout -s KILL 290 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcv_fetch -o run --output-format csv -- python3 tools/pmc_variants.py --config c2 --manifest gpurun_out/pmcv_manifest.json" \
  "pmcv_write|300|timeout -s KILL 290 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcv_write -o run --output-format csv -- python3 tools/pmc_variants.py --config c2 --manifest gpurun_out/pmcv_manifest.json" \
  "prof_c2_conv_trace|300|rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2_conv_trace -o run --output-format csv -- python3 bench.py --op conv --steps 200 --warmup 5 --no-cpu" \
  "prof_c2_conv_fetch|180|timeout -s KILL 170 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_c2_conv_fetch -o run --output-format csv -- python3 bench.py --op conv --steps 5 --warmup 1 --no-cpu" \
  "prof_c2_conv_write|180|timeout -s KILL 170 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_c2_conv_write -o run --output-format csv -- python3 bench.py --op conv --steps 5 --warmup 1 --no-cpu"
