# round-2 session: full regression on the current tree — GPU suite, smoke, default bench, the
# extension and subset bench lines, and rocprofv3 of the default command
exec tools/gpu_session.sh \
  "gputest_r02x|600|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "smoke_r02x|120|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench_c2_r02x|300|python3 bench.py" \
  "bench_subset_c2_r02x|300|python3 bench.py --op subset --no-cpu" \
  "bench_conv_c2_r02x|200|python3 bench.py --op conv --no-cpu" \
  "prof_default_r02x|300|rocprofv3 --kernel-trace --stats -d gpurun_out/prof_default_r02x -o run --output-format csv -- python3 bench.py --no-cpu"
