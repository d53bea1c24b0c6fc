# round-2 session: final-tree evidence — rocprofv3 of the default command (kernel average vs the
# bench line's kernel_ms), the subset / convolution / re-entry bench lines, config 4 and 5 lines
exec tools/gpu_session.sh \
  "prof_default_r02ak|300|rocprofv3 --kernel-trace --stats -d gpurun_out/prof_default_r02ak -o run --output-format csv -- python3 bench.py --no-cpu" \
  "bench_subset_c2_r02ak|200|python3 bench.py --op subset --no-cpu" \
  "bench_conv_c2_r02ak|200|python3 bench.py --op conv --no-cpu" \
  "bench_regen_c2_r02ak|200|python3 bench.py --op regen --no-cpu" \
  "bench_c4_r02ak|300|python3 bench.py --config c4 --steps 10 --warmup 2 --no-cpu" \
  "bench_c5_r02ak|300|python3 bench.py --config c5 --steps 20 --warmup 3 --no-cpu" \
  "bench_c3_r02ak|300|python3 bench.py --config c3 --steps 20 --warmup 3 --no-cpu"
