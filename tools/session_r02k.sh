# round-2 session: GenerateDoG_nomp_dynamic (AVX-512 x OpenMP semantics) on the GPU — parity, host
# ASan of the new exports, bench line, rocprof stats and PMC traffic of the subset build kernel
exec tools/gpu_session.sh \
  "a512_tests_r02k|300|python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k 'subset or a512'" \
  "asan_r02k|300|make -s -C tools/asan run" \
  "bench_subset_c2_r02k|300|python3 bench.py --op subset" \
  "a512_time_r02k|120|examples/a512_hip" \
  "prof_subset_r02k|300|rocprofv3 --kernel-trace --stats -d gpurun_out/prof_subset_r02k -o run --output-format csv -- python3 bench.py --op subset --steps 200 --warmup 5 --no-cpu" \
  "pmc_subset_fetch_r02k|200|timeout -s KILL 190 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_subset_fetch_r02k -o run --output-format csv -- python3 bench.py --op subset --steps 20 --warmup 2 --no-cpu --no-autotune --variant 15 --tile-order 0" \
  "pmc_subset_write_r02k|200|timeout -s KILL 190 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_subset_write_r02k -o run --output-format csv -- python3 bench.py --op subset --steps 20 --warmup 2 --no-cpu --no-autotune --variant 15 --tile-order 0"
