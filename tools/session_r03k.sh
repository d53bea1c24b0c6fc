# round-3 session k: final-tree bench lines of configs 3-5 and of the other ops on config 2
exec tools/gpu_session.sh \
  "bench_c4_r03k|300|python3 bench.py --config c4 --steps 10 --warmup 2 --no-cpu" \
  "bench_c5_r03k|300|python3 bench.py --config c5 --steps 20 --warmup 3 --no-cpu" \
  "bench_c3_r03k|300|python3 bench.py --config c3 --steps 20 --warmup 3 --no-cpu" \
  "bench_conv_c2_r03k|200|python3 bench.py --op conv --no-cpu" \
  "bench_subset_c2_r03k|200|python3 bench.py --op subset --no-cpu" \
  "bench_regen_c2_r03k|200|python3 bench.py --op regen --no-cpu" \
  "bench_gauss_c2_r03k|200|python3 bench.py --op gauss --no-cpu" \
  "bench_regen_c4_r03k|300|python3 bench.py --op regen --config c4 --steps 10 --warmup 2 --no-cpu"
