# round-2 session: bench --op regen / gauss with the in-place block shape autotuned
exec tools/gpu_session.sh \
  "bench_regen_c2_r02af|200|python3 bench.py --op regen --no-cpu" \
  "bench_gauss_c2_r02af|200|python3 bench.py --op gauss --no-cpu" \
  "bench_regen_c4_r02af|300|python3 bench.py --op regen --config c4 --steps 20 --warmup 3 --no-cpu"
