# round-2 session: full GPU suite, build bench lines for configs 3 and 5, and self-launched gloo
# rehearsals of the driver's multi-rank command on one GPU (8 ranks of config 2, 2 ranks of config 4).
exec tools/gpu_session.sh \
  "gputest_r02e|600|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "smoke_r02e|120|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench_c3_r02|300|python3 bench.py --config c3 --steps 50 --warmup 5" \
  "bench_c5_r02|300|python3 bench.py --config c5 --steps 50 --warmup 5 --no-cpu" \
  "selflaunch_gloo8_c2_r02|400|GDP_BENCH_BACKEND=gloo python3 bench.py --gpus 8 --steps 50 --warmup 5" \
  "selflaunch_gloo2_c4_r02|400|GDP_BENCH_BACKEND=gloo python3 bench.py --gpus 2 --config c4 --steps 10 --warmup 2"
