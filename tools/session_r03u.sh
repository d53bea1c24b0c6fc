# round-3 session u: the driver's bench command three times back to back on one box (run-to-run spread)
exec tools/gpu_session.sh \
  "bench_repeat1_r03u|300|python3 bench.py --gpus 1 --steps 20 --warmup 5" \
  "bench_repeat2_r03u|300|python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu" \
  "bench_repeat3_r03u|300|python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu"
