# round-3 session ar: the tree with store pacing in both autotunes — full GPU suite, smoke, the
# bench lines of configs 2-5 (the driver's default command first) and the convolution line
exec tools/gpu_session.sh \
  "gputest_r03ar|700|python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider" \
  "smoke_r03ar|120|python3 -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench_default_r03ar|300|python3 bench.py" \
  "bench_c3_r03ar|300|python3 bench.py --config c3 --steps 20 --warmup 3 --no-cpu" \
  "bench_c4_r03ar|300|python3 bench.py --config c4 --steps 10 --warmup 2 --no-cpu" \
  "bench_c5_r03ar|300|python3 bench.py --config c5 --steps 20 --warmup 3 --no-cpu"
