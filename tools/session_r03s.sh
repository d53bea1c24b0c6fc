# round-3 session s: the final tree once more — GPU suite, smoke, the driver's default command
exec tools/gpu_session.sh \
  "gputest_r03s|600|python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider" \
  "smoke_r03s|120|python3 -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench_c2_r03s|300|python3 bench.py --gpus 1 --steps 20 --warmup 5"
