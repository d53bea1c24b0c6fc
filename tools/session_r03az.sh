# round-3 session az: final tree after the convolution default change — GPU suite, smoke, the
# driver's default command, the convolution line
exec tools/gpu_session.sh \
  "gputest_r03az|700|python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider" \
  "smoke_r03az|120|python3 -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench_default_r03az|300|python3 bench.py" \
  "bench_conv_c2_r03az|200|python3 bench.py --op conv --no-cpu" \
  "bench_conv_c4_r03az|300|python3 bench.py --op conv --config c4 --steps 10 --warmup 2 --no-cpu"
