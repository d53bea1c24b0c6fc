# round-2 session: full GPU suite + smoke + default bench on the current tree.
exec tools/gpu_session.sh \
  "gputest_r02o|600|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "smoke_r02o|120|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench_c2_r02o|300|python3 bench.py" \
  "bench_conv_c2_r02o|200|python3 bench.py --op conv --no-cpu"
