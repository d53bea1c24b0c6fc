# round-2 session (re-created container): full regression on the rebuilt tree — GPU suite, smoke,
# default bench
exec tools/gpu_session.sh \
  "gputest_r02ag|600|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "smoke_r02ag|120|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench_c2_r02ag|300|python3 bench.py"
