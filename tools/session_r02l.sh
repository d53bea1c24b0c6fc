# round-2 session: subset build (LT = 5 specialisation) parity + interleaved A/B against the full build
exec tools/gpu_session.sh \
  "a512_tests_r02l|300|python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k 'subset or a512'" \
  "ab_subset_r02l|300|python3 tools/tune.py --config c2 --rotate 5 --rounds 9 --iters 40 --variants 'v=15;v=15,op=subset;v=16;v=16,op=subset;v=15,nt=1,op=build'" \
  "bench_subset_c2_r02l|300|python3 bench.py --op subset" \
  "bench_c2_r02l|300|python3 bench.py"
