# round-2 session: subset build with paced stores (s_waitcnt vmcnt(0) after each) vs the full build
exec tools/gpu_session.sh \
  "subset_tests_r02s|300|python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k 'subset_build_matches_reference'" \
  "ab_subset_c2_r02s|300|python3 tools/tune.py --config c2 --rotate 5 --rounds 9 --iters 40 --variants 'v=15;v=15,op=subset;v=16;v=16,op=subset;v=8;v=8,op=subset'" \
  "ab_subset_c4_r02s|300|python3 tools/tune.py --config c4 --rounds 5 --iters 4 --variants 'v=15;v=15,op=subset'" \
  "bench_subset_c2_r02s|300|python3 bench.py --op subset"
