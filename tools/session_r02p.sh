# round-2 session: subset-semantics fuzz + band test + Python mirrors
exec tools/gpu_session.sh \
  "subset_tests_r02p|400|python -u -m pytest tests/test_gpu_fuzz.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k 'subset or a512'"
