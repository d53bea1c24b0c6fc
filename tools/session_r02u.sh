# round-2 session: a512 drop-ins after gdp_dog_range, host ASan of the new exports
exec tools/gpu_session.sh \
  "a512_tests_r02u|300|python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 250 --timeout-method thread -k 'subset or a512'" \
  "asan_r02u|300|make -s -C tools/asan run"
