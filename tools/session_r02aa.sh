# round-2 session: the self-launched gloo rehearsals with loopback-pinned pairs
exec tools/gpu_session.sh \
  "selflaunch_r02aa|400|python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread -k 'selflaunch or scatter_and_gather'"
