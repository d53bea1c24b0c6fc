# round-2 session: hunt the intermittent rank-0 exit of the 2-rank banded-convolution self-launch
# (seen once after 214 tests of the suite): the self-launch tests after the rest of the parity file, twice
exec tools/gpu_session.sh \
  "hunt1_r02z|400|python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread" \
  "hunt2_r02z|400|python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread -k 'selflaunch or band or conv or mpi or cpp'"
