# After the mirrored-call drain guard and the gather image checks (round 5): the comm failure test,
# the mirrored GenerateDoG tests, the host ASan driver
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_state.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "comm or mirror" > gpurun_out/gputest_comm_mirror_r05m.log 2>&1
timeout -k 10 600 make -C tools/asan run > gpurun_out/asan_r05m.log 2>&1
echo done
