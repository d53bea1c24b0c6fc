# round-3 session x: the extended randomized sweep (window centres, tile order 2, in-place
# follow-ups with random block splits) at the suite's size, then a 5x longer sweep on other seeds
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -x -v --timeout 280 --timeout-method thread \
  --durations=0 > gpurun_out/fuzz_default_r03x.log 2>&1 &&
GDP_FUZZ_SCALE=5 GDP_FUZZ_SEED=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -x -v -s \
  --timeout 880 --timeout-method thread --durations=0 > gpurun_out/fuzz_x5_seed1_r03x.log 2>&1
rc=$?; tail -5 gpurun_out/fuzz_default_r03x.log; tail -8 gpurun_out/fuzz_x5_seed1_r03x.log; exit $rc
