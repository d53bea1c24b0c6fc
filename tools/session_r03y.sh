# round-3 session y: long randomized sweeps — 50x the suite's case count on another seed, and
# 5x with sides up to 2048 (build / subset sweeps)
set -o pipefail
mkdir -p gpurun_out
GDP_FUZZ_SCALE=50 GDP_FUZZ_SEED=2 timeout -k 10 900 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -x -v -s \
  --timeout 880 --timeout-method thread --durations=0 > gpurun_out/fuzz_x50_seed2_r03y.log 2>&1 &&
GDP_FUZZ_SCALE=5 GDP_FUZZ_SEED=3 GDP_FUZZ_MAXDIM=2048 timeout -k 10 900 python -u -m pytest tests/test_gpu_fuzz.py -m gpu \
  -x -v -s -k "parity or subset" --timeout 880 --timeout-method thread --durations=0 > gpurun_out/fuzz_x5_2048_seed3_r03y.log 2>&1
rc=$?; tail -6 gpurun_out/fuzz_x50_seed2_r03y.log; tail -6 gpurun_out/fuzz_x5_2048_seed3_r03y.log; exit $rc
