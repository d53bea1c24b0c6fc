# examples/serve_threads: concurrent contexts from host threads (round 5)
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "serve_threads" > gpurun_out/gputest_serve_threads_r05s.log 2>&1
for t in 1 2 4 6; do
  timeout -k 10 120 examples/serve_threads 4096 $t 100 >> gpurun_out/serve_threads_c2_r05s.log 2>&1
done
echo done
