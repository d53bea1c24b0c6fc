# Interleaved A/B of the convolution-extension kernels (tools/tune.py --op conv) on configs 2-5;
# VARIANTS overrides the candidate list.
set -o pipefail
S="${VARIANTS:-ck=0,cr=16,co=0;ck=0,cr=16,co=5;ck=2,cr=32,co=4;ck=2,cr=48,co=4;ck=2,cr=32,co=5;ck=2,cr=16,co=4}"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "convolution or row_bands_with_halo or config5_bands" --timeout 120 --timeout-method thread > gpurun_out/convtest.log 2>&1 || { tail -20 gpurun_out/convtest.log; exit 1; }
tail -1 gpurun_out/convtest.log
timeout -k 10 200 python -u tools/tune.py --op conv --config c2 --rotate 5 --iters 20 --rounds 5 --variants "$S" > gpurun_out/conv_ab_c2.log 2>&1 &&
timeout -k 10 200 python -u tools/tune.py --op conv --config c3 --iters 3 --rounds 3 --variants "$S" > gpurun_out/conv_ab_c3.log 2>&1 &&
timeout -k 10 300 python -u tools/tune.py --op conv --config c4 --iters 2 --rounds 3 --variants "$S" > gpurun_out/conv_ab_c4.log 2>&1 &&
timeout -k 10 200 python -u tools/tune.py --op conv --config c5 --iters 5 --rounds 3 --variants "$S" > gpurun_out/conv_ab_c5.log 2>&1
rc=$?; cat gpurun_out/conv_ab_*.log | grep variant; exit $rc
