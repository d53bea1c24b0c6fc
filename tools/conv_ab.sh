# Interleaved A/B of the convolution-extension kernels (tools/tune.py --op conv) on configs 2-5.
set -o pipefail
S="ck=0,cr=16,co=0;ck=0,cr=16,co=4;ck=0,cr=16,co=5;ck=2,cr=32,co=0;ck=2,cr=32,co=1;ck=2,cr=32,co=4;ck=2,cr=32,co=5;ck=2,cr=48,co=4;ck=2,cr=48,co=5"
timeout -k 10 200 python -u tools/tune.py --op conv --config c2 --rotate 5 --iters 20 --rounds 5 --variants "$S" > gpurun_out/conv_ab_c2.log 2>&1 &&
timeout -k 10 200 python -u tools/tune.py --op conv --config c3 --iters 3 --rounds 3 --variants "$S" > gpurun_out/conv_ab_c3.log 2>&1 &&
timeout -k 10 300 python -u tools/tune.py --op conv --config c4 --iters 2 --rounds 3 --variants "$S" > gpurun_out/conv_ab_c4.log 2>&1 &&
timeout -k 10 200 python -u tools/tune.py --op conv --config c5 --iters 5 --rounds 3 --variants "$S" > gpurun_out/conv_ab_c5.log 2>&1
rc=$?; cat gpurun_out/conv_ab_*.log | grep variant; exit $rc
