# Timing decomposition of the block-tile convolution kernel (GDP_CONV_DIAG bits: 1 no global
# loads, 2 no filter arithmetic, 4 no octave-0 loads, 16 no octave>0 loads, 8 plain stores) on
# cold 4096^2 (c2, 5 rotated sets) and 64 x 4096^2 (c4).
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k convolution --timeout 120 --timeout-method thread > gpurun_out/convtest.log 2>&1 || { tail gpurun_out/convtest.log; exit 1; }
for d in ${DIAGS:-0 1 4 16}; do
  GDP_CONV_DIAG=$d timeout -k 10 120 python -u tools/tune.py --op conv --config c2 --rotate 5 --iters 20 --rounds 5 --no-check \
     --variants "${VC2:-ck=0,cr=16,co=0;ck=2,cr=16,co=0;ck=2,cr=16,co=4}" | sed "s/^/diag=$d /" >> gpurun_out/conv_diag.log || exit 1
  GDP_CONV_DIAG=$d timeout -k 10 120 python -u tools/tune.py --op conv --config c4 --iters 2 --rounds 2 --no-check \
     --variants "${VC4:-ck=0,cr=16,co=5;ck=2,cr=16,co=1;ck=2,cr=16,co=5}" | sed "s/^/diag=$d /" >> gpurun_out/conv_diag.log || exit 1
done
tail -1 gpurun_out/convtest.log
cat gpurun_out/conv_diag.log
