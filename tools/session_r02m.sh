# round-2 session: XCD-band block order of k_conv_blk (conv order bit 3) — correctness (randomized
# convolution sweep incl. the new orders, row bands) then interleaved cold A/B on configs 2-5
V='ck=2,cr=32,co=4;ck=2,cr=32,co=12;ck=2,cr=32,co=28;ck=2,cr=32,co=44;ck=2,cr=32,co=140;ck=2,cr=48,co=44'
exec tools/gpu_session.sh \
  "conv_fuzz_r02m|300|python -u -m pytest tests/test_gpu_fuzz.py -m gpu -x -v --timeout 280 --timeout-method thread -k convolution" \
  "ab_xcdband_c2_r02m|300|python3 tools/tune.py --op conv --config c2 --rotate 5 --rounds 7 --iters 40 --variants '$V'" \
  "ab_xcdband_c4_r02m|300|python3 tools/tune.py --op conv --config c4 --rounds 5 --iters 4 --variants '$V'" \
  "ab_xcdband_c5_r02m|300|python3 tools/tune.py --op conv --config c5 --rounds 5 --iters 10 --variants '$V'" \
  "ab_xcdband_c3_r02m|300|python3 tools/tune.py --op conv --config c3 --rotate 2 --rounds 5 --iters 10 --variants '$V'"
