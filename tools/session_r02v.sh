# round-2 session: block-tile convolution for S = 4 / 5 (L = 7 / 8) — parity sweep + row bands
exec tools/gpu_session.sh \
  "conv_s45_r02v|600|python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 500 --timeout-method thread -k 'convolution or conv_row_bands'" \
  "ab_conv_s5_r02v|300|python3 tools/tune.py --op conv --config c2 --rotate 2 --rounds 5 --iters 20 --S 5 --variants 'ck=2,cr=32,co=4;ck=1'"
