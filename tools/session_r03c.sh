# round-3 session c: the [row][scale] row-window layout — parity of the non-square paths under it,
# then its A/B; the 64-row convolution tile A/B (test ids fixed)
exec tools/gpu_session.sh \
  "rowtap_parity_r03c|400|GDP_ROWTAP_LAYOUT=1 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -k 'shapes or variant or intlen or config3 or inplace or gauss_range or subset or row_bands or taps or fuzz or random'" \
  "ab_rowtap_r03c|700|bash tools/ab_rowtap.sh" \
  "conv_ab_r03c|600|VARIANTS='ck=2,cr=32,co=4;ck=2,cr=48,co=4;ck=2,cr=64,co=4;ck=2,cr=64,co=5' bash tools/conv_ab.sh"
