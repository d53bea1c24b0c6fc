# round-3 session q (experiment): conv kernel 3 — row windows in registers, no LDS, no barrier —
# against the block tiles; convolution tests first
V="ck=2,cr=32,co=4;ck=3,cr=32,co=4;ck=3,cr=16,co=4;ck=3,cr=32,cw=8,co=4;ck=3,cr=16,cw=8,co=4;ck=3,cr=32,co=0"
exec tools/gpu_session.sh \
  "conv_tests_r03q|400|python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -k 'convolution or conv_row or conv_config5 or conv_block'" \
  "conv_rows_c2_r03q|300|python tools/tune.py --op conv --config c2 --rotate 5 --iters 20 --rounds 5 --variants '$V'" \
  "conv_rows_c4_r03q|300|python tools/tune.py --op conv --config c4 --iters 2 --rounds 3 --variants 'ck=2,cr=32,co=4;ck=3,cr=32,co=4;ck=3,cr=32,cw=8,co=4'" \
  "conv_rows_c5_r03q|300|python tools/tune.py --op conv --config c5 --iters 5 --rounds 3 --variants 'ck=2,cr=32,co=4;ck=3,cr=32,co=4;ck=3,cr=32,cw=8,co=4'" \
  "conv_rows_c3_r03q|300|python tools/tune.py --op conv --config c3 --iters 3 --rounds 3 --variants 'ck=2,cr=32,co=4;ck=3,cr=32,co=4;ck=3,cr=32,cw=8,co=4'"
