# round-3 session t: 224-column conv block tiles (4 halo lanes per side, every tile and wave store on
# whole 128-B lines) — tests, then the A/B against the 240-column default on configs 2-5
exec tools/gpu_session.sh \
  "conv_h4_tests_r03t|400|python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -k 'convolution or conv_row or conv_block'" \
  "conv_h4_c2_r03t|300|python tools/tune.py --op conv --config c2 --rotate 5 --iters 20 --rounds 5 --variants 'ck=2,cr=32,co=4;ck=2,cr=32,co=4,ch=4;ck=2,cr=32,co=0,ch=4'" \
  "conv_h4_c4_r03t|300|python tools/tune.py --op conv --config c4 --iters 2 --rounds 3 --variants 'ck=2,cr=32,co=4;ck=2,cr=32,co=4,ch=4'" \
  "conv_h4_c5_r03t|300|python tools/tune.py --op conv --config c5 --iters 5 --rounds 3 --variants 'ck=2,cr=32,co=4;ck=2,cr=32,co=4,ch=4'" \
  "conv_h4_c3_r03t|300|python tools/tune.py --op conv --config c3 --iters 3 --rounds 3 --variants 'ck=2,cr=32,co=4;ck=2,cr=32,co=4,ch=4'"
