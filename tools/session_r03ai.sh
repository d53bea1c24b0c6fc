# round-3 session ai: GDP_TUNE_ZERO_WINDOW (groups outside every window's support store their
# input-independent DoG levels without waiting for the input) — parity, then interleaved A/B
T="python tools/tune.py --rounds 7"
exec tools/gpu_session.sh \
  "zw_parity_r03ai|300|python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k 'zero_window or every_build_variant or negative'" \
  "zw_c2_r03ai|300|$T --config c2 --rotate 5 --iters 20 --variants 'v=15;v=15,zw=1;v=16;v=16,zw=1;v=0;v=0,zw=1'" \
  "zw_c3_r03ai|300|$T --config c3 --iters 3 --variants 'v=11;v=11,zw=1;v=4;v=4,zw=1;v=16;v=16,zw=1'" \
  "zw_c4_r03ai|400|$T --config c4 --iters 3 --variants 'v=15;v=15,zw=1;v=16;v=16,zw=1'" \
  "zw_c5_r03ai|300|$T --config c5 --iters 3 --variants 'v=15;v=15,zw=1;v=16;v=16,zw=1'"
