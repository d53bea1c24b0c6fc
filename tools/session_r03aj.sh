# round-3 session aj: GDP_TUNE_ZERO_WINDOW mode 2 (outside-support groups skip their window loads
# and multiplies but form the zero DoG levels as x - x, so the stores keep waiting for the input)
# — parity, then interleaved A/B against mode 0 and 1 (session ai: mode 1 slower except c5)
T="python tools/tune.py --rounds 7"
exec tools/gpu_session.sh \
  "zw2_parity_r03aj|300|python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k 'zero_window'" \
  "zw2_c2_r03aj|300|$T --config c2 --rotate 5 --iters 20 --variants 'v=15;v=15,zw=2;v=16;v=16,zw=2;v=15,zw=1'" \
  "zw2_c3_r03aj|300|$T --config c3 --iters 3 --variants 'v=11;v=11,zw=2;v=16;v=16,zw=2'" \
  "zw2_c4_r03aj|400|$T --config c4 --iters 3 --variants 'v=15;v=15,zw=2;v=16;v=16,zw=2'" \
  "zw2_c5_r03aj|300|$T --config c5 --iters 3 --variants 'v=15;v=15,zw=2;v=15,zw=1;v=16;v=16,zw=2'"
