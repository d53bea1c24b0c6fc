# round-3 session au: zero window mode 2 (the input of an outside-support group loaded AFTER its
# paced zero stores, so a launch's first stores do not wait for its first cold loads) vs mode 1
T="python tools/tune.py --rounds 9"
exec tools/gpu_session.sh \
  "zl_parity_r03au|300|python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k 'zero_window or every_build_variant'" \
  "zl_c2_r03au|300|$T --config c2 --rotate 5 --iters 20 --variants 'v=15;v=15,zw=1,sp=0;v=15,zw=2,sp=0;v=16,zw=1,sp=0;v=16,zw=2,sp=0;v=17,zw=1,sp=0;v=17,zw=2,sp=0;v=8,zw=1,sp=0;v=8,zw=2,sp=0;v=15,zw=2,sp=1'" \
  "zl_c4_r03au|400|$T --config c4 --iters 2 --rounds 5 --variants 'v=15,ord=1;v=0,ord=1,zw=1,sp=0;v=0,ord=1,zw=2,sp=0;v=15,ord=1,zw=2,sp=0'" \
  "zl_c5_r03au|300|$T --config c5 --iters 3 --variants 'v=15;v=0,zw=1,sp=0;v=0,zw=2,sp=0;v=8,zw=2,sp=0'" \
  "zl_c3_r03au|300|$T --config c3 --iters 3 --variants 'v=11;v=11,ord=1,zw=1,sp=0;v=11,ord=1,zw=2,sp=0;v=11,sp=1'"
