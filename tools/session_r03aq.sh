# round-3 session aq: store pacing on the full build path too (s_waitcnt vmcnt(n) after each store,
# GDP_TUNE_STORE_PACE) and with the zero window — session ap: zero window + vmcnt(0) beat the
# default on config 2 (0.0871 vs 0.0886 ms) and config 5 (1.275 vs 1.381)
T="python tools/tune.py --rounds 7"
exec tools/gpu_session.sh \
  "sp2_parity_r03aq|300|python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k 'zero_window or every_build_variant'" \
  "sp2_c2_r03aq|300|$T --config c2 --rotate 5 --iters 20 --variants 'v=15;v=15,sp=0;v=15,sp=1;v=15,zw=1,sp=0;v=16;v=16,sp=0;v=16,zw=1,sp=0;v=0,zw=1,sp=0;v=8,zw=1,sp=0'" \
  "sp2_c4_r03aq|400|$T --config c4 --iters 2 --rounds 5 --variants 'v=15,ord=1;v=15,ord=1,sp=0;v=15,ord=1,sp=1;v=15,ord=1,zw=1,sp=0;v=0,ord=1,zw=1,sp=0;v=16,ord=1,zw=1,sp=0'" \
  "sp2_c3_r03aq|300|$T --config c3 --iters 3 --variants 'v=11;v=11,sp=0;v=11,sp=1;v=11,zw=1,sp=0;v=4,zw=1,sp=0;v=16,zw=1,sp=0'" \
  "sp2_c5_r03aq|300|$T --config c5 --iters 3 --variants 'v=15;v=15,sp=0;v=0,zw=1,sp=0;v=15,zw=1,sp=0;v=8,zw=1,sp=0'"
