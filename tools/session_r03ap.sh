# round-3 session ap: store pacing (GDP_TUNE_STORE_PACE: s_waitcnt vmcnt(n) after each pyramid store)
# for the convolution block tiles (their five stores per row go out back to back; SQ counters show
# 44 % issue stalls) and for the build's outside-support groups (zero window) — A/B, one process each
T="python tools/tune.py --rounds 7 --no-check"
C="op=conv,ck=2,cr=32,co=4"
exec tools/gpu_session.sh \
  "sp_parity_r03ap|300|python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k 'zero_window or conv'" \
  "sp_conv_c2_r03ap|300|$T --config c2 --rotate 5 --iters 20 --variants '$C;$C,sp=0;$C,sp=1;$C,sp=2;$C,sp=3'" \
  "sp_conv_c4_r03ap|400|$T --config c4 --iters 2 --rounds 5 --variants '$C;$C,sp=0;$C,sp=1;$C,sp=2;$C,sp=3'" \
  "sp_conv_c5_r03ap|300|$T --config c5 --iters 3 --variants '$C;$C,sp=0;$C,sp=1;$C,sp=3'" \
  "sp_zw_c2_r03ap|300|$T --config c2 --rotate 5 --iters 20 --variants 'v=15;v=15,zw=1;v=15,zw=1,sp=0;v=15,zw=1,sp=1;v=15,zw=1,sp=2;v=16;v=16,zw=1,sp=0;v=16,zw=1,sp=1'" \
  "sp_zw_c4_r03ap|400|$T --config c4 --iters 2 --rounds 5 --variants 'v=15,ord=1;v=15,ord=1,zw=1;v=15,ord=1,zw=1,sp=0;v=15,ord=1,zw=1,sp=1'" \
  "sp_zw_c5_r03ap|300|$T --config c5 --iters 3 --variants 'v=15;v=0,zw=1;v=0,zw=1,sp=0;v=0,zw=1,sp=1;v=16,zw=1,sp=0'"
