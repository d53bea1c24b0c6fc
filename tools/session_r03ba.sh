# round-3 session ba: the launch's drain — the last N blocks of a build do not pace their stores
# (GDP_TUNE_PACE_TAIL; paced waves take five round trips each, which only lengthens the tail)
T="python tools/tune.py --rounds 9"
Z="zw=1,sp=0"
exec tools/gpu_session.sh \
  "pt_parity_r03ba|300|python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k 'zero_window or every_build_variant'" \
  "pt_c2_r03ba|300|$T --config c2 --rotate 5 --iters 20 --variants 'v=8,$Z;v=8,$Z,pt=256;v=8,$Z,pt=512;v=8,$Z,pt=1024;v=8,$Z,pt=2048;v=15,$Z;v=15,$Z,pt=256;v=15,$Z,pt=512;v=15,$Z,pt=1024;v=16,$Z,pt=1024'" \
  "pt_c4_r03ba|400|$T --config c4 --iters 2 --rounds 5 --variants 'v=0,ord=1,$Z;v=0,ord=1,$Z,pt=512;v=0,ord=1,$Z,pt=2048'" \
  "pt_c5_r03ba|300|$T --config c5 --iters 3 --rounds 5 --variants 'v=8,$Z;v=8,$Z,pt=512;v=8,$Z,pt=2048;v=0,$Z;v=0,$Z,pt=1024'"
