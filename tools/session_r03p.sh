# round-3 session p (experiment): 4-wave blocks for the fused build, flattened (v19 16x64, v20 8x128)
exec tools/gpu_session.sh \
  "ab_small_c2_r03p|200|python tools/tune.py --config c2 --rotate 5 --iters 30 --rounds 5 --variants 'v=15;v=16;v=19;v=20'" \
  "ab_small_c5_r03p|200|python tools/tune.py --config c5 --iters 5 --rounds 3 --variants 'v=15;v=16;v=19;v=20'" \
  "ab_small_c4_r03p|300|python tools/tune.py --config c4 --iters 3 --rounds 3 --variants 'v=15;v=15,ord=1;v=0,ord=1;v=19;v=20'" \
  "ab_small_c3_r03p|200|python tools/tune.py --config c3 --iters 10 --rounds 3 --variants 'v=11;v=19;v=20'"
