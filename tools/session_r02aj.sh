# round-2 session: EXPERIMENT — XCD-chunked build tile order with each XCD's walk rotated by x * K
# tiles (tile_order 16 + K), against linear (0) and plain chunked (1), cold, interleaved
V="v=15,ord=0;v=15,ord=1;v=15,ord=17;v=15,ord=33;v=15,ord=81;v=15,ord=273;v=15,ord=145"
exec tools/gpu_session.sh \
  "ab_skew_c2_r02aj|240|python3 tools/tune.py --config c2 --rotate 5 --iters 20 --rounds 9 --variants '$V'" \
  "ab_skew_c5_r02aj|240|python3 tools/tune.py --config c5 --iters 5 --rounds 7 --variants '$V'" \
  "ab_skew_c4_r02aj|300|python3 tools/tune.py --config c4 --iters 3 --rounds 5 --variants 'v=15,ord=0;v=15,ord=1;v=15,ord=17;v=15,ord=81;v=15,ord=273'"
