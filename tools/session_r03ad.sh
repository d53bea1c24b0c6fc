# round-3 session ad: the batched 3840-wide slowdown is mostly the OUTPUT side (session ac: an
# input pitch of 4096 recovers 5 % of 20 %).  Which tile widths / tile orders avoid it?  Tiles per
# row: v15 15, v10 20, v11 10, v13 8, v14 12, v4 30; order 2 = whole tile rows per XCD
exec tools/gpu_session.sh \
  "tiles_w3840b16_r03ad|400|python tools/tune.py --shape 4096x3840x16 --iters 3 --rounds 5 --no-check --variants 'v=15;v=15,ord=2;v=10;v=11;v=11,ord=2;v=13;v=14;v=4;v=17'" \
  "tiles_w4096b16_r03ad|300|python tools/tune.py --shape 4096x4096x16 --iters 3 --rounds 5 --no-check --variants 'v=15;v=15,ord=2;v=11;v=4'" \
  "tiles_c3_r03ad|300|python tools/tune.py --config c3 --iters 3 --rounds 5 --no-check --variants 'v=11;v=11,ord=2;v=13;v=14;v=10;v=4'"
