# round-3 session aa: does the conv block tiles' partial last tile column cost? 4096 = 17 x 240 + 16
# (an 18th column of blocks with 16 output columns) vs 3840 = 16 x 240 (no partial tiles), cold;
# k_build (256-wide tiles, no partial tiles on either) as the control
exec tools/gpu_session.sh \
  "convw_4096_r03aa|200|python tools/tune.py --op conv --shape 4096x4096x1 --rotate 5 --iters 30 --rounds 5 --no-check --variants 'ck=2,cr=32,co=4;op=build,v=15'" \
  "convw_3840_r03aa|200|python tools/tune.py --op conv --shape 4096x3840x1 --rotate 5 --iters 30 --rounds 5 --no-check --variants 'ck=2,cr=32,co=4;op=build,v=15'" \
  "convw_4096b16_r03aa|200|python tools/tune.py --op conv --shape 4096x4096x16 --iters 3 --rounds 5 --no-check --variants 'ck=2,cr=32,co=4;op=build,v=15'" \
  "convw_3840b16_r03aa|200|python tools/tune.py --op conv --shape 4096x3840x16 --iters 3 --rounds 5 --no-check --variants 'ck=2,cr=32,co=4;op=build,v=15'"
