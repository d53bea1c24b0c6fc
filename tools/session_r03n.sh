# round-3 session n: the convolution block tiles' height on single images after the staging fix
# (shorter blocks = shorter launch drain, more re-staged rows): T = 8 / 16 / 24 / 32 / 48 rows,
# 16 or 8 waves, cold 4096^2 and 16384^2, batch 64 x 4096^2
exec tools/gpu_session.sh \
  "conv_T_c2_r03n|300|python tools/tune.py --op conv --config c2 --rotate 5 --iters 20 --rounds 5 --variants 'ck=2,cr=32,co=4;ck=2,cr=16,co=4;ck=2,cr=16,cw=8,co=4;ck=2,cr=24,cw=8,co=4;ck=2,cr=8,cw=8,co=4;ck=2,cr=32,cw=8,co=4;ck=2,cr=48,co=4'" \
  "conv_T_c5_r03n|300|python tools/tune.py --op conv --config c5 --iters 5 --rounds 3 --variants 'ck=2,cr=32,co=4;ck=2,cr=16,co=4;ck=2,cr=16,cw=8,co=4;ck=2,cr=24,cw=8,co=4'" \
  "conv_T_c4_r03n|300|python tools/tune.py --op conv --config c4 --iters 2 --rounds 3 --variants 'ck=2,cr=32,co=4;ck=2,cr=16,co=4;ck=2,cr=24,cw=8,co=4'"
