# round-3 session aw: do the convolution's other block shapes / orders change rank once its stores
# are paced?  (T = 16 / 32 / 48 on 16 waves, T = 16 / 32 on 8 waves, orders 4 / 5 / 0; cp = pace)
T="python tools/tune.py --rounds 7 --no-check"
V="op=conv,ck=2,cr=32,co=4,cp=2;op=conv,ck=2,cr=32,co=4,cp=-1;op=conv,ck=2,cr=48,co=4,cp=2;op=conv,ck=2,cr=16,co=4,cp=2;op=conv,ck=2,cr=32,cw=8,co=4,cp=2;op=conv,ck=2,cr=16,cw=8,co=4,cp=2;op=conv,ck=2,cr=32,co=5,cp=2;op=conv,ck=2,cr=32,co=0,cp=2;op=conv,ck=2,cr=32,co=4,cp=0"
exec tools/gpu_session.sh \
  "cpw_conv_c2_r03aw|300|$T --config c2 --rotate 5 --iters 20 --variants '$V'" \
  "cpw_conv_c4_r03aw|500|$T --config c4 --iters 2 --rounds 5 --variants '$V'" \
  "cpw_conv_c5_r03aw|300|$T --config c5 --iters 3 --rounds 5 --variants '$V'"
