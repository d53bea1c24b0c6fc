# round-3 session ay: paced convolution — pace depth on 48-row tiles, 64-row tiles (80 KB of LDS, two
# blocks per CU; unpaced they lost to 32 rows), 32 rows on 8 waves
T="python tools/tune.py --rounds 7 --no-check"
V="op=conv,ck=2,cr=48,co=4,cp=2;op=conv,ck=2,cr=48,co=4,cp=1;op=conv,ck=2,cr=48,co=4,cp=3;op=conv,ck=2,cr=48,co=4,cp=0;op=conv,ck=2,cr=64,co=4,cp=2;op=conv,ck=2,cr=64,co=4,cp=1;op=conv,ck=2,cr=32,cw=8,co=4,cp=1;op=conv,ck=2,cr=48,co=4,cp=-1"
exec tools/gpu_session.sh \
  "cpy_parity_r03ay|300|python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k 'conv'" \
  "cpy_conv_c2_r03ay|300|$T --config c2 --rotate 5 --iters 20 --variants '$V'" \
  "cpy_conv_c4_r03ay|500|$T --config c4 --iters 2 --rounds 5 --variants '$V'" \
  "cpy_conv_c5_r03ay|300|$T --config c5 --iters 3 --rounds 5 --variants '$V'"
