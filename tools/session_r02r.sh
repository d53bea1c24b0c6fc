# round-2 session: non-temporal input loads in k_build (timing-only build tools/ab/libgdp_inNT.so) vs default
L=sift-parallel-optimization_amd/lib/libgdp.so
N=tools/ab/libgdp_inNT.so
exec tools/gpu_session.sh \
  "ab_inNT_c2_r02r|400|TUNE_EXTRA='--rotate 5' bash tools/ab/run_ab.sh c2 40 7 'v=15;v=16' $L $N $L $N" \
  "ab_inNT_c4_r02r|400|bash tools/ab/run_ab.sh c4 4 5 'v=15' $L $N $L $N" \
  "ab_inNT_c5_r02r|400|bash tools/ab/run_ab.sh c5 10 5 'v=15;v=15,ord=1' $L $N $L $N"
