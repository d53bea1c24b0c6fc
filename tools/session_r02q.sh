# round-2 session: store cache policy of the streaming pyramid stores (timing-only library builds,
# tools/ab/libgdp_*.so from -DGDP_STORE_POLICY): nt (default) vs sc0 sc1 / sc1 / nt sc1, alternated
L=sift-parallel-optimization_amd/lib/libgdp.so
exec tools/gpu_session.sh \
  "ab_store_c2_r02q|400|TUNE_EXTRA='--rotate 5' bash tools/ab/run_ab.sh c2 40 7 'v=15;v=16' $L tools/ab/libgdp_sc0sc1.so tools/ab/libgdp_sc1.so tools/ab/libgdp_ntsc1.so $L tools/ab/libgdp_sc0sc1.so" \
  "ab_store_c4_r02q|400|bash tools/ab/run_ab.sh c4 4 5 'v=15' $L tools/ab/libgdp_sc0sc1.so tools/ab/libgdp_sc1.so tools/ab/libgdp_ntsc1.so $L tools/ab/libgdp_sc0sc1.so"
