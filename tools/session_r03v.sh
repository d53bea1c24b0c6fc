# round-3 session v: config 3 store policy and tile orders for v11 (plain vs non-temporal stores)
exec tools/gpu_session.sh \
  "ab_c3_nt_r03v|300|python tools/tune.py --config c3 --iters 10 --rounds 5 --variants 'v=11;v=11,nt=0;v=11,ord=1;v=11,ord=2;v=11,ord=1,nt=0;v=14;v=14,nt=0'"
