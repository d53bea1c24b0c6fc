# round-2 session: the in-place passes (re-entry GenerateDoG, GaussFilter window) on the current tree
exec tools/gpu_session.sh \
  "bench_regen_c2_r02ad|200|python3 bench.py --op regen --no-cpu" \
  "bench_gauss_c2_r02ad|200|python3 bench.py --op gauss --no-cpu" \
  "ab_regen_r02ad|300|python3 tools/tune.py --op regen --config c2 --rotate 3 --rounds 7 --iters 20 --variants 'sub=0;sub=1;sub=2;sub=4;sub=0,nt=0;sub=1,nt=0'"
