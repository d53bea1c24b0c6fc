# round-2 session: 8-rank gloo rehearsal (one GPU) of the row-band config with the input scatter and
# the collector's band gather to rank 0 (the N = 8 code path of --scatter / --gather)
exec tools/gpu_session.sh \
  "collect_c5_gloo8_r02t|600|env GDP_BENCH_BACKEND=gloo python3 bench.py --gpus 8 --config c5 --steps 5 --warmup 2 --no-cpu --no-autotune --scatter --gather"
