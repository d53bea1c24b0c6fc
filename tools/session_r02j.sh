# round-2 session: band scatter / gather collector paths of bench.py (gloo ranks on one GPU)
exec tools/gpu_session.sh \
  "collect_c5_gloo2_r02j|300|python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 290 --timeout-method thread -k band_scatter_and_gather" \
  "collect_c5_gloo2_line_r02j|300|env GDP_BENCH_BACKEND=gloo python3 bench.py --gpus 2 --config c5 --steps 5 --warmup 2 --no-cpu --scatter --gather"
