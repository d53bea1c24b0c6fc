# round-2 session: reproduce the 2-rank banded-convolution self-launch failure with full stderr
exec tools/gpu_session.sh \
  "conv_band2_r02y|300|env GDP_BENCH_BACKEND=gloo python3 bench.py --gpus 2 --op conv --config c5 --steps 2 --warmup 1"
