# round-2 session: banded convolution with halo rows (GPU tests), 2-rank self-launched gloo
# rehearsal of the banded convolution bench (halo exchange every step) on one GPU.
exec tools/gpu_session.sh \
  "gputest_conv_bands|400|python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k 'row_bands_with_halo or config5_bands_checksums or convolution' --timeout 300 --timeout-method thread" \
  "selflaunch_gloo2_conv_c5|300|GDP_BENCH_BACKEND=gloo python3 bench.py --gpus 2 --op conv --config c5 --steps 10 --warmup 2" \
  "bench_conv_c5_r02|300|python3 bench.py --op conv --config c5 --steps 50 --warmup 5 --no-cpu"
