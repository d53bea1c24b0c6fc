# round-3 session a: the GPU suite (GenerateDoG_mpi centre fix, refused conv pairs, topology /
# file-rendezvous self-launch), the default bench line, the in-place lines with their new parity,
# and the PATH 3 preload A/B (tools/ab_preload.sh)
exec tools/gpu_session.sh \
  "gputest_r03a|600|python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider" \
  "bench_c2_r03a|300|python3 bench.py" \
  "bench_regen_c2_r03a|200|python3 bench.py --op regen --no-cpu" \
  "bench_gauss_c2_r03a|200|python3 bench.py --op gauss --no-cpu" \
  "ab_preload_r03a|1000|bash tools/ab_preload.sh"
