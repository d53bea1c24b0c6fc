# round-3 session ao: window support in the in-place passes — parity (the zero-window test now
# covers k_levels / k_levels_x / k_window re-entry, and every in-place test), and the in-place bench
# lines with the (shape x zero window) autotune; then (chained in the gpurun command) PMC records of
# every zero-window in-place instance: ZW=1 tools/pmc_inplace.sh c2 / c4
exec tools/gpu_session.sh \
  "zwi2_parity_r03ao|500|python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k 'zero_window or inplace or regen or gauss or generate_dog or window'" \
  "bench_regen_c2_r03ao|200|python3 bench.py --op regen --no-cpu" \
  "bench_gauss_c2_r03ao|200|python3 bench.py --op gauss --no-cpu" \
  "bench_regen_c4_r03ao|300|python3 bench.py --op regen --config c4 --steps 10 --warmup 2 --no-cpu" \
  "bench_gauss_c4_r03ao|300|python3 bench.py --op gauss --config c4 --steps 10 --warmup 2 --no-cpu"
