# round-3 session ak: the zero-window knob in the autotune — parity (incl. the autotune and the
# bench's own checks), bench lines of configs 5 and 2 with the extended autotune, and PMC records of
# every zero-window instance on configs 5 and 2 (FETCH_SIZE / WRITE_SIZE, each its own pass)
PV="python3 tools/pmc_variants.py --zero-window 1"
exec tools/gpu_session.sh \
  "zwk_parity_r03ak|400|python -u -m pytest tests/test_gpu_parity.py tests/test_bench_accounting.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k 'zero_window or autotune or every_build_variant or bench'" \
  "bench_c5_r03ak|300|python3 bench.py --config c5 --steps 20 --warmup 3 --no-cpu" \
  "bench_c2_r03ak|300|python3 bench.py --no-cpu" \
  "pmcz_fetch_c5_r03ak|300|timeout -s KILL 290 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcz_fetch_c5 -o run --output-format csv -- $PV --config c5 --manifest gpurun_out/pmcz_manifest_c5.json" \
  "pmcz_write_c5_r03ak|300|timeout -s KILL 290 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcz_write_c5 -o run --output-format csv -- $PV --config c5 --manifest gpurun_out/pmcz_manifest_c5.json" \
  "pmcz_fetch_c2_r03ak|300|timeout -s KILL 290 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcz_fetch_c2 -o run --output-format csv -- $PV --config c2 --manifest gpurun_out/pmcz_manifest_c2.json" \
  "pmcz_write_c2_r03ak|300|timeout -s KILL 290 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcz_write_c2 -o run --output-format csv -- $PV --config c2 --manifest gpurun_out/pmcz_manifest_c2.json"
