# round-3 session d: the full GPU suite with the [row][scale] row-window default, config 3's PMC
# records of every build instance re-taken with it (tools/pmc_variants.py), the config 3 bench line
exec tools/gpu_session.sh \
  "gputest_r03d|600|python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider" \
  "pmcv_fetch_c3_r03d|300|timeout -s KILL 290 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcv_fetch_c3 -o run --output-format csv -- python3 tools/pmc_variants.py --config c3 --manifest gpurun_out/pmcv_manifest_c3.json" \
  "pmcv_write_c3_r03d|300|timeout -s KILL 290 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcv_write_c3 -o run --output-format csv -- python3 tools/pmc_variants.py --config c3 --manifest gpurun_out/pmcv_manifest_c3.json" \
  "bench_c3_r03d|300|python3 bench.py --config c3 --steps 20 --warmup 3 --no-cpu"
