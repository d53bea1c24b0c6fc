# round-3 session al: PMC records of every zero-window build instance on configs 3 and 4 (each
# counter its own pass), and the bench lines of configs 3 / 4 with the extended autotune
PV="python3 tools/pmc_variants.py --zero-window 1"
exec tools/gpu_session.sh \
  "pmcz_fetch_c3_r03al|300|timeout -s KILL 290 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcz_fetch_c3 -o run --output-format csv -- $PV --config c3 --manifest gpurun_out/pmcz_manifest_c3.json" \
  "pmcz_write_c3_r03al|300|timeout -s KILL 290 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcz_write_c3 -o run --output-format csv -- $PV --config c3 --manifest gpurun_out/pmcz_manifest_c3.json" \
  "pmcz_fetch_c4_r03al|300|timeout -s KILL 290 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcz_fetch_c4 -o run --output-format csv -- $PV --config c4 --manifest gpurun_out/pmcz_manifest_c4.json" \
  "pmcz_write_c4_r03al|300|timeout -s KILL 290 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcz_write_c4 -o run --output-format csv -- $PV --config c4 --manifest gpurun_out/pmcz_manifest_c4.json" \
  "bench_c3_r03al|300|python3 bench.py --config c3 --steps 20 --warmup 3 --no-cpu" \
  "bench_c4_r03al|300|python3 bench.py --config c4 --steps 10 --warmup 2 --no-cpu" \
  "bench_c5_r03al|300|python3 bench.py --config c5 --steps 20 --warmup 3 --no-cpu"
