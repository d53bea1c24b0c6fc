# round-2 session: PMC traffic of every subset-build instance (bench.py --op subset's autotune
# picks among them), one rocprofv3 --pmc pass per counter; then the subset bench line
exec tools/gpu_session.sh \
  "pmcs_fetch|300|timeout -s KILL 290 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcs_fetch -o run --output-format csv -- python3 tools/pmc_variants.py --config c2 --op subset --manifest gpurun_out/pmcs_manifest.json" \
  "pmcs_write|300|timeout -s KILL 290 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcs_write -o run --output-format csv -- python3 tools/pmc_variants.py --config c2 --op subset --manifest gpurun_out/pmcs_manifest.json" \
  "bench_subset_c2_r02n|300|python3 bench.py --op subset"
