# round-2 session: FETCH_SIZE / WRITE_SIZE of every build-kernel instance on configs 3, 4 and 5
# (tools/pmc_variants.py; each counter in its own rocprofv3 pass).
steps=()
for c in c3 c4 c5; do
  steps+=("pmcv_fetch_$c|300|timeout -s KILL 290 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcv_fetch_$c -o run --output-format csv -- python3 tools/pmc_variants.py --config $c --manifest gpurun_out/pmcv_manifest_$c.json")
  steps+=("pmcv_write_$c|300|timeout -s KILL 290 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcv_write_$c -o run --output-format csv -- python3 tools/pmc_variants.py --config $c --manifest gpurun_out/pmcv_manifest_$c.json")
done
exec tools/gpu_session.sh "${steps[@]}"
