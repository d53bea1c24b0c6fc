#!/usr/bin/env bash
# PMC traffic of the row-band config's per-rank launch (bench.py --gpus N --config c5): every
# build instance the autotune can pick, on rank 0's band of N, one GPU; FETCH_SIZE and WRITE_SIZE
# in passes of their own.  Summarise in the container:
#   python3 tools/pmc_variants.py --summarise --config c5 --round r04 --manifest gpurun_out/pmcb<N>z<Z>_manifest.json \
#       --fetch gpurun_out/pmcb<N>z<Z>_fetch --write gpurun_out/pmcb<N>z<Z>_write
#   tools/pmc_band.sh "2 4 8" "0 1"
specs=()
for n in $1; do
  for z in $2; do
    t="pmcb${n}z${z}"
    run="python3 tools/pmc_variants.py --config c5 --band-of ${n} --zero-window ${z} --manifest gpurun_out/${t}_manifest.json"
    specs+=("${t}_fetch|120|timeout -s KILL 110 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${t}_fetch -o run --output-format csv -- ${run}")
    specs+=("${t}_write|120|timeout -s KILL 110 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${t}_write -o run --output-format csv -- ${run}")
  done
done
exec tools/gpu_session.sh "${specs[@]}"
