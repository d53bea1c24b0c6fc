# FETCH_SIZE (its own rocprofv3 pass) of the convolution kernels on config 4 / config 2, one run per
# kernel / block order: tag:kernel:order
set -o pipefail
for spec in ${SPECS:-c4s:0:5 c4b:2:1 c4b5:2:5 c4r:3:1 c2s:0:0 c2b:2:4}; do
  IFS=: read tag ck co <<< "$spec"
  cfg=c${tag:1:1}
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcconv_$tag -o run --output-format csv -- \
    python3 bench.py --op conv --config $cfg --conv-kernel $ck --conv-order $co --steps 3 --warmup 1 --no-cpu \
    > gpurun_out/pmcconv_$tag.log 2>&1 || { tail -5 gpurun_out/pmcconv_$tag.log; exit 1; }
done
