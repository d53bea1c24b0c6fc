# Convolution block order 4 (octave-interleaved) vs 5 (the same sequence XCD-chunked, so an
# octave-o block row runs on the XCD whose L2 just staged its input rows): time + DRAM reads (round 5)
set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
for rep in a b; do
  for o in 4 5; do
    timeout -k 10 200 python3 bench.py --op conv --conv-order $o --no-cpu > gpurun_out/conv_o${o}_c2_${rep}_r05v.log 2>&1
    timeout -k 10 300 python3 bench.py --op conv --conv-order $o --config c4 --no-cpu --steps 10 --warmup 2 > gpurun_out/conv_o${o}_c4_${rep}_r05v.log 2>&1
  done
done
cd /tmp && export TMPDIR=/tmp
for o in 4 5; do
  timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_WRREQ_WRITE_DRAM_32B_sum -d $R/gpurun_out/p32_conv_o$o -o run --output-format csv -- python3 $R/bench.py --op conv --conv-order $o --steps 5 --warmup 1 --no-cpu > $R/gpurun_out/p32_conv_o$o.log 2>&1
done
echo done
