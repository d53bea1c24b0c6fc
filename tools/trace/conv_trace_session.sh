# Per-wave trace of one cold k_conv_blk launch at 4096^2 for 48 / 32 / 16 rows per block (round 5)
set -e
mkdir -p gpurun_out
for T in 48 32 16; do
  timeout -k 10 180 python tools/trace/trace_blocks.py --op conv --conv-rows $T --conv-waves 16 --conv-order 4 \
    > gpurun_out/trace_conv_c2_t${T}_r05j.log 2>&1
done
echo done
