# Convolution block order 5: 48 vs 32 rows per block (16 waves) and 32 rows x 8 waves, c2 / c4 (round 5)
set -e
mkdir -p gpurun_out
for rep in a b; do
  for rw in "48 16" "32 16" "32 8"; do
    set -- $rw
    timeout -k 10 200 python3 bench.py --op conv --conv-rows $1 --conv-waves $2 --no-cpu > gpurun_out/conv_r$1w$2_c2_${rep}_r05z.log 2>&1
    timeout -k 10 300 python3 bench.py --op conv --conv-rows $1 --conv-waves $2 --config c4 --no-cpu --steps 10 --warmup 2 > gpurun_out/conv_r$1w$2_c4_${rep}_r05z.log 2>&1
  done
done
echo done
