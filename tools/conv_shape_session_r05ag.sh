# Convolution block tiles under order 5: 8-wave shapes that fit 4 blocks per CU (24 / 16 rows) vs
# the 48-row 16-wave default, c2 and c4, alternated (round 5)
set -e
mkdir -p gpurun_out
for rep in a b; do
  for rw in "48 16" "24 8" "16 8"; do
    set -- $rw
    timeout -k 10 200 python3 bench.py --op conv --conv-rows $1 --conv-waves $2 --no-cpu > gpurun_out/conv_r$1w$2_c2_${rep}_r05ag.log 2>&1
    timeout -k 10 300 python3 bench.py --op conv --conv-rows $1 --conv-waves $2 --config c4 --no-cpu --steps 10 --warmup 2 > gpurun_out/conv_r$1w$2_c4_${rep}_r05ag.log 2>&1
  done
done
echo done
