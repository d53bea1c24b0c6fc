# Convolution block order 4 vs 5 on configs 3 and 5, then the order-5 PMC records of configs 2-5 (round 5)
set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
for rep in a b; do
  for o in 4 5; do
    timeout -k 10 300 python3 bench.py --op conv --conv-order $o --config c3 --no-cpu --steps 10 --warmup 2 > gpurun_out/conv_o${o}_c3_${rep}_r05w.log 2>&1
    timeout -k 10 300 python3 bench.py --op conv --conv-order $o --config c5 --no-cpu --steps 10 --warmup 2 > gpurun_out/conv_o${o}_c5_${rep}_r05w.log 2>&1
  done
done
cd /tmp && export TMPDIR=/tmp
for cfg in c2 c3 c4 c5; do
  A="$R/bench.py --op conv --conv-order 5 --config $cfg --steps 3 --warmup 1 --no-cpu"
  timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pf_conv5_$cfg -o run --output-format csv -- python3 $A > $R/gpurun_out/pf_conv5_$cfg.log 2>&1
  timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pw_conv5_$cfg -o run --output-format csv -- python3 $A > $R/gpurun_out/pw_conv5_$cfg.log 2>&1
done
echo done
