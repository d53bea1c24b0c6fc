# Within-box spread of the headline: the default command five times back to back (no CPU sample)
set -e
mkdir -p gpurun_out
for k in 1 2 3 4 5; do
  timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench_default_rep${k}_r05ae.log 2>&1
done
echo done
