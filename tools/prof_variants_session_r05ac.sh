# rocprofv3 kernel traces (--stats) of the default command pinned to v15 / v16 / v17 and of the
# default command itself, after the streams figure became opt-in (round 5)
set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for v in 15 16 17; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c2_v${v}_r05ac -o run --output-format csv -- \
    python3 $R/bench.py --steps 200 --warmup 5 --no-cpu --variant $v --tile-order 0 --zero-window 1 > $R/gpurun_out/prof_c2_v${v}_r05ac.log 2>&1
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_default_r05ac -o run --output-format csv -- \
  python3 $R/bench.py > $R/gpurun_out/prof_default_r05ac.log 2>&1
echo done
