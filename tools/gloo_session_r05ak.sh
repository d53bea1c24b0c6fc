# Two-rank gloo rehearsal after the gpu_state field (round 5)
set -e
mkdir -p gpurun_out
GDP_BENCH_BACKEND=gloo timeout -k 10 280 python3 bench.py --gpus 2 --steps 50 --warmup 5 > gpurun_out/selflaunch_gloo2_c2_r05ak.log 2>&1
echo done
