# Two-rank gloo rehearsals on one GPU on the final tree (round 5): c2 build, c5 row bands, c5 conv
# row bands with the halo exchange every step (block order 5 on the bands)
set -e
mkdir -p gpurun_out
GDP_BENCH_BACKEND=gloo timeout -k 10 280 python3 bench.py --gpus 2 --steps 50 --warmup 5 > gpurun_out/selflaunch_gloo2_c2_r05y.log 2>&1
GDP_BENCH_BACKEND=gloo timeout -k 10 280 python3 bench.py --config c5 --gpus 2 --steps 20 --warmup 3 > gpurun_out/selflaunch_gloo2_c5_r05y.log 2>&1
GDP_BENCH_BACKEND=gloo timeout -k 10 280 python3 bench.py --gpus 2 --op conv --config c5 --steps 10 --warmup 2 --no-cpu > gpurun_out/selflaunch_gloo2_conv_c5_r05y.log 2>&1
echo done
