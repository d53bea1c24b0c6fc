# round-2 session: rocprofv3 --stats of the default workload with the autotune's pick fixed
# (variant 15, tile order 0), so the stats file's k_build average covers only warm-up + timed steps
exec tools/gpu_session.sh \
  "prof_fixed_r02al|300|rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fixed_r02al -o run --output-format csv -- python3 bench.py --no-cpu --variant 15 --tile-order 0"
