# round-2 session: the driver's default bench command under rocprofv3 --kernel-trace --stats (the
# timed region's k_build dispatches averaged against the bench line's kernel_ms).
exec tools/gpu_session.sh \
  "prof_default_r02|400|rocprofv3 --kernel-trace --stats -d gpurun_out/prof_default_r02 -o run --output-format csv -- python3 bench.py"
