# round-3 session av: final tree — GPU suite, smoke, the driver's default command plain and under
# rocprofv3 --kernel-trace --stats, the bench lines of configs 3-5 and of the convolution (now
# paced at vmcnt(2) by default) with its A/B against no pacing
T="python tools/tune.py --rounds 7 --no-check"
C="op=conv,ck=2,cr=32,co=4"
exec tools/gpu_session.sh \
  "gputest_r03av|700|python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider" \
  "smoke_r03av|120|python3 -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench_default_r03av|300|python3 bench.py" \
  "prof_default_r03av|300|rocprofv3 --kernel-trace --stats -d gpurun_out/prof_default_r03av -o run --output-format csv -- python3 bench.py --no-cpu" \
  "bench_c3_r03av|300|python3 bench.py --config c3 --steps 20 --warmup 3 --no-cpu" \
  "bench_c4_r03av|300|python3 bench.py --config c4 --steps 10 --warmup 2 --no-cpu" \
  "bench_c5_r03av|300|python3 bench.py --config c5 --steps 20 --warmup 3 --no-cpu" \
  "bench_conv_c2_r03av|200|python3 bench.py --op conv --no-cpu" \
  "bench_conv_c4_r03av|300|python3 bench.py --op conv --config c4 --steps 10 --warmup 2 --no-cpu" \
  "cp_conv_c2_r03av|300|$T --config c2 --rotate 5 --iters 20 --variants '$C,cp=-1;$C,cp=2;$C,cp=1'" \
  "cp_conv_c4_r03av|400|$T --config c4 --iters 2 --rounds 5 --variants '$C,cp=-1;$C,cp=2;$C,cp=1'"
