# round-3 session am: zero-window A/B on one box over more variants (session al's bench picked
# v0 + zero window on config 5 at 1.20 ms; session ak's v8 + zero window at 1.32 ms on another box)
T="python tools/tune.py --rounds 7"
exec tools/gpu_session.sh \
  "zw3_c5_r03am|400|$T --config c5 --iters 3 --variants 'v=0;v=0,zw=1;v=8;v=8,zw=1;v=15;v=15,zw=1;v=16;v=16,zw=1;v=2;v=2,zw=1;v=5;v=5,zw=1'" \
  "zw3_c4_r03am|400|$T --config c4 --iters 3 --variants 'v=0;v=0,zw=1;v=15;v=15,zw=1;v=15,ord=1;v=15,ord=1,zw=1;v=8,zw=1'" \
  "zw3_c2_r03am|300|$T --config c2 --rotate 5 --iters 20 --variants 'v=0;v=0,zw=1;v=15;v=15,zw=1;v=16;v=16,zw=1;v=8;v=8,zw=1'" \
  "bench_c5_r03am|300|python3 bench.py --config c5 --steps 20 --warmup 3 --no-cpu"
