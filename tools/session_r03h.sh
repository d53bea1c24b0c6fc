# round-3 session h: where the convolution extension's time goes, octave by octave — cold timings
# of the block tiles (and of k_build for comparison) with 1, 2, 3 and 5 octaves on 4096^2 and
# 64 x 4096^2, and FETCH_SIZE / WRITE_SIZE of the 1-octave launch (octave 0 alone)
T="python tools/tune.py --config"
exec tools/gpu_session.sh \
  "conv_oct_c2_r03h|400|for O in 1 2 3 5; do $T c2 --rotate 5 --octaves \$O --iters 20 --rounds 5 --no-check --variants 'ck=2,cr=32,co=4,op=conv;ck=2,cr=32,co=0,op=conv;v=15' | grep variant | sed \"s/^/O=\$O /\" || exit 1; done" \
  "conv_oct_c4_r03h|400|for O in 1 5; do $T c4 --octaves \$O --iters 3 --rounds 3 --no-check --variants 'ck=2,cr=32,co=4,op=conv;v=15' | grep variant | sed \"s/^/O=\$O /\" || exit 1; done" \
  "conv_o1_fetch_r03h|120|timeout -s KILL 110 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/conv_o1_fetch -o run --output-format csv -- python3 tools/tune.py --config c2 --rotate 5 --octaves 1 --iters 5 --rounds 2 --no-check --op conv --variants 'ck=2,cr=32,co=4'" \
  "conv_o1_write_r03h|120|timeout -s KILL 110 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/conv_o1_write -o run --output-format csv -- python3 tools/tune.py --config c2 --rotate 5 --octaves 1 --iters 5 --rounds 2 --no-check --op conv --variants 'ck=2,cr=32,co=4'" \
  "conv_o5_fetch_r03h|120|timeout -s KILL 110 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/conv_o5_fetch -o run --output-format csv -- python3 tools/tune.py --config c2 --rotate 5 --octaves 5 --iters 5 --rounds 2 --no-check --op conv --variants 'ck=2,cr=32,co=4;ck=2,cr=32,co=0'"
