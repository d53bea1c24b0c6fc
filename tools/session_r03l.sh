# round-3 session l: HBM bytes of the tall 65536 x 4096 build (v15) with each row-window layout
# (PMC traffic beside the tune.py A/B), each counter in its own pass
T="python3 tools/tune.py --config c2 --shape 65536x4096x1 --iters 5 --rounds 1 --no-check --variants v=15"
exec tools/gpu_session.sh \
  "tall_l0_fetch_r03l|120|GDP_ROWTAP_LAYOUT=0 timeout -s KILL 110 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/tall_l0_fetch -o run --output-format csv -- $T" \
  "tall_l0_write_r03l|120|GDP_ROWTAP_LAYOUT=0 timeout -s KILL 110 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/tall_l0_write -o run --output-format csv -- $T" \
  "tall_l1_fetch_r03l|120|GDP_ROWTAP_LAYOUT=1 timeout -s KILL 110 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/tall_l1_fetch -o run --output-format csv -- $T" \
  "tall_l1_write_r03l|120|GDP_ROWTAP_LAYOUT=1 timeout -s KILL 110 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/tall_l1_write -o run --output-format csv -- $T" \
  "tall_trace_r03l|200|rocprofv3 --kernel-trace --stats -d gpurun_out/tall_trace -o run --output-format csv -- python3 tools/tune.py --config c2 --shape 65536x4096x1 --iters 20 --rounds 3 --no-check --variants v=15"
