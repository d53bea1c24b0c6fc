# round-3 session ag (re-entry after a container rebuild): the tree as committed — GPU suite, smoke,
# the driver's default command, the convolution line — and SQ counters of k_conv_blk (VALU / LDS /
# wait breakdown) to decide where its remaining time goes
P="timeout -s KILL 90 rocprofv3"
CONV="python3 bench.py --op conv --steps 20 --warmup 3 --no-cpu"
exec tools/gpu_session.sh \
  "gputest_r03ag|700|python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider" \
  "smoke_r03ag|120|python3 -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench_default_r03ag|300|python3 bench.py" \
  "bench_conv_c2_r03ag|200|python3 bench.py --op conv --no-cpu" \
  "counters_list_r03ag|60|rocprofv3 -L" \
  "sq1_conv_c2_r03ag|100|$P --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d gpurun_out/sq1_conv_c2 -o run --output-format csv -- $CONV" \
  "sq2_conv_c2_r03ag|100|$P --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE -d gpurun_out/sq2_conv_c2 -o run --output-format csv -- $CONV" \
  "sq1_build_c2_r03ag|100|$P --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d gpurun_out/sq1_build_c2 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu"
