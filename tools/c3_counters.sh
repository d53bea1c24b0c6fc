#!/usr/bin/env bash
# which counter separates config 3 (64 x 1080x1920, v11) from same-byte batches of
# larger images that stream faster (16 x 2048^2, 64 x 1024x2048 with v15)?  One SQ pass and one TCC
# pass per shape, each its own rocprofv3 run (counters never combined with trace domains).
sq="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY"
tcc="TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_STALL_sum TCC_EA0_RDREQ_sum TCC_TAG_STALL_sum"
steps=()
for spec in "c3:1080x1920x64:11" "c3:1080x1920x64:15" "c2:2048x2048x16:15" "c2:1024x2048x64:15"; do
  IFS=: read -r cfg shape v <<< "$spec"
  tag="${shape}_v${v}"
  cmd="python3 tools/tune.py --config ${cfg} --shape ${shape} --variants v=${v} --rounds 1 --iters 5 --no-check"
  steps+=("cnt_${tag}_sq|90|timeout -s KILL 80 rocprofv3 --pmc ${sq} -d gpurun_out/cnt_${tag}_sq -o run --output-format csv -- ${cmd}")
  steps+=("cnt_${tag}_tcc|90|timeout -s KILL 80 rocprofv3 --pmc ${tcc} -d gpurun_out/cnt_${tag}_tcc -o run --output-format csv -- ${cmd}")
done
exec tools/gpu_session.sh "${steps[@]}"
