# Re-entry (k_levels) with loads interleaved between stores (GDP_TUNE_INPLACE_PACE = 4) vs the
# current order, alternated on one box, plus the parity tests that cover the new order (round 5)
# (historical: GDP_TUNE_INPLACE_PACE = 4 existed only in the build this A/B measured; see DESIGN_HISTORY §10)
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_state.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "zero_window_path or mirrored" > gpurun_out/gputest_regen_pace_r05l.log 2>&1
for rep in a b; do
  for p in -1 4; do
    for sub in 2 1; do
      timeout -k 10 200 python bench.py --no-cpu --op regen --inplace-sub $sub --zero-window 1 --store-pace $p \
        > gpurun_out/regen_c2_s${sub}_p${p}_${rep}_r05l.log 2>&1
    done
  done
done
timeout -k 10 300 python bench.py --no-cpu --op regen > gpurun_out/bench_regen_c2_r05l.log 2>&1
timeout -k 10 300 python bench.py --no-cpu --op regen --config c4 > gpurun_out/bench_regen_c4_r05l.log 2>&1
echo done
