# round-3 session o: parity of the in-place passes with the 128 / 64-thread shapes, PMC records of
# the new shapes (configs 2 and 4), the conv tile-height A/B (session n) and the regen / gauss
# bench lines with the widened autotune
exec tools/gpu_session.sh \
  "inplace_tests_r03o|300|python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k 'inplace or gauss_range or reentry or mirror or a512 or dropin or single_gpu'" \
  "pmc_sub_c2_r03o|400|REGEN_SUBS='8 16' GAUSS_SUBS='8 16' bash tools/pmc_inplace.sh c2 r03" \
  "pmc_sub_c4_r03o|400|REGEN_SUBS='8 16' GAUSS_SUBS='8 16' bash tools/pmc_inplace.sh c4 r03" \
  "conv_T_r03o|700|bash tools/session_r03n.sh" \
  "bench_regen_c2_r03o|200|python3 bench.py --op regen --no-cpu" \
  "bench_gauss_c2_r03o|200|python3 bench.py --op gauss --no-cpu" \
  "bench_regen_c5_r03o|300|python3 bench.py --op regen --config c5 --steps 20 --warmup 3 --no-cpu"
