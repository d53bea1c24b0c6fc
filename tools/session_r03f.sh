# round-3 session f: k_levels_w (the levels of a group across one wave's lanes, no barrier) — the
# in-place parity tests, its A/B against the other re-entry shapes on configs 2-5, the regen bench
# lines with it in the autotune, and PMC records of its instance on configs 2 and 4
exec tools/gpu_session.sh \
  "inplace_tests_r03f|300|python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k 'inplace or gauss_range or reentry or mirror_surface or a512'" \
  "ab_regen_c2_r03f|200|python tools/tune.py --op regen --config c2 --rotate 5 --iters 20 --rounds 5 --variants 'sub=1;sub=4;sub=2;sub=0;sub=8'" \
  "ab_regen_c4_r03f|300|python tools/tune.py --op regen --config c4 --iters 3 --rounds 3 --variants 'sub=1;sub=4;sub=0;sub=8'" \
  "ab_regen_c5_r03f|200|python tools/tune.py --op regen --config c5 --iters 5 --rounds 3 --variants 'sub=1;sub=4;sub=0;sub=8'" \
  "ab_regen_c3_r03f|200|python tools/tune.py --op regen --config c3 --iters 5 --rounds 3 --variants 'sub=1;sub=2;sub=0;sub=8'" \
  "bench_regen_c2_r03f|200|python3 bench.py --op regen --no-cpu" \
  "bench_regen_c4_r03f|300|python3 bench.py --op regen --config c4 --steps 10 --warmup 2 --no-cpu" \
  "pmc_w_c2_r03f|300|REGEN_SUBS=8 GAUSS_SUBS= bash tools/pmc_inplace.sh c2 r03" \
  "pmc_w_c4_r03f|300|REGEN_SUBS=8 GAUSS_SUBS= bash tools/pmc_inplace.sh c4 r03"
