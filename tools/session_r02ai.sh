# round-2 session: k_levels_x with 16 / L chunks per block (GDP_TUNE_INPLACE_SUB = 3) — parity of the
# in-place passes, then interleaved A/B of the re-entry pass's block shapes on configs 2 / 4 / 5
V="v=15,sub=0;v=15,sub=3;v=15,sub=4;v=15,sub=1"
exec tools/gpu_session.sh \
  "inplace_tests_r02ai|300|python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k 'inplace or gauss_range or reentry or re_entry'" \
  "ab_regen_c2_r02ai|240|python3 tools/tune.py --config c2 --op regen --rotate 3 --iters 20 --rounds 9 --variants '$V'" \
  "ab_regen_c4_r02ai|300|python3 tools/tune.py --config c4 --op regen --iters 3 --rounds 5 --variants '$V'" \
  "ab_regen_c5_r02ai|240|python3 tools/tune.py --config c5 --op regen --iters 5 --rounds 7 --variants '$V'"
