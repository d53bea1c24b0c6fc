# round-2 session: in-place re-entry pass block size (GDP_TUNE_INPLACE_SUB) on configs 2 / 4 / 5
V='sub=1;sub=4;sub=2;sub=0;sub=4;sub=1'
exec tools/gpu_session.sh \
  "ab_regen_c2_r02ae|300|python3 tools/tune.py --op regen --config c2 --rotate 3 --rounds 9 --iters 20 --variants '$V'" \
  "ab_regen_c4_r02ae|300|python3 tools/tune.py --op regen --config c4 --rounds 5 --iters 3 --variants '$V'" \
  "ab_regen_c5_r02ae|300|python3 tools/tune.py --op regen --config c5 --rounds 5 --iters 6 --variants '$V'" \
  "ab_regen_c3_r02ae|300|python3 tools/tune.py --op regen --config c3 --rotate 2 --rounds 5 --iters 6 --variants '$V'"
