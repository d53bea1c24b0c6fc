# round-3 session m: smaller blocks for the in-place passes (128 / 64 threads: GDP_TUNE_*_SUB 8 / 16)
# against the shipped shapes, re-entry and window pass, configs 2-5; parity of the in-place tests
exec tools/gpu_session.sh \
  "inplace_tests_r03m|300|python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k 'inplace or gauss_range or reentry'" \
  "ab_sub_c2_r03m|200|python tools/tune.py --op regen --config c2 --rotate 5 --iters 20 --rounds 5 --variants 'sub=1;sub=4;sub=2;sub=8;sub=16;sub=0'" \
  "ab_sub_c4_r03m|300|python tools/tune.py --op regen --config c4 --iters 3 --rounds 3 --variants 'sub=1;sub=4;sub=8;sub=16;sub=0'" \
  "ab_sub_c5_r03m|200|python tools/tune.py --op regen --config c5 --iters 5 --rounds 3 --variants 'sub=1;sub=4;sub=8;sub=16'" \
  "ab_sub_c3_r03m|200|python tools/tune.py --op regen --config c3 --iters 5 --rounds 3 --variants 'sub=1;sub=2;sub=8;sub=16'" \
  "ab_wsub_c2_r03m|200|python tools/tune.py --op gauss --config c2 --rotate 5 --iters 20 --rounds 5 --variants 'wsub=4;wsub=2;wsub=8;wsub=16'" \
  "ab_wsub_c4_r03m|300|python tools/tune.py --op gauss --config c4 --iters 3 --rounds 3 --variants 'wsub=4;wsub=1;wsub=8;wsub=16'"
