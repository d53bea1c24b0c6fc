# round-3 session i: flattened (PATH 3) forms of the tiles that divide 1920 (v19 16x192, v20 8x320,
# v21 8x480) against config 3's v11 / v17 and on the square configs; parity of the new variants
exec tools/gpu_session.sh \
  "variant_parity_r03i|200|python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k 'every_build_variant'" \
  "ab_c3_r03i|300|python tools/tune.py --config c3 --iters 10 --rounds 5 --variants 'v=11;v=17;v=19;v=20;v=21;v=10;v=14;v=13;v=11,ord=1;v=20,ord=1'" \
  "ab_c2_r03i|200|python tools/tune.py --config c2 --rotate 5 --iters 30 --rounds 5 --variants 'v=15;v=16;v=19;v=20;v=21'" \
  "ab_c4_r03i|300|python tools/tune.py --config c4 --iters 3 --rounds 3 --variants 'v=15;v=15,ord=1;v=19;v=20;v=21'"
