# round-3 session ah: whole-row build tiles (variants 19-22: 2 / 4 x 1920, 2 / 4 x 960) — parity,
# then interleaved A/B against v11 (config 3's default) and v15 / v16 on configs 3 / 2 / 4
T="python tools/tune.py --iters 3 --rounds 5"
exec tools/gpu_session.sh \
  "rowtile_parity_r03ah|300|python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k 'every_build_variant'" \
  "rowtile_c3_r03ah|400|$T --config c3 --rotate 1 --variants 'v=11;v=19;v=20;v=21;v=22;v=4;v=16'" \
  "rowtile_c2_r03ah|300|$T --config c2 --rotate 5 --iters 20 --variants 'v=15;v=16;v=20;v=22'" \
  "rowtile_c4_r03ah|400|$T --config c4 --variants 'v=15;v=16;v=20;v=22'"
