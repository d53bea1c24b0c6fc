# round-3 session an: window support in the in-place passes (k_levels / k_levels_x / k_window skip
# the window loads outside it: v * 0.0f) — parity, then interleaved A/B on configs 2 / 4 / 5
T="python tools/tune.py --rounds 7"
R="op=regen,sub=1;op=regen,sub=1,zw=1;op=regen,sub=4;op=regen,sub=4,zw=1;op=regen,sub=16;op=regen,sub=16,zw=1;op=regen,sub=0;op=regen,sub=0,zw=1"
G="op=gauss,wsub=4;op=gauss,wsub=4,zw=1;op=gauss,wsub=1;op=gauss,wsub=1,zw=1;op=gauss,wsub=16;op=gauss,wsub=16,zw=1"
exec tools/gpu_session.sh \
  "zwi_parity_r03an|400|python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k 'zero_window'" \
  "zwi_regen_c2_r03an|300|$T --config c2 --rotate 5 --iters 10 --variants '$R'" \
  "zwi_gauss_c2_r03an|300|$T --config c2 --rotate 5 --iters 10 --variants '$G'" \
  "zwi_regen_c5_r03an|300|$T --config c5 --iters 2 --variants '$R'" \
  "zwi_gauss_c5_r03an|300|$T --config c5 --iters 2 --variants '$G'" \
  "zwi_regen_c4_r03an|400|$T --config c4 --iters 2 --rounds 5 --variants '$R'" \
  "zwi_gauss_c4_r03an|400|$T --config c4 --iters 2 --rounds 5 --variants '$G'"
