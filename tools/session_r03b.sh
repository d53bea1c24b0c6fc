# round-3 session b: PMC records of the in-place passes on config 2 (every block shape the autotune
# can pick), the 64-row convolution tile A/B (tests first), and the hot-row-window timing bound of a
# tall non-square image (libgdp_hotrt.so: timing only, wrong values)
L=sift-parallel-optimization_amd/lib
exec tools/gpu_session.sh \
  "hotrt_r03b|300|for lib in \$PWD/$L/libgdp.so \$PWD/$L/libgdp_hotrt.so \$PWD/$L/libgdp.so \$PWD/$L/libgdp_hotrt.so; do echo \"## \$lib\"; GDP_LIBRARY=\$lib timeout -k 10 120 python tools/tune.py --config c2 --shape 65536x4096x1 --iters 30 --rounds 5 --no-check --variants 'v=15;v=16;v=0;v=15,ord=1' | grep variant || exit 1; done" \
  "conv_ab_r03b|900|VARIANTS='ck=2,cr=32,co=4;ck=2,cr=48,co=4;ck=2,cr=64,co=4;ck=2,cr=64,co=5' bash tools/conv_ab.sh" \
  "pmc_inplace_c2_r03b|780|bash tools/pmc_inplace.sh c2 r03"
