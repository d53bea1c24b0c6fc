# round-3 session ae: the OUTPUT row pitch (timing-only GDP_OUT_PITCH: 1 = next power of two,
# N > 1 = cols + N floats at octave 0; only k_build honours it, values elsewhere wrong: --no-check).
# Each setting its own process (the pitch is fixed at context creation), default first and last.
T="python tools/tune.py --iters 3 --rounds 5 --no-check"
exec tools/gpu_session.sh \
  "opitch_w3840b16_def_r03ae|200|$T --shape 4096x3840x16 --variants 'v=15;v=11'" \
  "opitch_w3840b16_p2_r03ae|200|GDP_OUT_PITCH=1 $T --shape 4096x3840x16 --variants 'v=15;v=11'" \
  "opitch_w4096b16_def_r03ae|200|$T --shape 4096x4096x16 --variants 'v=15;v=11'" \
  "opitch_w4096b16_p64_r03ae|200|GDP_OUT_PITCH=64 $T --shape 4096x4096x16 --variants 'v=15;v=11'" \
  "opitch_c3_def_r03ae|200|$T --config c3 --variants 'v=11;v=15;v=4'" \
  "opitch_c3_p2_r03ae|200|GDP_OUT_PITCH=1 $T --config c3 --variants 'v=11;v=15;v=4'" \
  "opitch_w3840b1_def_r03ae|200|$T --shape 4096x3840x1 --rotate 5 --iters 20 --variants 'v=15;v=16'" \
  "opitch_w3840b1_p2_r03ae|200|GDP_OUT_PITCH=1 $T --shape 4096x3840x1 --rotate 5 --iters 20 --variants 'v=15;v=16'" \
  "opitch_w3840b16_def2_r03ae|200|$T --shape 4096x3840x16 --variants 'v=15;v=11'"
