# round-3 session af: output row pitch / stride alignment, wider sweep.  (ae: a 4096-float pitch
# takes 16 x 4096x3840 from 1.55 to 1.31 ms with v15, and a 4160 pitch takes 16 x 4096^2 from 1.31
# to 1.59 ms; config 3's v11 unchanged at a 2048 pitch.)
T="python tools/tune.py --iters 3 --rounds 4 --no-check"
ALL="v=0;v=1;v=2;v=3;v=4;v=5;v=7;v=8;v=9;v=10;v=11;v=12;v=13;v=14;v=15;v=16;v=17;v=18"
exec tools/gpu_session.sh \
  "opitch_c3_p2_all_r03af|400|GDP_OUT_PITCH=1 $T --config c3 --variants '$ALL'" \
  "opitch_c3_def_all_r03af|400|$T --config c3 --variants '$ALL'" \
  "opitch_w3840_sweep_r03af|500|for p in 0 64 128 512 768 1280 2304 4352; do echo PITCH+\$p; GDP_OUT_PITCH=\$p $T --shape 4096x3840x16 --variants 'v=15;v=11'; done" \
  "align_c3_r03af|300|for a in 64 4096 65536 524288; do echo ALIGN \$a; GDP_LEVEL_ALIGN=\$a $T --config c3 --variants 'v=11;v=15'; done" \
  "align_w3840_r03af|300|for a in 64 524288; do echo ALIGN \$a; GDP_LEVEL_ALIGN=\$a $T --shape 4096x3840x16 --variants 'v=15;v=11'; done"
