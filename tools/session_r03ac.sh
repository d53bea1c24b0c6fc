# round-3 session ac: is k_build's slowdown on batches of 3840-wide images (session ab) the INPUT
# pitch / image stride?  Same output layout, input read from a caller buffer with a padded pitch
# (4096) or a padded image stride; config 3 (1920 wide) the same way
exec tools/gpu_session.sh \
  "inpitch_w3840b16_r03ac|300|python tools/tune.py --shape 4096x3840x16 --iters 3 --rounds 5 --no-check --variants 'v=15;v=15,ip=3840;v=15,ip=4096;v=15,ip=3840,is=15729664;v=15,ip=3968'" \
  "inpitch_c3_r03ac|300|python tools/tune.py --config c3 --iters 3 --rounds 5 --no-check --variants 'v=11;v=11,ip=1920;v=11,ip=2048;v=11,ip=1920,is=2074624;v=15;v=15,ip=2048'" \
  "inpitch_w4096b16_r03ac|300|python tools/tune.py --shape 4096x4096x16 --iters 3 --rounds 5 --no-check --variants 'v=15;v=15,ip=4096;v=15,ip=4224'"
