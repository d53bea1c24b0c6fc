# round-3 session ab: k_build on batches of 3840-wide images streamed 20 % below 4096-wide ones
# (session aa: 16 x 4096x3840 1.53 ms vs 16 x 4096^2 1.31 ms, while one 4096x3840 image is fine) —
# which geometry does it: width, height, tile columns (odd / even), batch size, tile order?
V="v=15;v=15,ord=1;v=0;v=16"
exec tools/gpu_session.sh \
  "w3840b16_r03ab|200|python tools/tune.py --shape 4096x3840x16 --iters 3 --rounds 5 --no-check --variants '$V'" \
  "h3840b16_r03ab|200|python tools/tune.py --shape 3840x4096x16 --iters 3 --rounds 5 --no-check --variants '$V'" \
  "w3584b16_r03ab|200|python tools/tune.py --shape 4096x3584x16 --iters 3 --rounds 5 --no-check --variants '$V'" \
  "w4096b16_r03ab|200|python tools/tune.py --shape 4096x4096x16 --iters 3 --rounds 5 --no-check --variants '$V'" \
  "w3840b4_r03ab|200|python tools/tune.py --shape 4096x3840x4 --rotate 2 --iters 5 --rounds 5 --no-check --variants '$V'" \
  "w3840b2_r03ab|200|python tools/tune.py --shape 4096x3840x2 --rotate 3 --iters 10 --rounds 5 --no-check --variants '$V'" \
  "w3840b1_r03ab|200|python tools/tune.py --shape 4096x3840x1 --rotate 5 --iters 20 --rounds 5 --no-check --variants '$V'"
