# round-3 session w: per-launch fixed cost of today's build — cold 4096^2 batches of 1 / 2 / 4 / 8
# images per launch (rotated sets >= 2 GiB), v15 and v16
exec tools/gpu_session.sh \
  "fixed_b1_r03w|200|python tools/tune.py --config c2 --shape 4096x4096x1 --rotate 5 --iters 40 --rounds 5 --no-check --variants 'v=15;v=16'" \
  "fixed_b2_r03w|200|python tools/tune.py --config c2 --shape 4096x4096x2 --rotate 3 --iters 20 --rounds 5 --no-check --variants 'v=15;v=16'" \
  "fixed_b4_r03w|200|python tools/tune.py --config c2 --shape 4096x4096x4 --rotate 2 --iters 10 --rounds 5 --no-check --variants 'v=15;v=16'" \
  "fixed_b8_r03w|200|python tools/tune.py --config c2 --shape 4096x4096x8 --rotate 1 --iters 5 --rounds 5 --no-check --variants 'v=15;v=16'"
