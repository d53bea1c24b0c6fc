# Research A/B: convolution block tiles with rows unrolled branch-free at a set register budget (round 5)
set -e
mkdir -p gpurun_out
timeout -k 10 900 python3 tools/conv_unroll_ab.py --reps 2 > gpurun_out/conv_unroll_c2_r05q.log 2>&1
echo done
