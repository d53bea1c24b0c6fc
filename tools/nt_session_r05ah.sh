# Non-temporal vs plain pyramid stores on the chunked backing (round 5): interleaved in one process,
# cold rotated sets, configs 2 and 4
set -e
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/tune.py --config c2 --rotate 5 --rounds 7 --iters 20 \
  --variants "v=15;v=15,nt=0;v=16;v=16,nt=0;v=17;v=17,nt=0" > gpurun_out/nt_ab_c2_r05ah.log 2>&1
timeout -k 10 400 python3 tools/tune.py --config c4 --rotate 1 --rounds 5 --iters 3 \
  --variants "v=0;v=0,nt=0;v=15;v=15,nt=0" > gpurun_out/nt_ab_c4_r05ah.log 2>&1
echo done
