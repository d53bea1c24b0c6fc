# round-3 session z: tile order 3 (each image's tail units right after its tiles) — parity first,
# then interleaved cold A/B against the current orders on the configs whose variants have tails
exec tools/gpu_session.sh \
  "gputest_tail_r03z|300|python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 120 --timeout-method thread -k 'variant or tail or randomized'" \
  "ab_tail_c3_r03z|300|python tools/tune.py --config c3 --iters 10 --rounds 5 --variants 'v=11,ord=0;v=11,ord=3;v=11,ord=1;v=16,ord=0;v=16,ord=3'" \
  "ab_tail_c2_r03z|200|python tools/tune.py --config c2 --rotate 5 --iters 30 --rounds 5 --variants 'v=16,ord=0;v=16,ord=3;v=15,ord=0'" \
  "ab_tail_c4_r03z|300|python tools/tune.py --config c4 --iters 3 --rounds 3 --variants 'v=16,ord=0;v=16,ord=3;v=0,ord=1;v=8,ord=0;v=8,ord=3'"
