# round-3 session r: conv octave split (octave 0 and octaves >= 1 as two concurrent launches) —
# bit-identity tests, then the A/B against the one-launch block tiles on configs 2-5
exec tools/gpu_session.sh \
  "conv_split_tests_r03r|400|python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -k 'convolution or conv_octave_split or conv_row or conv_block'" \
  "conv_split_c2_r03r|300|python tools/tune.py --op conv --config c2 --rotate 5 --iters 20 --rounds 5 --variants 'ck=2,cr=32,co=4;ck=2,cr=32,co=4,cs=1;ck=2,cr=32,co=0,cs=1;ck=2,cr=32,co=1,cs=1'" \
  "conv_split_c4_r03r|300|python tools/tune.py --op conv --config c4 --iters 2 --rounds 3 --variants 'ck=2,cr=32,co=4;ck=2,cr=32,co=4,cs=1;ck=2,cr=32,co=1,cs=1'" \
  "conv_split_c5_r03r|300|python tools/tune.py --op conv --config c5 --iters 5 --rounds 3 --variants 'ck=2,cr=32,co=4;ck=2,cr=32,co=4,cs=1;ck=2,cr=32,co=1,cs=1'" \
  "conv_split_c3_r03r|300|python tools/tune.py --op conv --config c3 --iters 3 --rounds 3 --variants 'ck=2,cr=32,co=4;ck=2,cr=32,co=4,cs=1'"
