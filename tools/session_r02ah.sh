# round-2 session: PATH 4 build variants (octave 0 register-resident, loads first, octaves 1.. flattened)
# against v15 / v16, cold rotated buffers, interleaved in one process; identical-output check on
V="v=15;v=19;v=20;v=21;v=16;v=15,ord=1;v=19,ord=1;v=20,ord=1"
exec tools/gpu_session.sh \
  "ab_path4_c2_r02ah|240|python3 tools/tune.py --config c2 --rotate 5 --iters 20 --rounds 9 --variants '$V'" \
  "ab_path4_c5_r02ah|240|python3 tools/tune.py --config c5 --iters 5 --rounds 7 --variants '$V'" \
  "ab_path4_c4_r02ah|300|python3 tools/tune.py --config c4 --iters 3 --rounds 5 --variants '$V'" \
  "ab_path4_c3_r02ah|240|python3 tools/tune.py --config c3 --iters 5 --rounds 7 --variants 'v=11;v=15;v=19;v=20;v=21;v=16'"
