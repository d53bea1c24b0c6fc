# round-3 session bb: the driver's exact default command three times on one box (final tree)
exec tools/gpu_session.sh \
  "repeat1_r03bb|300|python3 bench.py" \
  "repeat2_r03bb|300|python3 bench.py" \
  "repeat3_r03bb|300|python3 bench.py"
