# round-2 session: stability — the whole GPU suite twice on one box (the driver runs it once at round end)
exec tools/gpu_session.sh \
  "stab1_r02ac|600|python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread" \
  "stab2_r02ac|600|python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread"
