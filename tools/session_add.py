#!/usr/bin/env python3
"""Record a GPU session in tools/sessions.json (run it with tools/run_session.sh <id>):
    python3 tools/session_add.py r04b "what the session measures" "name|limit_s|command" ...
An existing id is replaced only with --replace."""
import json
import os
import sys

path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "sessions.json")
args = sys.argv[1:]
replace = "--replace" in args
args = [a for a in args if a != "--replace"]
if len(args) < 3:
    sys.exit(__doc__)
sid, comment, specs = args[0], args[1], args[2:]
with open(path) as f:
    m = json.load(f)
if sid in m and not replace:
    sys.exit(f"session {sid} exists (--replace to overwrite)")
steps = []
for spec in specs:
    name, limit, cmd = spec.split("|", 2)
    steps.append({"name": name, "limit": int(limit), "cmd": cmd})
m[sid] = {"comment": comment, "steps": steps}
with open(path, "w") as f:
    json.dump(m, f, indent=1)
print(f"{sid}: {len(steps)} steps")
