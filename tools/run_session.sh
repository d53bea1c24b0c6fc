#!/usr/bin/env bash
# Run one recorded GPU session of tools/sessions.json on the gpurun box:
#     /usr/local/graft/bin/gpurun -- tools/run_session.sh r04b
# Each session is a list of steps (name, time limit, command) handed to tools/gpu_session.sh
# (every step under its own `timeout -k 10`, output to gpurun_out/<name>.log, a fatal exit ends
# the session); two round-3 sessions are plain scripts ("script").  The manifest replaces the
# ~90 one-off session_r0*.sh files rounds 2-3 left: the profiles/<name>.log
# files are those steps' logs.  `tools/run_session.sh --list` prints every session and step.
set -u
id="${1:?usage: tools/run_session.sh <session id> | --list}"
if [ "$id" = "--list" ]; then
  exec python3 - <<'PY'
import json
m = json.load(open("tools/sessions.json"))
for sid, s in m.items():
    print(f"{sid}: {s['comment']}")
    for st in s.get("steps", []):
        print(f"    {st['name']} ({st['limit']} s): {st['cmd']}")
    if "script" in s:
        print("    (script) " + s["script"].replace("\n", "\n             "))
PY
fi
mapfile -d '' specs < <(python3 - "$id" <<'PY'
import json, sys
s = json.load(open("tools/sessions.json"))[sys.argv[1]]
if "script" in s:
    sys.stdout.write("script\0" + s["script"] + "\0")
else:
    for st in s["steps"]:
        sys.stdout.write(f"{st['name']}|{st['limit']}|{st['cmd']}\0")
PY
)
[ "${#specs[@]}" -gt 0 ] || { echo "no session $id" >&2; exit 2; }
if [ "${specs[0]}" = "script" ]; then
  exec bash -c "${specs[1]}"
fi
exec tools/gpu_session.sh "${specs[@]}"
