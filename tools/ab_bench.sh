#!/bin/bash
# A/B of the C3 bench against a previous build kept in ab_old/ (a copy of the package, bench.py and
# oracle at that commit, library built there): new, old, new, old, each under its own time limit
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/abb_new_$i.log 2>&1 || exit $?
  timeout -k 10 300 python ab_old/bench.py --no-cpu-baseline > gpurun_out/abb_old_$i.log 2>&1 || exit $?
done
for f in gpurun_out/abb_*.log; do
  python - "$f" <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l)
print(sys.argv[1], d["ms_per_step"], d["ms_per_step_all_rows_last_layer"], d["ms_per_step_serialized"], d.get("kernel_ms"))
PY
done
