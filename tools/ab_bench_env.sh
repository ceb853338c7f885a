#!/bin/bash
# Interleaved A/B of environment settings on the C3 bench (bench.py --no-cpu-baseline
# --no-kernel-breakdown): each round runs every variant once, each under its own time limit.
# A variant is a comma-separated list of VAR=value settings ("-": none), e.g.
#   bash tools/ab_bench_env.sh "L3_SPLIT_NOJOIN=0 L3_SPLIT_NOJOIN=1" [rounds]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
specs=$1; rounds=${2:-3}
for i in $(seq 1 "$rounds"); do
  k=0
  for sp in $specs; do
    k=$((k + 1))
    envs=""; [ "$sp" != "-" ] && envs=${sp//,/ }
    env $envs timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernel-breakdown > gpurun_out/abbe_v${k}_$i.log 2>&1 || exit $?
  done
done
k=0
for sp in $specs; do
  k=$((k + 1))
  for f in gpurun_out/abbe_v${k}_*.log; do
    echo "$sp $(basename $f) $(python3 -c 'import json,sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print("ms", d["ms_per_step"], "median", d["ms_per_step_median"], "host", d["ms_per_step_with_logits_d2h"], "all_rows", d["ms_per_step_all_rows_last_layer"], "x6", (d.get("gemm_x6") or {}).get("ms_per_step"))' $f)"
  done
done
