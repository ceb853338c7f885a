# Interleaved A/B of environment settings on the decode bench (tools/bench_decode.py: batch 1
# and the batched device loops); each round runs every variant once.  A variant is a
# comma-separated list of VAR=value settings ("-": none), e.g.
#   bash tools/ab_env.sh "L3_DECODE_PERSIST_FOLD=0 L3_DECODE_PERSIST_FOLD=1,L3_DECODE_PERSIST_LM_DELAY=300" [rounds]
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
specs=$1; rounds=${2:-3}
for i in $(seq 1 "$rounds"); do
  k=0
  for sp in $specs; do
    k=$((k + 1))
    envs=""; [ "$sp" != "-" ] && envs=${sp//,/ }
    env $envs timeout -k 10 200 python tools/bench_decode.py > gpurun_out/abe_v${k}_$i.log 2>&1 || exit $?
  done
done
k=0
for sp in $specs; do
  k=$((k + 1))
  for f in gpurun_out/abe_v${k}_*.log; do
    echo "$sp $(basename $f) $(python3 -c 'import json,sys
j = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
b = j.get("batched_device_loop", {})
print("lazy", j["ms_per_step"], "loop", j["device_loop_ms_per_step"], j["device_loop_ids_exact"],
      " ".join("B%s %s" % (k, v["ms_per_step"]) for k, v in b.items()))' $f)"
  done
done
