# Interleaved A/B of environment settings on the Llama-3-shape batch-1 decode (bench.py
# --workload c5decode); each round runs every variant once.  A variant is a comma-separated list
# of VAR=value settings ("-": none), e.g.
#   bash tools/ab_env_c5dec.sh "L3_DECODE_PF_MB=0 L3_DECODE_PF_MB=48" [rounds]
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
specs=$1; rounds=${2:-3}
for i in $(seq 1 "$rounds"); do
  k=0
  for sp in $specs; do
    k=$((k + 1))
    envs=""; [ "$sp" != "-" ] && envs=${sp//,/ }
    env $envs timeout -k 10 300 python bench.py --workload c5decode --steps 30 > gpurun_out/abc5_v${k}_$i.log 2>&1 || exit $?
  done
done
k=0
for sp in $specs; do
  k=$((k + 1))
  for f in gpurun_out/abc5_v${k}_*.log; do
    echo "$sp $(basename $f) $(python3 -c 'import json,sys
j = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print("loop", j["device_loop_ms_per_token"], "lazy", j["lazy_generate_ms_per_token"], "ids_equal", j["ids_equal_lazy_vs_device_loop"])' $f)"
  done
done
