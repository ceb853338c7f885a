# Interleaved A/B of environment settings on the Llama-3-shape prefill (bench.py --workload c5,
# 32 layers, B=64 L=2048, one step after one warm-up); variants as in tools/ab_env.sh
#   bash tools/ab_c5.sh "L3_GEMM_GROUP_M=0 -" [rounds]
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
specs=$1; rounds=${2:-2}
for i in $(seq 1 "$rounds"); do
  k=0
  for sp in $specs; do
    k=$((k + 1))
    envs=""; [ "$sp" != "-" ] && envs=${sp//,/ }
    env $envs timeout -k 10 400 python bench.py --workload c5 --steps 1 --warmup 1 > gpurun_out/abc5p_v${k}_$i.log 2>&1 || exit $?
  done
done
k=0
for sp in $specs; do
  k=$((k + 1))
  for f in gpurun_out/abc5p_v${k}_*.log; do
    echo "$sp $(basename $f) $(python3 -c 'import json,sys
j = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
k = j["kernels"]
print("tokens/s", j["value"], "ms", j["ms_per_step"], "frac", j["whole_forward_frac"], "gateup", k["gateup"]["TFLOP/s"], "qkv", k["qkv"]["TFLOP/s"])' $f)"
  done
done
