set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for i in 1 2; do
 for v in "2 128" "6 128" "12 128" "2 256" "12 256"; do
  set -- $v
  L3_SKINNY_CH=$1 L3_SKINNY_TN2_MIN=$2 timeout -k 10 200 python tools/bench_decode.py > gpurun_out/skab_ch$1_tn$2_$i.log 2>&1 || exit $?
 done
done
for f in gpurun_out/skab_*.log; do echo "$f $(grep -o '"batched_device_loop": .*' $f)"; done
