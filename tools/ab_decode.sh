set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 200 python tools/bench_decode.py > gpurun_out/ab_new_$i.log 2>&1 || exit $?
  timeout -k 10 200 python ab_old/tools/bench_decode.py > gpurun_out/ab_old_$i.log 2>&1 || exit $?
done
for f in gpurun_out/ab_*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f | head -1) $(grep -o '"device_loop_ms_per_step": [0-9.]*' $f)"; done
