# Persistent batch-1 decode step (L3_DECODE_PERSIST=1) against the graph-launched step:
# decode parity tests with it on, then interleaved bench_decode pairs (stops at the first
# fault / timeout: exit codes other than 0 / 1 end the script).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
L3_DECODE_PERSIST=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -rf \
  -k "persistent or greedy or generate or speculative or run_ahead or tiny or cli or argmax_ties or cache_edges or ragged or last_layer" \
  --timeout 300 --timeout-method thread > gpurun_out/persist_tests.log 2>&1
rc=$?; echo "persist tests rc=$rc"; tail -5 gpurun_out/persist_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for i in 1 2 3; do
  L3_DECODE_PERSIST=1 timeout -k 10 200 python tools/bench_decode.py > gpurun_out/pab_on_$i.log 2>&1 || exit $?
  L3_DECODE_PERSIST=0 timeout -k 10 200 python tools/bench_decode.py > gpurun_out/pab_off_$i.log 2>&1 || exit $?
done
for f in gpurun_out/pab_*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f | head -1) $(grep -o '"device_loop_ms_per_step": [0-9.]*' $f) $(grep -o '"[a-z_]*ids_exact[a-z_]*": [a-z]*' $f | tr '\n' ' ')"; done
