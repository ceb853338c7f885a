#!/bin/bash
# C5 (Llama-3 shape) prefill with rocm-smi sampling of clocks / power / temperature every 2 s,
# to see whether the sustained 16 s forward is power- or thermal-limited.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
( for i in $(seq 1 150); do date +%T; rocm-smi --showpower --showclocks --showtemp 2>/dev/null | grep -E "^(GPU|0 |card)|Power|sclk|Temp|fclk|mclk" ; sleep 2; done ) > gpurun_out/smi.log 2>&1 &
SMI=$!
timeout -k 10 600 python bench.py --workload c5 --steps ${1:-1} --warmup 1 --layers ${2:-32} > gpurun_out/c5p.log 2>&1
rc=$?
kill $SMI 2>/dev/null
wait $SMI 2>/dev/null
cat gpurun_out/c5p.log | tail -2
exit $rc
