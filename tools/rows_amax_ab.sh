# Batched decode: the lm_head's per-row argmax partials (L3_DECODE_ROWS_AMAX=1, default) against
# logits + the full-row argmax (0); interleaved bench_decode runs
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for i in 1 2 3; do
  for v in 1 0; do
    L3_DECODE_ROWS_AMAX=$v timeout -k 10 200 python tools/bench_decode.py > gpurun_out/ramax_${v}_$i.log 2>&1 || exit $?
  done
done
for f in gpurun_out/ramax_*.log; do echo "$f $(grep -o '"batched_device_loop": .*' $f)"; done
