# Batched decode: the persistent layers step (L3_DECODE_PBATCH=1, decode_batch.hip) against the
# per-kernel graph (0); interleaved bench_decode runs
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for i in 1 2 3; do
  for v in 1 0; do
    L3_DECODE_PBATCH=$v timeout -k 10 200 python tools/bench_decode.py > gpurun_out/pbab_${v}_$i.log 2>&1 || exit $?
  done
done
for f in gpurun_out/pbab_*.log; do echo "$f $(grep -o '"batched_device_loop": .*' $f | sed 's/"roofline": {[^}]*}//g')"; done
