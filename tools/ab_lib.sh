# Interleaved A/B of library builds and decode modes on the batch-1 decode bench: each round runs
# every variant once.  A variant is <lib>:<L3_DECODE_PERSIST>[:<L3_DECODE_PERSIST_FOLD>], <lib> =
# "tree" (the in-tree build) or a name under tools/variants/libllama3hip_<name>.so (built from
# variant sources outside the tree).
#   bash tools/ab_lib.sh "r4:1 tree:1 tree:1:1 tree:0" [rounds]
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
specs=$1; rounds=${2:-3}
for i in $(seq 1 "$rounds"); do
  for sp in $specs; do
    v=${sp%%:*}; r=${sp#*:}; m=${r%%:*}; f=0; [ "$r" != "$m" ] && f=${r#*:}
    lib=""; [ "$v" != tree ] && lib=tools/variants/libllama3hip_$v.so
    L3_LIB_PATH=$lib L3_DECODE_PERSIST=$m L3_DECODE_PERSIST_FOLD=$f timeout -k 10 200 python tools/bench_decode.py > gpurun_out/abl_${v}_m${m}f${f}_$i.log 2>&1 || exit $?
  done
done
for f in gpurun_out/abl_*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f | head -1) $(grep -o '"device_loop_ms_per_step": [0-9.]*' $f) $(grep -o '"device_loop_ids_exact": [a-z]*' $f)"; done
