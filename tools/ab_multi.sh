# Interleaved A/B: the committed library (tools/variants/libllama3hip_r5.so) against the tree with
# the multi-step persistent launch off / on (L3_DECODE_PERSIST_MULTI), tools/bench_decode.py.
# (L3_DECODE_PERSIST_MULTI exists only in the research build: tools/research/decode_persist_multistep.hip
# in place of llama3.np_amd/csrc/decode_persist.hip; the product library ignores it)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for i in 1 2 3; do
  L3_LIB_PATH=tools/variants/libllama3hip_r5.so timeout -k 10 200 python tools/bench_decode.py > gpurun_out/abm_r5_$i.log 2>&1 || exit $?
  L3_DECODE_PERSIST_MULTI=0 timeout -k 10 200 python tools/bench_decode.py > gpurun_out/abm_m0_$i.log 2>&1 || exit $?
  L3_DECODE_PERSIST_MULTI=1 timeout -k 10 200 python tools/bench_decode.py > gpurun_out/abm_m1_$i.log 2>&1 || exit $?
done
for f in gpurun_out/abm_*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f | head -1) $(grep -o '"device_loop_ms_per_step": [0-9.]*' $f) $(grep -o '"device_loop_ids_exact": [a-z]*' $f)"; done
