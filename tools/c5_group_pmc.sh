# Round 6 (verdict r05 item 6): the Llama-3-shape gate|up's L2-miss traffic (PMC FETCH_SIZE, one
# pass per setting) against the grouped tile order's group size (L3_GEMM_GROUP_M: row tiles per
# group, walked column by column; 8 is the product's), plus one WRITE pass; each step under its
# own limit, stopping at the first fault / timeout.  Summary: tools/pmc_traffic.py per directory.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for g in ${GROUPS_TO_TRY:-4 8 16 32}; do
  L3_GEMM_GROUP_M=$g timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/c5g_fetch_$g -o run --output-format csv -- \
    python bench.py --workload c5 --layers 2 --steps 1 --warmup 1 > gpurun_out/c5g_fetch_$g.log 2>&1 || exit $?
done
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/c5g_write -o run --output-format csv -- \
  python bench.py --workload c5 --layers 2 --steps 1 --warmup 1 > gpurun_out/c5g_write.log 2>&1 || exit $?
for g in ${GROUPS_TO_TRY:-4 8 16 32}; do
  L3_GEMM_GROUP_M=$g timeout -k 10 300 python bench.py --workload c5 --layers 2 --steps 2 --warmup 1 > gpurun_out/c5g_bench_$g.log 2>&1 || exit $?
done
