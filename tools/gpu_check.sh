#!/bin/bash
# Run GPU steps in order; each under its own time limit.  Exit status 0 (pass) or 1
# (assertion / test failures) lets the next step run; anything else (fault, abort,
# segfault, timeout) ends the call so nothing more touches the GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {
  local name=$1 limit=$2; shift 2
  echo "=== [$name] $(date +%T) limit ${limit}s: $*"
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== [$name] rc=$rc"
  tail -n 40 "gpurun_out/$name.log"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "fatal rc=$rc: stopping"; exit "$rc"; fi
}
for s in "$@"; do
  case "$s" in
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) step tests 1200 python -m pytest tests -m gpu -q -rf --timeout 600 ;;
    c5slice) step c5slice 900 python -u -m pytest tests/test_gpu_parity.py -k c5_ -x -v --timeout 900 --timeout-method thread ;;
    testsx) step tests 1200 python -m pytest tests -m gpu -q -x -rf --timeout 600 ;;
    bench) step bench 600 python bench.py ;;
    benchq) step benchq 300 python bench.py --no-cpu-baseline ;;
    split[1-4]) L3_BATCH_SPLIT=${s#split} step $s 300 python bench.py --no-cpu-baseline ;;
    prof) step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-kernel-breakdown --no-x6 ;;
    profx6) L3_GEMM_X6=1 step profx6 600 rocprofv3 --kernel-trace --stats -d gpurun_out/profx6 -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-kernel-breakdown --no-x6 ;;
    x6tune) step x6tune 600 tools/gemm_tune 5 10 x6 ;;
    x6acc) step x6acc 300 tools/gemm_tune 1 1 x6acc ;;
    pmc) step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-breakdown --split 1 --no-x6
         step pmc_write 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-breakdown --split 1 --no-x6 ;;
    pmcx6) L3_GEMM_X6=1 step pmc_x6_fetch 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_x6_fetch -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-breakdown --split 1 --no-x6
         L3_GEMM_X6=1 step pmc_x6_write 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_x6_write -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-breakdown --split 1 --no-x6 ;;
    pmcc5) step pmc_c5_fetch 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_c5_fetch -o run --output-format csv -- python bench.py --workload c5 --layers 2 --steps 1 --warmup 1 --no-x6
         step pmc_c5_write 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_c5_write -o run --output-format csv -- python bench.py --workload c5 --layers 2 --steps 1 --warmup 1 --no-x6 ;;
    tune) step tune 600 tools/gemm_tune 5 10 ;;
    tunerows) step tunerows 600 tools/gemm_tune 5 10 rows ;;
    tunering) step tunering 600 tools/gemm_tune 5 10 ring ;;
    tunelm) step tunelm 300 tools/gemm_tune 5 20 lmhead ;;
    tunesk) step tunesk 300 tools/gemm_tune 5 50 skinny ;;
    tuneqkv18) step tuneqkv18 300 tools/gemm_tune 5 10 qkv18 ;;
    tunec5) step tunec5 900 tools/gemm_tune 3 3 c5 ;;
    pmcsq) step pmcA 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d gpurun_out/pmcA -o run --output-format csv -- tools/attn_tune 1 2
           step pmcB 600 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE -d gpurun_out/pmcB -o run --output-format csv -- tools/attn_tune 1 2
           step pmcC 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d gpurun_out/pmcC -o run --output-format csv -- tools/gemm_tune 1 2
           step pmcD 600 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE -d gpurun_out/pmcD -o run --output-format csv -- tools/gemm_tune 1 2 ;;
    stamps) step stamps 300 tools/gemm_tune 1 1 stamps ;;
    attntune) step attntune 600 tools/attn_tune ;;
    attnabl) step attnabl 300 tools/attn_tune 5 10 abl ;;
    attnpf2) step attnpf2 300 tools/attn_tune 5 10 pf2 ;;
    attnprio) step attnprio 300 tools/attn_tune 5 10 prio ;;
    attndefer) step attndefer 300 tools/attn_tune 5 10 defer ;;
    attnstamps) step attnstamps 120 tools/attn_tune 3 1 stamps gpurun_out/attn_stamps.bin ;;
    attnearly) step attnearly 300 tools/attn_tune 5 10 early ;;
    profr) step profr 600 rocprofv3 --kernel-trace --stats -d gpurun_out/profr -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-kernel-breakdown --rccl ;;
    floor) step floor 120 tools/launch_floor ;;
    handoff) step handoff 180 tools/handoff_chain ;;
    hostprobe) step hostprobe 300 python tools/host_path_probe.py ;;
    decode) step decode 300 python tools/bench_decode.py ;;
    decode32) L3_GEMV_LPU=32 step decode32 300 python tools/bench_decode.py ;;
    decode64) L3_GEMV_LPU=64 step decode64 300 python tools/bench_decode.py ;;
    decgs1) L3_DECODE_GRAPH_STEPS=1 step decgs1 300 python tools/bench_decode.py ;;
    decgs4) L3_DECODE_GRAPH_STEPS=4 step decgs4 300 python tools/bench_decode.py ;;
    decgs16) L3_DECODE_GRAPH_STEPS=16 step decgs16 300 python tools/bench_decode.py ;;
    decgs32) L3_DECODE_GRAPH_STEPS=32 step decgs32 300 python tools/bench_decode.py ;;
    decspec0) L3_DECODE_SPECULATE=0 step decspec0 300 python tools/bench_decode.py ;;
    decamax0) L3_LM_AMAX=0 step decamax0 300 python tools/bench_decode.py ;;
    decfold0) L3_DECODE_FOLD_ARGMAX=0 step decfold0 300 python tools/bench_decode.py ;;
    declayer0) L3_DECODE_LAYER=0 step declayer0 300 python tools/bench_decode.py ;;
    decnofuse) L3_DECODE_FUSE_O=0 step decnofuse 300 python tools/bench_decode.py ;;
    testsdec) step testsdec 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "greedy or generate or decode or head_dims or cli or cache_edges or tiny or golden or speculative or run_ahead" --timeout 300 --timeout-method thread ;;
    decsk0) L3_SKINNY=0 step decsk0 300 python tools/bench_decode.py ;;
    decskmin2) L3_SKINNY_MIN=2 step decskmin2 300 python tools/bench_decode.py ;;
    decmr2) L3_GEMV_MR=2 step decmr2 300 python tools/bench_decode.py ;;
    decmr4) L3_GEMV_MR=4 step decmr4 300 python tools/bench_decode.py ;;
    decode16) L3_GEMV_LPU=16 step decode16 300 python tools/bench_decode.py ;;
    decprofb*) step $s 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$s -o run --output-format csv -- python tools/bench_decode.py --eager-batch ${s#decprofb} ;;
    decprofp) step decprofp 300 rocprofv3 --kernel-trace --stats -d gpurun_out/decprofp -o run --output-format csv -- python tools/bench_decode.py ;;
    persistab) step persistab 600 bash tools/ab_lib.sh "tree:1 tree:0" 3 ;;
    decprof) step decprof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/decprof -o run --output-format csv -- python tools/bench_decode.py --eager ;;
    c5) step c5 900 python bench.py --workload c5 --steps 1 --warmup 1 ;;
    c4) step c4 300 python bench.py --global-batch 2048 --steps 5 --warmup 1 --no-cpu-baseline --no-kernel-breakdown ;;
    c5dec) step c5dec 600 python bench.py --workload c5decode --steps 30 ;;
    c5decnt0) L3_GEMV_NT=0 step c5decnt0 600 python bench.py --workload c5decode --steps 30 ;;
    c5declpu*) L3_GEMV_LPU=${s#c5declpu} step $s 600 python bench.py --workload c5decode --steps 30 ;;
    c5decsk0) L3_SPLITK=0 step c5decsk0 600 python bench.py --workload c5decode --steps 30 ;;
    c5decb*) L3_SPLITK_BLOCKS=${s#c5decb} step $s 600 python bench.py --workload c5decode --steps 30 ;;
    c5deckt*) L3_SPLITK_MINKT=${s#c5deckt} step $s 600 python bench.py --workload c5decode --steps 30 ;;
    c5deccfg[1-4]) L3_SPLITK_CFG=${s#c5deccfg} step $s 600 python bench.py --workload c5decode --steps 30 ;;
    splitk) step splitk 900 python -u -m pytest tests/test_gpu_parity.py -k "c5_short or c5_slice_llama3" -x -v --timeout 900 --timeout-method thread ;;
    c5decprof) L3_DECODE_GRAPH=0 step c5decprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/c5decprof -o run --output-format csv -- python bench.py --workload c5decode --steps 6 ;;
    c5small) step c5small 600 python bench.py --workload c5 --layers 2 --steps 2 --warmup 1 ;;
    c5small1) L3_BATCH_SPLIT=1 step c5small1 600 python bench.py --workload c5 --layers 2 --steps 2 --warmup 1 ;;
    rccl) step rccl 180 python tools/rccl_selftest.py --world 2 --same-device ;;
    rccl1) step rccl1 180 python tools/rccl_selftest.py --world 1 ;;
    torchrun1) step torchrun1 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 5 --warmup 2 --no-cpu-baseline --rccl ;;
    torchrun1p0) L3_COMM_PRIORITY=0 step torchrun1p0 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 1 --steps 20 --warmup 3 --no-cpu-baseline --rccl ;;
    torchrun1n) step torchrun1n 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 1 --steps 20 --warmup 3 --no-cpu-baseline ;;
    torchrun1r) step torchrun1r 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29520 bench.py --gpus 1 --steps 20 --warmup 3 --no-cpu-baseline --rccl ;;
    spawn1) step spawn1 300 python bench.py --spawn --rccl --steps 20 --warmup 3 --no-cpu-baseline ;;
    c5deep) step c5deep 900 python -u -m pytest tests/test_gpu_parity.py -k c5_full_depth -x -v -s --timeout 900 --timeout-method thread ;;
    testsv) step tests 1200 python -u -m pytest tests -m gpu -v -rfP --timeout 900 --timeout-method thread ;;
    ragged) step ragged 300 python -u -m pytest tests/test_gpu_parity.py -k "ragged or cache_edges or head_dims or chunk" -x -q --timeout 300 --timeout-method thread ;;
    benchr) step benchr 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --rccl ;;
    benchrp0) L3_COMM_PRIORITY=0 step benchrp0 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --rccl ;;
    benchrng) step benchrng 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --rccl --no-step-gather ;;
    benchrq8) GPU_MAX_HW_QUEUES=8 step benchrq8 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --rccl ;;
    benchrm1) L3_COMM_MODE=1 step benchrm1 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --rccl ;;
    benchrm2) L3_COMM_MODE=2 step benchrm2 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --rccl ;;
    benchq8) GPU_MAX_HW_QUEUES=8 step benchq8 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline ;;
    pmcattn) step pmcattnA 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d gpurun_out/pmcattnA -o run --output-format csv -- tools/attn_tune 1 2 c3
           step pmcattnB 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE -d gpurun_out/pmcattnB -o run --output-format csv -- tools/attn_tune 1 2 c3 ;;
    pmcgemm) step pmcgemmA 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d gpurun_out/pmcgemmA -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-breakdown --split 1 --no-x6
             step pmcgemmB 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE -d gpurun_out/pmcgemmB -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-breakdown --split 1 --no-x6 ;;
    attnprof) step attnprof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/attnprof -o run --output-format csv -- tools/attn_tune 3 10 ;;
    loadprobe) step loadprobe 600 python tools/load_probe.py ;;
    new4) step new4 1100 python -u -m pytest tests/test_gpu_parity.py -x -v -rfP -k "group or comm_info or gather or c4_full or c5_full_depth_full_size" --timeout 900 --timeout-method thread ;;
    single1) step single1 300 python bench.py --single-process --gpus 1 --steps 20 --warmup 3 --no-cpu-baseline ;;
    single1m) L3_GROUP_MULTI_PATH=1 step single1m 300 python bench.py --single-process --gpus 1 --steps 20 --warmup 3 --no-cpu-baseline ;;
    spawn1o) step spawn1o 300 python bench.py --spawn --rccl --comm-overlap --steps 20 --warmup 3 --no-cpu-baseline ;;
    gathov) step gathov 300 python tools/gather_race_check.py 10 ;;
    cabi) step cabi 300 python -u -m pytest tests/test_c_abi_gpu.py -x -v --timeout 120 --timeout-method thread ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
