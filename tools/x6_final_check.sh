set -u
mkdir -p gpurun_out
timeout -k 10 300 tools/gemm_tune_snop 1 1 x6detq 20 > gpurun_out/x6detq_final_snop.log 2>&1 || exit $?
timeout -k 10 300 tools/gemm_tune 1 1 x6det 100 > gpurun_out/x6det_final.log 2>&1 || exit $?
(timeout -k 10 200 python tools/x6_determinism.py && timeout -k 10 200 python tools/x6_determinism.py --dev) > gpurun_out/x6det_model_final.log 2>&1 || exit $?
timeout -k 10 300 tools/gemm_tune 5 10 x6 > gpurun_out/x6_final_speed.log 2>&1 || exit $?
