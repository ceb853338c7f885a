// fp32 MFMA GEMM dispatch (kernel templates and design notes: gemm_kernel.h).
// Only the (tile, epilogue) pairs used below are instantiated.
#include "gemm_kernel.h"

namespace l3 {

template <int EPI, int WM, int WN, int TM, int TN, int WPE, int BK = 32>
static hipError_t launch(const GemmArgs& a, hipStream_t s) {
    constexpr int BM = WM * TM * 16, BN = WN * TN * 16;
    const int64_t tiles = (int64_t)((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
    hipLaunchKernelGGL((gemm_lds_kernel<WM, WN, TM, TN, EPI, WPE, false, BK>), dim3((unsigned)tiles),
                       dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_gemm(int epi, const GemmArgs& a, hipStream_t s) {
    if (a.M <= 0 || a.N <= 0) return hipSuccess;
    if (a.K % 32 != 0 || a.K <= 0) return hipErrorInvalidValue;  // whole 32-deep k-tiles
    if (epi == EPI_SWIGLU && a.N % 32 != 0) return hipErrorInvalidValue;
    if (a.N % 4 != 0 || a.ldc % 4 != 0 || a.lda % 4 != 0) return hipErrorInvalidValue;  // 16-B rows
    // Configurations chosen with tools/gemm_tune (interleaved A/B on MI355X).
    const bool small_m = a.M <= 32;  // decode / tiny M: 16 x 128 tile
    switch (epi) {
        case EPI_SWIGLU:  // 128 x 128, BK 16: 142 VGPRs + 48 KB LDS -> 3 blocks per CU
            if (small_m) return launch<EPI_SWIGLU, 1, 4, 1, 2, 2>(a, s);
            return launch<EPI_SWIGLU, 2, 2, 4, 4, 2, 16>(a, s);
        case EPI_QKV:     // N = 864 (stories15M) / 6144 (Llama-3 shape) are multiples of 96
            if (small_m) return launch<EPI_QKV, 1, 4, 1, 2, 2>(a, s);
            if (a.N % 96 == 0)
                return a.K <= 1024 ? launch<EPI_QKV, 2, 2, 2, 3, 3, 16>(a, s)   // 64 x 96
                                   : launch<EPI_QKV, 2, 2, 4, 3, 3, 16>(a, s);  // 128 x 96
            return launch<EPI_QKV, 2, 2, 2, 4, 3, 16>(a, s);                    // 64 x 128
        case EPI_RESID:   // O-proj / down
            if (small_m) return launch<EPI_RESID, 1, 4, 1, 2, 2>(a, s);
            if (a.N % 96 == 0)
                return a.K <= 512 ? launch<EPI_RESID, 2, 2, 2, 3, 2>(a, s)   // 64 x 96
                                  : launch<EPI_RESID, 2, 2, 4, 3, 2>(a, s);  // 128 x 96
            return launch<EPI_RESID, 2, 2, 4, 4, 2, 16>(a, s);               // 128 x 128
        case EPI_STORE:   // lm_head, op-level linear
            if (small_m) return launch<EPI_STORE, 1, 4, 1, 2, 2>(a, s);
            return launch<EPI_STORE, 2, 2, 4, 4, 2>(a, s);
        default:
            return hipErrorInvalidValue;
    }
}

}  // namespace l3
