// fp32 MFMA GEMM dispatch (kernel templates and design notes: gemm_kernel.h).
#include "gemm_kernel.h"

namespace l3 {

#define L3_GEMM_LAUNCH(KERNEL)                                                                   \
    template <int WM, int WN, int TM, int TN, int WPE>                                           \
    static hipError_t launch_##KERNEL(int epi, const GemmArgs& a, hipStream_t s) {               \
        constexpr int BM = WM * TM * 16, BN = WN * TN * 16;                                      \
        const int64_t tiles = (int64_t)((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);            \
        dim3 grid((unsigned)tiles), block(256);                                                  \
        switch (epi) {                                                                           \
            case EPI_STORE: hipLaunchKernelGGL((KERNEL<WM, WN, TM, TN, EPI_STORE, WPE, false>), grid, block, 0, s, a); break;   \
            case EPI_RESID: hipLaunchKernelGGL((KERNEL<WM, WN, TM, TN, EPI_RESID, WPE, false>), grid, block, 0, s, a); break;   \
            case EPI_SWIGLU: hipLaunchKernelGGL((KERNEL<WM, WN, TM, TN, EPI_SWIGLU, WPE, false>), grid, block, 0, s, a); break; \
            case EPI_QKV: hipLaunchKernelGGL((KERNEL<WM, WN, TM, TN, EPI_QKV, WPE, false>), grid, block, 0, s, a); break;       \
            default: return hipErrorInvalidValue;                                                \
        }                                                                                        \
        return hipGetLastError();                                                                \
    }

L3_GEMM_LAUNCH(gemm_lds_kernel)

hipError_t launch_gemm(int epi, const GemmArgs& a, hipStream_t s) {
    if (a.M <= 0 || a.N <= 0) return hipSuccess;
    if (a.K % 32 != 0 || a.K <= 0) return hipErrorInvalidValue;
    if (epi == EPI_SWIGLU && a.N % 32 != 0) return hipErrorInvalidValue;
    if (a.N % 4 != 0 || a.ldc % 4 != 0 || a.lda % 4 != 0) return hipErrorInvalidValue;  // 16-B rows
    if (a.M <= 32) return launch_gemm_lds_kernel<1, 4, 1, 2, 2>(epi, a, s);  // 16 x 128: decode / tiny M
    // SwiGLU needs an even TN (gate/up 16-row groups pair up inside one wave).
    if (epi == EPI_SWIGLU || a.N % 96 != 0) return launch_gemm_lds_kernel<2, 2, 4, 4, 2>(epi, a, s);  // 128 x 128
    return launch_gemm_lds_kernel<2, 2, 4, 3, 2>(epi, a, s);  // 128 x 96: N = 288 (O, down), 864 (QKV)
}

}  // namespace l3
