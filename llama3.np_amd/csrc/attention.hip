// Fused causal attention dispatch (kernel template and design notes: attn_kernel.h).
#include "attn_kernel.h"

namespace l3 {

template <int HD, int QBW, bool VT = false>
static hipError_t launch_hd(const AttnArgs& a, hipStream_t s) {
    constexpr int QW = 64 * QBW;
    dim3 grid((a.L + QW - 1) / QW, a.H, a.B), block(256);
    hipLaunchKernelGGL((attn_fwd_kernel<HD, QBW, VT>), grid, block, 0, s, a);
    return hipGetLastError();
}

hipError_t launch_attention(const AttnArgs& a, hipStream_t s) {
    if (a.B <= 0 || a.L <= 0) return hipSuccess;
    if (a.H % a.KVH != 0) return hipErrorInvalidValue;
    // small L (decode, short prompts): one 16-query block per wave is enough
    const bool small = a.L <= 64;
    switch (a.HD) {
        case 16: return small ? launch_hd<16, 1>(a, s) : launch_hd<16, 4>(a, s);
        case 48: return small ? launch_hd<48, 1>(a, s) : launch_hd<48, 4>(a, s);
        case 64: return small ? launch_hd<64, 1>(a, s) : launch_hd<64, 2>(a, s);
        case 128: return small ? launch_hd<128, 1>(a, s) : launch_hd<128, 2>(a, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace l3
