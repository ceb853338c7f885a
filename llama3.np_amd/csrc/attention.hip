// Fused causal attention dispatch (kernel template and design notes: attn_kernel.h).  Every
// launch takes the PK body (round 6: interleaved score chains, packed softmax pass; C3
// 117.9-119.4 -> 116.3-116.7 us, the Llama-3 shape 829 -> 800 us, profiles/r06_attn_pk.txt)
#include "attn_kernel.h"

namespace l3 {

template <int HD, int QBW, int G, int KT>
static hipError_t launch(const AttnArgs& a, hipStream_t s) {
    constexpr int QW = 16 * QBW * (4 / G);
    dim3 grid((a.L + QW - 1) / QW, a.H / G, a.B), block(256);
    hipLaunchKernelGGL((attn_fwd_kernel<HD, QBW, G, KT, true>), grid, block, 0, s, a);
    return hipGetLastError();
}

// G = heads per workgroup sharing one KV head; QBW = 16-query blocks per wave (chosen so a
// workgroup's query range does not far exceed L; QBIG for long prompts, tools/attn_tune).
template <int HD, int KT, int QBIG, int G>
static hipError_t launch_g(const AttnArgs& a, hipStream_t s) {
    constexpr int WPH = 4 / G;
    if (a.L <= 16 * WPH) return launch<HD, 1, G, KT>(a, s);
    if (QBIG > 2 && a.L <= 32 * WPH) return launch<HD, 2, G, KT>(a, s);
    return launch<HD, QBIG, G, KT>(a, s);
}

template <int HD, int KT, int QBIG>
static hipError_t launch_hd(const AttnArgs& a, hipStream_t s) {
    const int n_rep = a.H / a.KVH;
    if (n_rep % 4 == 0) return launch_g<HD, KT, QBIG, 4>(a, s);
    if (n_rep % 2 == 0) return launch_g<HD, KT, QBIG, 2>(a, s);
    return launch_g<HD, KT, QBIG, 1>(a, s);
}

template <int HD>
static hipError_t launch_decode(const AttnArgs& a, hipStream_t s) {
    constexpr int R = 256 / (HD / 4);
    const size_t lds = ((size_t)R * HD + a.Smax) * 4;
    if (a.wo) {  // O-proj fused: 64 output rows per block along z
        if (!a.parts || a.D <= 0 || a.D % 4) return hipErrorInvalidValue;
        hipLaunchKernelGGL((attn_decode_kernel<HD, true>), dim3(a.H, a.B, (a.D + 63) / 64), dim3(256), lds, s, a);
    } else {
        hipLaunchKernelGGL((attn_decode_kernel<HD, false>), dim3(a.H, a.B), dim3(256), lds, s, a);
    }
    return hipGetLastError();
}

// The last query rows of each sequence only (a pruned last block, runtime.hip run_layer): one
// workgroup per (batch, head group) with one q-block per wave over rows [L - QW, L) — the
// same kernel and per-query arithmetic as the full launch, so those rows are bit-identical
template <int HD, int KT>
static hipError_t launch_last_hd(AttnArgs a, hipStream_t s) {
    const int n_rep = a.H / a.KVH;
    const int G = n_rep % 4 == 0 ? 4 : n_rep % 2 == 0 ? 2 : 1;
    const int QW = 16 * (4 / G);
    a.q_first = a.L > QW ? a.L - QW : 0;
    dim3 grid(1, a.H / G, a.B), block(256);
    if (G == 4) hipLaunchKernelGGL((attn_fwd_kernel<HD, 1, 4, KT, true>), grid, block, 0, s, a);
    else if (G == 2) hipLaunchKernelGGL((attn_fwd_kernel<HD, 1, 2, KT, true>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((attn_fwd_kernel<HD, 1, 1, KT, true>), grid, block, 0, s, a);
    return hipGetLastError();
}

hipError_t launch_attention_last(const AttnArgs& a, hipStream_t s) {
    if (a.B <= 0 || a.L <= 0) return hipSuccess;
    if (a.KVH <= 0 || a.H % a.KVH != 0 || a.wo || a.pos_dev) return hipErrorInvalidValue;
    switch (a.HD) {
        case 16: return launch_last_hd<16, 64>(a, s);
        case 32: return launch_last_hd<32, 64>(a, s);
        case 48: return launch_last_hd<48, 64>(a, s);
        case 64: return launch_last_hd<64, 64>(a, s);
        case 96: return launch_last_hd<96, 32>(a, s);
        case 128: return launch_last_hd<128, 32>(a, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_attention(const AttnArgs& a, hipStream_t s) {
    if (a.B <= 0 || a.L <= 0) return hipSuccess;
    if (a.KVH <= 0 || a.H % a.KVH != 0) return hipErrorInvalidValue;
    if (a.wo && (a.L != 1 || a.Smax > 8192)) return hipErrorInvalidValue;  // fused O-proj: decode only
    if (a.L == 1 && a.Smax <= 8192) {  // decode: one query per (b, h)
        switch (a.HD) {
            case 16: return launch_decode<16>(a, s);
            case 32: return launch_decode<32>(a, s);
            case 48: return launch_decode<48>(a, s);
            case 64: return launch_decode<64>(a, s);
            case 96: return launch_decode<96>(a, s);
            case 128: return launch_decode<128>(a, s);
            default: return hipErrorInvalidValue;
        }
    }
    switch (a.HD) {
        case 16: return launch_hd<16, 64, 4>(a, s);
        case 32: return launch_hd<32, 64, 4>(a, s);
        case 48: return launch_hd<48, 64, 4>(a, s);
        case 64: return launch_hd<64, 64, 4>(a, s);
        case 96: return launch_hd<96, 32, 1>(a, s);   // KT 32: 52 KB LDS -> 2 workgroups per CU
        case 128: return launch_hd<128, 32, 1>(a, s);  // KT 32: 72 KB LDS -> 2 workgroups per CU
        default: return hipErrorInvalidValue;
    }
}

hipError_t dcheck_collect_attention(unsigned* out) { return dcheck_collect(out); }

}  // namespace l3
