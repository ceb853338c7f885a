// fp32 GEMM from bf16 MFMAs ("x6"): C[M,N] = A[M,K] * W[N,K]^T to fp32 accuracy, opt-in
// (l3_set_gemm_x6 / L3_GEMM_X6=1; the default path is gemm_kernel.h's v_mfma_f32_16x16x4_f32).
//
// Each fp32 operand x is cut into three bf16 pieces by truncation, x = hi + mid + lo EXACTLY
// (hi = the top 8 significand bits, mid the next 8, lo the last 8: each piece fits a bf16 and the
// two subtractions that produce them are exact), and C is summed from the six products of weight
// at least 2^-16 of hi*hi:  hi*hi + hi*mid + mid*hi + hi*lo + lo*hi + mid*mid.  Every bf16 x bf16
// product is exact in the MFMA's fp32 accumulator; the dropped mid*lo, lo*mid and lo*lo are each
// below 2^-22 of |a w| (about 2^-24 typically), at the size of fp32's own rounding of one product.
// tools/gemm_tune x6acc measures both paths against an fp64 product.
// v_mfma_f32_16x16x32_bf16 does 16x the FLOP per clock of v_mfma_f32_16x16x4_f32
// (MI355X_MICROARCH.md, matrix cores), so the six cost 6/16 of the fp32 MFMA time.
//
// Layout: W is split once at l3_finalize into W3[n][piece][K] (bf16, after the RMSNorm fold);
// the activation tile is staged in fp32 by global_load_lds as in gemm_lds_kernel (the embedding
// gather of layer 0 included) and each wave splits its own fragments after the LDS read (a
// pre-split activation measured slower: its 1.5x image leaves one block per CU).  Fragment maps:
// v_mfma_f32_16x16x32_bf16 takes lane l's eight k values 8(l>>4) .. 8(l>>4)+7 of row l & 15 for
// both operands; W is the A operand and the activation B, so the accumulator map is
// gemm_lds_kernel's and its epilogues (RMSNorm row factor, RoPE / KV append, SwiGLU, residual)
// apply unchanged.  The row factor's sum of squares comes from the fp32 fragments.
#pragma once
#include "gemm_kernel.h"

namespace l3 {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma_bf16(u32x4 a, u32x4 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c,
                                                   0, 0, 0);
}

__host__ __device__ inline unsigned f2u(float x) {
    unsigned u;
    __builtin_memcpy(&u, &x, 4);
    return u;
}
__host__ __device__ inline float u2f(unsigned u) {
    float x;
    __builtin_memcpy(&x, &u, 4);
    return x;
}

// x = hi + mid + lo exactly; each piece's fp32 bits have a zero low half (a bf16 in the top half)
__host__ __device__ inline void split3_one(float x, unsigned& h, unsigned& m, unsigned& l) {
    h = f2u(x);
    const float r = x - u2f(h & 0xffff0000u);
    m = f2u(r);
    const float r2 = r - u2f(m & 0xffff0000u);
    l = f2u(r2);
}

// eight fp32 (k order) -> three planes of eight bf16 (packed pairs, element 2p in the low half)
__device__ __forceinline__ void split3(const f32x4& x0, const f32x4& x1, u32x4& h, u32x4& m, u32x4& l) {
    const float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
    unsigned hu[8], mu[8], lu[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) split3_one(v[e], hu[e], mu[e], lu[e]);
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        h[p] = __builtin_amdgcn_perm(hu[2 * p + 1], hu[2 * p], 0x07060302u);
        m[p] = __builtin_amdgcn_perm(mu[2 * p + 1], mu[2 * p], 0x07060302u);
        l[p] = __builtin_amdgcn_perm(lu[2 * p + 1], lu[2 * p], 0x07060302u);
    }
}

// src [rows][K] fp32 -> dst [rows][3][K] bf16 (one thread per element; gemm.hip launch_split_planes)
__global__ void split_planes_kernel(const float* src, unsigned short* dst, int64_t rows, int K) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (int64_t)rows * K) return;
    const int64_t r = i / K, k = i - r * K;
    unsigned h, m, l;
    split3_one(src[i], h, m, l);
    unsigned short* d = dst + r * 3 * K + k;
    d[0] = (unsigned short)(h >> 16);
    d[K] = (unsigned short)(m >> 16);
    d[2 * K] = (unsigned short)(l >> 16);
}

// bf16 plane image row: 32 bf16 = 4 quads of 16 B; quad q of row r at q ^ ((r >> 2) & 3): the 16
// lanes that read one quad index from 16 consecutive rows cover the 64 banks once
__device__ __forceinline__ int swz_p(int r) { return (r >> 2) & 3; }
// fp32 image row: 32 floats = 8 quads; quad q of row r at q ^ ((r >> 1) & 7)
__device__ __forceinline__ int swz_f(int r) { return (r >> 1) & 7; }

template <int WM, int WN, int TM, int TN, int EPI, int WPE = 2>
__global__ void __launch_bounds__(64 * WM * WN, WPE) gemm_x6_kernel(GemmArgs p) {
    constexpr int NW = WM * WN;
    constexpr int BM = WM * TM * 16, BN = WN * TN * 16, BK = 32;
    constexpr int A_BYTES = BM * 128;
    constexpr int W_BYTES = 3 * BN * 64;
    __shared__ __attribute__((aligned(16))) char smem[2 * (A_BYTES + W_BYTES)];
    auto a_img = [&](int buf) { return smem + buf * A_BYTES; };
    auto w_img = [&](int buf) { return smem + 2 * A_BYTES + buf * W_BYTES; };

#ifndef L3_X6_VGPR_FORM
    // an AGPR reference: hipcc then gives the MFMAs the AGPR form (accumulators in a[], D = C in
    // place) instead of VGPR chains renamed around the VALU work; tools/gemm_tune x6 at C3: QKV
    // 158.8 vs 153.5, O-proj 154.6 vs 148.7, down 185.2 vs 175.3 fp32-equivalent TF/s
    asm volatile("" ::: "a0");
#endif
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid / WN, wn = wid % WN;
    const int ntn = (p.N + BN - 1) / BN;
    const int t = xcd_remap(blockIdx.x, gridDim.x);
    int mt = t / ntn, nt = t - mt * ntn;
    if (p.group_m > 1) {
        const int ntm = (p.M + BM - 1) / BM;
        const int g = t / (p.group_m * ntn), first = g * p.group_m;
        const int gm = min(ntm - first, p.group_m), local = t - g * p.group_m * ntn;
        mt = first + local % gm;
        nt = local / gm;
    }
    const int m0 = mt * BM, n0 = nt * BN;
    const int nk = p.K / BK;

    // k-tile fill by global_load_lds: a 1 KB piece = 64 lanes x 16 B
    //   plane images: 16 rows of one plane (lane i: row i / 4, slot i % 4)
    //   fp32 image: 8 rows (lane i: row i / 8, slot i % 8)
    constexpr int WP = 3 * BN / 16;                    // weight pieces
    constexpr int AP = BM / 8;                         // activation pieces
    const unsigned short* W3 = p.W3;
    // A-row source addresses are fixed for the tile (an embedding row's index is read once)
    constexpr int A_PIECES = (AP + NW - 1) / NW;
    const float* a_src[A_PIECES];
#pragma unroll
    for (int it = 0; it < A_PIECES; ++it) {
        const int r = (wid + NW * it) * 8 + lane / 8;
        a_src[it] = a_row(p, min(m0 + r, p.M - 1)) + 4 * ((lane & 7) ^ swz_f(r));
    }
    auto fill = [&](int buf, int k0) {
        for (int piece = wid; piece < WP; piece += NW) {
            const int pl = piece / (BN / 16), r = (piece % (BN / 16)) * 16 + lane / 4;
            const int q = (lane & 3) ^ swz_p(r);
            const int gn = min(n0 + r, p.N - 1);
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void*)(W3 + ((int64_t)gn * 3 + pl) * p.K + k0 + 8 * q),
                (__attribute__((address_space(3))) void*)(w_img(buf) + piece * 1024), 16, 0, 0);
        }
#pragma unroll
        for (int it = 0; it < A_PIECES; ++it) {
            const int piece = wid + NW * it;
            if (AP % NW == 0 || piece < AP)
                __builtin_amdgcn_global_load_lds(
                    (const __attribute__((address_space(1))) void*)(a_src[it] + k0),
                    (__attribute__((address_space(3))) void*)(a_img(buf) + piece * 1024), 16, 0, 0);
        }
    };

    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    float ss[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) ss[i] = 0.f;

    const int frow = lane & 15, g = lane >> 4;
    const int arow0 = wm * TM * 16, brow0 = wn * TN * 16;

    auto compute = [&](int buf) {
        u32x4 ah[TM], am[TM], al[TM];
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const int r = arow0 + i * 16 + frow;
            const float* b = reinterpret_cast<const float*>(a_img(buf)) + r * 32;
            const f32x4 x0 = *reinterpret_cast<const f32x4*>(b + 4 * ((2 * g) ^ swz_f(r)));
            const f32x4 x1 = *reinterpret_cast<const f32x4*>(b + 4 * ((2 * g + 1) ^ swz_f(r)));
            ss[i] += x0.x * x0.x + x0.y * x0.y + x0.z * x0.z + x0.w * x0.w + x1.x * x1.x + x1.y * x1.y +
                     x1.z * x1.z + x1.w * x1.w;
            split3(x0, x1, ah[i], am[i], al[i]);
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int r = brow0 + j * 16 + frow;
            const char* b = w_img(buf);
            const int off = r * 64 + 16 * (g ^ swz_p(r));
            const u32x4 wh = *reinterpret_cast<const u32x4*>(b + off);
            const u32x4 wmd = *reinterpret_cast<const u32x4*>(b + BN * 64 + off);
            const u32x4 wl = *reinterpret_cast<const u32x4*>(b + 2 * BN * 64 + off);
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                // small terms first: they meet an accumulator not yet carrying this step's hi*hi
                acc[i][j] = mfma_bf16(wmd, am[i], acc[i][j]);
                acc[i][j] = mfma_bf16(wl, ah[i], acc[i][j]);
                acc[i][j] = mfma_bf16(wh, al[i], acc[i][j]);
                acc[i][j] = mfma_bf16(wmd, ah[i], acc[i][j]);
                acc[i][j] = mfma_bf16(wh, am[i], acc[i][j]);
                acc[i][j] = mfma_bf16(wh, ah[i], acc[i][j]);
            }
        }
    };

    fill(0, 0);
    __syncthreads();
    for (int kt = 0; kt < nk - 1; ++kt) {
        fill((kt + 1) & 1, (kt + 1) * BK);
        compute(kt & 1);
        __syncthreads();
    }
    compute((nk - 1) & 1);

    float rs[TM];
    const float inv_k = 1.0f / (float)p.K;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        const float v = sum_xor16_32(ss[i]);
        rs[i] = p.norm ? __builtin_amdgcn_rsqf(v * inv_k + p.eps) : 1.0f;
    }
    if constexpr (EPI == EPI_QKV) {
        if (p.qkv_fast && m0 + BM <= p.M && n0 + BN <= p.N)
            qkv_epilogue_full<TM, TN>(p, acc, rs, m0 + arow0, n0 + brow0, lane);
        else
            qkv_epilogue<TM, TN>(p, acc, rs, m0 + arow0, n0 + brow0, lane);
    } else {
        f32x4 res[1];
        direct_epilogue<TM, TN, EPI, false, 1>(p, acc, rs, res, m0 + arow0, n0 + brow0, lane);
    }
}

}  // namespace l3
