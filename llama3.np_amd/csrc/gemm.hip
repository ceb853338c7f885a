// fp32 MFMA GEMM for gfx950:  C[M,N] = A[M,K] * W[N,K]^T  with fused epilogues.
//
// Replaces every dense contraction of the reference forward:
//   QKV projections      llama3.py:166-168  (+ RMSNorm :248/:111-114 fused, + RoPE :181,
//                                            + KV-cache append :184-185)  -> EPI_QKV
//   O projection         llama3.py:211      (+ residual :253)             -> EPI_RESID
//   gate/up projections  llama3.py:99-101   (+ RMSNorm :256, SwiGLU)      -> EPI_SWIGLU
//   down projection      llama3.py:102      (+ residual :259)             -> EPI_RESID
//   lm_head              llama3.py:304-307  (+ final RMSNorm, last row)   -> EPI_STORE
//
// Matrix core: v_mfma_f32_16x16x4_f32 (exact fp32 in / fp32 accumulate, 64 FLOP/clk/SIMD,
// 157.3 TF/s chip peak).  Fragment maps (cdna_hip_programming.md section 3):
//   A: lane l supplies A[i = l&15][k = l>>4];  B: lane l supplies B[k = l>>4][j = l&15];
//   C/D: lane l holds C[row = 4*(l>>4) + r][col = l&15], r = 0..3.
// K-permutation trick: a sum over k may visit k in any order as long as A and B agree, so
// at sub-step s lane l feeds k = 4*(l>>4) + s.  One ds_read_b128 of a [row][k] LDS image then
// yields the operands of four consecutive MFMAs, for A and for W alike (both K-contiguous).
//
// Block: 256 threads = 4 waves arranged WM x WN, each wave a TM x TN grid of 16x16 tiles.
// K is staged 32 deep, register-prefetched one tile ahead into a double-buffered LDS image
// with row stride 40 floats (== 8 mod 16: conflict-free for the b128 fragment reads).
//
// RMSNorm fusion: rmsnorm(x) @ W^T = diag(1/rms(x)) * (x * w_norm) @ W^T.  The norm weight
// multiplies the A values as they are staged (one extra f32x4 load per k-tile per thread), the
// per-row sum of squares is accumulated from the same registers, and 1/rms scales the rows in
// the epilogue — the normalised activations are never written to HBM and W stays as stored.
#include "kernels.h"

namespace l3 {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int BK = 32;
constexpr int LDS_STRIDE = BK + 8;

__device__ __forceinline__ float silu_f(float x) { return x * (1.0f / (1.0f + __expf(-x))); }

template <int WM, int WN, int TM, int TN, int EPI>
__global__ void __launch_bounds__(256, 2) gemm_nt_kernel(GemmArgs p) {
    constexpr int BM = WM * TM * 16;
    constexpr int BN = WN * TN * 16;
    constexpr int A_F4 = BM * BK / 4;
    constexpr int B_F4 = BN * BK / 4;
    constexpr int A_IT = (A_F4 + 255) / 256;
    constexpr int B_IT = (B_F4 + 255) / 256;

    __shared__ __attribute__((aligned(16))) float As[2][BM][LDS_STRIDE];
    __shared__ __attribute__((aligned(16))) float Bs[2][BN][LDS_STRIDE];
    __shared__ float row_scale[BM];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = tid >> 6;
    const int wm = wid / WN;
    const int wn = wid % WN;

    // XCD-aware bijective remap: blocks b and b+8 share an XCD (L2); give each XCD a
    // contiguous run of tiles so the tiles that re-read one A row panel share its L2.
    const int ntn = (p.N + BN - 1) / BN;
    const int nwg = gridDim.x;
    const int b = blockIdx.x;
    const int xcd = b & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
    const int tm = t / ntn, tn = t % ntn;
    const int m0 = tm * BM, n0 = tn * BN;

    f32x4 ra[A_IT], rb[B_IT];
    float ss[A_IT];
#pragma unroll
    for (int i = 0; i < A_IT; ++i) ss[i] = 0.f;

    auto gload = [&](int k0) {
#pragma unroll
        for (int i = 0; i < A_IT; ++i) {
            const int f = tid + 256 * i;
            const int row = f >> 3, c = (f & 7) * 4;
            const int gm = m0 + row;
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            if ((A_F4 % 256 == 0 || f < A_F4) && gm < p.M)
                v = *reinterpret_cast<const f32x4*>(p.A + (int64_t)gm * p.lda + k0 + c);
            ra[i] = v;
        }
#pragma unroll
        for (int i = 0; i < B_IT; ++i) {
            const int f = tid + 256 * i;
            const int row = f >> 3, c = (f & 7) * 4;
            const int gn = n0 + row;
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            if ((B_F4 % 256 == 0 || f < B_F4) && gn < p.N)
                v = *reinterpret_cast<const f32x4*>(p.W + (int64_t)gn * p.K + k0 + c);
            rb[i] = v;
        }
    };
    auto sstore = [&](int buf, int k0) {
        f32x4 wv = {1.f, 1.f, 1.f, 1.f};
        if (p.norm) wv = *reinterpret_cast<const f32x4*>(p.norm_w + k0 + (tid & 7) * 4);
#pragma unroll
        for (int i = 0; i < A_IT; ++i) {
            const int f = tid + 256 * i;  // (f & 7) == (tid & 7): one norm-weight quad per thread
            if (A_F4 % 256 == 0 || f < A_F4) {
                f32x4 v = ra[i];
                if (p.norm) {
                    ss[i] += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
                    v *= wv;
                }
                *reinterpret_cast<f32x4*>(&As[buf][f >> 3][(f & 7) * 4]) = v;
            }
        }
#pragma unroll
        for (int i = 0; i < B_IT; ++i) {
            const int f = tid + 256 * i;
            if (B_F4 % 256 == 0 || f < B_F4)
                *reinterpret_cast<f32x4*>(&Bs[buf][f >> 3][(f & 7) * 4]) = rb[i];
        }
    };

    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int frow = lane & 15;
    const int fk = 4 * (lane >> 4);
    const int arow0 = wm * TM * 16;
    const int brow0 = wn * TN * 16;

    auto compute = [&](int buf) {
#pragma unroll
        for (int kg = 0; kg < BK / 16; ++kg) {
            f32x4 a[TM], bw[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i)
                a[i] = *reinterpret_cast<const f32x4*>(&As[buf][arow0 + i * 16 + frow][kg * 16 + fk]);
#pragma unroll
            for (int j = 0; j < TN; ++j)
                bw[j] = *reinterpret_cast<const f32x4*>(&Bs[buf][brow0 + j * 16 + frow][kg * 16 + fk]);
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][s], bw[j][s], acc[i][j],
                                                                         0, 0, 0);
        }
    };

    const int nk = p.K / BK;
    gload(0);
    sstore(0, 0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
        const int cur = kt & 1;
        if (kt + 1 < nk) gload((kt + 1) * BK);
        compute(cur);
        if (kt + 1 < nk) sstore(cur ^ 1, (kt + 1) * BK);
        __syncthreads();
    }

    if (p.norm) {
        const float inv_k = 1.0f / (float)p.K;
#pragma unroll
        for (int i = 0; i < A_IT; ++i) {
            float v = ss[i];
            v += __shfl_xor(v, 1);
            v += __shfl_xor(v, 2);
            v += __shfl_xor(v, 4);
            const int f = tid + 256 * i;
            if ((tid & 7) == 0 && (A_F4 % 256 == 0 || f < A_F4))
                row_scale[f >> 3] = 1.0f / sqrtf(v * inv_k + p.eps);
        }
        __syncthreads();
    }

    // ---- epilogue ----
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int lrow = arow0 + i * 16 + fk + r;  // fk == 4*(lane>>4)
            const int row = m0 + lrow;
            const float sc = p.norm ? row_scale[lrow] : 1.0f;
            if constexpr (EPI == EPI_STORE || EPI == EPI_RESID) {
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const int col = n0 + brow0 + j * 16 + frow;
                    if (row < p.M && col < p.N) {
                        float* dst = p.C + (int64_t)row * p.ldc + col;
                        if constexpr (EPI == EPI_STORE) *dst = acc[i][j][r] * sc;
                        else *dst += acc[i][j][r];
                    }
                }
            } else if constexpr (EPI == EPI_SWIGLU) {
#pragma unroll
                for (int j = 0; j < TN; j += 2) {
                    const int hcol = (n0 + brow0 + j * 16) / 2 + frow;
                    const float g = acc[i][j][r] * sc;
                    const float u = acc[i][j + 1][r] * sc;
                    if (row < p.M && hcol < p.N / 2)
                        p.C[(int64_t)row * p.ldc + hcol] = silu_f(g) * u;
                }
            } else {  // EPI_QKV
                const int qdim = p.H * p.HD, kvdim = p.KVH * p.HD;
                const int bidx = row / p.L;
                const int pos = p.start_pos + (row - bidx * p.L);
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const int col = n0 + brow0 + j * 16 + frow;
                    float v = acc[i][j][r] * sc;
                    const float partner = __shfl_xor(v, 1);  // every lane participates
                    if (row < p.M && col < p.N) {
                        if (col < qdim + kvdim) {  // q or k: interleaved-pair RoPE
                            const int d = (col < qdim ? col : col - qdim) % p.HD;
                            const int half = p.HD >> 1;
                            const float c = p.rope_cos[pos * half + (d >> 1)];
                            const float sn = p.rope_sin[pos * half + (d >> 1)];
                            v = (d & 1) ? (partner * sn + v * c) : (v * c - partner * sn);
                        }
                        if (col < qdim) {
                            p.q_out[(int64_t)row * qdim + col] = v * p.q_scale;
                        } else {
                            const bool is_k = col < qdim + kvdim;
                            const int c2 = is_k ? col - qdim : col - qdim - kvdim;
                            const int kvh = c2 / p.HD, d = c2 % p.HD;
                            float* cache = is_k ? p.cache_k : p.cache_v;
                            cache[(((int64_t)bidx * p.KVH + kvh) * p.Smax + pos) * p.HD + d] = v;
                        }
                    }
                }
            }
        }
    }
}

template <int WM, int WN, int TM, int TN>
static hipError_t launch_cfg(int epi, const GemmArgs& a, hipStream_t s) {
    constexpr int BM = WM * TM * 16, BN = WN * TN * 16;
    const int64_t tiles = (int64_t)((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
    dim3 grid((unsigned)tiles), block(256);
    switch (epi) {
        case EPI_STORE: hipLaunchKernelGGL((gemm_nt_kernel<WM, WN, TM, TN, EPI_STORE>), grid, block, 0, s, a); break;
        case EPI_RESID: hipLaunchKernelGGL((gemm_nt_kernel<WM, WN, TM, TN, EPI_RESID>), grid, block, 0, s, a); break;
        case EPI_SWIGLU: hipLaunchKernelGGL((gemm_nt_kernel<WM, WN, TM, TN, EPI_SWIGLU>), grid, block, 0, s, a); break;
        case EPI_QKV: hipLaunchKernelGGL((gemm_nt_kernel<WM, WN, TM, TN, EPI_QKV>), grid, block, 0, s, a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_gemm(int epi, const GemmArgs& a, hipStream_t s) {
    if (a.M <= 0 || a.N <= 0) return hipSuccess;
    if (a.K % BK != 0 || a.K <= 0) return hipErrorInvalidValue;
    if (epi == EPI_SWIGLU && a.N % 32 != 0) return hipErrorInvalidValue;
    if (a.M <= 32) return launch_cfg<1, 4, 1, 2>(epi, a, s);  // 16 x 128: decode / tiny M
    // SwiGLU needs an even TN (gate/up 16-row groups pair up inside one wave).
    if (epi == EPI_SWIGLU || a.N % 96 != 0) return launch_cfg<2, 2, 4, 4>(epi, a, s);  // 128 x 128
    return launch_cfg<2, 2, 4, 3>(epi, a, s);  // 128 x 96: N = 288 (O, down), 864 (QKV)
}

}  // namespace l3
