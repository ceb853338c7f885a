// fp32 MFMA GEMM kernels for gfx950:  C[M,N] = A[M,K] * W[N,K]^T  with fused epilogues.
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
//   A operand: lane l supplies A[i = l&15][k = l>>4];  B operand: lane l supplies B[k = l>>4][j = l&15];
//   C/D: lane l holds C[row = 4*(l>>4) + r][col = l&15], r = 0..3.
// K-permutation trick: a sum over k may visit k in any order as long as both operands agree,
// so at sub-step s lane l feeds k = 4*(l>>4) + s of a 16-deep group: one 16-byte LDS read of a
// K-contiguous row yields the operands of four consecutive MFMAs, for the activations and for
// W alike (both K-contiguous: W is the reference's [out, in]).
//
// Operands are swapped (W fragment as the A operand, activation fragment as B), so every
// accumulator is C^T: lane l holds C[row = 16i + (l&15)][col = 16j + 4(l>>4) + r] — four
// consecutive columns of one row, stored with one 16-byte write straight from registers (no
// LDS staging, no block barrier after the main loop).
//
// Main loop: K staged BK (16 or 32) deep through a double-buffered, unpadded, XOR-swizzled LDS
// image, one tile in flight ahead, one barrier per k-tile.  The next tile is filled either by
// global_load_lds (GLDS, the product path: no staging VGPRs, 128 x 128 fits 4 blocks/CU) or by
// register staging + ds_write_b128.  Rejected after measurement (tools/gemm_tune):
// fragment-shaped global loads straight to VGPRs (-35 %), a persistent flattened (tile, k)
// pipeline (-7 %), an LDS-staged row-major epilogue (-4 %).
//
// RMSNorm fusion: rmsnorm(x) @ W^T = diag(1/rms(x)) * x @ (W * w_norm)^T.  The norm weight is
// folded into W's columns once (l3_finalize, fold_cols_kernel); each lane accumulates the sum
// of squares of the A values its own fragments carry (a quarter of K of its row), two
// shuffles complete the row, and 1/rms scales the accumulators — the normalised activations
// are never materialised and A is copied to LDS as stored.
#pragma once
#include "kernels.h"

namespace l3 {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// silu (llama3.py:27-28) with v_rcp_f32 (1 ulp) instead of the IEEE division sequence: the
// SwiGLU epilogue's VALU share drops, gate|up 123.5 -> 126.4 TF/s (tools/gemm_tune A/B)
__device__ __forceinline__ float silu_f(float x) { return x * __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// XCD-aware bijective remap of the block id: blocks b and b+8 share an XCD (L2); each XCD
// gets a contiguous run of tile ids, so the tiles that re-read one A row panel share its L2.
__device__ __forceinline__ int xcd_remap(int b, int nwg) {
    const int xcd = b & 7, q8 = nwg >> 3, r8 = nwg & 7;
    return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
}

// Quad swizzle of row r of the unpadded LDS image: float4 quad q is stored at q ^ lds_swz(r).
// BK 16 -> (r >> 1) & 3, BK 32 -> r & 7: the ds_write_b128 groups (8 lanes: two rows at BK 16,
// one at BK 32) and the ds_read_b128 fragment reads (the four 16-lane groups of
// MI355X_MICROARCH.md section LDS) are conflict-free — enumerated, and the padded stride-24
// image it replaced measured SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE = 0.32 from its writes.
template <int BK>
__device__ __forceinline__ int lds_swz(int r) {
    return BK == 16 ? (r >> 1) & 3 : r & 7;
}

// QKV epilogue (same register-direct fragment map as direct_epilogue): RMSNorm row factor,
// RoPE on the two (even, odd) pairs of each float4 (llama3.py:41-76), then q (scaled) to the q
// buffer, k / v appended to the KV cache (llama3.py:184-185).  Branch-free over the q/k/v
// sections (a V tile rotates by cos = 1, sin = 0, which is exact), and the RoPE table loads of
// each row-half are issued before its stores: a load's vmcnt wait also waits for all older stores.
// output column (the first of a lane's float4) -> q / k / v section, head, column in the head
__device__ __forceinline__ void qkv_col(const GemmArgs& p, int col, int& sec, int& head, int& d) {
    const int qdim = p.H * p.HD, kvdim = p.KVH * p.HD;
    sec = col < qdim ? 0 : (col < qdim + kvdim ? 1 : 2);
    const int cc = col - (sec == 0 ? 0 : (sec == 1 ? qdim : qdim + kvdim));
    head = cc / p.HD;
    d = cc - head * p.HD;
}

// the RoPE table pairs of a one-row-tile QKV epilogue (TM = 1), fetched before the dot products
// by a kernel that has them to spare (gemm_skinny_kernel): qkv_epilogue<1, TN, true> takes them
template <int TN>
__device__ __forceinline__ void qkv_tables(const GemmArgs& p, int mrow0, int ncol0, int lane,
                                           float2 (&cs)[TN], float2 (&sn)[TN]) {
    const int frow = lane & 15, fq4 = 4 * (lane >> 4);
    const int rowc = min(mrow0 + frow, p.M - 1);
    const int pos = start_of(p) + rowc - rowc / p.L * p.L;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        int sec, head, d;
        qkv_col(p, min(ncol0 + j * 16 + fq4, p.N - 4) + p.col_base, sec, head, d);
        const int t = pos * (p.HD >> 1) + (d >> 1);
        cs[j] = *reinterpret_cast<const float2*>(p.rope_cos + t);
        sn[j] = *reinterpret_cast<const float2*>(p.rope_sin + t);
    }
}

template <int TM, int TN, bool PRE = false>
__device__ __forceinline__ void qkv_epilogue(const GemmArgs& p, const f32x4 (&acc)[TM][TN],
                                             const float (&rs)[TM], int mrow0, int ncol0,
                                             int lane, const float2* pre_cs = nullptr,
                                             const float2* pre_sn = nullptr) {
    static_assert(!PRE || TM == 1, "prefetched RoPE pairs: one row tile");
    const int frow = lane & 15, fq4 = 4 * (lane >> 4);
    const int qdim = p.H * p.HD, hd2 = p.HD >> 1;
    const int sp = start_of(p);
    int rowc[TM], bidx[TM], pos[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        rowc[i] = min(mrow0 + i * 16 + frow, p.M - 1);
        bidx[i] = rowc[i] / p.L;
        pos[i] = sp + rowc[i] - bidx[i] * p.L;
    }
    int sec[TN], head[TN], d[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) qkv_col(p, min(ncol0 + j * 16 + fq4, p.N - 4) + p.col_base, sec[j], head[j], d[j]);
    // two row-halves: each issues its RoPE loads (TM/2 x TN pairs) before its stores, so a
    // wave waits twice rather than once per float4, and the 4-block/CU register budget holds
    constexpr int TH = TM > 1 ? TM / 2 : 1;
#pragma unroll
    for (int i0 = 0; i0 < TM; i0 += TH) {
        float2 cs[TH][TN], sn[TH][TN];
#pragma unroll
        for (int ii = 0; ii < TH; ++ii)
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                if constexpr (PRE) {
                    cs[ii][j] = pre_cs[j];
                    sn[ii][j] = pre_sn[j];
                } else {
                    const int t = pos[i0 + ii] * hd2 + (d[j] >> 1);
                    cs[ii][j] = *reinterpret_cast<const float2*>(p.rope_cos + t);
                    sn[ii][j] = *reinterpret_cast<const float2*>(p.rope_sin + t);
                }
            }
#pragma unroll
        for (int ii = 0; ii < TH; ++ii) {
            const int i = i0 + ii;
            const int row = mrow0 + i * 16 + frow;
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int col = ncol0 + j * 16 + fq4;
                if (row >= p.M || col >= p.N) continue;
                const bool rot = sec[j] < 2;
                const float2 c = rot ? cs[ii][j] : float2{1.f, 1.f};
                const float2 s = rot ? sn[ii][j] : float2{0.f, 0.f};
                const f32x4 v = acc[i][j] * (sec[j] == 0 ? rs[i] * p.q_scale : rs[i]);
                const f32x4 r = {v.x * c.x - v.y * s.x, v.x * s.x + v.y * c.x,
                                 v.z * c.y - v.w * s.y, v.z * s.y + v.w * c.y};
                float* base = sec[j] == 0 ? p.q_out : (sec[j] == 1 ? p.cache_k : p.cache_v);
                const int64_t off = sec[j] == 0
                                        ? (int64_t)row * qdim + col
                                        : (((int64_t)bidx[i] * p.KVH + head[j]) * p.Smax + pos[i]) * p.HD + d[j];
                L3_DCHECK(sec[j] == 0 || (pos[i] >= 0 && pos[i] < p.Smax), CHK_KV_SLOT);
                *reinterpret_cast<f32x4*>(base + off) = r;
            }
        }
    }
}

// The QKV epilogue of a tile that lies wholly inside the launch (block-uniform: the product C3 /
// C4 / C5 shapes are multiples of their tiles) with HD % 16 == 0 and L >= the wave's TM x 16
// rows: the same arithmetic as qkv_epilogue, without its per-element work — no bounds guards,
// no integer division per row or column (each wave's first row and each 16-column group, which
// a head never straddles, are split once on the scalar unit; a lane's rows add at most one
// sequence wrap), each output address a row part plus a column part, and the q / k / v choice
// per column group wave-uniform.  In-kernel stamps (tools/gemm_tune qkvstamps, round 6): the
// generic epilogue took 21.5k cycles per block against 6.0k for a plain store of the same tile
template <int TM, int TN, int TH = (TM > 1 ? TM / 2 : 1)>
__device__ __forceinline__ void qkv_epilogue_full(const GemmArgs& p, const f32x4 (&acc)[TM][TN],
                                                  const float (&rs)[TM], int mrow0, int ncol0, int lane) {
    const int frow = lane & 15, fq4 = 4 * (lane >> 4);
    const int qdim = p.H * p.HD, kvdim = p.KVH * p.HD, hd2 = p.HD >> 1;
    const int sp = start_of(p);
    const int L = p.L;
    // rows: mrow0 (wave-uniform) = b0 * L + r0; lane row i: r0 + 16 i + frow < 2L
    const int b0 = __builtin_amdgcn_readfirstlane(mrow0) / L;
    const int r0 = __builtin_amdgcn_readfirstlane(mrow0) - b0 * L;
    const int64_t bstride = (int64_t)p.KVH * p.Smax * p.HD;
    int pos[TM];
    int64_t qoff[TM], koff[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        const int local = r0 + i * 16 + frow;
        const bool wrap = local >= L;
        const int ps = wrap ? local - L : local;
        pos[i] = sp + ps;
        qoff[i] = (int64_t)(mrow0 + i * 16 + frow) * qdim;
        koff[i] = (int64_t)(b0 + (wrap ? 1 : 0)) * bstride + (int64_t)pos[i] * p.HD;
        L3_DCHECK(pos[i] >= 0 && pos[i] < p.Smax, CHK_KV_SLOT);
    }
    // column groups: section, head and the group's first d, all wave-uniform
    int sec[TN];
    int coff[TN], d[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int c0 = __builtin_amdgcn_readfirstlane(ncol0 + j * 16) + p.col_base;
        const int sc = c0 < qdim ? 0 : (c0 < qdim + kvdim ? 1 : 2);
        const int cc = c0 - (sc == 0 ? 0 : (sc == 1 ? qdim : qdim + kvdim));
        const int head = cc / p.HD;
        sec[j] = sc;
        d[j] = cc - head * p.HD + fq4;
        coff[j] = sc == 0 ? ncol0 + j * 16 + fq4 : head * p.Smax * p.HD + d[j];
    }
    // TH rows of tables per pass: every load of a pass is issued before its stores (a load's
    // vmcnt wait also waits for older stores)
#pragma unroll
    for (int i0 = 0; i0 < TM; i0 += TH) {
        float2 cs[TH][TN], sn[TH][TN];
#pragma unroll
        for (int ii = 0; ii < TH; ++ii)
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int t = pos[i0 + ii] * hd2 + (d[j] >> 1);
                cs[ii][j] = *reinterpret_cast<const float2*>(p.rope_cos + t);
                sn[ii][j] = *reinterpret_cast<const float2*>(p.rope_sin + t);
            }
#pragma unroll
        for (int ii = 0; ii < TH; ++ii) {
            const int i = i0 + ii;
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const bool rot = sec[j] < 2;
                const float2 c = rot ? cs[ii][j] : float2{1.f, 1.f};
                const float2 s = rot ? sn[ii][j] : float2{0.f, 0.f};
                const f32x4 v = acc[i][j] * (sec[j] == 0 ? rs[i] * p.q_scale : rs[i]);
                const f32x4 r = {v.x * c.x - v.y * s.x, v.x * s.x + v.y * c.x,
                                 v.z * c.y - v.w * s.y, v.z * s.y + v.w * c.y};
                float* base = sec[j] == 0 ? p.q_out : (sec[j] == 1 ? p.cache_k : p.cache_v);
                const int64_t off = (sec[j] == 0 ? qoff[i] : koff[i]) + coff[j];
                *reinterpret_cast<f32x4*>(base + off) = r;
            }
        }
    }
}

// Register-direct epilogue (EPI_STORE / EPI_RESID / EPI_SWIGLU).  The MFMA operands are swapped
// (W fragment as the A operand, activation fragment as B), so the accumulator of tile (i, j) is C^T: lane l
// holds C[row = 16i + (l&15)][col = 16j + 4(l>>4) + r], r = 0..3 — four consecutive columns
// of one row, i.e. one 16-byte store, with no LDS staging and no block barrier.  rs[i] is the
// lane's RMSNorm factor for its row of tile i (1 without norm); res the prefetched residual.
template <int TM, int TN, int EPI, bool RES_PREFETCH, int NR>
__device__ __forceinline__ void direct_epilogue(const GemmArgs& p, const f32x4 (&acc)[TM][TN],
                                                const float (&rs)[TM], const f32x4 (&res)[NR],
                                                int mrow0, int ncol0, int lane) {
    const int frow = lane & 15, fq4 = 4 * (lane >> 4);
    if constexpr (EPI == EPI_STORE) {
        if (p.amax_rows) {
            // greedy argmax partials instead of the logits (llama3.py:320 over this wave's 16 * TN
            // columns of each row): the lane's own columns in rising order ("strictly greater, or
            // the first NaN" keeps the first index on ties), then the four lanes of the row
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const int row = mrow0 + i * 16 + frow;
                float best = -INFINITY;
                int bi = 0x7fffffff;
#pragma unroll
                for (int j = 0; j < TN; ++j)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int col = ncol0 + j * 16 + fq4 + r;
                        const float v = acc[i][j][r] * rs[i];
                        const bool vn = v != v, bn = best != best;
                        const bool take = col < p.N && (bi == 0x7fffffff || v > best || (vn && !bn));
                        best = take ? v : best;
                        bi = take ? col : bi;
                    }
                argmax_xor16_32<true, true>(best, bi, lane);
                if (lane < 16 && row < p.M)
                    p.amax_rows[(int64_t)row * p.amax_nct + ncol0 / (16 * TN)] = ArgmaxPart{best, bi};
            }
            return;
        }
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        const int row = mrow0 + i * 16 + frow;
        if (row >= p.M) continue;
        const float sc = rs[i];
        if constexpr (EPI == EPI_SWIGLU) {
            // fused W rows in 16-row groups: tile j (even) = gate, j + 1 = up of the same
            // 16 hidden units (ncol0 + 16j is a multiple of 32)
#pragma unroll
            for (int j = 0; j < TN; j += 2) {
                const int hcol = (ncol0 + j * 16) / 2 + fq4;
                if (hcol >= p.N / 2) continue;
                const f32x4 g = acc[i][j] * sc, u = acc[i][j + 1] * sc;
                const f32x4 v = {silu_f(g.x) * u.x, silu_f(g.y) * u.y, silu_f(g.z) * u.z, silu_f(g.w) * u.w};
                *reinterpret_cast<f32x4*>(p.C + (int64_t)row * p.ldc + hcol) = v;
            }
        } else {
            // EPI_RESID without the prefetch: the row's TN residual float4s are loaded together
            // (unpredicated, clamped column) before the first add — a predicated load per tile
            // compiled to a branch that waited for it before the next was issued
            f32x4 rrow[(EPI == EPI_RESID && !RES_PREFETCH) ? TN : 1];
            if constexpr (EPI == EPI_RESID && !RES_PREFETCH) {
                const float* rb = res_row(p, row);
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    rrow[j] = *reinterpret_cast<const f32x4*>(rb + min(ncol0 + j * 16 + fq4, p.N - 4));
            }
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int col = ncol0 + j * 16 + fq4;
                if (col >= p.N) continue;
                f32x4 v = acc[i][j];
                float* dst = p.C + (int64_t)row * p.ldc + col;
                if constexpr (EPI == EPI_RESID) {
                    if constexpr (RES_PREFETCH) v += res[i * TN + j];
                    else v += rrow[j];
                } else {
                    v *= sc;
                }
                *reinterpret_cast<f32x4*>(dst) = v;
            }
        }
    }
}

// Split-K epilogue: the raw accumulators of k-slice ks to p.ws[ks][M][N] (same register-direct
// fragment map, 16-byte stores) and, with the norm, the rows' partial sums of squares to
// p.ws[splits * M * N + ks * M + row] (one wave column writes them)
template <int TM, int TN>
__device__ __forceinline__ void split_epilogue(const GemmArgs& p, const f32x4 (&acc)[TM][TN],
                                               const float (&ss)[TM], int ks, int mrow0, int ncol0,
                                               int lane, bool ss_writer) {
    const int frow = lane & 15, fq4 = 4 * (lane >> 4);
    const int64_t MN = (int64_t)p.M * p.N;
    float* part = p.ws + ks * MN;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        const int row = mrow0 + i * 16 + frow;
        const float v = sum_xor16_32(ss[i]);  // every lane takes part in the exchange
        if (row >= p.M) continue;
        if (p.norm && ss_writer && lane < 16) p.ws[p.splits * MN + (int64_t)ks * p.M + row] = v;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int col = ncol0 + j * 16 + fq4;
            if (col < p.N) *reinterpret_cast<f32x4*>(part + (int64_t)row * p.N + col) = acc[i][j];
        }
    }
}

// Split-K finish: one thread per output float4 (EPI_SWIGLU: per float4 of hidden units) sums
// the p.splits partial tiles in slice order, forms the RMSNorm row factor from the partial sums
// of squares, and applies the same epilogue math as direct_epilogue / qkv_epilogue
template <int EPI>
__global__ void __launch_bounds__(256) splitk_finish_kernel(GemmArgs p) {
    const int nc = (EPI == EPI_SWIGLU ? p.N / 2 : p.N) / 4;
    const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (idx >= (int64_t)p.M * nc) return;
    const int row = (int)(idx / nc), c4 = (int)(idx - (int64_t)row * nc);
    const int S = p.splits;
    const int64_t MN = (int64_t)p.M * p.N;
    // every slice's load is issued before the first add (unpredicated, clamped slice index;
    // slices past S add zero): a loop of dependent loads cost one round trip per slice
    constexpr int SMAX = 16;  // launch_split_cfg: S <= 16
    float rs = 1.0f;
    if (p.norm) {
        float t[SMAX];
#pragma unroll
        for (int k = 0; k < SMAX; ++k) t[k] = p.ws[S * MN + (int64_t)min(k, S - 1) * p.M + row];
        float v = 0.f;
#pragma unroll
        for (int k = 0; k < SMAX; ++k) v += k < S ? t[k] : 0.f;
        rs = __builtin_amdgcn_rsqf(v * (1.0f / (float)p.K) + p.eps);
    }
    auto sum_at = [&](int col) {
        const float* src = p.ws + (int64_t)row * p.N + col;
        f32x4 t[SMAX];
#pragma unroll
        for (int k = 0; k < SMAX; ++k) t[k] = *reinterpret_cast<const f32x4*>(src + (int64_t)min(k, S - 1) * MN);
        f32x4 v = t[0];
#pragma unroll
        for (int k = 1; k < SMAX; ++k) v += k < S ? t[k] : f32x4{0.f, 0.f, 0.f, 0.f};
        return v;
    };
    if constexpr (EPI == EPI_SWIGLU) {
        // hidden units 16g + q: gate column 32g + q, up column 32g + 16 + q (fused W row groups)
        const int hcol = 4 * c4, g = hcol >> 4, q = hcol & 15;
        const f32x4 gt = sum_at(32 * g + q) * rs, up = sum_at(32 * g + 16 + q) * rs;
        const f32x4 v = {silu_f(gt.x) * up.x, silu_f(gt.y) * up.y, silu_f(gt.z) * up.z, silu_f(gt.w) * up.w};
        *reinterpret_cast<f32x4*>(p.C + (int64_t)row * p.ldc + hcol) = v;
    } else if constexpr (EPI == EPI_QKV) {
        const int col = 4 * c4;
        const int qdim = p.H * p.HD, kvdim = p.KVH * p.HD;
        const int sec = col < qdim ? 0 : (col < qdim + kvdim ? 1 : 2);
        const int cc = col - (sec == 0 ? 0 : (sec == 1 ? qdim : qdim + kvdim));
        const int head = cc / p.HD, d = cc - head * p.HD;
        const int bidx = row / p.L, pos = start_of(p) + row - bidx * p.L;
        const f32x4 v = sum_at(col) * (sec == 0 ? rs * p.q_scale : rs);
        float2 c = {1.f, 1.f}, sn = {0.f, 0.f};
        if (sec < 2) {
            const int t = pos * (p.HD >> 1) + (d >> 1);
            c = *reinterpret_cast<const float2*>(p.rope_cos + t);
            sn = *reinterpret_cast<const float2*>(p.rope_sin + t);
        }
        const f32x4 r = {v.x * c.x - v.y * sn.x, v.x * sn.x + v.y * c.x,
                         v.z * c.y - v.w * sn.y, v.z * sn.y + v.w * c.y};
        float* base = sec == 0 ? p.q_out : (sec == 1 ? p.cache_k : p.cache_v);
        const int64_t off = sec == 0 ? (int64_t)row * qdim + col
                                     : (((int64_t)bidx * p.KVH + head) * p.Smax + pos) * p.HD + d;
        L3_DCHECK(sec == 0 || (pos >= 0 && pos < p.Smax), CHK_KV_SLOT);
        *reinterpret_cast<f32x4*>(base + off) = r;
    } else {
        const int col = 4 * c4;
        f32x4 v = sum_at(col);
        if constexpr (EPI == EPI_RESID) v += *reinterpret_cast<const f32x4*>(res_at(p, row, col));
        else v *= rs;
        *reinterpret_cast<f32x4*>(p.C + (int64_t)row * p.ldc + col) = v;
    }
}

// In-kernel clock stamps for diagnostic builds (never in the product path): shader-clock
// counter and the 100 MHz real-time counter, read together.
__device__ __forceinline__ void stamp_pair(unsigned long long* dst) {
    unsigned long long t, rt;
    asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(t), "=s"(rt)::"memory");
    dst[0] = t;
    dst[1] = rt;
}

#define L3_STAMP(slot)                             \
    if constexpr (STAMP) {                         \
        __builtin_amdgcn_sched_barrier(0);         \
        stamp_pair(stamps + 2 * (slot));           \
        __builtin_amdgcn_sched_barrier(0);         \
    }

// ---------------------------------------------------------------------------------------
// Tiled kernel: 64 * WM * WN threads = WM x WN waves (the product tiles: 2 x 2), wave tile
// (TM x 16) x (TN x 16).
// counted wait for this wave's vector-memory ops (loads, stores and LDS-DMA alike, in order)
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}

// SPLIT: block b of a tiles x p.splits grid runs k-slice b / tiles of tile b % tiles (slice-major:
// the blocks of one XCD share that slice of A in L2) and leaves its raw accumulators and partial
// row sums of squares in p.ws (split_epilogue); splitk_finish_kernel sums the slices in order
template <int WM, int WN, int TM, int TN, int EPI, int WAVES_PER_EU = 2, bool STAMP = false,
          int BK = 32, bool GLDS = true, int NS = 2, bool SPLIT = false>
__global__ void __launch_bounds__(64 * WM * WN, WAVES_PER_EU) gemm_lds_kernel(GemmArgs p) {
    constexpr int NW = WM * WN, NT = 64 * NW;  // waves, threads
    constexpr int BM = WM * TM * 16;
    constexpr int BN = WN * TN * 16;
    static_assert(BK == 16 || BK == 32, "BK must be 16 or 32");
    static_assert(NS == 2 || (NS > 2 && GLDS), "deeper rings are filled by global_load_lds");
    constexpr int Q = BK / 4;        // float4 per image row
    constexpr int RP = 256 / BK;     // image rows per 1 KB global_load_lds piece
    constexpr int A_F4 = BM * Q, B_F4 = BN * Q;
    constexpr int A_IT = (A_F4 + NT - 1) / NT, B_IT = (B_F4 + NT - 1) / NT;

    // one LDS array: [NS][BM][BK] A image, then [NS][BN][BK] W image
    __shared__ __attribute__((aligned(16))) float smem[NS * (BM + BN) * BK];
    float (*As)[BM][BK] = reinterpret_cast<float (*)[BM][BK]>(smem);
    float (*Bs)[BN][BK] = reinterpret_cast<float (*)[BN][BK]>(smem + NS * BM * BK);

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid / WN, wn = wid % WN;
    const int ntn = (p.N + BN - 1) / BN;
    const int tb = xcd_remap(blockIdx.x, gridDim.x);
    const int ntiles = SPLIT ? ((p.M + BM - 1) / BM) * ntn : 1;
    const int ks = SPLIT ? tb / ntiles : 0;      // k-slice
    const int t = SPLIT ? tb - ks * ntiles : tb;  // tile
    int mt = t / ntn, nt = t - mt * ntn;
    if (p.group_m > 1) {  // GemmArgs::group_m: group of group_m row tiles, column-major inside
        const int ntm = (p.M + BM - 1) / BM;
        const int g = t / (p.group_m * ntn), first = g * p.group_m;
        const int gm = min(ntm - first, p.group_m), local = t - g * p.group_m * ntn;
        mt = first + local % gm;
        nt = local / gm;
    }
    const int m0 = mt * BM, n0 = nt * BN;
    const int nk = SPLIT ? p.K / BK / p.splits : p.K / BK;  // k-tiles of this block
    const int kb = ks * nk * BK;                           // its first k
    unsigned long long stamps[8];
    L3_STAMP(0);

    // ---- k-tile fill, GLDS: one wave-instruction writes 1 KB = RP image rows (lane i at byte
    // 16 i); the swizzle moves to the source address.  Pieces go round-robin over the waves;
    // rows past M / N are clamped (their outputs are never stored).
    // A-row source addresses are fixed for the tile: resolved once (a gathered embedding row
    // costs one index load per lane here, never inside the k-loop beside the DMA)
    constexpr int A_PIECES = (BM / RP + NW - 1) / NW;
    const float* a_src[A_PIECES];
#pragma unroll
    for (int it = 0; it < A_PIECES; ++it) {
        const int piece = wid + NW * it, r = piece * RP + lane / Q;
        a_src[it] = a_row(p, min(m0 + r, p.M - 1)) + 4 * ((lane % Q) ^ lds_swz<BK>(r));
    }
    auto glds_tile = [&](int buf, int k0) {
        const int rl = lane / Q, pq = lane % Q;
#pragma unroll
        for (int it = 0; it < A_PIECES; ++it) {
            const int piece = wid + NW * it;
            if ((BM / RP) % NW == 0 || piece < BM / RP) {
                __builtin_amdgcn_global_load_lds(
                    (const __attribute__((address_space(1))) void*)(a_src[it] + k0),
                    (__attribute__((address_space(3))) void*)&As[buf][piece * RP][0], 16, 0, 0);
            }
        }
#pragma unroll
        for (int it = 0; it < (BN / RP + NW - 1) / NW; ++it) {
            const int piece = wid + NW * it, r = piece * RP + rl;
            if ((BN / RP) % NW == 0 || piece < BN / RP) {
                const int gn = min(n0 + r, p.N - 1), q = pq ^ lds_swz<BK>(r);
                __builtin_amdgcn_global_load_lds(
                    (const __attribute__((address_space(1))) void*)(p.W + (int64_t)gn * p.K + k0 + 4 * q),
                    (__attribute__((address_space(3))) void*)&Bs[buf][piece * RP][0], 16, 0, 0);
            }
        }
    };
    // ---- k-tile fill, register staging: float4 f of the tile -> row f / Q, quad f % Q
    f32x4 ra[GLDS ? 1 : A_IT], rb[GLDS ? 1 : B_IT];
    auto gload = [&](int k0) {
#pragma unroll
        for (int i = 0; i < A_IT; ++i) {
            const int f = tid + NT * i, row = f / Q, c = (f % Q) * 4, gm = m0 + row;
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            if ((A_F4 % NT == 0 || f < A_F4) && gm < p.M)
                v = *reinterpret_cast<const f32x4*>(a_row(p, gm) + k0 + c);
            ra[i] = v;
        }
#pragma unroll
        for (int i = 0; i < B_IT; ++i) {
            const int f = tid + NT * i, row = f / Q, c = (f % Q) * 4, gn = n0 + row;
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            if ((B_F4 % NT == 0 || f < B_F4) && gn < p.N)
                v = *reinterpret_cast<const f32x4*>(p.W + (int64_t)gn * p.K + k0 + c);
            rb[i] = v;
        }
    };
    auto sstore = [&](int buf) {
#pragma unroll
        for (int i = 0; i < A_IT; ++i) {
            const int f = tid + NT * i, r = f / Q, q = f % Q;
            if (A_F4 % NT == 0 || f < A_F4)
                *reinterpret_cast<f32x4*>(&As[buf][r][(q ^ lds_swz<BK>(r)) * 4]) = ra[i];
        }
#pragma unroll
        for (int i = 0; i < B_IT; ++i) {
            const int f = tid + NT * i, r = f / Q, q = f % Q;
            if (B_F4 % NT == 0 || f < B_F4)
                *reinterpret_cast<f32x4*>(&Bs[buf][r][(q ^ lds_swz<BK>(r)) * 4]) = rb[i];
        }
    };

    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    float ss[TM];  // RMSNorm: sum of squares of this lane's quarter of row 16i + (lane & 15)
#pragma unroll
    for (int i = 0; i < TM; ++i) ss[i] = 0.f;

    const int frow = lane & 15, fk = 4 * (lane >> 4);
    const int arow0 = wm * TM * 16, brow0 = wn * TN * 16;
    const int fswz = lds_swz<BK>(frow);  // rows 16i + frow share it (16 | row base)

    auto compute = [&](int buf) {
#pragma unroll
        for (int kg = 0; kg < BK / 16; ++kg) {
            f32x4 a[TM], bw[TN];
            const int fcol = 4 * ((kg * 4 + (lane >> 4)) ^ fswz);
#pragma unroll
            for (int i = 0; i < TM; ++i)
                a[i] = *reinterpret_cast<const f32x4*>(&As[buf][arow0 + i * 16 + frow][fcol]);
#pragma unroll
            for (int j = 0; j < TN; ++j)
                bw[j] = *reinterpret_cast<const f32x4*>(&Bs[buf][brow0 + j * 16 + frow][fcol]);
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j) acc[i][j] = mfma4(bw[j][s], a[i][s], acc[i][j]);
#pragma unroll
            for (int i = 0; i < TM; ++i)
                ss[i] += a[i].x * a[i].x + a[i].y * a[i].y + a[i].z * a[i].z + a[i].w * a[i].w;
        }
    };

    // EPI_RESID: the lane's residual float4s, prefetched during the last k-tile when at most 12
    constexpr bool RES_PREFETCH = EPI == EPI_RESID && TM * TN <= 12;
    f32x4 res[RES_PREFETCH ? TM * TN : 1];

    if constexpr (NS > 2) {
        // NS-deep LDS ring for latency-bound shapes (few blocks, weights streamed from HBM):
        // NS - 1 k-tiles in flight; counted vmcnt + raw s_barrier so the DMA spans barriers
        // (__syncthreads would drain every outstanding glds).  Per iteration: wait until tile
        // kt has landed (this wave's pieces), barrier (everyone's pieces landed, everyone done
        // with tile kt - 1), refill the slot of tile kt - 1 with tile kt + NS - 1, compute.
        // glds per wave per tile: pieces go round-robin over the 4 waves, so when a tile's
        // piece count is not a multiple of 4 the first (count % 4) waves issue one more; each
        // wave's counted wait must use its own count (with the larger count for every wave, a
        // wave issuing fewer would not wait for its own pieces of tile kt: stale LDS rows)
        constexpr int AP = BM / RP, BP = BN / RP;
        constexpr int GA_HI = (AP + NW - 1) / NW, GA_LO = AP / NW, GB_HI = (BP + NW - 1) / NW, GB_LO = BP / NW;
        // the per-wave counts cover every piece exactly once: (AP % 4) waves issue GA_HI, the
        // rest GA_LO (when AP % 4 == 0 all four issue GA_HI == GA_LO); same for B
        static_assert((AP % NW) * GA_HI + (NW - AP % NW) * GA_LO == AP, "A pieces per wave");
        static_assert((BP % NW) * GB_HI + (NW - BP % NW) * GB_LO == BP, "B pieces per wave");
        static_assert(AP % NW != 0 || GA_HI == GA_LO, "A pieces: equal counts");
        static_assert(BP % NW != 0 || GB_HI == GB_LO, "B pieces: equal counts");
        const bool a_hi = AP % NW == 0 || wid < AP % NW, b_hi = BP % NW == 0 || wid < BP % NW;
        auto wait_ring = [&]() {  // wave-uniform branches over compile-time counts
            if (a_hi) {
                if (b_hi) wait_vmcnt<(NS - 2) * (GA_HI + GB_HI)>();
                else wait_vmcnt<(NS - 2) * (GA_HI + GB_LO)>();
            } else {
                if (b_hi) wait_vmcnt<(NS - 2) * (GA_LO + GB_HI)>();
                else wait_vmcnt<(NS - 2) * (GA_LO + GB_LO)>();
            }
        };
#pragma unroll
        for (int i = 0; i < NS - 1; ++i)
            if (i < nk) glds_tile(i, kb + i * BK);
        for (int kt = 0; kt < nk; ++kt) {
            if (kt + NS - 2 < nk) wait_ring();
            else wait_vmcnt<0>();
            // this wave's LDS reads of tile kt - 1 are done before anyone refills its slot
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            __builtin_amdgcn_sched_barrier(0);
            if (kt + NS - 1 < nk) glds_tile((kt + NS - 1) % NS, kb + (kt + NS - 1) * BK);
            if constexpr (RES_PREFETCH) {
                if (kt == nk - 1) {
                    const float* rb[TM];
#pragma unroll
                    for (int i = 0; i < TM; ++i) rb[i] = res_row(p, min(m0 + arow0 + i * 16 + frow, p.M - 1));
#pragma unroll
                    for (int i = 0; i < TM; ++i)
#pragma unroll
                        for (int j = 0; j < TN; ++j)
                            res[i * TN + j] = *reinterpret_cast<const f32x4*>(rb[i] + min(n0 + brow0 + j * 16 + fk, p.N - 4));
                }
            }
            compute(kt % NS);
        }
    } else {
    if constexpr (GLDS) {
        glds_tile(0, kb);
    } else {
        gload(kb);
        sstore(0);
    }
    __syncthreads();
    L3_STAMP(1);
    for (int kt = 0; kt < nk - 1; ++kt) {
        const int cur = kt & 1;
        if constexpr (GLDS) {
            glds_tile(cur ^ 1, kb + (kt + 1) * BK);  // lands while this tile computes
            compute(cur);
        } else {
            gload(kb + (kt + 1) * BK);
            compute(cur);
            sstore(cur ^ 1);
        }
        __syncthreads();  // (GLDS: its fence waits vmcnt(0), retiring the DMA)
    }
    // last k-tile, peeled: the residual loads are issued first so their latency hides behind
    // this tile's MFMAs
    // (unpredicated, from clamped rows / columns — rows and columns past the edge are never
    // stored — so all TM x TN loads are in flight together: predicated ones compiled to
    // branches that waited for each load before issuing the next)
    if constexpr (RES_PREFETCH) {
        const float* rb[TM];  // a gathered embedding row's index is read once per row
#pragma unroll
        for (int i = 0; i < TM; ++i) rb[i] = res_row(p, min(m0 + arow0 + i * 16 + frow, p.M - 1));
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
                res[i * TN + j] = *reinterpret_cast<const f32x4*>(rb[i] + min(n0 + brow0 + j * 16 + fk, p.N - 4));
    }
    compute((nk - 1) & 1);
    }

    // no barrier: each wave finishes its own tile from registers
    if constexpr (SPLIT) {
        split_epilogue<TM, TN>(p, acc, ss, ks, m0 + arow0, n0 + brow0, lane, wn == 0);
        return;
    }
    float rs[TM];
    const float inv_k = 1.0f / (float)p.K;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        float v = ss[i];
        v = sum_xor16_32(v);  // the four k-quarters of the row
        // v_rsq_f32 (1 ulp) rather than sqrt + IEEE division: QKV +1.2 %, gate|up +0.5 %
        rs[i] = p.norm ? __builtin_amdgcn_rsqf(v * inv_k + p.eps) : 1.0f;
    }
    L3_STAMP(2);
    if constexpr (EPI == EPI_QKV) {
        // whole tile inside the launch (block-uniform), heads in whole 16-column groups, at most
        // one sequence wrap per wave row range: the division-free epilogue (L3_QKV_FAST_EPI=0
        // in the launcher keeps the generic one for A/B)
        if (p.qkv_fast && m0 + BM <= p.M && n0 + BN <= p.N)
#ifdef L3_QKV_TH_ALL  // tools: every table load before the first store (register A/B)
            qkv_epilogue_full<TM, TN, TM>(p, acc, rs, m0 + arow0, n0 + brow0, lane);
#else
            qkv_epilogue_full<TM, TN>(p, acc, rs, m0 + arow0, n0 + brow0, lane);
#endif
        else
            qkv_epilogue<TM, TN>(p, acc, rs, m0 + arow0, n0 + brow0, lane);
    }
    else direct_epilogue<TM, TN, EPI, RES_PREFETCH>(p, acc, rs, res, m0 + arow0, n0 + brow0, lane);
    L3_STAMP(3);
    if constexpr (STAMP) {
        if (tid == 0) {
            unsigned long long* d = p.stamps + (size_t)blockIdx.x * 10;
            for (int i = 0; i < 8; ++i) d[i] = stamps[i];
            unsigned xcc;
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
            d[8] = xcc;
            d[9] = t;
        }
    }
}

#undef L3_STAMP

// ---------------------------------------------------------------------------------------
// Skinny MFMA GEMM for 9..256 rows against a small (L2-resident) weight: batched decode and
// short prompts (llama3.py:166-178,211,99-102 at B x 1 tokens).  A block owns one 16-row x
// 16*TN-column output tile and its four waves split K; no LDS staging: every lane loads its own
// fragments straight from global memory (A row m0 + (l&15) and W rows n0 + 16j + (l&15),
// 16-byte pieces at k = 16kb + 4(l>>4): the K-permutation of gemm_lds_kernel), up to CH
// k-blocks of them in flight per memory round trip, then 4 MFMAs per k-block and W row.  The
// four partial tiles (and row sums of squares) meet in LDS and wave 0 adds them in wave order
// and runs the tiled kernel's epilogue (RMSNorm row factor, RoPE / KV append, SwiGLU pairs,
// residual).  The weight-streaming GEMV keeps M <= 8, where its lanes' wider K split wins.
//
// STAMP (diagnostic builds, tools/gemm_tune skinnystamps; never in the product): wave 0 of each
// block leaves s_memrealtime (100 MHz) stamps in p.stamps[block][8]: entry, first fragments
// landed, k-loop done, partials reduced (after the barrier), epilogue issued, its stores acked
template <int EPI, int TN, int CH, int NW = 4, bool STAMP = false>
__global__ void __launch_bounds__(64 * NW) gemm_skinny_kernel(GemmArgs p) {
    static_assert(EPI != EPI_SWIGLU || TN % 2 == 0, "SwiGLU pairs gate / up tiles");
    auto sk_stamp = [&](int k) {
        if constexpr (STAMP) {
            __builtin_amdgcn_sched_barrier(0);
            const unsigned long long t = __builtin_amdgcn_s_memrealtime();
            if ((threadIdx.x & 255) == 0) p.stamps[(size_t)blockIdx.x * 8 + k] = t;
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    sk_stamp(0);
    constexpr int WN = 16 * TN;  // columns per tile
    __shared__ f32x4 red[NW][TN][64];
    __shared__ float rss[NW][64];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int frow = lane & 15, kq = 4 * (lane >> 4);
    const int ntn = (p.N + WN - 1) / WN;
    int mt, nt;
    if (p.skinny_xcd) {  // contiguous run of tiles per XCD, column-major: W tiles stay on one XCD
        const int nmt = (p.M + 15) / 16, t = xcd_remap(blockIdx.x, gridDim.x);
        nt = t / nmt;
        mt = t - nt * nmt;
    } else {
        mt = blockIdx.x / ntn;
        nt = blockIdx.x - mt * ntn;
    }
    const int m0 = mt * 16, n0 = nt * WN;
    const float* arow = a_row(p, min(m0 + frow, p.M - 1));
    const float* wrow[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) wrow[j] = p.W + (int64_t)min(n0 + 16 * j + frow, p.N - 1) * p.K;
    // the epilogue's own operands (EPI_RESID: the residual float4s of the lane's row; EPI_QKV: the
    // RoPE table pairs) do not depend on the dot products: fetched now, with the fragments, not
    // after the reduction (one memory round trip less per launch); every wave issues them, wave 0
    // uses them (unpredicated: a wave-dependent branch would cost the others nothing but the
    // waits hipcc places after it)
    const int fq4 = 4 * (lane >> 4);
    f32x4 res[EPI == EPI_RESID ? TN : 1];
    float2 pcs[EPI == EPI_QKV ? TN : 1], psn[EPI == EPI_QKV ? TN : 1];
    if constexpr (EPI == EPI_RESID) {
        const float* rb = res_row(p, min(m0 + frow, p.M - 1));
#pragma unroll
        for (int j = 0; j < TN; ++j) res[j] = *reinterpret_cast<const f32x4*>(rb + min(n0 + j * 16 + fq4, p.N - 4));
    } else if constexpr (EPI == EPI_QKV) {
        qkv_tables<TN>(p, m0, n0, lane, pcs, psn);
    }
    f32x4 acc[1][TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[0][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    float ss = 0.f;
    const int nkb = p.K >> 4;
    const int kb_lo = wid * nkb / NW, kb_hi = (wid + 1) * nkb / NW;  // this wave's k-blocks
    for (int kb0 = kb_lo; kb0 < kb_hi; kb0 += CH) {
        f32x4 av[CH], wv[CH][TN];
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            const int k = 16 * min(kb0 + c, kb_hi - 1) + kq;
            av[c] = *reinterpret_cast<const f32x4*>(arow + k);
#pragma unroll
            for (int j = 0; j < TN; ++j) wv[c][j] = *reinterpret_cast<const f32x4*>(wrow[j] + k);
        }
        if constexpr (STAMP) {
            if (kb0 == kb_lo) {
                __builtin_amdgcn_s_waitcnt(0);  // (diagnostic) the first fragments landed
                sk_stamp(1);
            }
        }
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            if (kb0 + c < kb_hi) {  // wave-uniform
                ss += av[c].x * av[c].x + av[c].y * av[c].y + av[c].z * av[c].z + av[c].w * av[c].w;
#pragma unroll
                for (int s = 0; s < 4; ++s)
#pragma unroll
                    for (int j = 0; j < TN; ++j) acc[0][j] = mfma4(wv[c][j][s], av[c][s], acc[0][j]);
            }
        }
    }
    sk_stamp(2);
#pragma unroll
    for (int j = 0; j < TN; ++j) red[wid][j][lane] = acc[0][j];
    rss[wid][lane] = ss;
    __syncthreads();
    if (wid != 0) return;
    sk_stamp(3);
#pragma unroll
    for (int w = 1; w < NW; ++w) {
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[0][j] += red[w][j][lane];
        ss += rss[w][lane];
    }
    float rs[1];
    {
        const float v = sum_xor16_32(ss);  // the four k-quarters of the row
        rs[0] = p.norm ? __builtin_amdgcn_rsqf(v * (1.0f / (float)p.K) + p.eps) : 1.0f;
    }
    if constexpr (EPI == EPI_QKV) {
        qkv_epilogue<1, TN, true>(p, acc, rs, m0, n0, lane, pcs, psn);
    } else if constexpr (EPI == EPI_RESID) {
        direct_epilogue<1, TN, EPI, true, TN>(p, acc, rs, res, m0, n0, lane);
    } else {
        direct_epilogue<1, TN, EPI, false, 1>(p, acc, rs, res, m0, n0, lane);
    }
    if constexpr (STAMP) {
        sk_stamp(4);
        __builtin_amdgcn_s_waitcnt(0);  // (diagnostic) the epilogue's stores acknowledged
        sk_stamp(5);
    }
}

// ---------------------------------------------------------------------------------------
// Skinny GEMM for short M (greedy decode, short prompts): weight-streaming, HBM / latency
// bound, so no MFMA; MR rows per block, grid.y row blocks beyond MR.  A unit is one W row (EPI_STORE / EPI_RESID), a RoPE pair (EPI_QKV: rows
// 2u, 2u + 1) or a gate/up pair (EPI_SWIGLU: fused rows 32(u/16) + u%16 and + 16).  LPU lanes
// share a unit and split its K: lane j streams float4 k4 = j + LPU t, with a whole chunk of CH
// loads per row in flight before the first FMA (one memory round trip per chunk, not one per
// load), and a butterfly over the LPU lanes completes the dot products.  The M input rows are
// staged in LDS once per block; the RMSNorm sum of squares comes from the same lane-split reads
// (the norm weight itself is folded into W, launch_fold_cols).
//
// PARTS (decode with the O-proj fused into attention, MR = 1 only): p.parts holds the per-head
// O-proj rows [M][nparts][D]; EPI_SWIGLU adds them to its input row (h + attention . Wo^T, the
// FFN's input, llama3.py:253), EPI_RESID to its residual (the down-proj's residual is that same
// row, :259), always in head order.  Their loads join the same round trip (GEMV_MAXP per
// piece, predicated past nparts, so CH drops to 4).
//
// NT: the W pieces are loaded non-temporal (global_load ... nt): weights that one wave streams
// once per call and that do not fit the caches anyway (Llama-3-shape decode: 67 MB - 2.1 GB per
// launch); the small layer weights of stories15M stay on the default policy (they are re-read
// from the caches every step).
//
// FOLD (EPI_QKV, MR = 1: layer 0 of a captured batch-1 decode step that follows another in the
// same graph): the previous step's greedy argmax (llama3.py:320) happens here instead of in a
// launch of its own — every block reduces that step's lm_head partials (GemmArgs::amax_in, a few
// KB from L2, loaded beside the W pieces) to the id whose embedding row is this step's input
// (:287); block 0 publishes the id (amax_ids, amax_st's history).
template <int EPI, int MR, int LPU, bool PARTS = false, bool NT = false, bool FOLD = false>
__global__ void __launch_bounds__(256) gemv_kernel(GemmArgs p) {
    extern __shared__ __attribute__((aligned(16))) float xs[];  // [MR][K]
    static_assert(!PARTS || MR == 1, "partial rows only on the one-row GEMV");
    static_assert(!FOLD || (MR == 1 && EPI == EPI_QKV && !PARTS), "the folded argmax feeds a one-row QKV");
    constexpr int ROWS = (EPI == EPI_SWIGLU || EPI == EPI_QKV) ? 2 : 1;
    constexpr int UPW = 64 / LPU;  // units per wave
    constexpr int CH = PARTS ? 4 : 8;  // float4 per W row per lane in flight
    constexpr bool XPARTS = PARTS && EPI == EPI_SWIGLU;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int K4 = p.K >> 2;
    const int j = lane % LPU;
    const int unit = (blockIdx.x * 4 + wid) * UPW + lane / LPU;
    const int nunits = ROWS == 2 ? p.N / 2 : p.N;
    const bool valid = unit < nunits;
    const int u = valid ? unit : 0;
    int wrow[ROWS];
    if constexpr (EPI == EPI_SWIGLU) {
        wrow[0] = 32 * (u / 16) + (u % 16);
        wrow[ROWS - 1] = wrow[0] + 16;
    } else if constexpr (EPI == EPI_QKV) {
        wrow[0] = 2 * u;
        wrow[ROWS - 1] = 2 * u + 1;
    } else {
        wrow[0] = u;
    }
    const f32x4* W4 = reinterpret_cast<const f32x4*>(p.W);
    // row block: rows [m0, m0 + Mb) of A (grid.y row blocks of MR rows re-read W through L2)
    const int m0 = blockIdx.y * MR, Mb = min(MR, p.M - m0);
    // MR == 1 (batch-1 decode): each lane loads its own float4s of the input row next to its W
    // pieces — one memory round trip, no LDS staging pass and no block barrier; MR > 1 stages
    // the rows once in LDS (re-read by every unit of the block)
    constexpr bool DIRECT = MR == 1;
    const f32x4* X4 = reinterpret_cast<const f32x4*>(FOLD ? p.A : a_row(p, m0));
    f32x4 w[ROWS][CH];
    f32x4 xv[DIRECT ? CH : 1];
    f32x4 xp[XPARTS ? CH : 1][XPARTS ? GEMV_MAXP : 1];
    const f32x4* P4 = reinterpret_cast<const f32x4*>(p.parts) + (int64_t)m0 * p.nparts * K4;
    // Row-blocked forms (MR > 1): W loads unpredicated from clamped addresses, x zeroed past K
    // where it is used (their predicated loads compiled to exec-masked branches that each waited
    // for the load before issuing the next).  The one-row form keeps predicated loads: there
    // hipcc already issued them all before the first wait, and the unpredicated form let it
    // interleave loads and waits instead.
    auto load_chunk = [&](int t0) {
#pragma unroll
        for (int t = 0; t < CH; ++t) {
            const int k4 = j + LPU * (t0 + t), kk = min(k4, K4 - 1);
#pragma unroll
            for (int r = 0; r < ROWS; ++r) {
                if constexpr (DIRECT)
                    w[r][t] = k4 >= K4 ? f32x4{0.f, 0.f, 0.f, 0.f}
                              : NT ? __builtin_nontemporal_load(&W4[(int64_t)wrow[r] * K4 + k4])
                                   : W4[(int64_t)wrow[r] * K4 + k4];
                else
                    w[r][t] = NT ? __builtin_nontemporal_load(&W4[(int64_t)wrow[r] * K4 + kk])
                                 : W4[(int64_t)wrow[r] * K4 + kk];
            }
            if constexpr (DIRECT) {
                if (!FOLD || t0) xv[t] = X4[kk];  // FOLD: chunk 0's x once the id is known
            }
            if constexpr (XPARTS) {
#pragma unroll
                for (int pp = 0; pp < GEMV_MAXP; ++pp)
                    xp[t][pp] = (pp < p.nparts && k4 < K4) ? P4[(int64_t)pp * K4 + k4] : f32x4{0.f, 0.f, 0.f, 0.f};
            }
        }
    };
    // x = A row + the heads' O-proj rows, summed in head order
    auto add_parts = [&]() {
        if constexpr (XPARTS) {
#pragma unroll
            for (int t = 0; t < CH; ++t)
#pragma unroll
                for (int pp = 0; pp < GEMV_MAXP; ++pp) xv[t] += xp[t][pp];
        }
    };
    // FOLD: the previous step's partials, loaded before the W pieces so the reduction waits for
    // them alone (clamped indices: a repeated partial does not change an argmax)
    constexpr int FU = 8;
    ArgmaxPart fq[FOLD ? FU : 1];
    int f_pos = 0, f_base = 0, f_cap = 0;  // block 0: the history fields, fetched up front
    int32_t* f_hist = nullptr;
    float* f_hist_val = nullptr;
    if constexpr (FOLD) {
#pragma unroll
        for (int u = 0; u < FU; ++u) fq[u] = p.amax_in[min(u * 256 + tid, p.amax_in_n - 1)];
        if (blockIdx.x == 0) {
            const DecState* st = p.amax_st;
            f_pos = st->pos;
            f_base = st->hist_base;
            f_cap = st->hist_cap;
            f_hist = st->hist;
            f_hist_val = st->hist_val;
        }
    }
    load_chunk(0);  // in flight while the input rows are staged
    // the epilogue's own operands (EPI_RESID: the residual; EPI_QKV: the RoPE cos / sin of the
    // pair) do not depend on the dot products: fetch them now, not after the reduction (one
    // memory round trip less per launch; decode runs three such launches per layer)
    const bool writer = j == 0 && valid;
    float pre0[MR], pre1[MR];
    float2 bak_old[EPI == EPI_QKV ? MR : 1];
    int qkv_sec = 0, qkv_head = 0, qkv_d = 0;  // EPI_QKV: 0 q, 1 k, 2 v; head; column in head
    if constexpr (EPI == EPI_QKV) {
        const int qdim = p.H * p.HD, kvdim = p.KVH * p.HD, col = 2 * u;
        qkv_sec = col < qdim ? 0 : col < qdim + kvdim ? 1 : 2;
        const int cc = col - (qkv_sec == 0 ? 0 : qkv_sec == 1 ? qdim : qdim + kvdim);
        qkv_head = cc / p.HD;
        qkv_d = cc - qkv_head * p.HD;
    }
#pragma unroll
    for (int mi = 0; mi < MR; ++mi) {
        pre0[mi] = 0.f;
        pre1[mi] = 0.f;
        if (!writer || mi >= Mb) continue;
        const int m = m0 + mi;
        if constexpr (EPI == EPI_RESID) {
            pre0[mi] = *res_at(p, m, unit);
            if constexpr (PARTS) {
                float pr[GEMV_MAXP];
#pragma unroll
                for (int pp = 0; pp < GEMV_MAXP; ++pp)
                    pr[pp] = pp < p.nparts ? p.parts[((int64_t)m * p.nparts + pp) * p.ldc + unit] : 0.f;
#pragma unroll
                for (int pp = 0; pp < GEMV_MAXP; ++pp) pre0[mi] += pr[pp];
            }
        } else if constexpr (EPI == EPI_QKV) {
            if (qkv_sec < 2) {
                const int bidx = m / p.L, pos = start_of(p) + m - bidx * p.L;
                const int t = pos * (p.HD >> 1) + (qkv_d >> 1);
                pre0[mi] = p.rope_cos[t];
                pre1[mi] = p.rope_sin[t];
            } else {
                pre0[mi] = 1.f;  // V: identity rotation
            }
            if (p.kv_bak && qkv_sec > 0) {  // the slot's previous K / V pair (see GemmArgs::kv_bak)
                const int bidx = m / p.L, pos = start_of(p) + m - bidx * p.L;
                bak_old[mi] = *reinterpret_cast<const float2*>(
                    (qkv_sec == 1 ? p.cache_k : p.cache_v) +
                    (((int64_t)bidx * p.KVH + qkv_head) * p.Smax + pos) * p.HD + qkv_d);
            }
        }
    }
    if constexpr (FOLD) {
        float bv = -INFINITY;
        int bi = 0x7fffffff;
        for (int base = 0;; base += FU * 256) {
#pragma unroll
            for (int u = 0; u < FU; ++u)
                if (argmax_better(fq[u].v, fq[u].i, bv, bi)) { bv = fq[u].v; bi = fq[u].i; }
            if (base + FU * 256 >= p.amax_in_n) break;
#pragma unroll
            for (int u = 0; u < FU; ++u) fq[u] = p.amax_in[min(base + FU * 256 + u * 256 + tid, p.amax_in_n - 1)];
        }
        group_argmax<64>(bv, bi, lane);
        __shared__ float fv[4];
        __shared__ int fi[4];
        if (lane == 0) {
            fv[wid] = bv;
            fi[wid] = bi;
        }
        __syncthreads();
        bv = fv[0];
        bi = fi[0];
#pragma unroll
        for (int w2 = 1; w2 < 4; ++w2)
            if (argmax_better(fv[w2], fi[w2], bv, bi)) {
                bv = fv[w2];
                bi = fi[w2];
            }
        X4 = reinterpret_cast<const f32x4*>(p.A + (int64_t)bi * p.lda);
#pragma unroll
        for (int t = 0; t < CH; ++t) xv[t] = X4[min(j + LPU * t, K4 - 1)];
        if (blockIdx.x == 0 && tid == 0) {
            p.amax_ids[0] = bi;
            // the previous step's position: its lm_head already moved pos on (pos_adv)
            const int q = f_pos - 1 - f_base;
            if (f_hist && q >= 0 && q < f_cap) f_hist[q] = bi;
            if (f_hist_val && q >= 0 && q < f_cap) f_hist_val[q] = bv;
        }
    }
    // stage the row block (rows past Mb zero: branch-free FMA loop), SU loads in flight per
    // thread before the first LDS store (a serial load -> store walk costs a round trip each)
    // (unpredicated loads from clamped addresses, zeroed after they land: predicated loads
    // compiled to exec-masked branches that waited for each load before issuing the next)
    constexpr int SU = 8;
    if constexpr (!DIRECT) {
        for (int f0 = tid; f0 < MR * K4; f0 += 256 * SU) {
            f32x4 v[SU];
#pragma unroll
            for (int u = 0; u < SU; ++u) {
                const int f = f0 + 256 * u, m = f / K4, k4 = f - m * K4;
                const bool ok = f < MR * K4 && m < Mb;
                v[u] = reinterpret_cast<const f32x4*>(a_row(p, m0 + (ok ? m : 0)))[ok ? k4 : 0];
            }
#pragma unroll
            for (int u = 0; u < SU; ++u) {
                const int f = f0 + 256 * u, m = f / K4;
                if (f < MR * K4) reinterpret_cast<f32x4*>(xs)[f] = m < Mb ? v[u] : f32x4{0.f, 0.f, 0.f, 0.f};
            }
        }
        __syncthreads();
    }

    float acc[ROWS][MR], ss[MR];
#pragma unroll
    for (int m = 0; m < MR; ++m) {
        ss[m] = 0.f;
#pragma unroll
        for (int r = 0; r < ROWS; ++r) acc[r][m] = 0.f;
    }
    const int nt = (K4 + LPU - 1) / LPU;
    for (int t0 = 0; t0 < nt; t0 += CH) {
        if (t0) load_chunk(t0);
        add_parts();
        if constexpr (XPARTS) {  // block 0's first unit holds every k4 of the summed row
            if (p.x_out && blockIdx.x == 0 && tid < LPU) {
#pragma unroll
                for (int t = 0; t < CH; ++t) {
                    const int k4 = j + LPU * (t0 + t);
                    if (k4 < K4) reinterpret_cast<f32x4*>(p.x_out + (int64_t)m0 * p.K)[k4] = xv[t];
                }
            }
        }
#pragma unroll
        for (int t = 0; t < CH; ++t) {
            if (t0 + t >= nt) break;  // wave-uniform
            // lanes past K: the one-row form reads a clamped (finite) x against its zero W and
            // counts no norm; the row-blocked form holds clamped W and zeroes x
            const int k4 = j + LPU * (t0 + t), kk = min(k4, K4 - 1);
            const float in = k4 < K4 ? 1.f : 0.f;
            f32x4 x[MR];
            if constexpr (DIRECT) {
                x[0] = xv[t];
            } else {
#pragma unroll
                for (int m = 0; m < MR; ++m)
                    x[m] = k4 < K4 ? reinterpret_cast<const f32x4*>(xs + m * p.K)[kk] : f32x4{0.f, 0.f, 0.f, 0.f};
            }
#pragma unroll
            for (int m = 0; m < MR; ++m) {
                ss[m] += in * (x[m].x * x[m].x + x[m].y * x[m].y + x[m].z * x[m].z + x[m].w * x[m].w);
#pragma unroll
                for (int r = 0; r < ROWS; ++r)
                    acc[r][m] += w[r][t].x * x[m].x + w[r][t].y * x[m].y + w[r][t].z * x[m].z + w[r][t].w * x[m].w;
            }
        }
    }
    // the LPU lanes of a unit are one aligned group: VALU-only reduction (no LDS round trips)
#pragma unroll
    for (int m = 0; m < MR; ++m) {
        ss[m] = group_sum<LPU>(ss[m]);
#pragma unroll
        for (int r = 0; r < ROWS; ++r) acc[r][m] = group_sum<LPU>(acc[r][m]);
    }
    if constexpr (EPI == EPI_STORE && MR == 1) {
        if (p.amax_part) {  // batch-1 lm_head: this block's (value, index) argmax (llama3.py:320)
            // every lane of a unit holds its sum; the value is the logit stored below, bit for bit
            const float sc = p.norm ? __builtin_amdgcn_rsqf(ss[0] / (float)p.K + p.eps) : 1.0f;
            float bv = valid ? acc[0][0] * sc : -INFINITY;
            int bi = valid ? unit : 0x7fffffff;
            group_argmax<64>(bv, bi, lane);
            __shared__ float sv[4];
            __shared__ int si[4];
            if (lane == 0) {
                sv[wid] = bv;
                si[wid] = bi;
            }
            __syncthreads();
            if (tid == 0) {
#pragma unroll
                for (int w2 = 1; w2 < 4; ++w2)
                    if (argmax_better(sv[w2], si[w2], bv, bi)) {
                        bv = sv[w2];
                        bi = si[w2];
                    }
                p.amax_part[blockIdx.x] = ArgmaxPart{bv, bi};
                if (p.pos_adv && blockIdx.x == 0) p.pos_adv->pos += 1;
            }
        }
    }
    if (!writer) return;
#pragma unroll
    for (int mi = 0; mi < MR; ++mi) {
        if (mi >= Mb) break;
        const int m = m0 + mi;  // global row
        const float sc = p.norm ? __builtin_amdgcn_rsqf(ss[mi] / (float)p.K + p.eps) : 1.0f;
        if constexpr (EPI == EPI_QKV) {
            // columns 2u, 2u + 1: one RoPE pair (llama3.py:41-76; V rotates by cos 1, sin 0,
            // exact), then q / KV-cache append
            const int qdim = p.H * p.HD;
            const int col = 2 * unit;
            const float v0 = acc[0][mi] * sc, v1 = acc[ROWS - 1][mi] * sc;
            const float cs = pre0[mi], sn = pre1[mi];
            const float r0 = v0 * cs - v1 * sn, r1 = v0 * sn + v1 * cs;
            const int bidx = m / p.L, pos = start_of(p) + m - bidx * p.L;
            float2* dst = qkv_sec == 0
                              ? reinterpret_cast<float2*>(p.q_out + (int64_t)m * qdim + col)
                              : reinterpret_cast<float2*>((qkv_sec == 1 ? p.cache_k : p.cache_v) +
                                                          (((int64_t)bidx * p.KVH + qkv_head) * p.Smax + pos) * p.HD + qkv_d);
            if (p.kv_bak && qkv_sec > 0)  // [pos % KV_BAK_SLOTS][k, v][batch row][KV head][HD]
                *reinterpret_cast<float2*>(p.kv_bak + (((((int64_t)(pos % KV_BAK_SLOTS) * 2 + qkv_sec - 1) * (p.M / p.L) + bidx) *
                                                        p.KVH + qkv_head) * p.HD + qkv_d)) = bak_old[mi];
            L3_DCHECK(qkv_sec == 0 || (pos >= 0 && pos < p.Smax), CHK_KV_SLOT);
            *dst = qkv_sec == 0 ? float2{r0 * p.q_scale, r1 * p.q_scale} : float2{r0, r1};
        } else {
            float* dst = p.C + (int64_t)m * p.ldc + unit;
            if constexpr (EPI == EPI_SWIGLU) *dst = silu_f(acc[0][mi] * sc) * (acc[ROWS - 1][mi] * sc);
            else if constexpr (EPI == EPI_RESID) *dst = pre0[mi] + acc[0][mi];
            else *dst = acc[0][mi] * sc;
        }
    }
}

}  // namespace l3
