// Fused causal attention for gfx950, fp32 MFMA (v_mfma_f32_16x16x4_f32), online softmax.
//
// Replaces llama3.py:186-210 — cache read (:186-187), repeat_kv (:190-191, here an index map
// h -> h / n_rep), scores q.k^T/sqrt(HD) (:200-202), causal mask (:204-205, built at :293-297),
// softmax (:206, :22-24), P.V (:207) and the head merge (:210).  The [B,H,L,S] score tensor
// is never materialised.
//
// Orientation ("q on the lane"): every tile is computed transposed so that the query index
// sits on lane&15 in all accumulators:
//   S^T[key][q] = sum_d K[key][d] * Q[q][d]      (A = K tile from LDS, B = Q from registers)
//   O^T[d][q]  += sum_key V[key][d] * P[q][key]  (A = V tile from LDS, B = P straight from the
//                                                 S^T accumulator: lane l holds
//                                                 P[q = l&15][key = 4(l>>4)+r], which is the
//                                                 B operand of sub-step s = r under the
//                                                 K-permutation trick, see gemm_kernel.h)
// so the running max / sum and the O rescale are lane-local, and the row max needs only two
// cross-lane steps (xor 16, xor 32).  q is pre-scaled by log2(e)/sqrt(HD) in the QKV epilogue,
// so p = exp2(s - m).
//
// Work split: a workgroup (4 waves) owns one (batch, KV head) pair's group of G query heads
// (G = gcd(n_rep, 4): the heads that read the same K/V, so every staged K/V tile serves G heads)
// and a range of queries.  Wave w works for head g = w % G; the 4/G waves of one head share its
// 16-query blocks, dealt zig-zag (w, 7-w, 8+w, 15-w for 4 waves) so causal work is balanced.
// K/V tiles of KT keys are staged through double-buffered LDS (K rows padded to HD+8 floats:
// conflict-free ds_read_b128).  Tiles / 16-key groups past a block's last query are skipped;
// only a q-block's diagonal tile runs the masked body (per-group liveness + causal compare),
// every other tile a branch-free one (C3 attention +3.8 %, bit-identical results).
#pragma once
#include <type_traits>

#include "kernels.h"

namespace l3 {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// Timing-study variants of this kernel (ablation bits, the rejected DEFER schedule) live in
// tools/attn_research.h, outside the product library.
// PK (round 6, the product's launches; tools/attn_tune pk A/Bs it): the unmasked body's score chains interleaved over the
// key groups (a d-group's four K fragments read together, one MFMA of each chain in turn) and
// the softmax's subtract / sum on packed pairs (v_pk_add_f32: half the VALU ops of that pass);
// the row sum then adds even and odd columns separately, so results differ in the last bits
template <int HD, int QBW, int G, int KT, bool PK = false>
__global__ void __launch_bounds__(256, 2) attn_fwd_kernel(AttnArgs p) {
    static_assert(HD % 16 == 0 && KT % 16 == 0 && (G == 1 || G == 2 || G == 4), "shape");
    constexpr int WPH = 4 / G;                // waves per head
    constexpr int NQB = QBW * WPH;            // 16-query blocks per head per workgroup
    constexpr int QW = 16 * NQB;              // queries per workgroup
    constexpr int ND = HD / 16;               // 16-wide d groups
    constexpr int KSTR = HD + 8;              // padded: == 8 mod 16 floats
    // P.V reads V[key = kg*16 + 4(lane>>4) + s][d = dg*16 + (lane&15)] with ds_read_b32: lanes
    // 0-15 and 16-31 (one bank group) are 4 rows apart, so 4*VSTR must be == 16 (mod 32):
    // VSTR == 4 (mod 8) puts the two 16-lane halves on disjoint banks (HD is a multiple of 16)
    constexpr int VSTR = HD + 4;
    constexpr int K_F4 = KT * HD / 4;
    constexpr int K_IT = (K_F4 + 255) / 256;
    constexpr int KG = KT / 16;               // 16-key groups per tile

    __shared__ __attribute__((aligned(16))) float Ks[2][KT][KSTR];
    __shared__ __attribute__((aligned(16))) float Vs[2][KT][VSTR];

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int g = wid % G, part = wid / G;
    const int qt = blockIdx.x, b = blockIdx.z;
    const int h = blockIdx.y * G + g;
    const int kvh = (blockIdx.y * G) / (p.H / p.KVH);
    const int qdim = p.H * HD;
    const int fq = lane & 15;       // query within a 16-block
    const int fk = 4 * (lane >> 4); // k offset of this lane's operand quad

    // this wave's q blocks (zig-zag over the WPH waves of its head)
    int qblk[QBW];
#pragma unroll
    for (int j = 0; j < QBW; ++j)
        qblk[j] = (j & 1) ? (2 * WPH * (j >> 1) + 2 * WPH - 1 - part) : (2 * WPH * (j >> 1) + part);

    const int start_pos = start_of(p);
    const int q_lo = p.q_first + qt * QW;
    const int q_hi = min(p.L, q_lo + QW);
    const int key_end = start_pos + q_hi;  // keys [0, key_end) are needed
    const int ntiles = (key_end + KT - 1) / KT;
    if (threadIdx.x == 0) L3_DCHECK(start_pos >= 0 && start_pos + p.L <= p.Smax, CHK_ATTN_KEYS);

    // Loads are unpredicated, from clamped (in-bounds) rows: a query lane past L computes on a
    // copy of row L - 1 and is never stored (each lane's softmax state is its own query's), and
    // a key past Smax is past key_end, so every valid query masks it.  Predicated loads compiled
    // to exec-masked branches whose register copies waited for every load in flight (an
    // s_waitcnt vmcnt(0) after the second q load of the prologue).
    f32x4 qreg[QBW][ND];
    f32x4 o[QBW][ND];
    float m_run[QBW], l_run[QBW];
#pragma unroll
    for (int j = 0; j < QBW; ++j) {
        const int ql = min(q_lo + qblk[j] * 16 + fq, p.L - 1);
        const float* src = p.q + ((int64_t)b * p.L + ql) * qdim + h * HD + fk;
#pragma unroll
        for (int dg = 0; dg < ND; ++dg) {
            qreg[j][dg] = *reinterpret_cast<const f32x4*>(src + dg * 16);
            o[j][dg] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
        m_run[j] = -INFINITY;
        l_run[j] = 0.f;
    }

    const int64_t kv_base = ((int64_t)b * p.KVH + kvh) * p.Smax;
    f32x4 rk[K_IT], rv[K_IT];
    auto gload = [&](int tile) {
#pragma unroll
        for (int i = 0; i < K_IT; ++i) {
            const int f = tid + 256 * i;
            const int row = f / (HD / 4), c = (f % (HD / 4)) * 4;
            const int key = min(tile * KT + row, p.Smax - 1);
            if (K_F4 % 256 == 0 || f < K_F4) {
                rk[i] = *reinterpret_cast<const f32x4*>(p.cache_k + (kv_base + key) * HD + c);
                rv[i] = *reinterpret_cast<const f32x4*>(p.cache_v + (kv_base + key) * HD + c);
            }
        }
    };
    auto sstore = [&](int buf) {
#pragma unroll
        for (int i = 0; i < K_IT; ++i) {
            const int f = tid + 256 * i;
            if (K_F4 % 256 == 0 || f < K_F4) {
                const int row = f / (HD / 4), c = (f % (HD / 4)) * 4;
                *reinterpret_cast<f32x4*>(&Ks[buf][row][c]) = rk[i];
                *reinterpret_cast<f32x4*>(&Vs[buf][row][c]) = rv[i];
            }
        }
    };

    gload(0);
    sstore(0);
    __syncthreads();
    int cur = 0;
    for (int tile = 0; tile < ntiles; ++tile) {
        if (tile + 1 < ntiles) gload(tile + 1);
        const int k0 = tile * KT;
        // one q-block against this K/V tile; MASKED: the diagonal tile (some key of the tile
        // is past some query of the block: per-16-key-group liveness + causal mask).  The
        // unmasked body has no wave-uniform branches, so hipcc can interleave the four key
        // groups' S chains and hoist the V reads
        auto qblock_tile = [&](const int j, const int qblock_first, const int qmax_abs, auto masked_tag) {
            constexpr bool MASKED = decltype(masked_tag)::value;
            const int q_abs = start_pos + qblock_first + fq;
            f32x4 sacc[KG];
            bool live[KG];
#pragma unroll
            for (int kg = 0; kg < KG; ++kg) {
                live[kg] = !MASKED || (k0 + kg * 16) <= qmax_abs;     // wave-uniform
                sacc[kg] = f32x4{0.f, 0.f, 0.f, 0.f};
            }
            if constexpr (PK && !MASKED) {  // KG independent chains, one MFMA of each in turn
#pragma unroll
                for (int dg = 0; dg < ND; ++dg) {
                    f32x4 kf[KG];
#pragma unroll
                    for (int kg = 0; kg < KG; ++kg)
                        kf[kg] = *reinterpret_cast<const f32x4*>(&Ks[cur][kg * 16 + fq][dg * 16 + fk]);
#pragma unroll
                    for (int s = 0; s < 4; ++s)
#pragma unroll
                        for (int kg = 0; kg < KG; ++kg)
                            sacc[kg] = __builtin_amdgcn_mfma_f32_16x16x4f32(kf[kg][s], qreg[j][dg][s], sacc[kg], 0, 0, 0);
                }
            } else {
#pragma unroll
                for (int kg = 0; kg < KG; ++kg) {
                    if (live[kg]) {
#pragma unroll
                        for (int dg = 0; dg < ND; ++dg) {
                            const f32x4 kf = *reinterpret_cast<const f32x4*>(&Ks[cur][kg * 16 + fq][dg * 16 + fk]);
#pragma unroll
                            for (int s = 0; s < 4; ++s)
                                sacc[kg] = __builtin_amdgcn_mfma_f32_16x16x4f32(kf[s], qreg[j][dg][s], sacc[kg], 0, 0, 0);
                        }
                    }
                }
            }
            // causal mask + tile max; lane holds keys k0 + kg*16 + fk + r for query q_abs
            float mt = -INFINITY;
#pragma unroll
            for (int kg = 0; kg < KG; ++kg)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    float v = sacc[kg][r];
                    if constexpr (MASKED) {
                        const int key = k0 + kg * 16 + fk + r;
                        v = (live[kg] && key <= q_abs) ? v : -INFINITY;
                    }
                    sacc[kg][r] = v;
                    mt = fmaxf(mt, v);
                }
            mt = max_xor16_32(mt);
            const float m_new = fmaxf(m_run[j], mt);
            // v_exp_f32 directly: arguments are <= 0 (exact 0 at -inf), so the libm
            // denormal-range guard around exp2f is dead weight (5 VALU per call)
            const float alpha = __builtin_amdgcn_exp2f(m_run[j] - m_new);  // 0 on the first tile
            m_run[j] = m_new;
            float psum = 0.f;
            if constexpr (PK) {
                typedef float f32x2 __attribute__((ext_vector_type(2)));
                const f32x2 mm = {m_new, m_new};
                f32x2 ps = {0.f, 0.f};
#pragma unroll
                for (int kg = 0; kg < KG; ++kg)
#pragma unroll
                    for (int r = 0; r < 4; r += 2) {
                        const f32x2 x = f32x2{sacc[kg][r], sacc[kg][r + 1]} - mm;
                        const f32x2 e = {__builtin_amdgcn_exp2f(x.x), __builtin_amdgcn_exp2f(x.y)};
                        sacc[kg][r] = e.x;
                        sacc[kg][r + 1] = e.y;
                        ps += e;
                    }
                psum = ps.x + ps.y;
            } else {
#pragma unroll
                for (int kg = 0; kg < KG; ++kg)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float pv = __builtin_amdgcn_exp2f(sacc[kg][r] - m_new);
                        sacc[kg][r] = pv;
                        psum += pv;
                    }
            }
            l_run[j] = l_run[j] * alpha + psum;
#pragma unroll
            for (int dg = 0; dg < ND; ++dg) o[j][dg] *= alpha;
#pragma unroll
            for (int kg = 0; kg < KG; ++kg) {
                if (!live[kg]) continue;
#pragma unroll
                for (int dg = 0; dg < ND; ++dg)
#pragma unroll
                    for (int s = 0; s < 4; ++s) {
                        const float vf = Vs[cur][kg * 16 + fk + s][dg * 16 + fq];
                        o[j][dg] = __builtin_amdgcn_mfma_f32_16x16x4f32(vf, sacc[kg][s], o[j][dg], 0, 0, 0);
                    }
            }
            // unmasked body: the P.V phase hand-ordered — each V read (ds_read_b32) two MFMAs
            // ahead of its use (round 4, tools/attn_tune sched: C3 117.8-119.8 -> 116.4-116.5 us,
            // bit-identical; the same for the score phase measured null)
            if constexpr (!MASKED) {
                __builtin_amdgcn_sched_group_barrier(0x100, 2, 1);  // DS read
#pragma unroll
                for (int i = 0; i < KG * ND * 4 - 2; ++i) {
                    __builtin_amdgcn_sched_group_barrier(0x100, 1, 1);
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);  // MFMA
                }
                __builtin_amdgcn_sched_group_barrier(0x008, 2, 1);
            }
        };
#pragma unroll
        for (int j = 0; j < QBW; ++j) {
            const int qblock_first = q_lo + qblk[j] * 16;
            if (qblock_first >= p.L) continue;                        // padding block
            const int qmax_abs = start_pos + min(qblock_first + 15, p.L - 1);
            if (k0 > qmax_abs) continue;                              // whole tile masked
            // every key of the tile <= every query of the block: no mask, all groups live
            if (k0 + KT - 1 <= start_pos + qblock_first)
                qblock_tile(j, qblock_first, qmax_abs, std::integral_constant<bool, false>{});
            else
                qblock_tile(j, qblock_first, qmax_abs, std::integral_constant<bool, true>{});
        }
        if (tile + 1 < ntiles) sstore(cur ^ 1);
        __syncthreads();
        cur ^= 1;
    }

    // finalize: l = sum over the 4 lane groups; lane holds O^T[d = dg*16 + fk + r][q = fq]
#pragma unroll
    for (int j = 0; j < QBW; ++j) {
        float l = l_run[j];
        l = sum_xor16_32(l);
        const int ql = q_lo + qblk[j] * 16 + fq;
        if (ql < p.L) {
            const float inv = 1.0f / l;
            float* dst = p.out + ((int64_t)b * p.L + ql) * qdim + h * HD + fk;
#pragma unroll
            for (int dg = 0; dg < ND; ++dg)
                *reinterpret_cast<f32x4*>(dst + dg * 16) = o[j][dg] * inv;
        }
    }
}

// ---------------------------------------------------------------------------------------
// Decode attention (L = 1: one query per (batch, head) at position pos attends keys [0, pos],
// no mask, llama3.py:186-210 with the cache slice :186-187).  A workgroup owns one (b, h);
// the work is three short memory-bound passes, so the kernel is built around round trips, not
// MFMA: (1) scores, one key per thread (its HD/4 float4 loads in flight together), kept in
// LDS; (2) block max and exp2 / sum; (3) P.V with rg = tid / (HD/4) key groups x HD/4 float4
// columns, the first VP rows of each thread's V prefetched at kernel entry so their latency
// hides under passes 1-2; partial O reduced through LDS.  q is pre-scaled by log2(e)/sqrt(HD).
//
// FUSE_O (decode, small D): the launch also does this head's share of the O-proj (llama3.py:211)
// — blockIdx.z picks 64 of the D output rows, 4 lanes per row each holding a quarter of the
// row's HD-wide Wo slice (fetched at kernel entry, beside the V prefetch) — and writes
// parts[b][h][row] = Wo[row, h*HD:(h+1)*HD] . out[b][h].  The z blocks of one (b, h) recompute
// the same attention (its K/V reads are small at these sizes) instead of handing it on: the
// partial rows go to the next kernels, which add them in head order (GemmArgs::parts), so no
// cross-block hand-off (and no agent-scope fence) is needed inside this launch.
template <int HD, bool FUSE_O = false>
__global__ void __launch_bounds__(256) attn_decode_kernel(AttnArgs p) {
    constexpr int D4 = HD / 4, R = 256 / D4, VP = 8;
    constexpr int WQ = HD / 16;  // FUSE_O: float4 of the Wo row slice per lane
    extern __shared__ __attribute__((aligned(16))) float dsm[];  // [R][HD] partials, [Smax] scores
    float* red = dsm;
    float* sc = dsm + R * HD;
    __shared__ float wred[8];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int h = blockIdx.x, b = blockIdx.y;
    const int kvh = h / (p.H / p.KVH);
    const int pos = start_of(p);
    const int S = pos + 1;
    if (tid == 0) L3_DCHECK(pos >= 0 && S <= p.Smax, CHK_ATTN_KEYS);
    const int64_t kv_base = ((int64_t)b * p.KVH + kvh) * p.Smax * HD;
    const f32x4* K4 = reinterpret_cast<const f32x4*>(p.cache_k + kv_base);
    const f32x4* V4 = reinterpret_cast<const f32x4*>(p.cache_v + kv_base);
    const int rg = tid / D4, d4 = tid - rg * D4;
    // the entry loads are unpredicated, from clamped (in-bounds) rows — a V row past S or an
    // O-proj row past D is loaded but never used; predicated loads compiled to exec-masked
    // branches whose register copies waited for every load in flight (one round trip more)
    f32x4 vpre[VP];
#pragma unroll
    for (int t = 0; t < VP; ++t) vpre[t] = V4[(int64_t)min(rg + t * R, S - 1) * D4 + d4];
    const int orow = blockIdx.z * 64 + (tid >> 2), opart = tid & 3;
    f32x4 wpre[FUSE_O ? WQ : 1];
    if constexpr (FUSE_O) {
        const f32x4* w4 = reinterpret_cast<const f32x4*>(p.wo + (int64_t)min(orow, p.D - 1) * (p.H * HD) + h * HD) + opart * WQ;
#pragma unroll
        for (int i = 0; i < WQ; ++i) wpre[i] = w4[i];
    }
    const f32x4* q4 = reinterpret_cast<const f32x4*>(p.q + ((int64_t)b * p.H + h) * HD);
    f32x4 q[D4];
#pragma unroll
    for (int i = 0; i < D4; ++i) q[i] = q4[i];

    // (1) scores
    float m = -INFINITY;
    for (int k = tid; k < S; k += 256) {
        f32x4 kv[D4];
#pragma unroll
        for (int i = 0; i < D4; ++i) kv[i] = K4[(int64_t)k * D4 + i];
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < D4; ++i) s += kv[i].x * q[i].x + kv[i].y * q[i].y + kv[i].z * q[i].z + kv[i].w * q[i].w;
        sc[k] = s;
        m = fmaxf(m, s);
    }
    m = group_max<64>(m);
    if (lane == 0) wred[wid] = m;
    __syncthreads();
    m = fmaxf(fmaxf(wred[0], wred[1]), fmaxf(wred[2], wred[3]));
    // (2) p = exp2(s - max), row sum
    float l = 0.f;
    for (int k = tid; k < S; k += 256) {
        const float e = __builtin_amdgcn_exp2f(sc[k] - m);
        sc[k] = e;
        l += e;
    }
    l = group_sum<64>(l);
    if (lane == 0) wred[4 + wid] = l;
    __syncthreads();  // p complete in LDS; row sum in wred[4..7]
    l = (wred[4] + wred[5]) + (wred[6] + wred[7]);
    // (3) P.V
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    if (rg < R) {
#pragma unroll
        for (int t = 0; t < VP; ++t) {
            const int k = rg + t * R;
            acc += (k < S ? sc[min(k, S - 1)] : 0.f) * vpre[t];
        }
        for (int k = rg + VP * R; k < S; k += R) acc += sc[k] * V4[(int64_t)k * D4 + d4];
        reinterpret_cast<f32x4*>(red)[rg * D4 + d4] = acc;
    }
    __syncthreads();
    __shared__ f32x4 oh[D4];
    if (tid < D4) {
        f32x4 o = {0.f, 0.f, 0.f, 0.f};
        for (int r = 0; r < R; ++r) o += reinterpret_cast<const f32x4*>(red)[r * D4 + tid];
        if constexpr (FUSE_O) oh[tid] = o * (1.0f / l);
        else reinterpret_cast<f32x4*>(p.out + ((int64_t)b * p.H + h) * HD)[tid] = o * (1.0f / l);
    }
    if constexpr (FUSE_O) {
        __syncthreads();
        float acc = 0.f;
#pragma unroll
        for (int i = 0; i < WQ; ++i) {
            const f32x4 ov = oh[opart * WQ + i];
            acc += wpre[i].x * ov.x + wpre[i].y * ov.y + wpre[i].z * ov.z + wpre[i].w * ov.w;
        }
        acc += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(acc), 0xB1, 0xF, 0xF, false));
        acc += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(acc), 0x4E, 0xF, 0xF, false));
        if (opart == 0 && orow < p.D) p.parts[((int64_t)b * p.H + h) * p.D + orow] = acc;
    }
}

}  // namespace l3
