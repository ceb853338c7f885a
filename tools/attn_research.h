// Research copy of the round-2 prefill attention kernel (tools only, never linked into the
// product library): the product attn_fwd_kernel (llama3.np_amd/csrc/attn_kernel.h) without the
// timing-study ablation bits (ABL) and the rejected DEFER schedule, kept here so tools/attn_tune
// can still time them (DESIGN.md decisions table; profiles/r02_attn_ablations.log,
// r02_attn_defer*.log).
#pragma once
#include <type_traits>

#include "../llama3.np_amd/csrc/attn_kernel.h"

namespace l3 {

// ABL & 512 (timing study, results correct): per-wave s_memtime stamps to g_attn_stamps,
// 16 uint64 per wave: [0] entry, [1] after the prologue barrier, [2 + 2t] tile t's compute
// done, [3 + 2t] after tile t's barrier (t < 4), [10] exit, [11] HW_REG_HW_ID, [12] XCC_ID
__device__ unsigned long long* g_attn_stamps;

// ABL & 2048 / 4096: hand-ordered score / P.V phases of the unmasked body (sched_group_barrier;
// verdict round 3 item 4).
// ABL: ablation bits for tools/attn_tune timing studies only (product launches use 0; results
// are wrong with any bit set): 1 every tile full and unmasked for every block (no causal
// structure), 2 p = s (no exp), 4 no K/V loads after tile 0, 8 no barrier in the tile loop,
// 16 no softmax bookkeeping (no max / rescale / sum); 32 (timing study, results correct): K/V
// tiles prefetched two ahead through two register sets; 64 / 128 / 256 (timing study, results
// correct): s_setprio(1) around both MFMA clusters / the score cluster / the P.V cluster;
// 1024 (timing study, results correct): K/V tile 0 before q, raw prologue barrier
//
// DEFER (HD 48): three K/V slots instead of two, and the diagonal (masked) units of the even
// q-block slots j (C3: the even tiles' diagonal units) run one barrier interval later, first
// thing after the next tile's barrier (the tile is still in its slot then; the store of tile
// t+1 goes to the slot of t-2).
// A q-block's units still run in tile order, so the output is bit-identical.  Why: with the
// zig-zag deal the busiest wave carries 16 / 12 / 8 / 4 key groups between the four barriers of
// C3 against 34 of work per wave (the diagonal unit of q-block 4t+r costs r+1 groups, and the
// wave holding r = 3 alternates); deferring the even tiles' diagonal units pairs r with 3 - r,
// so every wave carries 12 / 13 / 4 / 5.  The third slot fits beside a second workgroup per CU
// only with an unpadded K image: rows of 48 floats, float4 quad q of row r stored at
// q ^ 3*((r>>3)&1), which keeps the 16-lane ds_read_b128 groups of the score reads on 16
// distinct bank quads (25 KB per slot, 75 KB in all).
template <int HD, int QBW, int G, int KT, int ABL = 0, bool DEFER = false>
__global__ void __launch_bounds__(256, 2) attn_research_kernel(AttnArgs p) {
    static_assert(HD % 16 == 0 && KT % 16 == 0 && (G == 1 || G == 2 || G == 4), "shape");
    static_assert(!DEFER || (HD == 48 && (ABL & 32) == 0), "DEFER: the swizzled K image is laid out for HD 48");
    constexpr int NS = DEFER ? 3 : 2;         // K/V slots
    constexpr int WPH = 4 / G;                // waves per head
    constexpr int NQB = QBW * WPH;            // 16-query blocks per head per workgroup
    constexpr int QW = 16 * NQB;              // queries per workgroup
    constexpr int ND = HD / 16;               // 16-wide d groups
    constexpr int KSTR = DEFER ? HD : HD + 8; // padded: == 8 mod 16 floats; DEFER: swizzled
    // P.V reads V[key = kg*16 + 4(lane>>4) + s][d = dg*16 + (lane&15)] with ds_read_b32: lanes
    // 0-15 and 16-31 (one bank group) are 4 rows apart, so 4*VSTR must be == 16 (mod 32):
    // VSTR == 4 (mod 8) puts the two 16-lane halves on disjoint banks (HD is a multiple of 16)
    constexpr int VSTR = HD + 4;
    constexpr int K_F4 = KT * HD / 4;
    constexpr int K_IT = (K_F4 + 255) / 256;
    constexpr int KG = KT / 16;               // 16-key groups per tile

    __shared__ __attribute__((aligned(16))) float Ks[NS][KT][KSTR];
    __shared__ __attribute__((aligned(16))) float Vs[NS][KT][VSTR];

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    unsigned long long* stp = nullptr;
    if constexpr ((ABL & 512) != 0)
        stp = g_attn_stamps + ((((size_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) * 4 + wid) * 16;
    auto stamp = [&](int i) {
        if constexpr ((ABL & 512) != 0) {
            const unsigned long long t = __builtin_amdgcn_s_memtime();
            if (lane == 0) stp[i] = t;
        }
    };
    stamp(0);
    const int g = wid % G, part = wid / G;
    const int qt = blockIdx.x, b = blockIdx.z;
    const int h = blockIdx.y * G + g;
    const int kvh = (blockIdx.y * G) / (p.H / p.KVH);
    const int qdim = p.H * HD;
    const int fq = lane & 15;       // query within a 16-block
    const int fk = 4 * (lane >> 4); // k offset of this lane's operand quad
    // column of this lane's K fragment quad within a 16-wide d group (DEFER: swizzled image;
    // the row's bit 3 is fq's, so the swizzle is a per-lane constant)
    const int fkx = DEFER ? 4 * ((lane >> 4) ^ (3 * ((fq >> 3) & 1))) : fk;

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

    const int64_t kv_base = ((int64_t)b * p.KVH + kvh) * p.Smax;
    f32x4 rk[K_IT], rv[K_IT];
    f32x4 rk2[(ABL & 32) ? K_IT : 1], rv2[(ABL & 32) ? K_IT : 1];
    auto gload_into = [&](int tile, f32x4* dk, f32x4* dv) {
#pragma unroll
        for (int i = 0; i < K_IT; ++i) {
            const int f = tid + 256 * i;
            const int row = f / (HD / 4), c = (f % (HD / 4)) * 4;
            const int key = tile * KT + row;
            f32x4 vk = {0.f, 0.f, 0.f, 0.f}, vv = vk;
            if ((K_F4 % 256 == 0 || f < K_F4) && key < p.Smax) {
                vk = *reinterpret_cast<const f32x4*>(p.cache_k + (kv_base + key) * HD + c);
                vv = *reinterpret_cast<const f32x4*>(p.cache_v + (kv_base + key) * HD + c);
            }
            dk[i] = vk;
            dv[i] = vv;
        }
    };
    auto sstore_from = [&](int buf, const f32x4* sk, const f32x4* sv) {
#pragma unroll
        for (int i = 0; i < K_IT; ++i) {
            const int f = tid + 256 * i;
            if (K_F4 % 256 == 0 || f < K_F4) {
                const int row = f / (HD / 4), c = (f % (HD / 4)) * 4;
                const int ck = DEFER ? (c ^ (12 * ((row >> 3) & 1))) : c;  // quad ^ 3 on rows 8-15 of 16
                *reinterpret_cast<f32x4*>(&Ks[buf][row][ck]) = sk[i];
                *reinterpret_cast<f32x4*>(&Vs[buf][row][c]) = sv[i];
            }
        }
    };
    auto gload = [&](int tile) { gload_into(tile, rk, rv); };
    auto sstore = [&](int buf) { sstore_from(buf, rk, rv); };
    // ABL & 1024 (timing study, results correct): K/V tile 0 is fetched before q, and the
    // prologue barrier waits only for its LDS stores, so the q loads land during tile 0
    if constexpr ((ABL & 1024) != 0) gload(0);
    f32x4 qreg[QBW][ND];
    f32x4 o[QBW][ND];
    float m_run[QBW], l_run[QBW];
#pragma unroll
    for (int j = 0; j < QBW; ++j) {
        const int ql = q_lo + qblk[j] * 16 + fq;
        const float* src = p.q + ((int64_t)b * p.L + ql) * qdim + h * HD + fk;
#pragma unroll
        for (int dg = 0; dg < ND; ++dg) {
            qreg[j][dg] = (ql < p.L) ? *reinterpret_cast<const f32x4*>(src + dg * 16)
                                     : f32x4{0.f, 0.f, 0.f, 0.f};
            o[j][dg] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
        m_run[j] = -INFINITY;
        l_run[j] = 0.f;
    }


    if constexpr ((ABL & 1024) == 0) gload(0);
    sstore(0);
    if constexpr ((ABL & 32) != 0) {
        if (ntiles > 1) gload(1);  // set A holds tile 1
    }
    if constexpr ((ABL & 1024) != 0) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
    } else {
        __syncthreads();
    }
    stamp(1);
    int cur = 0;  // slot of this tile (tile % NS)
    for (int tile = 0; tile < ntiles; ++tile) {
        const int nxt = (cur + 1 == NS) ? 0 : cur + 1;
        if constexpr ((ABL & 32) != 0) {  // tile + 2 into the set that held tile (its store is done)
            if (tile + 2 < ntiles) {
                if (tile & 1) gload_into(tile + 2, rk, rv);
                else gload_into(tile + 2, rk2, rv2);
            }
        } else if (!(ABL & 4) && tile + 1 < ntiles) {
            gload(tile + 1);
        }
        const int k0 = tile * KT;
        {
            // one q-block against this K/V tile; MASKED: the diagonal tile (some key of the tile
            // is past some query of the block: per-16-key-group liveness + causal mask).  The
            // unmasked body has no wave-uniform branches, so hipcc can interleave the four
            // key groups' S chains and hoist the V reads
            auto qblock_tile = [&](const int j, const int qblock_first, const int qmax_abs,
                                   const int cur, const int k0, auto masked_tag) {
                constexpr bool MASKED = decltype(masked_tag)::value;
                const int q_abs = start_pos + qblock_first + fq;
                f32x4 sacc[KG];
                bool live[KG];
                if constexpr ((ABL & (64 | 128)) != 0) __builtin_amdgcn_s_setprio(1);
#pragma unroll
                for (int kg = 0; kg < KG; ++kg) {
                    live[kg] = !MASKED || (k0 + kg * 16) <= qmax_abs;     // wave-uniform
                    sacc[kg] = f32x4{0.f, 0.f, 0.f, 0.f};
                    if (live[kg]) {
#pragma unroll
                        for (int dg = 0; dg < ND; ++dg) {
                            const f32x4 kf = *reinterpret_cast<const f32x4*>(&Ks[cur][kg * 16 + fq][dg * 16 + fkx]);
#pragma unroll
                            for (int s = 0; s < 4; ++s)
                                sacc[kg] = __builtin_amdgcn_mfma_f32_16x16x4f32(kf[s], qreg[j][dg][s], sacc[kg], 0, 0, 0);
                        }
                    }
                }
                if constexpr ((ABL & (64 | 128)) != 0) __builtin_amdgcn_s_setprio(0);
                // ABL & 2048 (unmasked body): the score phase hand-ordered — K fragment reads
                // (ds_read_b128) two fragments ahead of their 4 MFMAs, the phase fenced off
                if constexpr ((ABL & 2048) != 0 && !MASKED) {
                    __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);  // DS reads, two fragments ahead
#pragma unroll
                    for (int i = 0; i < KG * ND - 2; ++i) {
                        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);  // MFMA
                        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
                    }
                    __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
                    __builtin_amdgcn_sched_barrier(0);
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
                if constexpr (!(ABL & 16)) {
                mt = max_xor16_32(mt);
                const float m_new = fmaxf(m_run[j], mt);
                // v_exp_f32 directly: arguments are <= 0 (exact 0 at -inf), so the libm
                // denormal-range guard around exp2f is dead weight (5 VALU per call)
                const float alpha = __builtin_amdgcn_exp2f(m_run[j] - m_new);  // 0 on the first tile
                m_run[j] = m_new;
                float psum = 0.f;
#pragma unroll
                for (int kg = 0; kg < KG; ++kg)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float pv = (ABL & 2) ? sacc[kg][r] - m_new
                                                   : __builtin_amdgcn_exp2f(sacc[kg][r] - m_new);
                        sacc[kg][r] = pv;
                        psum += pv;
                    }
                l_run[j] = l_run[j] * alpha + psum;
#pragma unroll
                for (int dg = 0; dg < ND; ++dg) o[j][dg] *= alpha;
                }
                if constexpr ((ABL & (64 | 256)) != 0) __builtin_amdgcn_s_setprio(1);
                if constexpr ((ABL & 4096) != 0 && !MASKED) __builtin_amdgcn_sched_barrier(0);
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
                // ABL & 4096 (unmasked body): the P.V phase hand-ordered — V reads (ds_read_b32) two
                // MFMAs ahead: 2 reads, then (1 read, 1 MFMA) pairs, then the last 2 MFMAs
                if constexpr ((ABL & 4096) != 0 && !MASKED) {
                    __builtin_amdgcn_sched_group_barrier(0x100, 2, 1);
#pragma unroll
                    for (int i = 0; i < KG * ND * 4 - 2; ++i) {
                        __builtin_amdgcn_sched_group_barrier(0x100, 1, 1);
                        __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
                    }
                    __builtin_amdgcn_sched_group_barrier(0x008, 2, 1);
                }
                if constexpr ((ABL & (64 | 256)) != 0) __builtin_amdgcn_s_setprio(0);
            };
            if constexpr (DEFER) {
                if (tile > 0) {  // the even q-block slots' diagonal units of tile - 1, deferred
                    const int pk0 = k0 - KT, prv = (cur == 0) ? NS - 1 : cur - 1;
#pragma unroll
                    for (int j = 0; j < QBW; j += 2) {
                        const int qblock_first = q_lo + qblk[j] * 16;
                        if (qblock_first >= p.L) continue;
                        const int qmax_abs = start_pos + min(qblock_first + 15, p.L - 1);
                        if (pk0 > qmax_abs || pk0 + KT - 1 <= start_pos + qblock_first) continue;
                        qblock_tile(j, qblock_first, qmax_abs, prv, pk0, std::integral_constant<bool, true>{});
                    }
                }
            }
            // DEFER: the diagonal units of the even q-block slots j wait for the next interval
            // (never the last tile's).  With the zig-zag deal at start_pos 0 and one workgroup per
            // 256 queries (C3), slot j's diagonal tile is tile j, so this defers the even tiles'
            // diagonal units; any other shape stays correct, only the balance differs
            const bool defer_even = DEFER && tile + 1 < ntiles;
#pragma unroll
            for (int j = 0; j < QBW; ++j) {
                const int qblock_first = q_lo + qblk[j] * 16;
                if (qblock_first >= p.L) continue;                        // padding block
                const int qmax_abs = start_pos + min(qblock_first + 15, p.L - 1);
                if (!(ABL & 1) && k0 > qmax_abs) continue;                // whole tile masked
                // every key of the tile <= every query of the block: no mask, all groups live
                if ((ABL & 1) || k0 + KT - 1 <= start_pos + qblock_first)
                    qblock_tile(j, qblock_first, qmax_abs, cur, k0, std::integral_constant<bool, false>{});
                else if (!(defer_even && (j & 1) == 0))
                    qblock_tile(j, qblock_first, qmax_abs, cur, k0, std::integral_constant<bool, true>{});
            }
        }
        if (tile < 4) stamp(2 + 2 * tile);
        if constexpr ((ABL & 32) != 0) {
            if (tile + 1 < ntiles) {
                if (tile & 1) sstore_from(nxt, rk2, rv2);
                else sstore_from(nxt, rk, rv);
            }
        } else if (!(ABL & 4) && tile + 1 < ntiles) {
            sstore(nxt);
        }
        if constexpr (!(ABL & 8)) __syncthreads();
        if (tile < 4) stamp(3 + 2 * tile);
        cur = nxt;
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
    stamp(10);
    if constexpr ((ABL & 512) != 0) {
        if (lane == 0) {
            stp[11] = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_REG_HW_ID
            stp[12] = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
        }
    }
}

}  // namespace l3
