// Multi-item attention grids (tools only; measured and rejected, DESIGN.md decisions table):
// the product attn_fwd_kernel (llama3.np_amd/csrc/attn_kernel.h) with its items — (q tile, head
// group, batch row) — flattened onto a 1-D grid of at most 2 workgroups per CU, each walking
// several items with the next item's first K / V tile (and, QEARLY, its q) fetched during the
// current item's last tile.  Bit-identical output.  C3: 126.7 -> 125.5 us (null), half batch
// 68.2 -> 79.5 us, C4 916 -> 931 us (profiles/r03_attn_persist.log).
#pragma once
#include <type_traits>

#include "../llama3.np_amd/csrc/kernels.h"

namespace l3 {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// QEARLY (multi-item grids): the next item's q loads are issued before this item's last K / V
// barrier instead of after it (+17 VGPRs at C3, tools/attn_tune persist)
template <int HD, int QBW, int G, int KT, bool QEARLY = false>
__global__ void __launch_bounds__(256, 2) attn_persist_kernel(AttnArgs p) {
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
    const int qdim = p.H * HD;
    const int fq = lane & 15;       // query within a 16-block
    const int fk = 4 * (lane >> 4); // k offset of this lane's operand quad

    // this wave's q blocks (zig-zag over the WPH waves of its head)
    int qblk[QBW];
#pragma unroll
    for (int j = 0; j < QBW; ++j)
        qblk[j] = (j & 1) ? (2 * WPH * (j >> 1) + 2 * WPH - 1 - part) : (2 * WPH * (j >> 1) + part);

    const int start_pos = start_of(p);
    // items (q tile, head group, batch row), q tile fastest: item i runs on block i % gridDim.x,
    // so a grid of fewer blocks than items walks several items per block (see launch_attn_persist)
    const int nqt = (p.L - p.q_first + QW - 1) / QW, ngy = p.H / G;
    const int nitems = nqt * ngy * p.B;
    struct Item {
        int q_lo, q_hi, ntiles, h, b;
        int64_t kv_base;
    };
    auto item_at = [&](int it) {
        Item r;
        const int qt = it % nqt, rest = it / nqt, hy = rest % ngy;
        r.b = rest / ngy;
        r.h = hy * G + g;
        r.q_lo = p.q_first + qt * QW;
        r.q_hi = min(p.L, r.q_lo + QW);
        r.ntiles = (start_pos + r.q_hi + KT - 1) / KT;  // keys [0, start_pos + q_hi) are needed
        r.kv_base = ((int64_t)r.b * p.KVH + (hy * G) / (p.H / p.KVH)) * p.Smax;
        return r;
    };
    int item = blockIdx.x;
    if (item >= nitems) return;  // whole workgroup
    Item cur_it = item_at(item);

    f32x4 qreg[QBW][ND];
    f32x4 o[QBW][ND];
    float m_run[QBW], l_run[QBW];
    auto load_q = [&](const Item& it) {
#pragma unroll
        for (int j = 0; j < QBW; ++j) {
            const int ql = it.q_lo + qblk[j] * 16 + fq;
            const float* src = p.q + ((int64_t)it.b * p.L + ql) * qdim + it.h * HD + fk;
#pragma unroll
            for (int dg = 0; dg < ND; ++dg)
                qreg[j][dg] = (ql < p.L) ? *reinterpret_cast<const f32x4*>(src + dg * 16)
                                         : f32x4{0.f, 0.f, 0.f, 0.f};
        }
    };
    auto reset = [&]() {
#pragma unroll
        for (int j = 0; j < QBW; ++j) {
#pragma unroll
            for (int dg = 0; dg < ND; ++dg) o[j][dg] = f32x4{0.f, 0.f, 0.f, 0.f};
            m_run[j] = -INFINITY;
            l_run[j] = 0.f;
        }
    };
    // l = sum over the 4 lane groups; lane holds O^T[d = dg*16 + fk + r][q = fq]
    auto finish = [&](const Item& it) {
#pragma unroll
        for (int j = 0; j < QBW; ++j) {
            const float l = sum_xor16_32(l_run[j]);
            const int ql = it.q_lo + qblk[j] * 16 + fq;
            if (ql < p.L) {
                const float inv = 1.0f / l;
                float* dst = p.out + ((int64_t)it.b * p.L + ql) * qdim + it.h * HD + fk;
#pragma unroll
                for (int dg = 0; dg < ND; ++dg)
                    *reinterpret_cast<f32x4*>(dst + dg * 16) = o[j][dg] * inv;
            }
        }
    };
    load_q(cur_it);
    reset();

    f32x4 rk[K_IT], rv[K_IT];
    auto gload = [&](int64_t kv_base, int tile) {
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
            rk[i] = vk;
            rv[i] = vv;
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

    gload(cur_it.kv_base, 0);
    sstore(0);
    __syncthreads();
    int cur = 0;
    // one (item, tile) pipeline: the next tile's K / V — the next item's first tile after an
    // item's last — is in flight while this one computes, and the next item's q loads are
    // issued before this item's output stores, so only a block's first item pays the prologue
    while (true) {
        const int next = item + (int)gridDim.x;
        const bool more = next < nitems;
        const int q_lo = cur_it.q_lo, ntiles = cur_it.ntiles;
        for (int tile = 0; tile < ntiles; ++tile) {
            const bool last = tile + 1 == ntiles;
            if (!last) gload(cur_it.kv_base, tile + 1);
            else if (more) gload(item_at(next).kv_base, 0);
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
    #pragma unroll
                for (int kg = 0; kg < KG; ++kg)
    #pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float pv = __builtin_amdgcn_exp2f(sacc[kg][r] - m_new);
                        sacc[kg][r] = pv;
                        psum += pv;
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
            if constexpr (QEARLY) {
                if (last) {
                    if (more) load_q(item_at(next));  // q is dead once the last tile has run
                    finish(cur_it);
                    if (!more) return;
                    reset();
                }
            }
            if (!last || more) sstore(cur ^ 1);
            __syncthreads();
            cur ^= 1;
        }
        if constexpr (!QEARLY) {
            finish(cur_it);
            if (!more) return;
            load_q(item_at(next));
            reset();
        }
        item = next;
        cur_it = item_at(next);
    }
}

// Grid of attn_persist_kernel: one block per item, or — for launches of more items than two
// workgroups per CU hold at once (every item one whole sequence, so all items cost the same)
// — blocks that walk ceil(items / (2 CUs)) items each: the K / V and q fetches of a block's
// next item overlap its current item (C3: a workgroup's prologue was 14 % of its life,
// profiles/r03_attn_stamps.txt).  cap: the blocks resident at once (0: one per item).
template <int HD, int QBW, int G, int KT, bool QEARLY = false>
inline hipError_t launch_attn_persist(const AttnArgs& a, hipStream_t s, int cap) {
    constexpr int QW = 16 * QBW * (4 / G);
    const int nqt = (a.L - a.q_first + QW - 1) / QW;
    const int items = nqt * (a.H / G) * a.B;
    int grid = items;
    if (cap > 0 && nqt == 1 && items > cap) {
        const int per = (items + cap - 1) / cap;
        grid = (items + per - 1) / per;
    }
    hipLaunchKernelGGL((attn_persist_kernel<HD, QBW, G, KT, QEARLY>), dim3(grid), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace l3
