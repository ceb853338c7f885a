// "rev" attention variant (tools only, A/B against the product attn_fwd_kernel): one 8-wave
// workgroup runs TWO (batch, head) items (heads 2y and 2y + 1 of one batch row, n_rep = 1) and
// walks the second one's K/V tiles in REVERSE order (online softmax takes keys in any order).
// Every wave owns the same two zig-zag q-blocks {w, 15 - w} of both items.  With 64-key tiles a
// q-block's live key groups per tile fall with the tile index, so item 0's work in interval t
// plus item 1's in interval (T - 1 - t) is nearly constant: at C3 every wave carries 8 or 9
// (q-block, 16-key group) units in every interval (busiest 36 over the four, against 34 of
// work), where the product's one-item workgroups put 16 / 12 / 8 / 4 on the busiest wave (40
// against 34).  Item 1's sums run in another key order: equal to the product within fp32
// rounding, not bit for bit.
#pragma once
#include <type_traits>

#include "../llama3.np_amd/csrc/attn_kernel.h"

namespace l3 {

template <int HD, int KT>
__global__ void __launch_bounds__(512, 2) attn_rev_kernel(AttnArgs p) {
    static_assert(HD % 16 == 0 && KT % 16 == 0, "shape");
    constexpr int NT = 512, QBI = 2, QW = 256;
    constexpr int ND = HD / 16;
    constexpr int KSTR = HD + 8;
    constexpr int VSTR = HD + 4;
    constexpr int K_F4 = KT * HD / 4;                 // float4 per item per tile
    constexpr int K_IT = (2 * K_F4 + NT - 1) / NT;
    constexpr int KG = KT / 16;

    __shared__ __attribute__((aligned(16))) float Ks[2][2][KT][KSTR];  // [item][buf]
    __shared__ __attribute__((aligned(16))) float Vs[2][2][KT][VSTR];

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int b = blockIdx.z;
    const int qdim = p.H * HD;
    const int fq = lane & 15;
    const int fk = 4 * (lane >> 4);
    const int qblk[QBI] = {wid, 15 - wid};

    const int start_pos = start_of(p);
    const int q_lo = p.q_first + blockIdx.x * QW;
    const int q_hi = min(p.L, q_lo + QW);
    const int key_end = start_pos + q_hi;
    const int ntiles = (key_end + KT - 1) / KT;

    f32x4 qreg[2][QBI][ND];
    f32x4 o[2][QBI][ND];
    float m_run[2][QBI], l_run[2][QBI];
#pragma unroll
    for (int it = 0; it < 2; ++it) {
        const int h = blockIdx.y * 2 + it;
#pragma unroll
        for (int j = 0; j < QBI; ++j) {
            const int ql = q_lo + qblk[j] * 16 + fq;
            const float* src = p.q + ((int64_t)b * p.L + ql) * qdim + h * HD + fk;
#pragma unroll
            for (int dg = 0; dg < ND; ++dg) {
                qreg[it][j][dg] = (ql < p.L) ? *reinterpret_cast<const f32x4*>(src + dg * 16)
                                             : f32x4{0.f, 0.f, 0.f, 0.f};
                o[it][j][dg] = f32x4{0.f, 0.f, 0.f, 0.f};
            }
            m_run[it][j] = -INFINITY;
            l_run[it][j] = 0.f;
        }
    }

    const int64_t kv_base0 = ((int64_t)b * p.KVH + blockIdx.y * 2) * p.Smax;
    f32x4 rk[K_IT], rv[K_IT];
    auto tile_of = [&](int item, int t) { return item ? ntiles - 1 - t : t; };
    auto gload = [&](int t) {
#pragma unroll
        for (int i = 0; i < K_IT; ++i) {
            const int f = tid + NT * i, item = f / K_F4, ff = f - item * K_F4;
            const int row = ff / (HD / 4), c = (ff % (HD / 4)) * 4;
            const int key = tile_of(item, t) * KT + row;
            f32x4 vk = {0.f, 0.f, 0.f, 0.f}, vv = vk;
            if (((2 * K_F4) % NT == 0 || f < 2 * K_F4) && key < p.Smax) {
                const int64_t off = (kv_base0 + (int64_t)item * p.Smax + key) * HD + c;
                vk = *reinterpret_cast<const f32x4*>(p.cache_k + off);
                vv = *reinterpret_cast<const f32x4*>(p.cache_v + off);
            }
            rk[i] = vk;
            rv[i] = vv;
        }
    };
    auto sstore = [&](int buf) {
#pragma unroll
        for (int i = 0; i < K_IT; ++i) {
            const int f = tid + NT * i, item = f / K_F4, ff = f - item * K_F4;
            if ((2 * K_F4) % NT == 0 || f < 2 * K_F4) {
                const int row = ff / (HD / 4), c = (ff % (HD / 4)) * 4;
                *reinterpret_cast<f32x4*>(&Ks[item][buf][row][c]) = rk[i];
                *reinterpret_cast<f32x4*>(&Vs[item][buf][row][c]) = rv[i];
            }
        }
    };

    gload(0);
    sstore(0);
    __syncthreads();
    int cur = 0;
    for (int t = 0; t < ntiles; ++t) {
        if (t + 1 < ntiles) gload(t + 1);
        auto qblock_tile = [&](const int it, const int j, const int k0, const int qblock_first,
                               const int qmax_abs, auto masked_tag) {
            constexpr bool MASKED = decltype(masked_tag)::value;
            const int q_abs = start_pos + qblock_first + fq;
            f32x4 sacc[KG];
            bool live[KG];
#pragma unroll
            for (int kg = 0; kg < KG; ++kg) {
                live[kg] = !MASKED || (k0 + kg * 16) <= qmax_abs;
                sacc[kg] = f32x4{0.f, 0.f, 0.f, 0.f};
                if (live[kg]) {
#pragma unroll
                    for (int dg = 0; dg < ND; ++dg) {
                        const f32x4 kf = *reinterpret_cast<const f32x4*>(&Ks[it][cur][kg * 16 + fq][dg * 16 + fk]);
#pragma unroll
                        for (int s = 0; s < 4; ++s)
                            sacc[kg] = __builtin_amdgcn_mfma_f32_16x16x4f32(kf[s], qreg[it][j][dg][s], sacc[kg], 0, 0, 0);
                    }
                }
            }
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
            const float m_new = fmaxf(m_run[it][j], mt);
            const float alpha = __builtin_amdgcn_exp2f(m_run[it][j] - m_new);
            m_run[it][j] = m_new;
            float psum = 0.f;
#pragma unroll
            for (int kg = 0; kg < KG; ++kg)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float pv = __builtin_amdgcn_exp2f(sacc[kg][r] - m_new);
                    sacc[kg][r] = pv;
                    psum += pv;
                }
            l_run[it][j] = l_run[it][j] * alpha + psum;
#pragma unroll
            for (int dg = 0; dg < ND; ++dg) o[it][j][dg] *= alpha;
#pragma unroll
            for (int kg = 0; kg < KG; ++kg) {
                if (!live[kg]) continue;
#pragma unroll
                for (int dg = 0; dg < ND; ++dg)
#pragma unroll
                    for (int s = 0; s < 4; ++s) {
                        const float vf = Vs[it][cur][kg * 16 + fk + s][dg * 16 + fq];
                        o[it][j][dg] = __builtin_amdgcn_mfma_f32_16x16x4f32(vf, sacc[kg][s], o[it][j][dg], 0, 0, 0);
                    }
            }
        };
#pragma unroll
        for (int it = 0; it < 2; ++it) {
            const int k0 = tile_of(it, t) * KT;
#pragma unroll
            for (int j = 0; j < QBI; ++j) {
                const int qblock_first = q_lo + qblk[j] * 16;
                if (qblock_first >= p.L) continue;
                const int qmax_abs = start_pos + min(qblock_first + 15, p.L - 1);
                if (k0 > qmax_abs) continue;
                if (k0 + KT - 1 <= start_pos + qblock_first)
                    qblock_tile(it, j, k0, qblock_first, qmax_abs, std::integral_constant<bool, false>{});
                else
                    qblock_tile(it, j, k0, qblock_first, qmax_abs, std::integral_constant<bool, true>{});
            }
        }
        if (t + 1 < ntiles) sstore(cur ^ 1);
        __syncthreads();
        cur ^= 1;
    }

#pragma unroll
    for (int it = 0; it < 2; ++it) {
        const int h = blockIdx.y * 2 + it;
#pragma unroll
        for (int j = 0; j < QBI; ++j) {
            float l = l_run[it][j];
            l = sum_xor16_32(l);
            const int ql = q_lo + qblk[j] * 16 + fq;
            if (ql < p.L) {
                const float inv = 1.0f / l;
                float* dst = p.out + ((int64_t)b * p.L + ql) * qdim + h * HD + fk;
#pragma unroll
                for (int dg = 0; dg < ND; ++dg)
                    *reinterpret_cast<f32x4*>(dst + dg * 16) = o[it][j][dg] * inv;
            }
        }
    }
}

}  // namespace l3
