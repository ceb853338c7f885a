// "pair" attention variant (tools only, A/B against the product attn_fwd_kernel): one 8-wave
// workgroup runs TWO (batch, head) items (heads 2y and 2y + 1 of one batch row, n_rep = 1), waves
// 0-3 the first with the product's zig-zag q-block deal, waves 4-7 the second with the mirrored
// deal (wave 4 + u takes the q-blocks the product deal gives wave 3 - u).  Waves w and w + 4 land
// on the same SIMD (a workgroup's waves are dealt to the 4 SIMDs cyclically), so each SIMD
// carries the same causal work in every tile interval: at C3 (KT 64, 16 q-blocks) wave u's
// key groups per tile are 13+u / 12-u / 5+u / 4-u, and u + (3 - u) pairs give 29 / 21 / 13 / 5 on
// every SIMD, where the product's one-item workgroups leave 16 / 12 / 8 / 4 on the busiest wave.
// Same per-query arithmetic as the product kernel (same q-block order per item, same unit order):
// bit-identical output.
#pragma once
#include <type_traits>

#include "../llama3.np_amd/csrc/attn_kernel.h"

namespace l3 {

template <int HD, int QBW, int KT, bool MIRROR = true>
__global__ void __launch_bounds__(512, 2) attn_pair_kernel(AttnArgs p) {
    static_assert(HD % 16 == 0 && KT % 16 == 0, "shape");
    constexpr int WPH = 4;
    constexpr int NQB = QBW * WPH;
    constexpr int QW = 16 * NQB;
    constexpr int ND = HD / 16;
    constexpr int KSTR = HD + 8;
    constexpr int VSTR = HD + 4;
    constexpr int K_F4 = KT * HD / 4;
    constexpr int K_IT = (K_F4 + 255) / 256;
    constexpr int KG = KT / 16;

    __shared__ __attribute__((aligned(16))) float Ks[2][2][KT][KSTR];  // [item][buf]
    __shared__ __attribute__((aligned(16))) float Vs[2][2][KT][VSTR];

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int item = wid >> 2, u = wid & 3, itid = tid & 255;
    const int part = (MIRROR && item) ? 3 - u : u;
    const int qt = blockIdx.x, b = blockIdx.z;
    const int h = blockIdx.y * 2 + item;
    const int kvh = h;  // n_rep = 1
    const int qdim = p.H * HD;
    const int fq = lane & 15;
    const int fk = 4 * (lane >> 4);

    int qblk[QBW];
#pragma unroll
    for (int j = 0; j < QBW; ++j)
        qblk[j] = (j & 1) ? (2 * WPH * (j >> 1) + 2 * WPH - 1 - part) : (2 * WPH * (j >> 1) + part);

    const int start_pos = start_of(p);
    const int q_lo = p.q_first + qt * QW;
    const int q_hi = min(p.L, q_lo + QW);
    const int key_end = start_pos + q_hi;
    const int ntiles = (key_end + KT - 1) / KT;

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

    const int64_t kv_base = ((int64_t)b * p.KVH + kvh) * p.Smax;
    f32x4 rk[K_IT], rv[K_IT];
    auto gload = [&](int tile) {
#pragma unroll
        for (int i = 0; i < K_IT; ++i) {
            const int f = itid + 256 * i;
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
            const int f = itid + 256 * i;
            if (K_F4 % 256 == 0 || f < K_F4) {
                const int row = f / (HD / 4), c = (f % (HD / 4)) * 4;
                *reinterpret_cast<f32x4*>(&Ks[item][buf][row][c]) = rk[i];
                *reinterpret_cast<f32x4*>(&Vs[item][buf][row][c]) = rv[i];
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
        auto qblock_tile = [&](const int j, const int qblock_first, const int qmax_abs, auto masked_tag) {
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
                        const f32x4 kf = *reinterpret_cast<const f32x4*>(&Ks[item][cur][kg * 16 + fq][dg * 16 + fk]);
#pragma unroll
                        for (int s = 0; s < 4; ++s)
                            sacc[kg] = __builtin_amdgcn_mfma_f32_16x16x4f32(kf[s], qreg[j][dg][s], sacc[kg], 0, 0, 0);
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
            const float m_new = fmaxf(m_run[j], mt);
            const float alpha = __builtin_amdgcn_exp2f(m_run[j] - m_new);
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
                        const float vf = Vs[item][cur][kg * 16 + fk + s][dg * 16 + fq];
                        o[j][dg] = __builtin_amdgcn_mfma_f32_16x16x4f32(vf, sacc[kg][s], o[j][dg], 0, 0, 0);
                    }
            }
        };
#pragma unroll
        for (int j = 0; j < QBW; ++j) {
            const int qblock_first = q_lo + qblk[j] * 16;
            if (qblock_first >= p.L) continue;
            const int qmax_abs = start_pos + min(qblock_first + 15, p.L - 1);
            if (k0 > qmax_abs) continue;
            if (k0 + KT - 1 <= start_pos + qblock_first)
                qblock_tile(j, qblock_first, qmax_abs, std::integral_constant<bool, false>{});
            else
                qblock_tile(j, qblock_first, qmax_abs, std::integral_constant<bool, true>{});
        }
        if (tile + 1 < ntiles) sstore(cur ^ 1);
        __syncthreads();
        cur ^= 1;
    }

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

}  // namespace l3
