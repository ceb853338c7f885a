// Attention v3 experiments (tools/attn_tune only; not part of libllama3hip): the product
// kernel's structure (attn_fwd_kernel, G = 1) with three independent options:
//   NW      waves per workgroup (4: product; 8: 2 q-blocks per wave, 4 waves per SIMD at
//           <= 128 VGPRs with two workgroups per CU)
//   LAZY    lazy rescale (cdna_hip_programming.md T13): the running max a wave uses moves only
//           when some lane's tile max exceeds it by more than 8 (base-2 logits, so p <= 256):
//           skips the alpha exp2 and the O / l rescale on almost every tile after the first
//   SKIPD   on a q-block's diagonal tile, exp2 / sum only over the live 16-key groups
// Results are mathematically the product's; LAZY changes the rounding (reference max).
#pragma once
#include <type_traits>

#include "../llama3.np_amd/csrc/attn_kernel.h"

namespace l3 {

template <int HD, int NW, int QBW, int KT, bool LAZY, bool SKIPD, bool ILV = false, bool PIPE = false>
__global__ void __launch_bounds__(64 * NW, NW == 8 ? 4 : 2) attn_v3_kernel(AttnArgs p) {
    static_assert(HD % 16 == 0 && KT % 16 == 0 && (NW == 4 || NW == 8), "shape");
    constexpr int NT = 64 * NW;
    constexpr int NQB = QBW * NW;             // 16-query blocks per workgroup (one head)
    constexpr int QW = 16 * NQB;
    constexpr int ND = HD / 16;
    constexpr int KSTR = HD + 8;
    constexpr int VSTR = HD + 4;
    constexpr int K_F4 = KT * HD / 4;
    constexpr int K_IT = (K_F4 + NT - 1) / NT;
    constexpr int KG = KT / 16;

    __shared__ __attribute__((aligned(16))) float Ks[2][KT][KSTR];
    __shared__ __attribute__((aligned(16))) float Vs[2][KT][VSTR];

    const int tid = threadIdx.x, lane = tid & 63, part = tid >> 6;
    const int qt = blockIdx.x, b = blockIdx.z, h = blockIdx.y;
    const int kvh = h / (p.H / p.KVH);
    const int qdim = p.H * HD;
    const int fq = lane & 15, fk = 4 * (lane >> 4);

    int qblk[QBW];
#pragma unroll
    for (int j = 0; j < QBW; ++j)
        qblk[j] = (j & 1) ? (2 * NW * (j >> 1) + 2 * NW - 1 - part) : (2 * NW * (j >> 1) + part);

    const int start_pos = start_of(p);
    const int q_lo = qt * QW;
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
            qreg[j][dg] = (ql < p.L) ? *reinterpret_cast<const f32x4*>(src + dg * 16) : f32x4{0.f, 0.f, 0.f, 0.f};
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
            const int f = tid + NT * i;
            const int row = f / (HD / 4), c = (f % (HD / 4)) * 4;
            const int key = tile * KT + row;
            f32x4 vk = {0.f, 0.f, 0.f, 0.f}, vv = vk;
            if ((K_F4 % NT == 0 || f < K_F4) && key < p.Smax) {
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
            const int f = tid + NT * i;
            if (K_F4 % NT == 0 || f < K_F4) {
                const int row = f / (HD / 4), c = (f % (HD / 4)) * 4;
                *reinterpret_cast<f32x4*>(&Ks[buf][row][c]) = rk[i];
                *reinterpret_cast<f32x4*>(&Vs[buf][row][c]) = rv[i];
            }
        }
    };

    gload(0);
    sstore(0);
    __syncthreads();
    for (int tile = 0; tile < ntiles; ++tile) {
        const int cur = tile & 1;
        if (tile + 1 < ntiles) gload(tile + 1);
        const int k0 = tile * KT;
        auto qblock_tile = [&](const int j, const int qblock_first, const int qmax_abs, auto masked_tag) {
            constexpr bool MASKED = decltype(masked_tag)::value;
            const int q_abs = start_pos + qblock_first + fq;
            f32x4 sacc[KG];
            bool live[KG];
            if constexpr (ILV && !MASKED) {
                // all key groups live: the KG accumulation chains interleaved (one MFMA of each
                // chain in turn), the d-group's KG fragments read together
#pragma unroll
                for (int kg = 0; kg < KG; ++kg) {
                    live[kg] = true;
                    sacc[kg] = f32x4{0.f, 0.f, 0.f, 0.f};
                }
                if constexpr (PIPE) {
                    // fragments of d-group dg + 1 read while d-group dg's 16 MFMAs issue; the
                    // order pinned by scheduling groups (DS read x KG, then MFMA x 16)
                    f32x4 kf[2][KG];
#pragma unroll
                    for (int kg = 0; kg < KG; ++kg)
                        kf[0][kg] = *reinterpret_cast<const f32x4*>(&Ks[cur][kg * 16 + fq][fk]);
#pragma unroll
                    for (int dg = 0; dg < ND; ++dg) {
                        if (dg + 1 < ND) {
#pragma unroll
                            for (int kg = 0; kg < KG; ++kg)
                                kf[(dg + 1) & 1][kg] = *reinterpret_cast<const f32x4*>(&Ks[cur][kg * 16 + fq][(dg + 1) * 16 + fk]);
                        }
#pragma unroll
                        for (int s = 0; s < 4; ++s)
#pragma unroll
                            for (int kg = 0; kg < KG; ++kg)
                                sacc[kg] = __builtin_amdgcn_mfma_f32_16x16x4f32(kf[dg & 1][kg][s], qreg[j][dg][s], sacc[kg], 0, 0, 0);
                    }
                    __builtin_amdgcn_sched_group_barrier(0x100, KG, 0);
                    __builtin_amdgcn_sched_group_barrier(0x100, KG, 0);
                    __builtin_amdgcn_sched_group_barrier(0x008, 4 * KG, 0);
                    __builtin_amdgcn_sched_group_barrier(0x100, KG, 0);
                    __builtin_amdgcn_sched_group_barrier(0x008, 4 * KG, 0);
                    __builtin_amdgcn_sched_group_barrier(0x008, 4 * KG, 0);
                } else {
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
                }
            } else {
#pragma unroll
            for (int kg = 0; kg < KG; ++kg) {
                live[kg] = !MASKED || (k0 + kg * 16) <= qmax_abs;
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
            }
            float mt = -INFINITY;
#pragma unroll
            for (int kg = 0; kg < KG; ++kg) {
                if (SKIPD && MASKED && !live[kg]) continue;
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
            }
            mt = max_xor16_32(mt);
            float m_use;
            if constexpr (LAZY) {
                // move the reference max only when some lane's tile max exceeds it by > 8
                // (p <= 2^8): the wave-uniform branch skips the rescale on almost every tile
                const bool move = mt > m_run[j] + 8.0f;
                if (__builtin_amdgcn_ballot_w64(move)) {
                    const float m_new = fmaxf(m_run[j], mt);
                    const float alpha = __builtin_amdgcn_exp2f(m_run[j] - m_new);
                    m_run[j] = m_new;
                    l_run[j] *= alpha;
#pragma unroll
                    for (int dg = 0; dg < ND; ++dg) o[j][dg] *= alpha;
                }
                m_use = m_run[j];
            } else {
                const float m_new = fmaxf(m_run[j], mt);
                const float alpha = __builtin_amdgcn_exp2f(m_run[j] - m_new);
                m_run[j] = m_new;
                l_run[j] *= alpha;
#pragma unroll
                for (int dg = 0; dg < ND; ++dg) o[j][dg] *= alpha;
                m_use = m_new;
            }
            float psum = 0.f;
#pragma unroll
            for (int kg = 0; kg < KG; ++kg) {
                if (SKIPD && MASKED && !live[kg]) continue;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float pv = __builtin_amdgcn_exp2f(sacc[kg][r] - m_use);
                    sacc[kg][r] = pv;
                    psum += pv;
                }
            }
            l_run[j] += psum;
            if constexpr (PIPE && !MASKED) {
                // V values of key group kg + 1 read while kg's 12 MFMAs issue
                float vv[2][ND][4];
#pragma unroll
                for (int dg = 0; dg < ND; ++dg)
#pragma unroll
                    for (int s2 = 0; s2 < 4; ++s2) vv[0][dg][s2] = Vs[cur][fk + s2][dg * 16 + fq];
#pragma unroll
                for (int kg = 0; kg < KG; ++kg) {
                    if (kg + 1 < KG) {
#pragma unroll
                        for (int dg = 0; dg < ND; ++dg)
#pragma unroll
                            for (int s2 = 0; s2 < 4; ++s2)
                                vv[(kg + 1) & 1][dg][s2] = Vs[cur][(kg + 1) * 16 + fk + s2][dg * 16 + fq];
                    }
#pragma unroll
                    for (int s2 = 0; s2 < 4; ++s2)
#pragma unroll
                        for (int dg = 0; dg < ND; ++dg)
                            o[j][dg] = __builtin_amdgcn_mfma_f32_16x16x4f32(vv[kg & 1][dg][s2], sacc[kg][s2], o[j][dg], 0, 0, 0);
                }
            } else {
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
    }
#pragma unroll
    for (int j = 0; j < QBW; ++j) {
        float l = sum_xor16_32(l_run[j]);
        const int ql = q_lo + qblk[j] * 16 + fq;
        if (ql < p.L) {
            const float inv = 1.0f / l;
            float* dst = p.out + ((int64_t)b * p.L + ql) * qdim + h * HD + fk;
#pragma unroll
            for (int dg = 0; dg < ND; ++dg) *reinterpret_cast<f32x4*>(dst + dg * 16) = o[j][dg] * inv;
        }
    }
}

}  // namespace l3
