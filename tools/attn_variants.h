// Attention variants measured against the product kernel (attn_fwd_kernel) and rejected;
// kept for tools/attn_tune only (decisions table, round 2).  Not part of libllama3hip.
#pragma once
#include <type_traits>

#include "../llama3.np_amd/csrc/attn_kernel.h"

namespace l3 {

// ---------------------------------------------------------------------------------------
// v2: the same work split and K/V staging as attn_fwd_kernel, but the inner loop runs per
// 16-key group (kg) over all of a wave's live q-blocks at once:
//   S   : one K fragment read per (kg, d-group) feeds the score MFMAs of every live q-block —
//         NL independent accumulation chains interleaved (v1 re-read K per q-block and ran one
//         dependent 12-MFMA chain at a time: rocprofv3 SQ_WAIT_INST_ANY 0.56, MFMA busy 0.53)
//   soft: online softmax per kg (running max / sum per query, lane-local as in v1)
//   PV  : one V value per (kg, d-group, sub-step) feeds the PV MFMAs of every live q-block.
// A wave's q-blocks are held in descending order (blocks past L last), so for any key group
// the live blocks are a prefix of NL blocks: the step is instantiated per NL (wave-uniform
// switch), with the causal compare only on steps that touch a diagonal.
template <int HD, int QBW, int G, int KT, int WPE = 2>
__global__ void __launch_bounds__(256, WPE) attn_fwd_v2_kernel(AttnArgs p) {
    static_assert(HD % 16 == 0 && KT % 16 == 0 && (G == 1 || G == 2 || G == 4), "shape");
    constexpr int WPH = 4 / G;                // waves per head
    constexpr int NQB = QBW * WPH;            // 16-query blocks per head per workgroup
    constexpr int QW = 16 * NQB;              // queries per workgroup
    constexpr int ND = HD / 16;               // 16-wide d groups
    constexpr int KSTR = HD + 8;              // == 8 mod 16 floats: conflict-free ds_read_b128
    constexpr int VSTR = HD + 4;              // rows 4 apart on disjoint banks (ds_read_b32)
    constexpr int K_F4 = KT * HD / 4;
    constexpr int K_IT = (K_F4 + 255) / 256;
    constexpr int KG = KT / 16;

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

    const int start_pos = start_of(p);
    const int q_lo = qt * QW;
    const int q_hi = min(p.L, q_lo + QW);
    const int key_end = start_pos + q_hi;  // keys [0, key_end) are needed
    const int ntiles = (key_end + KT - 1) / KT;

    // this wave's q-blocks (zig-zag deal over the WPH waves of its head: ascending in j), held
    // descending with the blocks past L moved last -> live blocks of any key group = a prefix
    int blk[QBW];
    {
        int asc[QBW], nval = 0;
#pragma unroll
        for (int j = 0; j < QBW; ++j) {
            asc[j] = (j & 1) ? (2 * WPH * (j >> 1) + 2 * WPH - 1 - part) : (2 * WPH * (j >> 1) + part);
            nval += (q_lo + 16 * asc[j] < p.L) ? 1 : 0;
        }
        // descending valid blocks are asc[nval - 1 - i]; invalid ones follow
#pragma unroll
        for (int i = 0; i < QBW; ++i) {
            int v = asc[0];
#pragma unroll
            for (int j = 0; j < QBW; ++j)
                if (i < nval ? (j == nval - 1 - i) : (j == i)) v = asc[j];
            blk[i] = v;
        }
    }
    // causal extent of each block: last query (absolute) and first query; invalid: never live
    int qlast[QBW], qfirst[QBW];
#pragma unroll
    for (int i = 0; i < QBW; ++i) {
        const int q0 = q_lo + 16 * blk[i];
        const bool valid = q0 < p.L;
        qfirst[i] = start_pos + q0;
        qlast[i] = valid ? start_pos + min(q0 + 15, p.L - 1) : -1;
    }

    f32x4 qreg[QBW][ND];
    f32x4 o[QBW][ND];
    float m_run[QBW], l_run[QBW];
#pragma unroll
    for (int i = 0; i < QBW; ++i) {
        const int ql = q_lo + blk[i] * 16 + fq;
        const float* src = p.q + ((int64_t)b * p.L + ql) * qdim + h * HD + fk;
#pragma unroll
        for (int dg = 0; dg < ND; ++dg) {
            qreg[i][dg] = (ql < p.L) ? *reinterpret_cast<const f32x4*>(src + dg * 16)
                                     : f32x4{0.f, 0.f, 0.f, 0.f};
            o[i][dg] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
        m_run[i] = -INFINITY;
        l_run[i] = 0.f;
    }

    const int64_t kv_base = ((int64_t)b * p.KVH + kvh) * p.Smax;
    f32x4 rk[K_IT], rv[K_IT];
    auto gload = [&](int tile) {
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

    // one key group against the NL live blocks 0 .. NL-1
    auto kg_step = [&](const int cur, const int kg, const int kk, auto nl_tag, auto masked_tag) {
        constexpr int NL = decltype(nl_tag)::value;
        constexpr bool MASKED = decltype(masked_tag)::value;
        f32x4 s[NL];
#pragma unroll
        for (int i = 0; i < NL; ++i) s[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int dg = 0; dg < ND; ++dg) {
            const f32x4 kf = *reinterpret_cast<const f32x4*>(&Ks[cur][kg * 16 + fq][dg * 16 + fk]);
#pragma unroll
            for (int t = 0; t < 4; ++t)
#pragma unroll
                for (int i = 0; i < NL; ++i)
                    s[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(kf[t], qreg[i][dg][t], s[i], 0, 0, 0);
        }
        // lane holds keys 16 kk + fk + r for query qfirst[i] + fq
#pragma unroll
        for (int i = 0; i < NL; ++i) {
            float mt = -INFINITY;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float v = s[i][r];
                if constexpr (MASKED) v = (16 * kk + fk + r <= qfirst[i] + fq) ? v : -INFINITY;
                s[i][r] = v;
                mt = fmaxf(mt, v);
            }
            mt = max_xor16_32(mt);
            const float m_new = fmaxf(m_run[i], mt);
            const float alpha = __builtin_amdgcn_exp2f(m_run[i] - m_new);  // 0 on the first group
            m_run[i] = m_new;
            float psum = 0.f;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float pv = __builtin_amdgcn_exp2f(s[i][r] - m_new);
                s[i][r] = pv;
                psum += pv;
            }
            l_run[i] = l_run[i] * alpha + psum;
#pragma unroll
            for (int dg = 0; dg < ND; ++dg) o[i][dg] *= alpha;
        }
#pragma unroll
        for (int dg = 0; dg < ND; ++dg)
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const float vf = Vs[cur][kg * 16 + fk + t][dg * 16 + fq];
#pragma unroll
                for (int i = 0; i < NL; ++i)
                    o[i][dg] = __builtin_amdgcn_mfma_f32_16x16x4f32(vf, s[i][t], o[i][dg], 0, 0, 0);
            }
    };

    gload(0);
    sstore(0);
    __syncthreads();
    for (int tile = 0; tile < ntiles; ++tile) {
        const int cur = tile & 1;
        if (tile + 1 < ntiles) gload(tile + 1);
#pragma unroll
        for (int kg = 0; kg < KG; ++kg) {
            const int kk = tile * KG + kg;  // absolute 16-key group
            // live blocks: the prefix with 16 kk <= qlast (wave-uniform)
            int nl = 0;
#pragma unroll
            for (int i = 0; i < QBW; ++i) nl += (16 * kk <= qlast[i]) ? 1 : 0;
            if (nl == 0) continue;
            // unmasked only if every key of the group <= the first query of the last live block
            int qf_last = qfirst[0];
#pragma unroll
            for (int i = 1; i < QBW; ++i)
                if (i == nl - 1) qf_last = qfirst[i];
            const bool masked = 16 * kk + 15 > qf_last;
            using T = std::true_type;
            using F = std::false_type;
            if constexpr (QBW >= 4) {
                if (nl == 4) { if (masked) kg_step(cur, kg, kk, std::integral_constant<int, 4>{}, T{}); else kg_step(cur, kg, kk, std::integral_constant<int, 4>{}, F{}); continue; }
            }
            if constexpr (QBW >= 3) {
                if (nl == 3) { if (masked) kg_step(cur, kg, kk, std::integral_constant<int, 3>{}, T{}); else kg_step(cur, kg, kk, std::integral_constant<int, 3>{}, F{}); continue; }
            }
            if constexpr (QBW >= 2) {
                if (nl == 2) { if (masked) kg_step(cur, kg, kk, std::integral_constant<int, 2>{}, T{}); else kg_step(cur, kg, kk, std::integral_constant<int, 2>{}, F{}); continue; }
            }
            if (masked) kg_step(cur, kg, kk, std::integral_constant<int, 1>{}, T{});
            else kg_step(cur, kg, kk, std::integral_constant<int, 1>{}, F{});
        }
        if (tile + 1 < ntiles) sstore(cur ^ 1);
        __syncthreads();
    }

    // finalize: l = sum over the 4 lane groups; lane holds O^T[d = dg*16 + fk + r][q = fq]
#pragma unroll
    for (int i = 0; i < QBW; ++i) {
        float l = l_run[i];
        l = sum_xor16_32(l);
        const int ql = q_lo + blk[i] * 16 + fq;
        if (ql < p.L) {
            const float inv = 1.0f / l;
            float* dst = p.out + ((int64_t)b * p.L + ql) * qdim + h * HD + fk;
#pragma unroll
            for (int dg = 0; dg < ND; ++dg)
                *reinterpret_cast<f32x4*>(dst + dg * 16) = o[i][dg] * inv;
        }
    }
}

}  // namespace l3
