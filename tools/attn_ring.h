// Causal attention, HD = 48 (stories15M), K/V staged by LDS-DMA into an NS-slot ring.
// MEASURED AND REJECTED (tools/attn_tune ring): 76-78 TF/s against the
// product kernel's 81.6 on the same box; kept for the tuner only, not part of libllama3hip.
//
// Same math, work split and fragment maps as attn_fwd_kernel (attn_kernel.h: "q on the lane",
// online softmax, zig-zag q-blocks, masked body on the diagonal tile only) — replaces
// llama3.py:186-210 — with a different K/V pipeline:
//   * tiles are written to LDS by global_load_lds (1 KiB per wave-instruction, no staging
//     VGPRs); the image is lane-linear per piece, so conflict-free layouts are made on the
//     SOURCE side: K rows unpadded (48 floats) with float4 quad q stored at q ^ 3*((r>>3)&1),
//     which makes the 16-lane ds_read_b128 groups of the S fragment reads conflict-free; V rows
//     unpadded with a 16-float gap after every 4 rows, which puts the two 16-lane halves of a
//     ds_read_b32 P.V read (rows 4 apart) on disjoint banks (checked by enumeration against the
//     MI355X_MICROARCH.md lane groups) — 25 KiB per 64-key slot instead of 27.6 padded;
//   * NS = 2: the classic double buffer (DMA of tile t+1 issued at the top of tile t, retired
//     by the closing __syncthreads); NS = 3: tile t+2 in flight across the barrier (counted
//     vmcnt per wave + raw s_barrier), so a short tile at the causal end never waits on HBM.
// All LDS is one __shared__ array (a second object makes hipcc drain vmcnt before ds_reads).
#pragma once
#include <type_traits>

#include "../llama3.np_amd/csrc/kernels.h"

namespace l3 {

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int N>
__device__ __forceinline__ void attn_wait_vmcnt() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}

template <int QBW, int KT, int NS, int WPE>
__global__ void __launch_bounds__(256, WPE) attn_ring_kernel(AttnArgs p) {
    constexpr int HD = 48, ND = 3, NQB = QBW * 4, QW = 16 * NQB, KG = KT / 16;
    static_assert(KT % 16 == 0 && (NS == 2 || NS == 3), "shape");
    constexpr int KIMG = KT * HD;                        // floats, K image (unpadded, swizzled)
    constexpr int VIMG = KT * HD + (KT / 4) * 16;        // floats, V image (16-float gap per 4 rows)
    constexpr int KP = (KIMG + 255) / 256;               // 1 KiB pieces
    constexpr int VP = (VIMG + 255) / 256;
    constexpr int P = KP + VP;                           // pieces per tile
    constexpr int SLOT = (KP + VP) * 256;                // floats per slot
    constexpr int PW = (P + 3) / 4;                      // pieces per wave (max)
    constexpr int P_HI = (P + 3) / 4, P_LO = P / 4;      // waves < P % 4 issue P_HI

    __shared__ __attribute__((aligned(16))) float smem[NS * SLOT];

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int qt = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
    const int kvh = h / (p.H / p.KVH);
    const int qdim = p.H * HD;
    const int fq = lane & 15, fk = 4 * (lane >> 4);

    int qblk[QBW];
#pragma unroll
    for (int j = 0; j < QBW; ++j)
        qblk[j] = (j & 1) ? (8 * (j >> 1) + 7 - wid) : (8 * (j >> 1) + wid);

    const int start_pos = start_of(p);
    const int q_lo = qt * QW;
    const int q_hi = min(p.L, q_lo + QW);
    const int key_end = start_pos + q_hi;
    const int ntiles = (key_end + KT - 1) / KT;

    // ---- DMA pieces of this wave: piece = wid + 4 it; lane slot s = 64 * piece + lane (quads)
    const int64_t kv_base = ((int64_t)b * p.KVH + kvh) * p.Smax;
    int prow[PW], pq[PW];  // source key row within the tile and float4 quad of each piece slot
#pragma unroll
    for (int it = 0; it < PW; ++it) {
        const int piece = wid + 4 * it;
        int row = 0, q = 0;
        if (piece < KP) {
            const int s = piece * 64 + lane;  // K image quad
            row = min(s / 12, KT - 1);
            q = (s % 12) ^ (3 * ((row >> 3) & 1));
            if (s >= KT * 12) q = 0;          // past the image (last piece): dummy source
        } else {
            const int s = (piece - KP) * 64 + lane, g = s / 52, w = s % 52;
            row = min(4 * g + (w < 48 ? w / 12 : 0), KT - 1);
            q = w < 48 ? w % 12 : 0;          // gap slots: dummy source (the row's first quad)
        }
        prow[it] = row;
        pq[it] = q;
    }
    auto issue = [&](int tile) {
        float* slot = smem + (tile % NS) * SLOT;
#pragma unroll
        for (int it = 0; it < PW; ++it) {
            const int piece = wid + 4 * it;
            if (P % 4 == 0 || piece < P) {
                const int key = min(tile * KT + prow[it], p.Smax - 1);
                const float* src = (piece < KP ? p.cache_k : p.cache_v) + (kv_base + key) * HD + 4 * pq[it];
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                                 (__attribute__((address_space(3))) void*)(slot + piece * 256),
                                                 16, 0, 0);
            }
        }
    };

    issue(0);
    if (NS == 3 && ntiles > 1) issue(1);

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

    // K fragment of row r (= kg*16 + fq), quad q: swizzled address; V element (row, col)
    const int kswz = 3 * ((fq >> 3) & 1);
    auto kfrag = [&](const float* ks, int kg, int dg) -> f32x4 {
        const int row = kg * 16 + fq, q = (dg * 4 + (lane >> 4)) ^ kswz;
        return *reinterpret_cast<const f32x4*>(ks + row * HD + 4 * q);
    };
    auto vval = [&](const float* vs, int row, int col) -> float {
        return vs[row * HD + (row >> 2) * 16 + col];
    };

    const bool p_hi = P % 4 == 0 || wid < P % 4;
    for (int tile = 0; tile < ntiles; ++tile) {
        if constexpr (NS == 2) {
            if (tile == 0) __syncthreads();  // tile 0 landed (drains the DMA)
            if (tile + 1 < ntiles) issue(tile + 1);
        } else {
            // this wave's pieces of tile `tile` landed (those of tile + 1 may stay in flight),
            // then everyone's (barrier), and everyone is past tile - 1: its slot is refilled
            if (tile + 1 < ntiles) {
                if (p_hi) attn_wait_vmcnt<P_HI>();
                else attn_wait_vmcnt<P_LO>();
            } else {
                attn_wait_vmcnt<0>();
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            __builtin_amdgcn_sched_barrier(0);
            if (tile + 2 < ntiles) issue(tile + 2);
        }
        const float* ks = smem + (tile % NS) * SLOT;
        const float* vs = ks + KP * 256;
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
                        const f32x4 kf = kfrag(ks, kg, dg);
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
                        const float vf = vval(vs, kg * 16 + fk + s, dg * 16 + fq);
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
        if constexpr (NS == 2) __syncthreads();  // tile + 1 landed; everyone done with tile
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
