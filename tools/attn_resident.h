// Attention "resident" experiment (tools/attn_tune only until measured): a persistent grid, one
// 8-wave workgroup per CU, each walking (batch, head) items.  An item's whole K and V (keys
// [0, start_pos + L), L <= 256) sit in LDS at once, so the compute loop has no barrier at all
// (the product kernel barriers once per 64-key tile and every wave waits for the one with the
// most live key groups); the next item's K / V / q are loaded into registers while this one
// computes (no exposed prologue after the first item).  Waves own two 16-query blocks dealt
// zig-zag ({w, 15 - w}: 17 key groups each), walked one after the other.  G = 1 (n_rep = 1).
#pragma once
#include <type_traits>

#include "../llama3.np_amd/csrc/attn_kernel.h"

namespace l3 {

template <int HD, int KMAX, bool TILE_OUTER = false>
__global__ void __launch_bounds__(512, 2) attn_resident_kernel(AttnArgs p) {
    constexpr int NW = 8, NT = 64 * NW, QBW = 2, KT = 64, KG = KT / 16;
    constexpr int ND = HD / 16;
    constexpr int KSTR = HD + 8, VSTR = HD + 4;
    constexpr int HD4 = HD / 4;
    constexpr int KV_IT = (KMAX * HD4 + NT - 1) / NT;  // float4 per thread per matrix
    __shared__ __attribute__((aligned(16))) float Ks[KMAX][KSTR];
    __shared__ __attribute__((aligned(16))) float Vs[KMAX][VSTR];

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int fq = lane & 15, fk = 4 * (lane >> 4);
    const int qdim = p.H * HD;
    const int start_pos = start_of(p);
    const int key_end = start_pos + p.L;
    const int nf4 = key_end * HD4;
    const int nf4_pad = (key_end + KT - 1) / KT * KT * HD4;  // the last tile's rows past key_end: zeros
    const int nitems = p.B * p.H;
    const int qb[QBW] = {w, 2 * NW - 1 - w};

    f32x4 rk[KV_IT], rv[KV_IT], rq[QBW][ND];
    auto prefetch = [&](int item) {
        const int b = item / p.H, h = item - b * p.H;
        const int kvh = h / (p.H / p.KVH);
        const float* kb = p.cache_k + ((int64_t)b * p.KVH + kvh) * p.Smax * HD;
        const float* vb = p.cache_v + ((int64_t)b * p.KVH + kvh) * p.Smax * HD;
#pragma unroll
        for (int i = 0; i < KV_IT; ++i) {
            const int f = tid + NT * i;
            rk[i] = f < nf4 ? reinterpret_cast<const f32x4*>(kb)[f] : f32x4{0.f, 0.f, 0.f, 0.f};
            rv[i] = f < nf4 ? reinterpret_cast<const f32x4*>(vb)[f] : f32x4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int j = 0; j < QBW; ++j) {
            const int ql = qb[j] * 16 + fq;
            const float* src = p.q + ((int64_t)b * p.L + ql) * qdim + h * HD + fk;
#pragma unroll
            for (int dg = 0; dg < ND; ++dg)
                rq[j][dg] = ql < p.L ? *reinterpret_cast<const f32x4*>(src + dg * 16) : f32x4{0.f, 0.f, 0.f, 0.f};
        }
    };

    int item = blockIdx.x;
    if (item < nitems) prefetch(item);
    for (; item < nitems; item += gridDim.x) {
        const int b = item / p.H, h = item - b * p.H;
        __syncthreads();  // the previous item's LDS reads are done
#pragma unroll
        for (int i = 0; i < KV_IT; ++i) {
            const int f = tid + NT * i;
            if (f < nf4_pad) {
                const int row = f / HD4, c = (f - row * HD4) * 4;
                *reinterpret_cast<f32x4*>(&Ks[row][c]) = rk[i];
                *reinterpret_cast<f32x4*>(&Vs[row][c]) = rv[i];
            }
        }
        f32x4 qreg[QBW][ND];
#pragma unroll
        for (int j = 0; j < QBW; ++j)
#pragma unroll
            for (int dg = 0; dg < ND; ++dg) qreg[j][dg] = rq[j][dg];
        __syncthreads();
        if (item + (int)gridDim.x < nitems) prefetch(item + gridDim.x);

        f32x4 oo[QBW][ND];
        float mm[QBW], ll[QBW];
#pragma unroll
        for (int j = 0; j < QBW; ++j) {
            mm[j] = -INFINITY;
            ll[j] = 0.f;
#pragma unroll
            for (int dg = 0; dg < ND; ++dg) oo[j][dg] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
        // one (q-block, key tile) step of the online softmax
        auto step = [&](const int j, const int tile) {
            const int qblock_first = qb[j] * 16;
            const int qmax_abs = start_pos + min(qblock_first + 15, p.L - 1);
            const int q_abs = start_pos + qblock_first + fq;
            f32x4* o = oo[j];
            float& m_run = mm[j];
            float& l_run = ll[j];
            {
                const int k0 = tile * KT;
                auto body = [&](auto masked_tag) {
                    constexpr bool MASKED = decltype(masked_tag)::value;
                    f32x4 sacc[KG];
                    bool live[KG];
#pragma unroll
                    for (int kg = 0; kg < KG; ++kg) {
                        live[kg] = !MASKED || (k0 + kg * 16) <= qmax_abs;
                        sacc[kg] = f32x4{0.f, 0.f, 0.f, 0.f};
                        if (live[kg]) {
#pragma unroll
                            for (int dg = 0; dg < ND; ++dg) {
                                const f32x4 kf = *reinterpret_cast<const f32x4*>(&Ks[k0 + kg * 16 + fq][dg * 16 + fk]);
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
                    const float m_new = fmaxf(m_run, mt);
                    const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
                    m_run = m_new;
                    float psum = 0.f;
#pragma unroll
                    for (int kg = 0; kg < KG; ++kg)
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const float pv = __builtin_amdgcn_exp2f(sacc[kg][r] - m_new);
                            sacc[kg][r] = pv;
                            psum += pv;
                        }
                    l_run = l_run * alpha + psum;
#pragma unroll
                    for (int dg = 0; dg < ND; ++dg) o[dg] *= alpha;
#pragma unroll
                    for (int kg = 0; kg < KG; ++kg) {
                        if (!live[kg]) continue;
#pragma unroll
                        for (int dg = 0; dg < ND; ++dg)
#pragma unroll
                            for (int s = 0; s < 4; ++s) {
                                const float vf = Vs[k0 + kg * 16 + fk + s][dg * 16 + fq];
                                o[dg] = __builtin_amdgcn_mfma_f32_16x16x4f32(vf, sacc[kg][s], o[dg], 0, 0, 0);
                            }
                    }
                };
                if (k0 + KT - 1 <= start_pos + qblock_first) body(std::integral_constant<bool, false>{});
                else body(std::integral_constant<bool, true>{});
            }
        };
        auto ntiles_of = [&](int j) {
            const int qblock_first = qb[j] * 16;
            return qblock_first >= p.L ? 0 : (start_pos + min(qblock_first + 15, p.L - 1)) / KT + 1;
        };
        if constexpr (TILE_OUTER) {  // both q-blocks advance tile by tile (two independent chains)
            const int n0 = ntiles_of(0), n1 = ntiles_of(1), nmax = n0 > n1 ? n0 : n1;
            for (int tile = 0; tile < nmax; ++tile) {
                if (tile < n0) step(0, tile);
                if (tile < n1) step(1, tile);
            }
        } else {
            // staggered partners: waves 4-7 (the other wave on each SIMD) take their long q-block
            // first, so the two waves of a SIMD are not in the same phase
#pragma unroll
            for (int jj = 0; jj < QBW; ++jj) {
                const int j = w >= 4 ? QBW - 1 - jj : jj;
                const int n = ntiles_of(j);
                for (int tile = 0; tile < n; ++tile) step(j, tile);
            }
        }
#pragma unroll
        for (int j = 0; j < QBW; ++j) {
            const int ql = qb[j] * 16 + fq;
            const float l = sum_xor16_32(ll[j]);
            if (qb[j] * 16 < p.L && ql < p.L) {
                const float inv = 1.0f / l;
                float* dst = p.out + ((int64_t)b * p.L + ql) * qdim + h * HD + fk;
#pragma unroll
                for (int dg = 0; dg < ND; ++dg) *reinterpret_cast<f32x4*>(dst + dg * 16) = oo[j][dg] * inv;
            }
        }
    }
}

}  // namespace l3
