// RESEARCH RECORD — not built into libllama3hip.so (round 5, measured and rejected; DESIGN.md
// decisions table, profiles/r05_pbatch_ab.txt, profiles/r05_pbatch_stamps_*.txt).  It was compiled
// from llama3.np_amd/csrc with the runtime hooks of commit history (capture_steps' batched path);
// kept as the record of the design and its per-stage timeline.
//
// Persistent batched greedy decode step (llama3.py:316-320 at B = 9..256 rows, L = 1): every
// layer of one step — RMSNorm + QKV + RoPE + KV append, attention, O-proj + residual, RMSNorm +
// gate|up + SwiGLU, down + residual — as ONE launch; the lm_head (its per-row argmax partials,
// GemmArgs::amax_rows) and the B-row argmax stay two launches after it.  Three launches per step
// instead of 32.
//
// Why: a batched step is ~30 dependent launches of 4-8 us each, every one latency-bound (the
// whole step moves 344 MB and 7.8 GFLOP at B = 256: a 49 us floor, against 0.30 ms measured,
// profiles/r05_batched_decode_b256_eager_kernel_stats.csv).  Batch rows never interact
// (llama3.py:163-211), so every stage depends only on the same rows' previous stage: the rows
// are split into groups of 16 (one MFMA tile of rows), each group's stages run on its own GW
// workgroups, and a stage's hand-off is all-to-all only within the group.  Each workgroup
// requests its next stage's weight fragments before waiting for that stage's input, so they
// land while the hand-off is in flight (the batch-1 persistent step's lesson, decode_persist.hip).
//
// Hand-offs: 8-byte {tag, value} granules, one agent-scope relaxed atomic store each (sc1
// write-through) and agent-scope loads re-read until every tag equals the launch's epoch
// (cdna_hip_programming.md Guideline 16, R2); per (layer, stage) slab, the epoch bumped by
// workgroup 0 at the end once every workgroup's start mark is in (decode_persist.hip's protocol
// and words: epoch[0] tag, epoch[1] sticky failure, err = failed position + 1).  Spins are
// bounded; a workgroup that gives up sets the words and leaves, every later launch returns at
// once, and the host re-runs the step on the graph path (runtime.hip persist_recover).  There is
// no run-ahead for B > 8, so the K / V append happens in stage A directly (a re-run overwrites
// the slot).
//
// GEMM stages: v_mfma_f32_16x16x4_f32 with the K-permutation and swapped operands of
// gemm_kernel.h — a 16-row x 16-column tile per wave (QKV, gate|up pairs) or per workgroup with
// the K split over its four waves (O-proj, down: few tiles); the group's input rows staged in
// LDS by the hand-off sweep (fp32, padded rows), the W fragments straight from global memory
// into registers.  Attention: one (row, head) item per wave.
#include "gemm_kernel.h"

namespace l3 {

// Persistent batched decode step (decode_batch.hip): the layers of one greedy step for B = 2..256
// rows in one launch (rows in groups of 16, each group's stages on its own workgroups with
// in-launch hand-offs); the lm_head and the argmax follow as launches of their own
struct DecodeBatchArgs {
    int B, Bcap;                   // rows of this step; rows the granule slabs hold
    int D, H, KVH, HD, FD, n_layers, Smax;
    int RG, GW;                    // row groups of 16; layer workgroups per group (decode_batch_setup)
    int Dp, Qp, Fp, AW;            // LDS row strides, per-wave attention scratch (floats)
    float eps, q_scale;
    const float* emb;              // [VS, D]
    const float* const* wqkv;      // per layer (device arrays of device pointers); norms folded
    const float* const* wo;
    const float* const* wgu;
    const float* const* wd;
    float* const* cache_k;         // per layer [maxB, KVH, Smax, HD]
    float* const* cache_v;
    const float* rope_cos; const float* rope_sin;
    const int32_t* ids;            // [B] this step's tokens
    const DecState* st;            // pos (the argmax after the lm_head moves it on)
    float* h_out;                  // [B, D] the last layer's output rows (the lm_head's input)
    unsigned long long* gran;      // per layer [qkv | o | h1 | hid | h2] x Bcap rows, then marks [256]
    int64_t slab;                  // granules per layer
    unsigned* flags;               // [n_layers][5 stages][16 groups][nflag] hand-off flags (zeroed once)
    int nflag;                     // flags per (stage, group): the most tiles / items of any stage
    unsigned* epoch;               // decode_persist.hip's words (shared tag space)
    unsigned* err;
    int fault_pos, fault_wg;       // test knob (L3_DECODE_PERSIST_FAULT)
    unsigned long long* stamps;    // diagnostic (null): [workgroup][128] s_memrealtime at stage points
};


namespace pbatch {

typedef unsigned long long u64;
constexpr int NT = 256;
typedef const __attribute__((address_space(1))) f32x4* gf4p;
__device__ __forceinline__ gf4p gf4(const void* p) { return (gf4p)(p); }

__device__ __forceinline__ void gput(u64* g, unsigned tag, float v) {
    __hip_atomic_store(g, ((u64)tag << 32) | __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ u64 gget(const u64* g) {
    return __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// LDS-only workgroup barrier (see decode_persist.hip lds_barrier)
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
// a wave's own LDS writes visible to its other lanes
__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

struct Ctx {
    const DecodeBatchArgs& p;
    unsigned tag;
    int pos;
    volatile int* bad;
};

__device__ __forceinline__ void give_up(const Ctx& c) {
    *c.bad = 1;
    __hip_atomic_store(c.p.err, (unsigned)c.pos + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(c.p.epoch + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool sticky(const Ctx& c) {
    return __hip_atomic_load(c.p.epoch + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
}
__device__ __forceinline__ bool spin_out(const Ctx& c, unsigned spin) {
    return spin > (1u << 20) || ((spin & 255) == 255 && (*c.bad || sticky(c)));
}

// i / ld for i < 16 * ld + 4096, ld <= 1536 (checked exhaustively on the host): a multiply-high by
// ceil(2^32 / ld) instead of the integer division sequence (a sweep splits up to 48 indices per
// thread into (row, column))
struct RowDiv {
    int ld;
    unsigned m;
    __device__ explicit RowDiv(int l) : ld(l), m(0xffffffffu / (unsigned)l + 1u) {}
    __device__ __forceinline__ int row(int i) const { return (int)__umulhi((unsigned)i, m); }
};

// n granules src(i) into *dst(i) (LDS) by the whole workgroup, CH per thread in flight per pass
// (sized so a stage's input is one or two passes: each pass is a memory round trip), each pass
// re-read until every tag is the launch's; then extra granules (not stored: workgroup 0's start
// marks) checked the same way.  Ends with a workgroup barrier; false if it gave up
template <int CH, typename Src, typename Dst>
__device__ bool sweep(const Ctx& c, int n, Src src, Dst dst, const u64* extra = nullptr, int n_extra = 0) {
    const int tid = threadIdx.x;
    for (int base = 0; base < n + n_extra; base += CH * NT) {
        for (unsigned spin = 0;; ++spin) {
            u64 x[CH];
            bool ok = true;
#pragma unroll
            for (int k = 0; k < CH; ++k) {
                const int i = min(base + k * NT + tid, n + n_extra - 1);
                x[k] = gget(i < n ? src(i) : extra + (i - n));
            }
#pragma unroll
            for (int k = 0; k < CH; ++k) ok &= (unsigned)(x[k] >> 32) == c.tag;
            if (ok) {
#pragma unroll
                for (int k = 0; k < CH; ++k) {
                    const int i = base + k * NT + tid;
                    if (i < n) *dst(i) = __uint_as_float((unsigned)x[k]);
                }
                break;
            }
            if (spin_out(c, spin)) {
                give_up(c);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        if (*c.bad) break;
    }
    lds_barrier();
    return !*c.bad;
}

// Hand-off flags (cdna_hip_programming.md Guideline 16, R1): a producing wave drains its payload
// stores (agent-scope granule stores write through) and one lane then stores the flag; consumers
// poll only the flags they need, then read the payload once (its tags are checked by the sweep
// that reads it).  Polling the payload itself — up to 48 granules per thread per poll round on
// every workgroup — loaded the memory system enough to make every hand-off 5-10 us.
__device__ __forceinline__ void publish(unsigned* flag, unsigned tag) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if ((threadIdx.x & 63) == 0) __hip_atomic_store(flag, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// the whole workgroup waits until flags f(i), i < n, all carry the launch's tag
template <typename F>
__device__ bool wait_flags(const Ctx& c, int n, F f) {
    for (unsigned spin = 0;; ++spin) {
        bool ok = true;
        for (int i = threadIdx.x; i < n; i += NT)
            ok &= __hip_atomic_load(f(i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == c.tag;
        if (__syncthreads_and(ok)) return true;
        if (spin > (1u << 20) || ((spin & 255) == 255 && sticky(c))) {
            if (threadIdx.x == 0) give_up(c);
            return false;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

// The linear form for a group's rows: granules src[i], i < n (rows of ld values, row-major), into
// dst[row * dstride + col].  No clamped indices: a pass may read past n into the slab that
// follows (always allocated), and those granules are neither checked nor stored
template <int CH>
__device__ bool sweep_rows(const Ctx& c, const u64* src, int n, float* dst, int ld, int dstride) {
    const int tid = threadIdx.x;
    const RowDiv dv(ld);
    for (int base = 0; base < n; base += CH * NT) {
        for (unsigned spin = 0;; ++spin) {
            u64 x[CH];
            bool ok = true;
#pragma unroll
            for (int k = 0; k < CH; ++k) x[k] = gget(src + base + k * NT + tid);
#pragma unroll
            for (int k = 0; k < CH; ++k) ok &= base + k * NT + tid >= n || (unsigned)(x[k] >> 32) == c.tag;
            if (ok) {
#pragma unroll
                for (int k = 0; k < CH; ++k) {
                    const int i = base + k * NT + tid;
                    const int r = dv.row(i);
                    if (i < n) dst[r * dstride + (i - r * ld)] = __uint_as_float((unsigned)x[k]);
                }
                break;
            }
            if (spin_out(c, spin)) {
                give_up(c);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        if (*c.bad) break;
    }
    lds_barrier();
    return !*c.bad;
}

// W fragments of one 16-column tile for k-blocks [kb0, kb0 + NK) (clamped: k-blocks past kb_hi
// are loaded from the last valid one and never used): lane l reads W row row0 + (l & 15) (clamped
// to rows < nrow), floats 16 kb + 4 (l >> 4) .. + 3 (gemm_kernel.h's K-permutation)
template <int NK>
__device__ __forceinline__ void load_w(const float* W, int row0, int nrow, int K, int kb0, int kb_hi,
                                       f32x4 (&wv)[NK]) {
    const int lane = threadIdx.x & 63;
    const int row = min(row0 + (lane & 15), nrow - 1);
    const gf4p w4 = gf4(W + (int64_t)row * K + 4 * (lane >> 4));
#pragma unroll
    for (int kb = 0; kb < NK; ++kb) wv[kb] = w4[4 * min(kb0 + kb, kb_hi - 1)];
}

// acc (C^T: lane l holds row l & 15, columns 4 (l >> 4) .. + 3 of the tile) += X . W^T over
// k-blocks [kb0, min(kb0 + NK, kb_hi)), X = 16 LDS rows of stride xs; ss += the lane's share of
// its row's sum of squares (the row's four lane quarters complete it, sum_xor16_32)
template <int NK>
__device__ __forceinline__ f32x4 tile_mma(const f32x4 (&wv)[NK], const float* x, int xs, int kb0, int kb_hi,
                                          f32x4 acc, float& ss) {
    const int lane = threadIdx.x & 63;
    const float* xr = x + (lane & 15) * xs + 4 * (lane >> 4);
#pragma unroll
    for (int kb = 0; kb < NK; ++kb) {
        if (kb0 + kb >= kb_hi) break;  // wave-uniform
        const f32x4 a = *reinterpret_cast<const f32x4*>(xr + 16 * (kb0 + kb));
        ss += a.x * a.x + a.y * a.y + a.z * a.z + a.w * a.w;
#pragma unroll
        for (int s = 0; s < 4; ++s) acc = mfma4(wv[kb][s], a[s], acc);
    }
    return acc;
}

// two tiles against the same 16 rows (gate and up of one hidden-unit block): each A fragment is
// read from LDS once for both (two separate chains had hipcc hold both copies: 74 registers)
template <int NK>
__device__ __forceinline__ void tile_mma2(const f32x4 (&wa)[NK], const f32x4 (&wb)[NK], const float* x, int xs,
                                          f32x4& acc_a, f32x4& acc_b, float& ss) {
    const int lane = threadIdx.x & 63;
    const float* xr = x + (lane & 15) * xs + 4 * (lane >> 4);
#pragma unroll
    for (int kb = 0; kb < NK; ++kb) {
        const f32x4 a = *reinterpret_cast<const f32x4*>(xr + 16 * kb);
        ss += a.x * a.x + a.y * a.y + a.z * a.z + a.w * a.w;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            acc_a = mfma4(wa[kb][s], a[s], acc_a);
            acc_b = mfma4(wb[kb][s], a[s], acc_b);
        }
    }
}

}  // namespace pbatch

// KD = D / 16 = H * HD / 16 k-blocks of the D-wide GEMMs (QKV, O-proj, gate|up); KF = FD / 16 of
// the down-proj (split over the four waves)
// One layer of the step for this workgroup (stages A-E).  Not inlined into the kernel's layer
// loop: inlined, hipcc hoisted every lane's loop-invariant address arithmetic out of that loop and
// kept it live across all five stages (512 registers and 165 spilled); false if it gave up.
template <int KD, int KF>
__device__ __noinline__ bool batch_layer(const DecodeBatchArgs& p, const pbatch::Ctx& c, int li, float* sm) {
    using namespace pbatch;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wg = blockIdx.x, G = gridDim.x;
    const unsigned tag = c.tag;
    const int pos = c.pos;
    u64* marks = p.gran + p.slab * p.n_layers;
    auto stamp = [&](int k) {  // diagnostic timeline (tools/pbatch_stamps.py)
        if (p.stamps && tid == 0) p.stamps[(int64_t)wg * 128 + k] = __builtin_amdgcn_s_memrealtime();  // 100 MHz
    };
    const int g = wg / p.GW, j = wg - g * p.GW;
    const int D = p.D, H = p.H, KVH = p.KVH, HD = p.HD, FD = p.FD;
    const int qdim = H * HD, kvdim = KVH * HD, qkvn = qdim + 2 * kvdim;
    const int r0 = 16 * g;                  // the group's first batch row
    const int ws = j * 4 + w, nws = 4 * p.GW;  // wave slot in the group
    const int brow = r0 + (lane & 15);      // the batch row of this lane's tile row
    const bool rvalid = brow < p.B;
    float* hin = sm;                        // [16][Dp] layer input (O-proj residual)
    float* xo = hin + 16 * p.Dp;            // [16][Qp] attention output rows
    float* h1 = xo + 16 * p.Qp;             // [16][Dp] FFN input (down residual)
    float* xh = h1 + 16 * p.Dp;             // [16][Fp] SwiGLU rows
    float* red = xh + 16 * p.Fp;            // [4][64][4] K-split partial tiles
    float* att = red + 4 * 256;             // attention scratch: q | k_new | v_new, scores, partials
    const int nrows = min(16, p.B - r0);
    // this layer's flags of group g: [stage][tile or item]
    unsigned* fl = p.flags + ((int64_t)li * 5 * 16 + g) * p.nflag;
    auto flag = [&](int stage, int i) { return fl + (int64_t)stage * 16 * p.nflag + i; };
    unsigned* flp = li > 0 ? p.flags + ((int64_t)(li - 1) * 5 * 16 + g) * p.nflag + (int64_t)4 * 16 * p.nflag : nullptr;
    u64* g_qkv = p.gran + p.slab * li;
    u64* g_o = g_qkv + (int64_t)p.Bcap * qkvn;
    u64* g_h1 = g_o + (int64_t)p.Bcap * qdim;
    u64* g_hid = g_h1 + (int64_t)p.Bcap * D;
    u64* g_h2 = g_hid + (int64_t)p.Bcap * FD;
    float* ck = p.cache_k[li];
    float* cv = p.cache_v[li];

    // ---- stage A: RMSNorm + QKV + RoPE + KV append (llama3.py:248, 166-185) ---------------
    {
        const int nt = qkvn / 16;
        f32x4 wv[KD];
        if (ws < nt) load_w<KD>(p.wqkv[li], 16 * ws, qkvn, D, 0, KD, wv);
        if (li == 0) {  // the tokens' embedding rows (llama3.py:287)
            for (int i = tid; i < 16 * (D / 4); i += NT) {
                const int r = i / (D / 4), k4 = i - r * (D / 4);
                const int b = min(r0 + r, p.B - 1);
                reinterpret_cast<f32x4*>(hin + r * p.Dp)[k4] = gf4(p.emb + (int64_t)p.ids[b] * D)[k4];
            }
            lds_barrier();
        } else {
            u64* g_prev = p.gran + p.slab * (li - 1) + (int64_t)p.Bcap * (qkvn + qdim + D + FD);
            if (!wait_flags(c, D / 16, [=](int i) { return flp + i; })) return false;
            if (!sweep_rows<KD>(c, g_prev + (int64_t)r0 * D, nrows * D, hin, D, p.Dp)) return false;
        }
        stamp(1 + 10 * li);
        // (the first tile's W prefetched above; a later tile, rare, loads its own: a W array
        // reassigned inside the loop made hipcc keep two copies live, 512 registers + spills)
        auto tile = [&](int t, const f32x4 (&wt)[KD]) {
            float ss = 0.f;
            f32x4 acc = tile_mma<KD>(wt, hin, p.Dp, 0, KD, f32x4{0.f, 0.f, 0.f, 0.f}, ss);
            ss = sum_xor16_32(ss);
            const float rs = __builtin_amdgcn_rsqf(ss * (1.0f / (float)D) + p.eps);
            const int col = 16 * t + 4 * (lane >> 4);
            const int sec = col < qdim ? 0 : col < qdim + kvdim ? 1 : 2;
            const int cc = col - (sec == 0 ? 0 : sec == 1 ? qdim : qdim + kvdim);
            const int head = cc / HD, d = cc - head * HD;
            f32x4 v = acc * rs;
            if (sec < 2) {  // RoPE on the pairs (d, d + 1), (d + 2, d + 3) (llama3.py:41-76)
                const int tt = pos * (HD >> 1) + (d >> 1);
                const float c0 = p.rope_cos[tt], s0 = p.rope_sin[tt], c1 = p.rope_cos[tt + 1], s1 = p.rope_sin[tt + 1];
                v = f32x4{v.x * c0 - v.y * s0, v.x * s0 + v.y * c0, v.z * c1 - v.w * s1, v.z * s1 + v.w * c1};
                if (sec == 0) v *= p.q_scale;
            }
            if (rvalid) {
                u64* gq = g_qkv + (int64_t)brow * qkvn + col;
                gput(gq + 0, tag, v.x);
                gput(gq + 1, tag, v.y);
                gput(gq + 2, tag, v.z);
                gput(gq + 3, tag, v.w);
                if (sec > 0)  // the cache slot (llama3.py:184-185); a re-run of the step overwrites it
                    *reinterpret_cast<f32x4*>((sec == 1 ? ck : cv) +
                                              (((int64_t)brow * KVH + head) * p.Smax + pos) * HD + d) = v;
            }
            publish(flag(0, t), tag);
        };
        if (ws < nt) tile(ws, wv);
        for (int t = ws + nws; t < nt; t += nws) {
            f32x4 w2[KD];
            load_w<KD>(p.wqkv[li], 16 * t, qkvn, D, 0, KD, w2);
            tile(t, w2);
        }
    }
    stamp(2 + 10 * li);
    // workgroup 0, last layer: every workgroup's start mark (they were written at launch; the
    // epoch bump at the end needs them), checked while the attention inputs are in flight
    if (wg == 0 && li + 1 == p.n_layers &&
        !sweep<1>(c, G, [=](int i) { return marks + i; }, [=](int i) { return att + i; }))
        return false;
    // ---- stage B: attention, one (row, head) item per workgroup at a time (llama3.py:186-210)
    // (the batch-1 step's stage B: every K row and the first 256 keys' V rows of the item in
    // flight before its q / k_new / v_new hand-off; an item per wave walked its keys in
    // dependent round trips, 13-35 us per layer at B = 256)
    {
        const int D4 = HD / 4;
        float* qs = att;                                       // q | k_new | v_new
        float* sc = att + 3 * HD;                              // scores [pos + 1]
        f32x4* part = reinterpret_cast<f32x4*>(sc + ((p.Smax + 4) & ~3));  // [64] P.V partials
        float* redm = reinterpret_cast<float*>(part + 64);     // [8] block max / sum slots
        constexpr int R = NT / 16, VPF = NT / R;               // 16 key groups x 16 float4 columns
        const int rg = tid >> 4, d4 = min(tid & 15, D4 - 1);
        const int kmax = pos > 0 ? pos - 1 : 0;
        for (int it = j; it < nrows * H; it += p.GW) {
            const int r = it / H, h = it - r * H, b = r0 + r;
            const int kvh = h / (H / KVH);
            const float* Kb = ck + ((int64_t)b * KVH + kvh) * p.Smax * HD;
            const float* Vb = cv + ((int64_t)b * KVH + kvh) * p.Smax * HD;
            f32x4 kr[16], vr[VPF];
#pragma unroll
            for (int i = 0; i < 16; ++i) kr[i] = gf4(Kb + (int64_t)min(tid, kmax) * HD)[min(i, D4 - 1)];
#pragma unroll
            for (int t = 0; t < VPF; ++t) vr[t] = gf4(Vb + (int64_t)min(rg + t * R, kmax) * HD)[d4];
            const int qo = h * HD, ko = qdim + kvh * HD, vo = qdim + kvdim + kvh * HD;
            u64* gb = g_qkv + (int64_t)b * qkvn;
            const int th = HD / 16;  // QKV tiles per head
            if (!wait_flags(c, 3 * th, [=](int i) {
                    return flag(0, i < th ? qo / 16 + i : i < 2 * th ? ko / 16 + i - th : vo / 16 + i - 2 * th); }))
                return false;
            if (!sweep<1>(c, 3 * HD, [=](int i) { return gb + (i < HD ? qo + i : i < 2 * HD ? ko + i - HD : vo + i - 2 * HD); },
                       [=](int i) { return qs + i; }))
                return false;
            if (it == j) stamp(3 + 10 * li);
            const f32x4* q4 = reinterpret_cast<const f32x4*>(qs);
            const f32x4* kn4 = reinterpret_cast<const f32x4*>(qs + HD);
            const f32x4* vn4 = reinterpret_cast<const f32x4*>(qs + 2 * HD);
            // scores: key tid from its prefetched row (chunks past HD zeroed), the new key (pos)
            // from every 16-lane group at once, keys past the first NT in a plain loop
            float s_own = 0.f;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const f32x4 qv = q4[min(i, D4 - 1)];
                const float d = kr[i].x * qv.x + kr[i].y * qv.y + kr[i].z * qv.z + kr[i].w * qv.w;
                s_own += i < D4 ? d : 0.f;
            }
            const int jn = min(tid & 15, D4 - 1);
            const f32x4 qn = q4[jn], kn = kn4[jn];
            float s_new = (tid & 15) < D4 ? qn.x * kn.x + qn.y * kn.y + qn.z * kn.z + qn.w * kn.w : 0.f;
            s_new = group_sum<16>(s_new);
            s_own = tid == pos ? s_new : s_own;
            float m = -INFINITY;
            if (tid <= pos) {
                sc[tid] = s_own;
                m = s_own;
            }
            for (int k = tid + NT; k <= pos; k += NT) {
                float s2 = 0.f;
                for (int i = 0; i < D4; ++i) {
                    const f32x4 av = k == pos ? kn4[i] : gf4(Kb + (int64_t)k * HD)[i], bq = q4[i];
                    s2 += av.x * bq.x + av.y * bq.y + av.z * bq.z + av.w * bq.w;
                }
                sc[k] = s2;
                m = fmaxf(m, s2);
            }
            m = group_max<64>(m);
            if ((tid & 63) == 0) redm[tid >> 6] = m;
            lds_barrier();
            m = fmaxf(fmaxf(redm[0], redm[1]), fmaxf(redm[2], redm[3]));
            float l = 0.f;
            for (int k = tid; k <= pos; k += NT) {
                const float e = __builtin_amdgcn_exp2f(sc[k] - m);  // q carries log2(e) / sqrt(HD)
                sc[k] = e;
                l += e;
            }
            l = group_sum<64>(l);
            if ((tid & 63) == 0) redm[4 + (tid >> 6)] = l;
            lds_barrier();  // also publishes sc
            l = (redm[4] + redm[5]) + (redm[6] + redm[7]);
            f32x4 acc = {0.f, 0.f, 0.f, 0.f};
            {
                float pk[VPF];
#pragma unroll
                for (int t = 0; t < VPF; ++t) pk[t] = sc[min(rg + t * R, pos)];
#pragma unroll
                for (int t = 0; t < VPF; ++t) acc += (rg + t * R < pos ? pk[t] : 0.f) * vr[t];
                for (int k = rg + VPF * R; k < pos; k += R) acc += sc[k] * gf4(Vb + (int64_t)k * HD)[d4];
                acc += (pos % R == rg ? sc[pos] : 0.f) * vn4[d4];
            }
            acc = f32x4{sum_xor16_32(acc.x), sum_xor16_32(acc.y), sum_xor16_32(acc.z), sum_xor16_32(acc.w)};
            if ((tid & 63) < 16) part[(tid >> 6) * 16 + (tid & 15)] = acc;
            lds_barrier();
            if (tid < D4) {
                f32x4 o = (part[tid] + part[16 + tid]) + (part[32 + tid] + part[48 + tid]);
                o *= 1.0f / l;
                u64* go = g_o + (int64_t)b * qdim + qo + 4 * tid;
                gput(go + 0, tag, o.x);
                gput(go + 1, tag, o.y);
                gput(go + 2, tag, o.z);
                gput(go + 3, tag, o.w);
            }
            if (w == 0) publish(flag(1, it), tag);
            lds_barrier();  // part / redm / qs reused by the next item
        }
    }
    stamp(4 + 10 * li);
    // ---- stage C: O-proj + residual (llama3.py:211, 253): a tile per workgroup, K over its waves
    {
        constexpr int NK = (KD + 3) / 4;
        const int nt = D / 16;
        const int kb0 = w * KD / 4, kb1 = (w + 1) * KD / 4;
        f32x4 wv[NK];
        if (j < nt) load_w<NK>(p.wo[li], 16 * j, D, qdim, kb0, kb1, wv);
        if (!wait_flags(c, nrows * H, [=](int i) { return flag(1, i); })) return false;
        if (!sweep_rows<KD>(c, g_o + (int64_t)r0 * qdim, nrows * qdim, xo, qdim, p.Qp)) return false;
        stamp(5 + 10 * li);
        auto tile = [&](int t, const f32x4 (&wt)[NK]) {
            float ss = 0.f;
            const f32x4 acc = tile_mma<NK>(wt, xo, p.Qp, kb0, kb1, f32x4{0.f, 0.f, 0.f, 0.f}, ss);
            reinterpret_cast<f32x4*>(red)[w * 64 + lane] = acc;
            lds_barrier();
            if (w == 0) {
                const f32x4* rp = reinterpret_cast<const f32x4*>(red);
                const f32x4 sum = ((rp[lane] + rp[64 + lane]) + rp[128 + lane]) + rp[192 + lane];
                const int col = 16 * t + 4 * (lane >> 4);
                const f32x4 v = *reinterpret_cast<const f32x4*>(hin + (lane & 15) * p.Dp + col) + sum;
                if (rvalid) {
                    u64* gh = g_h1 + (int64_t)brow * D + col;
                    gput(gh + 0, tag, v.x);
                    gput(gh + 1, tag, v.y);
                    gput(gh + 2, tag, v.z);
                    gput(gh + 3, tag, v.w);
                }
                publish(flag(2, t), tag);
            }
        };
        if (j < nt) tile(j, wv);
        for (int t = j + p.GW; t < nt; t += p.GW) {
            f32x4 w2[NK];
            load_w<NK>(p.wo[li], 16 * t, D, qdim, kb0, kb1, w2);
            lds_barrier();  // the previous tile's partials read
            tile(t, w2);
        }
    }
    stamp(6 + 10 * li);
    // ---- stage D: RMSNorm + gate|up + SwiGLU (llama3.py:256, 97-101): a 16-unit pair per wave
    {
        const int np = FD / 16;  // hidden units 16 pp .. + 15: fused rows 32 pp + (0..15) gate, + 16 up
        f32x4 wg_[KD], wu[KD];
        if (ws < np) {
            load_w<KD>(p.wgu[li], 32 * ws, 2 * FD, D, 0, KD, wg_);
            load_w<KD>(p.wgu[li], 32 * ws + 16, 2 * FD, D, 0, KD, wu);
        }
        if (!wait_flags(c, D / 16, [=](int i) { return flag(2, i); })) return false;
        if (!sweep_rows<KD>(c, g_h1 + (int64_t)r0 * D, nrows * D, h1, D, p.Dp)) return false;
        stamp(7 + 10 * li);
        auto unit = [&](int pp, const f32x4 (&tg)[KD], const f32x4 (&tu)[KD]) {
            float ss = 0.f;
            f32x4 ag = {0.f, 0.f, 0.f, 0.f}, au = {0.f, 0.f, 0.f, 0.f};
            tile_mma2<KD>(tg, tu, h1, p.Dp, ag, au, ss);
            ss = sum_xor16_32(ss);
            const float rs = __builtin_amdgcn_rsqf(ss * (1.0f / (float)D) + p.eps);
            const f32x4 gt = ag * rs, up = au * rs;
            const f32x4 v = {silu_f(gt.x) * up.x, silu_f(gt.y) * up.y, silu_f(gt.z) * up.z, silu_f(gt.w) * up.w};
            if (rvalid) {
                u64* gh = g_hid + (int64_t)brow * FD + 16 * pp + 4 * (lane >> 4);
                gput(gh + 0, tag, v.x);
                gput(gh + 1, tag, v.y);
                gput(gh + 2, tag, v.z);
                gput(gh + 3, tag, v.w);
            }
            publish(flag(3, pp), tag);
        };
        if (ws < np) unit(ws, wg_, wu);
        for (int pp = ws + nws; pp < np; pp += nws) {
            f32x4 g2[KD], u2[KD];
            load_w<KD>(p.wgu[li], 32 * pp, 2 * FD, D, 0, KD, g2);
            load_w<KD>(p.wgu[li], 32 * pp + 16, 2 * FD, D, 0, KD, u2);
            unit(pp, g2, u2);
        }
    }
    stamp(8 + 10 * li);
    // ---- stage E: down + residual (llama3.py:102, 259): a tile per workgroup, K over its waves
    {
        constexpr int NK = (KF + 3) / 4;
        const int nt = D / 16;
        const int kb0 = w * KF / 4, kb1 = (w + 1) * KF / 4;
        f32x4 wv[NK];
        if (j < nt) load_w<NK>(p.wd[li], 16 * j, D, FD, kb0, kb1, wv);
        if (!wait_flags(c, FD / 16, [=](int i) { return flag(3, i); })) return false;
        if (!sweep_rows<(KF + 1) / 2>(c, g_hid + (int64_t)r0 * FD, nrows * FD, xh, FD, p.Fp)) return false;
        stamp(9 + 10 * li);
        auto tile = [&](int t, const f32x4 (&wt)[NK]) {
            float ss = 0.f;
            const f32x4 acc = tile_mma<NK>(wt, xh, p.Fp, kb0, kb1, f32x4{0.f, 0.f, 0.f, 0.f}, ss);
            reinterpret_cast<f32x4*>(red)[w * 64 + lane] = acc;
            lds_barrier();
            if (w == 0) {
                const f32x4* rp = reinterpret_cast<const f32x4*>(red);
                const f32x4 sum = ((rp[lane] + rp[64 + lane]) + rp[128 + lane]) + rp[192 + lane];
                const int col = 16 * t + 4 * (lane >> 4);
                const f32x4 v = *reinterpret_cast<const f32x4*>(h1 + (lane & 15) * p.Dp + col) + sum;
                if (rvalid) {
                    u64* gh = g_h2 + (int64_t)brow * D + col;
                    gput(gh + 0, tag, v.x);
                    gput(gh + 1, tag, v.y);
                    gput(gh + 2, tag, v.z);
                    gput(gh + 3, tag, v.w);
                    if (li + 1 == p.n_layers)  // the lm_head's input rows (llama3.py:304)
                        *reinterpret_cast<f32x4*>(p.h_out + (int64_t)brow * D + col) = v;
                }
                publish(flag(4, t), tag);
            }
        };
        if (j < nt) tile(j, wv);
        for (int t = j + p.GW; t < nt; t += p.GW) {
            f32x4 w2[NK];
            load_w<NK>(p.wd[li], 16 * t, D, FD, kb0, kb1, w2);
            lds_barrier();  // the previous tile's partials read
            tile(t, w2);
        }
    }
    stamp(10 + 10 * li);
    return true;
}

template <int KD, int KF>
__global__ void __launch_bounds__(256, 1) decode_batch_kernel(DecodeBatchArgs p) {
    using namespace pbatch;
    extern __shared__ __attribute__((aligned(16))) float sm[];
    __shared__ int bad_s;
    const int tid = threadIdx.x, wg = blockIdx.x;
    if (tid == 0) bad_s = 0;
    const unsigned tag = p.epoch[0];
    const int pos = p.st->pos;
    if (p.epoch[1]) return;  // an earlier launch gave up: the host recovers
    u64* marks = p.gran + p.slab * p.n_layers;
    if (tid == 0) gput(marks + wg, tag, 0.f);
    lds_barrier();
    Ctx c{p, tag, pos, &bad_s};
    if (p.stamps && tid == 0) p.stamps[(int64_t)wg * 128] = __builtin_amdgcn_s_memrealtime();
    if (pos == p.fault_pos && wg == p.fault_wg) {  // test knob (L3_DECODE_PERSIST_FAULT)
        if (tid == 0) give_up(c);
        return;
    }
    if (wg / p.GW >= p.RG) return;  // no rows for this workgroup (its start mark is in)
    for (int li = 0; li < p.n_layers; ++li)
        if (!batch_layer<KD, KF>(p, c, li, sm)) return;
    if (wg == 0 && tid == 0) *p.epoch = tag + 1;  // every workgroup has read this launch's tag
}

// ---------------------------------------------------------------------------------------
#define L3_BATCH_INSTANCES(X) \
    X(18, 48)  /* stories15M: D 288, FD 768 */ \
    X(4, 12)   /* tiny: D 64, FD 192 */

static const void* batch_kernel(int kd, int kf) {
#define L3_FN(A, B) if (kd == A && kf == B) return reinterpret_cast<const void*>(&decode_batch_kernel<A, B>);
    L3_BATCH_INSTANCES(L3_FN)
#undef L3_FN
    return nullptr;
}

static size_t batch_lds(const DecodeBatchArgs& a) {
    return ((size_t)16 * (2 * a.Dp + a.Qp + a.Fp) + 4 * 256 + (size_t)a.AW) * 4;
}

bool decode_batch_ok(const DecodeBatchArgs& a) {
    const int qdim = a.H * a.HD;
    return a.B >= 2 && a.B <= 256 && a.B <= a.Bcap && a.D % 16 == 0 && a.FD % 16 == 0 && a.HD % 16 == 0 &&
           a.HD <= 64 && a.KVH >= 1 && a.H % a.KVH == 0 && qdim == a.D && a.Smax >= 1 && a.Smax <= 1024 &&
           a.n_layers >= 1 && batch_kernel(a.D / 16, a.FD / 16) != nullptr;
}

// the grid's shape for B rows: groups of 16 rows, GW layer workgroups per group (all 256 CUs for
// the layers: 16 per group at B = 256, 64 for B <= 64), LDS strides; 0 when the step cannot run
int decode_batch_setup(DecodeBatchArgs& a) {
    if (!decode_batch_ok(a)) return 0;
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return 0;
    const int cap = env_knob("L3_DECODE_PERSIST_MAX_CUS", 0);
    if (cap > 0 && cap < cus) cus = cap;
    const int grid = cus < 256 ? cus : 256;
    a.RG = (a.B + 15) / 16;
    a.GW = grid / a.RG < 64 ? grid / a.RG : 64;
    if (a.GW < 4) return 0;
    a.Dp = a.D + 4;
    a.Qp = a.H * a.HD + 4;
    a.Fp = a.FD + 4;
    a.AW = ((3 * a.HD + a.Smax + 8 + 3) & ~3) + 4 * 64 + 8;
    const size_t lds = batch_lds(a);
    int max_lds = 0;
    if (hipDeviceGetAttribute(&max_lds, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev) != hipSuccess ||
        lds + 2048 > (size_t)max_lds)
        return 0;
    const void* fn = batch_kernel(a.D / 16, a.FD / 16);
    if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) return 0;
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 256, lds) != hipSuccess || per_cu < 1) return 0;
    return grid;
}

hipError_t launch_decode_batch(const DecodeBatchArgs& a, int grid, hipStream_t s) {
    if (grid < 1 || grid > 256 || !decode_batch_ok(a) || a.RG * a.GW > grid) return hipErrorNotSupported;
    const size_t lds = batch_lds(a);
#define L3_LAUNCH(A, B)                                                                          \
    if (a.D / 16 == A && a.FD / 16 == B) {                                                       \
        hipLaunchKernelGGL((decode_batch_kernel<A, B>), dim3(grid), dim3(256), lds, s, a);     \
        return hipGetLastError();                                                                \
    }
    L3_BATCH_INSTANCES(L3_LAUNCH)
#undef L3_LAUNCH
    return hipErrorNotSupported;
}

}  // namespace l3
