// Persistent batch-1 greedy decode step (llama3.py:316-320 at B = 1, L = 1): the whole step —
// every layer's RMSNorm + QKV + RoPE + KV append, attention, O-proj + residual, RMSNorm + gate|up
// + SwiGLU, down + residual, then the final norm + lm_head and the greedy argmax — as ONE launch
// instead of 25 graph-replayed kernels.
//
// Why: a batch-1 stories15M step is ~60 MB of L2/MALL-resident weights and a chain of ~30
// all-to-all dependencies (every output of a stage needs the stage's whole input vector).  As
// separate launches each dependency costs a kernel boundary plus the kernel's dependent memory
// round trips (tools/launch_floor: 1.8 us empty, 2.4 us with one load round trip; the product
// step averages 3.8 us per kernel).  Inside one launch an all-to-all hand-off measured 1.85-2.3
// us (tools/handoff_chain, profiles/r04_handoff_chain.log), about a boundary — so the gain must
// come from what a boundary forbids: every workgroup issues the NEXT stage's weight loads right
// after publishing the current stage, and they land while it waits for the hand-off.  Measured:
// 0.076 ms per greedy step in the device loop against 0.096-0.098 for the 25-kernel graph
// (profiles/r04_persist_decode_ab.log); the stages are VALU-bound at one wave per SIMD, so every
// select, branch and workgroup reduction on the critical path shows (DESIGN.md decisions table).
//
// Hand-offs (cdna_hip_programming.md Guideline 16, R2): every stage output value travels as one
// 8-byte {tag, value} granule written by ONE agent-scope relaxed atomic store (sc1 write-through);
// consumers re-read the granules they need with agent-scope relaxed loads (sc1, L1-bypassing)
// until every tag equals the launch's epoch.  Each (layer, stage) has its own granule slab, so no
// slab is rewritten inside a launch; the epoch (a device word, +1 at the end of every launch by
// workgroup 0, once every workgroup of the launch has published its start mark, i.e. has read the
// launch's tag) makes the previous launch's granules stale without a memset.  Only values produced
// in THIS launch travel as granules; everything older (weights, the KV rows of earlier positions,
// the token id) is read with plain loads, which a kernel boundary makes visible.
//
// Failure is all-or-nothing for the KV caches.  Spins are bounded: a workgroup that waits ~1 s
// (the layer chain), or that finds the sticky failure word another workgroup set (the lm_head
// and the final argmax), gives up — it sets that word and the host-mapped error word (the step's
// position + 1) and leaves — so a fault ends the launch instead of hanging it, and every later
// launch returns at once until the host has recovered (runtime.hip persist_recover: undo, then
// the 25-kernel graph path).  A layer workgroup keeps the K / V rows its stage A computes (and,
// for the run-ahead undo, the slots' previous contents) in LDS and writes them to the caches only
// after its last wait of the step, which every layer workgroup passes exactly when every stage of
// every layer has published, and then stores its write mark (the launch's tag); a workgroup that
// gives up records the failing launch's tag in epoch[2].  After a failure the undo
// (kv_restore_kernel, KvGuard) therefore restores exactly the units whose workgroup's mark equals
// that tag — all of them, none, or (a hand-off arriving at the edge of one workgroup's ~1 s bound)
// some — and never a slot the failed launch did not write.
//
// Work split (grid = 256 workgroups x 256 threads, all resident: 1 per CU by resources, checked
// against the device by decode_persist_grid before a capture): the layer stages run on workgroups
// 0..GL-1 (GL = 64); the attention of head h on workgroup h; the lm_head's 32000 rows on the
// workgroups >= GL (they load their rows while the layers run).  GEMV stages: 16 lanes per output
// unit (a row, or a RoPE / gate-up row pair), the unit's W rows in registers, the input vector
// staged once per workgroup in LDS.
#include "kernels.h"

namespace l3 {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned long long u64;

namespace persist {

constexpr int NT = 256;          // threads per workgroup
constexpr int LPR = 16;          // lanes per unit in the GEMV stages
constexpr int UPP = NT / LPR;    // units per pass

__device__ __forceinline__ void gput(u64* g, unsigned tag, float v) {
    __hip_atomic_store(g, ((u64)tag << 32) | __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ u64 gget(u64* g) {
    return __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Workgroup barrier for LDS traffic only: __syncthreads() is also a workgroup-scope release of
// global memory, i.e. an s_waitcnt vmcnt(0) that waits for this wave's write-through granule /
// cache / stamp stores to be acknowledged (~1 us) before the barrier.  Nothing in this kernel
// reads through global memory what another wave of its own workgroup wrote in the same launch,
// so the stage-internal barriers only need the LDS writes done (asm: the compiler neither moves
// memory accesses across it nor sees a barrier it would pad with waits).
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

struct Ctx {
    const DecodePersistArgs& p;
    unsigned tag;
    int pos;
    volatile int* bad;  // LDS flag: this workgroup gave up on a hand-off
    float* red;         // LDS scratch [NT]
};

// the step's position + 1 to the host-mapped error word; epoch[1] sticky (every workgroup still
// waiting gives up at its next check, every later launch returns at once)
__device__ __forceinline__ void give_up(const Ctx& c) {
    *c.bad = 1;
    __hip_atomic_store(c.p.epoch + 2, c.tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // the failing launch
    __hip_atomic_store(c.p.err, (unsigned)c.pos + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(c.p.epoch + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool sticky(const Ctx& c) {
    return __hip_atomic_load(c.p.epoch + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
}

// granules g[idx(i)] for i < n, the first nst of them into dst[i] (LDS; the rest only waited
// for), every thread its i = tid + NT*k, all of a thread's loads in flight per pass; re-read until
// every tag is the launch's.  Ends with a workgroup barrier; false if this workgroup gave up
// (caller returns).  stick: also give up once another workgroup has (the sticky word) — not in
// the layer chain, whose workgroups wait the full bound instead, so that the chain either
// completes for every layer workgroup or for none (the K / V write, see the header)
template <int PER, typename Idx>
__device__ __forceinline__ bool sweep(const Ctx& c, u64* g, int n, float* dst, Idx idx, int sleep, bool stick, int nst) {
    const int tid = threadIdx.x;
    bool ok = false;
    for (unsigned spin = 0;; ++spin) {
        ok = true;
        u64 x[PER];
        // unpredicated (a clamped index past n: a predicated load is a branch that waits)
#pragma unroll
        for (int k = 0; k < PER; ++k) x[k] = gget(g + idx(min(tid + NT * k, n - 1)));
#pragma unroll
        for (int k = 0; k < PER; ++k) ok &= (unsigned)(x[k] >> 32) == c.tag;
        if (ok) {
#pragma unroll
            for (int k = 0; k < PER; ++k) {
                const int i = tid + NT * k;
                if (i < nst) dst[i] = __uint_as_float((unsigned)x[k]);
            }
            break;
        }
        // ~1 s, or another wave of this workgroup / (stick) another workgroup gave up
        if (spin > (1u << 20) || ((spin & 255) == 255 && (*c.bad || (stick && sticky(c))))) {
            give_up(c);
            break;
        }
        if (sleep == 1) __builtin_amdgcn_s_sleep(1);
        else __builtin_amdgcn_s_sleep(8);
    }
    lds_barrier();
    return !*c.bad;
}

template <typename Idx>
__device__ __forceinline__ bool sweep_n(const Ctx& c, u64* g, int n, float* dst, Idx idx, int sleep = 1,
                                        bool stick = false, int nst = -1) {
    if (nst < 0) nst = n;
    if (n <= NT) return sweep<1>(c, g, n, dst, idx, sleep, stick, nst);
    if (n <= 2 * NT) return sweep<2>(c, g, n, dst, idx, sleep, stick, nst);
    if (n <= 4 * NT) return sweep<4>(c, g, n, dst, idx, sleep, stick, nst);
    return sweep<5>(c, g, n, dst, idx, sleep, stick, nst);  // n <= 1280
}

// block max / sum of one value per thread (every thread gets it), one barrier each: the two use
// their own red slots (the attention stage calls max, then sum, once per layer; between two
// uses of a slot every wave has passed other barriers, so its last reads are done)
__device__ __forceinline__ float block_max(const Ctx& c, float v) {
    v = group_max<64>(v);
    const int tid = threadIdx.x;
    if ((tid & 63) == 0) c.red[tid >> 6] = v;
    lds_barrier();
    return fmaxf(fmaxf(c.red[0], c.red[1]), fmaxf(c.red[2], c.red[3]));
}
__device__ __forceinline__ float block_sum(const Ctx& c, float v) {
    v = group_sum<64>(v);
    const int tid = threadIdx.x;
    if ((tid & 63) == 0) c.red[4 + (tid >> 6)] = v;
    lds_barrier();
    return (c.red[4] + c.red[5]) + (c.red[6] + c.red[7]);
}

// global (not flat) 16-byte loads: flat loads also count in lgkmcnt, so every LDS wait would
// wait for them too
typedef const __attribute__((address_space(1))) f32x4* gf4p;
__device__ __forceinline__ gf4p gf4(const void* p) { return (gf4p)(p); }

// W rows of one unit into registers: lane j of the unit holds float4s k4 = j + LPR * t, t < NC.
// Unpredicated loads from clamped (in-bounds) addresses: a predicated load compiles to an
// exec-masked branch that waits for every load in flight before the next one is issued (one round
// trip per float4).  Nothing is zeroed here: the chunks past K meet zeroed x chunks in the dot
// (read_x), and an invalid unit's (clamped, finite) rows give a result nobody publishes — zeroing
// the rows cost a v_cndmask per element of W after the loads landed, on every stage
template <int ROWS, int NC>
__device__ __forceinline__ void load_rows(const float* W, const int (&row)[ROWS], int K4, f32x4 (&w)[ROWS][NC]) {
    const int j = threadIdx.x % LPR;
    const gf4p W4 = gf4(W);
#pragma unroll
    for (int t = 0; t < NC; ++t) {
        const int kk = min(j + LPR * t, K4 - 1);
#pragma unroll
        for (int r = 0; r < ROWS; ++r) w[r][t] = W4[(int64_t)row[r] * K4 + kk];
    }
}

// x chunks of this lane (LDS), zero past K
template <int NC>
__device__ __forceinline__ void read_x(const float* x, int K4, f32x4 (&xv)[NC]) {
    const int j = threadIdx.x % LPR;
    const f32x4* X4 = reinterpret_cast<const f32x4*>(x);
#pragma unroll
    for (int t = 0; t < NC; ++t) xv[t] = X4[min(j + LPR * t, K4 - 1)];
#pragma unroll
    for (int t = 0; t < NC; ++t) xv[t] = j + LPR * t < K4 ? xv[t] : f32x4{0.f, 0.f, 0.f, 0.f};
}

// branch-free: every chunk's LDS read is issued before the first FMA; a per-chunk bound check
// compiled to a branch and an LDS wait per chunk (the lm_head's eight passes took 3 us)
template <int ROWS, int NC>
__device__ __forceinline__ void dot_rows(const f32x4 (&w)[ROWS][NC], const float* x, int K4, float (&acc)[ROWS]) {
    f32x4 xv[NC];
    read_x<NC>(x, K4, xv);
#pragma unroll
    for (int r = 0; r < ROWS; ++r) acc[r] = 0.f;
#pragma unroll
    for (int t = 0; t < NC; ++t)
#pragma unroll
        for (int r = 0; r < ROWS; ++r)
            acc[r] += w[r][t].x * xv[t].x + w[r][t].y * xv[t].y + w[r][t].z * xv[t].z + w[r][t].w * xv[t].w;
#pragma unroll
    for (int r = 0; r < ROWS; ++r) acc[r] = group_sum<LPR>(acc[r]);
}

// 1 / rms of x from the chunks a 16-lane unit holds (read_x: together they cover x once), so no
// workgroup reduction — inv_rms's block sum cost two barriers and a predicated loop per stage
template <int NC>
__device__ __forceinline__ float unit_inv_rms(const f32x4 (&xv)[NC], int n, float eps) {
    float ss = 0.f;
#pragma unroll
    for (int t = 0; t < NC; ++t) ss += xv[t].x * xv[t].x + xv[t].y * xv[t].y + xv[t].z * xv[t].z + xv[t].w * xv[t].w;
    ss = group_sum<LPR>(ss);
    return __builtin_amdgcn_rsqf(ss / (float)n + eps);
}
// dot_rows plus the RMSNorm scale of x (RMSNorm, llama3.py:111-114; the weight is folded into W)
template <int ROWS, int NC>
__device__ __forceinline__ float dot_rows_rms(const f32x4 (&w)[ROWS][NC], const float* x, int K4, float eps,
                                              float (&acc)[ROWS]) {
    f32x4 xv[NC];
    read_x<NC>(x, K4, xv);
#pragma unroll
    for (int r = 0; r < ROWS; ++r) acc[r] = 0.f;
#pragma unroll
    for (int t = 0; t < NC; ++t)
#pragma unroll
        for (int r = 0; r < ROWS; ++r)
            acc[r] += w[r][t].x * xv[t].x + w[r][t].y * xv[t].y + w[r][t].z * xv[t].z + w[r][t].w * xv[t].w;
#pragma unroll
    for (int r = 0; r < ROWS; ++r) acc[r] = group_sum<LPR>(acc[r]);
    return unit_inv_rms<NC>(xv, 4 * K4, eps);
}

// one row's dot with x already in registers (read_x): the lm_head's passes share one x
template <int NC>
__device__ __forceinline__ float dot_row_x(const f32x4 (&w)[NC], const f32x4 (&xv)[NC]) {
    float acc = 0.f;
#pragma unroll
    for (int t = 0; t < NC; ++t) acc += w[t].x * xv[t].x + w[t].y * xv[t].y + w[t].z * xv[t].z + w[t].w * xv[t].w;
    return acc;
}

// this workgroup's unit range of a layer stage with n units over GL workgroups (one pass: the
// eligibility keeps ceil(n / GL) <= UPP)
__device__ __forceinline__ int stage_unit(const DecodePersistArgs& p, int n, int wg, bool& valid) {
    const int per = (n + p.GL - 1) / p.GL;
    const int i = threadIdx.x / LPR;
    const int u = wg * per + i;
    valid = i < per && u < n;
    return valid ? u : 0;
}

}  // namespace persist

// One launch = one decode step.  Granule slab per layer: [qkv | o | h1 | hid | h2]
// (decode_persist_slab), then the lm_head partials [2 * 256], the start marks [256] and the layer
// workgroups' write marks [GL] (32-bit, in a 256-granule block).
// NCD / NCF: float4 per lane of a W row with K = D / K = FD (>= ceil(K / 64)); KPF >= HD / 4 (the
// old keys' chunks each attention lane holds); LMPF: lm_head passes of 16 rows each workgroup
// holds in registers.
template <int NCD, int NCF, int KPF, int LMPF>
__global__ void __launch_bounds__(256, 1) decode_persist_kernel(DecodePersistArgs p) {
    using namespace persist;
    extern __shared__ __attribute__((aligned(16))) float sm[];
    __shared__ int bad_s;
    __shared__ float red_s[NT];
    const int D = p.D, HD = p.HD, H = p.H, KVH = p.KVH, FD = p.FD;
    const int qdim = H * HD, kvdim = KVH * HD, qkvn = qdim + 2 * kvdim;
    f32x4* kvs = reinterpret_cast<f32x4*>(sm);  // [n_layers][UPP] this workgroup's K / V pairs: new, old
    float* hin = sm + 4 * UPP * p.n_layers;     // [D]  layer input (residual of the O-proj)
    float* h1s = hin + p.Dp;      // [D]  FFN input (residual of the down-proj)
    float* xs = h1s + p.Dp;       // [max(qkvn, FD, qdim)] stage input
    float* sc = xs + p.Xp;        // [Smax] attention scores
    const int tid = threadIdx.x, wg = blockIdx.x, G = gridDim.x;
    if (tid == 0) bad_s = 0;
    const unsigned tag = p.epoch[0];
    const int pos = p.st->pos;
    int id = p.ids[0];
    // an earlier launch gave up (epoch[1], sticky): do nothing, the host recovers
    if (p.epoch[1]) return;
    const int64_t slab = decode_persist_slab(H, KVH, HD, D, FD);
    u64* lm_g = p.gran + slab * p.n_layers;
    u64* marks = lm_g + 2 * 256;
    unsigned* wmarks = reinterpret_cast<unsigned*>(marks + 256);
    // start mark: this workgroup has read the launch's tag (workgroup 0 moves the epoch on only
    // after seeing every mark, so no workgroup dispatched late can read the next launch's tag)
    if (tid == 0) gput(marks + wg, tag, 0.f);
    lds_barrier();
    Ctx c{p, tag, pos, &bad_s, red_s};
    auto stamp = [&](int k) {  // diagnostic timeline (DecodePersistArgs::stamps)
        if (p.stamps && tid == 0) p.stamps[(int64_t)wg * 128 + k] = __builtin_amdgcn_s_memrealtime();  // 100 MHz
    };
    stamp(0);
    // test knob (L3_DECODE_PERSIST_FAULT): workgroup fault_wg gives up at once in the step at
    // fault_pos (a layer workgroup after reducing the previous step's partials, as every layer
    // workgroup does before its first wait: the previous step's id always reaches the history)
    // fault_late: a layer workgroup gives up at its last wait instead (stage E of the last layer,
    // every stage before it published: the other layer workgroups pass and write their slots)
    const bool fault_late = pos == p.fault_pos && wg == p.fault_wg && p.fault_late;
    const bool fault = pos == p.fault_pos && wg == p.fault_wg && !fault_late;
    const int64_t h2_off = (int64_t)qkvn + qdim + D + FD;  // h2 within a slab
    const int K4d = D / 4, K4f = FD / 4, K4q = qdim / 4;
    // roles: layer workgroup (the layer stages; the attention of head wg < H) or lm workgroup lwg
    const bool layer_wg = wg < p.GL;

    // lm_head rows of this workgroup: [r0, r1); unit = one row, LPR lanes.  Only the workgroups
    // past GL take rows: they load them at launch, while the layers run (rows on the layer
    // workgroups were loaded after their last stage and made the final argmax wait ~1 us)
    const int nlm = G - p.GL, lwg = wg - p.GL;
    const int lm_per = (p.VS + nlm - 1) / nlm;
    const int lm_r0 = layer_wg ? p.VS : lwg * lm_per, lm_r1 = min(p.VS, lm_r0 + lm_per);
    const int lm_passes = lm_r1 > lm_r0 ? (lm_r1 - lm_r0 + UPP - 1) / UPP : 0;
    // the generate-history fields workgroup 0 writes at the end, fetched now (off the final path)
    const int hist_base = p.st->hist_base, hist_cap = p.st->hist_cap;
    int32_t* const hist = p.st->hist;
    float* const hist_val = p.st->hist_val;
    // from_parts: the previous step (the launch before this one in the same graph) left its
    // lm_head partials and no id; every layer workgroup reduces them itself (plain loads: written
    // by the previous launch) — its final argmax hand-off and reduction come off that step's tail.
    // This launch's own partials overwrite them only after every layer workgroup has started
    // (the lm stage waits for the whole layer chain, which needs every layer workgroup).
    // (called before layer 0's W rows are requested: called after them, in stage A, the
    // partials' loads waited for the W rows in the in-order memory counter and the step measured
    // 0.088-0.089 against 0.086 ms)
    auto reduce_parts = [&]() {
        float best = -INFINITY;
        int bi = 0x7fffffff;
        for (int i = tid; i < nlm; i += NT) {
            const u64 v = lm_g[2 * i], x = lm_g[2 * i + 1];
            const float bv = __uint_as_float((unsigned)v);
            const int ix = (int)(unsigned)x;
            const bool take = argmax_better(bv, ix, best, bi);
            best = take ? bv : best;
            bi = take ? ix : bi;
        }
        group_argmax<64>(best, bi, tid & 63);
        __shared__ float pb[4];
        __shared__ int pi[4];
        if ((tid & 63) == 0) { pb[tid >> 6] = best; pi[tid >> 6] = bi; }
        lds_barrier();
        best = pb[0];
        bi = pi[0];
        for (int w2 = 1; w2 < 4; ++w2) {
            const bool take = argmax_better(pb[w2], pi[w2], best, bi);
            best = take ? pb[w2] : best;
            bi = take ? pi[w2] : bi;
        }
        id = bi;
        if (wg == 0 && tid == 0) {  // the previous step's id (and its logit): its generate history entry
            L3_DCHECK(id >= 0 && id < p.VS, CHK_TOKEN_ID);
            const int q = pos - 1 - hist_base;
            if (hist && q >= 0 && q < hist_cap) hist[q] = id;
            if (hist_val && q >= 0 && q < hist_cap) hist_val[q] = best;
        }
    };
    if (!layer_wg) {
        // ---- final RMSNorm + lm_head (llama3.py:304-307) + this workgroup's argmax (:320) ---------
        if (fault) {
            if (tid == 0) give_up(c);
            return;
        }
        f32x4 lw[LMPF][1][NCD];  // live on this path only (not across the layer loop)
#pragma unroll
        for (int ps = 0; ps < LMPF; ++ps) {  // nothing else to do: the rows land while the layers run
            const int r = lm_r0 + ps * UPP + tid / LPR;
            const int row[1] = {min(r, p.VS - 1)};
            load_rows<1, NCD>(p.lm_head, row, K4d, lw[ps]);  // clamped rows
        }
        u64* g_last = p.gran + slab * (p.n_layers - 1) + h2_off;
        if (tid == 0) {  // a long wait: one lane polls the last granule, sleeping
            for (unsigned spin = 0; (unsigned)(gget(g_last + D - 1) >> 32) != tag; ++spin) {
                if (spin > (1u << 20) || ((spin & 255) == 255 && sticky(c))) break;
                __builtin_amdgcn_s_sleep(16);
            }
        }
        if (!sweep_n(c, g_last, D, xs, [](int i) { return i; }, 8, true)) return;
        stamp(100);
        f32x4 xv[NCD];
        read_x<NCD>(xs, K4d, xv);
        const float rs = unit_inv_rms<NCD>(xv, D, p.eps);
        stamp(103);
        float best = -INFINITY;
        int bi = 0x7fffffff;
        auto consider = [&](int r, float dot) {
            const float v = dot * rs;
            const bool take = r < lm_r1 && argmax_better(v, r, best, bi);
            best = take ? v : best;
            bi = take ? r : bi;
        };
        // the passes held in registers since the launch: x read from LDS once for all of them (a
        // dot_rows per pass re-read it: 11 x 20 KB of LDS traffic per workgroup), the LPR-lane sums
        // after all the dots (independent chains)
        float lacc[LMPF];
#pragma unroll
        for (int ps = 0; ps < LMPF; ++ps) lacc[ps] = dot_row_x<NCD>(lw[ps][0], xv);
#pragma unroll
        for (int ps = 0; ps < LMPF; ++ps) lacc[ps] = group_sum<LPR>(lacc[ps]);
        // this lane's rows rise with the pass, so "strictly greater, or the first NaN" in pass
        // order is argmax_better (first index on ties, NaN first) without its index compares and
        // branches (the eleven branchy compares and the zeroing of the rows were ~3 us of VALU)
#pragma unroll
        for (int ps = 0; ps < LMPF; ++ps) {
            const int r = lm_r0 + ps * UPP + tid / LPR;
            const float v = lacc[ps] * rs;
            const bool vn = v != v, bn = best != best;
            const bool take = r < lm_r1 && (bi == 0x7fffffff || v > best || (vn && !bn));
            best = take ? v : best;
            bi = take ? r : bi;
        }
        for (int ps = LMPF; ps < lm_passes; ++ps) {  // rows past them, streamed now
            const int r = lm_r0 + ps * UPP + tid / LPR;
            f32x4 w[1][NCD];
            const int row[1] = {min(r, p.VS - 1)};
            load_rows<1, NCD>(p.lm_head, row, K4d, w);
            float acc[1];
            dot_rows<1, NCD>(w, xs, K4d, acc);
            consider(r, acc[0]);
        }
        stamp(104);
        group_argmax<64>(best, bi, tid & 63);
        __shared__ float bv_s[4];
        __shared__ int bi_s[4];
        if ((tid & 63) == 0) { bv_s[tid >> 6] = best; bi_s[tid >> 6] = bi; }
        lds_barrier();
        if (tid == 0) {
            for (int w2 = 1; w2 < 4; ++w2)
                if (argmax_better(bv_s[w2], bi_s[w2], best, bi)) { best = bv_s[w2]; bi = bi_s[w2]; }
            gput(lm_g + 2 * lwg, tag, best);
            gput(lm_g + 2 * lwg + 1, tag, __int_as_float(bi));
        }
        stamp(101);
        return;
    }

    if (p.from_parts) reduce_parts();
    if (fault) {
        if (tid == 0) give_up(c);
        return;
    }
    for (int li = 0; li < p.n_layers; ++li) {
        u64* g_qkv = p.gran + slab * li;
        u64* g_o = g_qkv + qkvn;
        u64* g_h1 = g_o + qdim;
        u64* g_hid = g_h1 + D;
        u64* g_h2 = g_hid + FD;
        const float* wqkv = p.wqkv[li];
        const float* ck = p.cache_k[li];
        const float* cv = p.cache_v[li];
        // the attention workgroup's K / V rows of this layer (keys before pos: written by earlier
        // launches), fetched in stage B before its hand-off wait (fetched at the layer's start
        // instead, ahead of the QKV rows, the step measured 0.091 against 0.087 ms)
        const int kvh = wg / (H / KVH);
        // P.V layout: 16 key groups (rg, one 16-lane row each) x 16 float4 columns (d4; the ones
        // past HD / 4 idle), so a wave's four key groups reduce across its rows on the VALU
        const int D4 = HD / 4;
        constexpr int R = NT / 16;
        const int rg = tid >> 4, d4 = min(tid & 15, D4 - 1);
        const f32x4* K4p = reinterpret_cast<const f32x4*>(ck + (int64_t)kvh * p.Smax * HD);
        const f32x4* V4p = reinterpret_cast<const f32x4*>(cv + (int64_t)kvh * p.Smax * HD);
        constexpr int VPF = NT / R;  // V rows per lane: the first NT keys
        // unpredicated loads from clamped rows (see load_rows), zeroed where used; row pos - 1 is
        // the last one an earlier launch wrote (pos >= 1 in a decode step)
        const int kmax = pos > 0 ? pos - 1 : 0;
        const gf4p Kg = gf4(K4p), Vg = gf4(V4p);
        f32x4 kr[KPF], vr[VPF];
        // ---- stage A: RMSNorm + QKV + RoPE (llama3.py:248, 166-181); the K / V append
        // (:184-185) waits for the end of the step (see the header) ----------------------------
        {
            bool valid;
            const int u = stage_unit(p, qkvn / 2, wg, valid);  // RoPE pair (rows 2u, 2u + 1)
            const int row[2] = {2 * u, 2 * u + 1};
            f32x4 w[2][NCD];
            load_rows<2, NCD>(wqkv, row, K4d, w);
            const int col = 2 * u;
            const int sec = col < qdim ? 0 : col < qdim + kvdim ? 1 : 2;
            const int cc = col - (sec == 0 ? 0 : sec == 1 ? qdim : qdim + kvdim);
            const int head = cc / HD, d = cc - head * HD;
            float2 cs = {1.f, 0.f};
            if (sec < 2) {
                const int t = pos * (HD >> 1) + (d >> 1);
                cs = float2{p.rope_cos[t], p.rope_sin[t]};
            }
            // the slot's previous contents, for the run-ahead undo (kv_bak, written at the end)
            float2 old = {0.f, 0.f};
            if (p.kv_bak && sec > 0 && valid)
                old = *reinterpret_cast<const float2*>((sec == 1 ? ck : cv) + ((int64_t)head * p.Smax + pos) * HD + d);
            // the layer input: the token's embedding row (llama3.py:287), else the previous
            // layer's output granules
            if (li == 0) {
                // one float4 per thread, one round trip (D / 4 <= NT by eligibility; a float per
                // thread took two dependent trips for D > NT)
                const gf4p E4 = gf4(p.emb + (int64_t)id * D);
                const f32x4 e = E4[min(tid, K4d - 1)];
                if (tid < K4d) reinterpret_cast<f32x4*>(hin)[tid] = e;
                lds_barrier();
            } else if (!sweep_n(c, p.gran + slab * (li - 1) + h2_off, D, hin, [](int i) { return i; })) {
                return;
            }
            stamp(1 + 10 * li);
            float acc[2];
            const float rs = dot_rows_rms<2, NCD>(w, hin, K4d, p.eps, acc);
            if (valid && tid % LPR == 0) {
                const float v0 = acc[0] * rs, v1 = acc[1] * rs;
                const float r0 = v0 * cs.x - v1 * cs.y, r1 = v0 * cs.y + v1 * cs.x;
                const float s = sec == 0 ? p.q_scale : 1.0f;
                gput(g_qkv + col, tag, r0 * s);
                gput(g_qkv + col + 1, tag, r1 * s);
                if (sec > 0) kvs[li * UPP + tid / LPR] = f32x4{r0, r1, old.x, old.y};
            }
            stamp(2 + 10 * li);
        }
        // ---- stage B: attention of head wg (llama3.py:186-210), the others go on ------------
        if (wg < H) {
            const int h = wg;
            float* qs = xs;                              // q | k_new | v_new of this head
            const int qo = h * HD, ko = qdim + kvh * HD, vo = qdim + kvdim + kvh * HD;
#pragma unroll
            for (int i = 0; i < KPF; ++i) kr[i] = Kg[(int64_t)min(tid, kmax) * D4 + min(i, D4 - 1)];
#pragma unroll
            for (int t = 0; t < VPF; ++t) vr[t] = Vg[(int64_t)min(rg + t * R, kmax) * D4 + d4];
            if (!sweep_n(c, g_qkv, 3 * HD, qs, [=](int i) { return i < HD ? qo + i : i < 2 * HD ? ko + i - HD : vo + i - 2 * HD; }))
                return;
            stamp(3 + 10 * li);
            // only the K chunks past HD need zeroing (the q4 reads there land in k_new); a lane's
            // score past pos is never kept and a V row past pos never used (P.V checks k < pos),
            // so nothing else is masked — a select per element was ~100 VALU on this critical path
            if (D4 < KPF) {  // uniform: none for HD = 4 KPF (stories15M)
#pragma unroll
                for (int i = 0; i < KPF; ++i)
                    if (i >= D4) kr[i] = f32x4{0.f, 0.f, 0.f, 0.f};
            }
            const f32x4* q4 = reinterpret_cast<const f32x4*>(qs);
            const f32x4* kn4 = reinterpret_cast<const f32x4*>(qs + HD);
            const f32x4* vn4 = reinterpret_cast<const f32x4*>(qs + 2 * HD);
            const int S = pos + 1;
            // key tid from the prefetched row (rows past HD are zero: the q4 reads past HD land
            // in the k / v part of qs and add nothing).  The new key's score (key pos, from k_new)
            // is computed by every 16-lane group at once — chunk j of q . k_new, summed over the
            // group — and selected by lane pos: loading k_new into that one lane's row was a
            // divergent branch that held its wave (and the block_max barrier) back ~0.3 us
            const int jn = min(tid & 15, D4 - 1);
            const f32x4 qn = q4[jn], kn = kn4[jn];
            float s_new = (tid & 15) < D4 ? qn.x * kn.x + qn.y * kn.y + qn.z * kn.z + qn.w * kn.w : 0.f;
            s_new = group_sum<16>(s_new);
            float s_own = 0.f;
#pragma unroll
            for (int i = 0; i < KPF; ++i) {
                const f32x4 b = q4[i];
                s_own += kr[i].x * b.x + kr[i].y * b.y + kr[i].z * b.z + kr[i].w * b.w;
            }
            s_own = tid == pos ? s_new : s_own;
            float m = -INFINITY;
            if (tid < S) {
                sc[tid] = s_own;
                m = s_own;
            }
            for (int k = tid + NT; k < S; k += NT) {
                float s = 0.f;
                // keys past the first NT (contexts longer than a workgroup; off the stories path):
                // a plain loop — an unrolled row here held registers over the whole stage
                for (int i = 0; i < D4; ++i) {
                    const f32x4 a = k == pos ? kn4[i] : K4p[(int64_t)k * D4 + i], b = q4[i];
                    s += a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w;
                }
                sc[k] = s;
                m = fmaxf(m, s);
            }
            if (li == 1) stamp(110);
            m = block_max(c, m);
            if (li == 1) stamp(111);
            float l = 0.f;
            for (int k = tid; k < S; k += NT) {
                const float e = __builtin_amdgcn_exp2f(sc[k] - m);  // q carries log2(e) / sqrt(HD)
                sc[k] = e;
                l += e;
            }
            l = block_sum(c, l);  // its barrier also publishes sc
            if (li == 1) stamp(112);
            f32x4 acc = {0.f, 0.f, 0.f, 0.f};
            {
                // every p read first (clamped index), then the FMAs with p zeroed past pos: a
                // predicated read per key was a branch and an LDS wait per key
                float pk[VPF];
#pragma unroll
                for (int t = 0; t < VPF; ++t) pk[t] = sc[min(rg + t * R, pos)];
#pragma unroll
                for (int t = 0; t < VPF; ++t) acc += (rg + t * R < pos ? pk[t] : 0.f) * vr[t];
                for (int k = rg + VPF * R; k < pos; k += R) acc += sc[k] * V4p[(int64_t)k * D4 + d4];
                // the new key's row: every lane reads it, the key group owning it adds it (no
                // divergent reads before the partials' barrier)
                const float pn = sc[pos];
                const f32x4 vn = vn4[d4];
                acc += (pos % R == rg ? pn : 0.f) * vn;
            }
            if (li == 1) stamp(113);
            // the four key groups of a wave summed across its 16-lane rows (permlane swaps), then
            // the four waves' sums through LDS (a chain of 21 dependent adds over LDS partials
            // was ~0.4 us)
            {
                auto rows = [](float v) {
                    const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
                    v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
                    const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
                    return __uint_as_float(b[0]) + __uint_as_float(b[1]);
                };
                acc = f32x4{rows(acc.x), rows(acc.y), rows(acc.z), rows(acc.w)};
            }
            f32x4* part = reinterpret_cast<f32x4*>(sc + ((S + 3) & ~3));
            if ((tid & 63) < 16) part[(tid >> 6) * 16 + (tid & 15)] = acc;
            lds_barrier();
            if (li == 1) stamp(114);
            if (tid < D4) {
                f32x4 o = (part[tid] + part[16 + tid]) + (part[32 + tid] + part[48 + tid]);
                o *= 1.0f / l;
                gput(g_o + qo + 4 * tid + 0, tag, o.x);
                gput(g_o + qo + 4 * tid + 1, tag, o.y);
                gput(g_o + qo + 4 * tid + 2, tag, o.z);
                gput(g_o + qo + 4 * tid + 3, tag, o.w);
            }
            stamp(4 + 10 * li);
        }
        // ---- stage C: O-proj + residual (llama3.py:211, 253) --------------------------------
        {
            bool valid;
            const int u = stage_unit(p, D, wg, valid);
            const int row[1] = {u};
            f32x4 w[1][NCD];
            load_rows<1, NCD>(p.wo[li], row, K4q, w);
            if (!sweep_n(c, g_o, qdim, xs, [](int i) { return i; })) return;
            stamp(5 + 10 * li);
            float acc[1];
            dot_rows<1, NCD>(w, xs, K4q, acc);
            if (valid && tid % LPR == 0) gput(g_h1 + u, tag, hin[u] + acc[0]);
            stamp(6 + 10 * li);
        }
        // ---- stage D: RMSNorm + gate|up + SwiGLU (llama3.py:256, 97-101) -----------------------
        {
            bool valid;
            // unit u: hidden unit u, fused rows 32(u/16) + u%16 (gate) and +16 (up)
            const int u = stage_unit(p, FD, wg, valid);
            int row[2];
            row[0] = 32 * (u / 16) + u % 16;
            row[1] = row[0] + 16;
            f32x4 w[2][NCD];
            load_rows<2, NCD>(p.wgu[li], row, K4d, w);
            if (!sweep_n(c, g_h1, D, h1s, [](int i) { return i; })) return;
            stamp(7 + 10 * li);
            float acc[2];
            const float rs = dot_rows_rms<2, NCD>(w, h1s, K4d, p.eps, acc);
            if (valid && tid % LPR == 0) {
                const float gt = acc[0] * rs, up = acc[1] * rs;
                gput(g_hid + u, tag, gt * __builtin_amdgcn_rcpf(1.0f + __expf(-gt)) * up);
            }
            stamp(8 + 10 * li);
        }
        // ---- stage E: down + residual (llama3.py:102, 259) ------------------------------------
        {
            bool valid;
            const int u = stage_unit(p, D, wg, valid);
            const int row[1] = {u};
            f32x4 w[1][NCF];
            load_rows<1, NCF>(p.wd[li], row, K4f, w);
            if (fault_late && li + 1 == p.n_layers) {
                if (tid == 0) give_up(c);
                return;
            }
            if (!sweep_n(c, g_hid, FD, xs, [](int i) { return i; })) return;
            stamp(9 + 10 * li);
            float acc[1];
            dot_rows<1, NCF>(w, xs, K4f, acc);
            if (valid && tid % LPR == 0) gput(g_h2 + u, tag, h1s[u] + acc[0]);  // the last layer's: to the lm workgroups
            stamp(10 + 10 * li);
        }
    }
    // ---- every layer workgroup past its last wait: every stage of every layer has published ----
    // the step's K / V rows into the caches (llama3.py:184-185), each slot's previous contents into
    // kv_bak [pos % KV_BAK_SLOTS][k, v][1][KVH][HD] (the run-ahead undo, GemmArgs::kv_bak): stores
    // only, from LDS (the next launch reads the rows with plain loads after the kernel boundary)
    {
        bool valid;
        const int u = stage_unit(p, qkvn / 2, wg, valid);
        const int col = 2 * u;
        const int sec = col < qdim ? 0 : col < qdim + kvdim ? 1 : 2;
        if (valid && sec > 0 && tid % LPR == 0) {
            const int cc = col - (sec == 1 ? qdim : qdim + kvdim);
            const int head = cc / HD, d = cc - head * HD;
            const int64_t coff = ((int64_t)head * p.Smax + pos) * HD + d;
            L3_DCHECK(pos >= 0 && pos < p.Smax, CHK_KV_SLOT);
            const int64_t boff = (((int64_t)(pos % KV_BAK_SLOTS) * 2 + sec - 1) * KVH + head) * HD + d;
            float* const* cache = sec == 1 ? p.cache_k : p.cache_v;
            for (int li = 0; li < p.n_layers; ++li) {
                const f32x4 e = kvs[li * UPP + tid / LPR];
                if (p.kv_bak) *reinterpret_cast<float2*>(p.kv_bak + (int64_t)li * p.bak_layer + boff) = float2{e.z, e.w};
                *reinterpret_cast<float2*>(cache[li] + coff) = float2{e.x, e.y};
            }
        }
        // this workgroup's write mark: every one of its threads is past the last wait (the sweep
        // ends in a barrier with no give-up), so each stores its slots above — nothing can stop it
        // between that barrier and here
        if (tid == 0) __hip_atomic_store(wmarks + wg, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (wg != 0) return;
    // ---- workgroup 0, its own slots written: every workgroup's start mark (every one has read this
    // launch's tag — an lm workgroup dispatched late, another kernel holding its CU, would
    // otherwise read the moved epoch and wait for granules no launch writes) before the epoch
    // moves on.  Waited for after the slot writes, so a give-up here (a workgroup never
    // dispatched) leaves this workgroup's mark set and its slots restorable (kv_bak) ------------
    if (!sweep_n(c, marks, G, xs, [](int i) { return i; }, 1, false, 0)) return;
    if (!p.write_id) {
        // the next launch reduces this step's partials itself; only the position moves on here
        // (every layer workgroup read it at its start: none could have finished layer 0 else)
        if (tid == 0) {
            p.st->pos = pos + 1;
            *p.epoch = tag + 1;
        }
        return;
    }

    // ---- (3) last step of a graph: the step's greedy id from the lm partials; generate history, position ----
    {
        float* pv = xs;  // [2 nlm]
        if (!sweep_n(c, lm_g, 2 * nlm, pv, [](int i) { return i; }, 1, true)) return;
        stamp(105);
        float best = -INFINITY;
        int bi = 0x7fffffff;
        for (int i = tid; i < nlm; i += NT) {
            const float v = pv[2 * i];
            const int ix = __float_as_int(pv[2 * i + 1]);
            const bool take = argmax_better(v, ix, best, bi);
            best = take ? v : best;
            bi = take ? ix : bi;
        }
        group_argmax<64>(best, bi, tid & 63);
        __shared__ float fb[4];
        __shared__ int fi[4];
        if ((tid & 63) == 0) { fb[tid >> 6] = best; fi[tid >> 6] = bi; }
        lds_barrier();
        if (tid == 0) {
            for (int w2 = 1; w2 < 4; ++w2)
                if (argmax_better(fb[w2], fi[w2], best, bi)) { best = fb[w2]; bi = fi[w2]; }
            p.ids[0] = bi;
            const int q = pos - hist_base;
            if (hist && q >= 0 && q < hist_cap) hist[q] = bi;
            if (hist_val && q >= 0 && q < hist_cap) hist_val[q] = best;
            p.st->pos = pos + 1;
            *p.epoch = tag + 1;
        }
        stamp(102);
    }
}

// Instances (chunk counts rounded up; the loads past K are clamped): X(NCD, NCF, KPF, LMPF)
#define L3_PERSIST_INSTANCES(X)                                                                   \
    X(1, 3, 16, 8)    /* tiny models (tests) */                                                   \
    X(5, 12, 12, 11)  /* stories15M: D 288, FD 768, HD 48 (167 lm rows per lm workgroup) */       \
    X(5, 12, 16, 8)   /* the same D / FD with HD 52..64 (D 256: 4 heads of 64) */                 \
    X(5, 16, 16, 4)                                                                               \
    X(8, 16, 16, 2)                                                                               \
    X(1, 12, 16, 8)                                                                               \
    X(5, 3, 16, 8)                                                                                \
    X(8, 12, 16, 2)

static int ncd_of(int D) { const int n = (D + 63) / 64; return n <= 1 ? 1 : n <= 5 ? 5 : n <= 8 ? 8 : 0; }
static int ncf_of(int FD) { const int n = (FD + 63) / 64; return n <= 3 ? 3 : n <= 12 ? 12 : n <= 16 ? 16 : 0; }

// the first instance that takes the shape: its (D, FD) chunking and KPF >= HD / 4 (a KPF short of
// HD / 4 would drop the old keys' last dims from their scores)
struct PersistInstance { int ncd, ncf, kpf, lmpf; };
static const PersistInstance kPersistInstances[] = {
#define L3_ROW(A, B, C, E) {A, B, C, E},
    L3_PERSIST_INSTANCES(L3_ROW)
#undef L3_ROW
};
static const PersistInstance* persist_instance(const DecodePersistArgs& a) {
    const int ncd = ncd_of(a.D), ncf = ncf_of(a.FD);
    for (const PersistInstance& x : kPersistInstances)
        if (x.ncd == ncd && x.ncf == ncf && a.HD / 4 <= x.kpf) return &x;
    return nullptr;
}

static const void* persist_kernel(const PersistInstance* x) {
#define L3_FN(A, B, C, E) \
    if (x->ncd == A && x->ncf == B && x->kpf == C && x->lmpf == E) return reinterpret_cast<const void*>(&decode_persist_kernel<A, B, C, E>);
    L3_PERSIST_INSTANCES(L3_FN)
#undef L3_FN
    return nullptr;
}

bool decode_persist_ok(const DecodePersistArgs& a) {
    const int qkvn = (a.H + 2 * a.KVH) * a.HD;
    return a.D % 4 == 0 && a.FD % 4 == 0 && a.HD % 4 == 0 && a.HD >= 4 && a.HD <= 64 && a.H <= a.GL &&
           a.H % a.KVH == 0 && a.H * a.HD == a.D && persist_instance(a) && qkvn % 2 == 0 &&
           (qkvn / 2 + a.GL - 1) / a.GL <= persist::UPP && (a.FD + a.GL - 1) / a.GL <= persist::UPP &&
           (a.D + a.GL - 1) / a.GL <= persist::UPP && a.D / 4 <= persist::NT && a.Smax >= 1 && a.Smax <= 8192 && a.VS >= 1 &&
           a.n_layers >= 1 && a.GL >= 1 && a.GL < 256;
}

static size_t persist_lds(const DecodePersistArgs& a) {  // K / V pairs, hin, h1s, xs, scores, P.V partials
    return ((size_t)4 * persist::UPP * a.n_layers + 2 * a.Dp + a.Xp + a.Smax + 4 + 256 * 4 + 64) * 4;
}

// Grid of one decode step, 0 when the step cannot run on this device: one workgroup per CU (256
// on MI355X), every one of them resident at once — the workgroups wait on each other, so the
// grid must not exceed the CUs times the blocks per CU the kernel's resources admit (its
// registers hold it to 1; checked with the occupancy query at the dynamic LDS).  Fewer CUs than
// the layer workgroups + the lm workgroups need (a CPX partition's 32) means no persistent step.
// L3_DECODE_PERSIST_MAX_CUS caps the CU count seen (test knob).
int decode_persist_grid(const DecodePersistArgs& a) {
    if (!decode_persist_ok(a)) return 0;
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return 0;
    const int cap = env_knob("L3_DECODE_PERSIST_MAX_CUS", 0);
    if (cap > 0 && cap < cus) cus = cap;
    const int grid = cus < 256 ? cus : 256;
    if (grid <= a.GL || 2 * (grid - a.GL) > a.Xp) return 0;
    const size_t lds = persist_lds(a);
    if (lds > 64 * 1024) return 0;  // (the default dynamic LDS cap)
    int per_cu = 0;
    const void* fn = persist_kernel(persist_instance(a));
    if (!fn || hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 256, lds) != hipSuccess || per_cu < 1)
        return 0;
    return grid;
}

hipError_t launch_decode_persist(const DecodePersistArgs& a, int grid, hipStream_t s) {
    if (grid < 1 || grid > 256 || grid <= a.GL || !decode_persist_ok(a)) return hipErrorNotSupported;
    const size_t lds = persist_lds(a);
    const PersistInstance* x = persist_instance(a);
#define L3_LAUNCH(A, B, C, E)                                                                            \
    if (x->ncd == A && x->ncf == B && x->kpf == C && x->lmpf == E) {                                     \
        hipLaunchKernelGGL((decode_persist_kernel<A, B, C, E>), dim3(grid), dim3(256), lds, s, a);      \
        return hipGetLastError();                                                                        \
    }
    L3_PERSIST_INSTANCES(L3_LAUNCH)
#undef L3_LAUNCH
    return hipErrorNotSupported;
}

hipError_t dcheck_collect_persist(unsigned* out) { return dcheck_collect(out); }

}  // namespace l3
