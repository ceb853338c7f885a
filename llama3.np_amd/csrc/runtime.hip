// libllama3hip runtime: device context, weight residency, forward orchestration, RCCL.
// Implements include/llama3hip.h.  Reference anchors are given per entry point.
//
// Device layout (one context per GPU, everything resident in HBM for the context's life):
//   emb        [VS, D]                       model.embed_tokens.weight
//   per layer  wqkv [H*HD + 2*KVH*HD, D]     q|k|v rows stacked (one GEMM)
//              wo   [D, H*HD]
//              wgu  [2*FD, D]                gate/up interleaved in 16-row groups (one GEMM
//                                            whose epilogue pairs gate_j with up_j)
//              wd   [D, FD]
//              n_attn / n_ffn [D]            RMSNorm weights, applied inside the GEMMs
//              cache_k / cache_v [maxB, KVH, M, HD]  zero-initialised, persistent
//   lm_head    [VS, D], final_norm [D]       (vocab_size 0: layer-only context, no tables)
//   rope cos/sin [M, HD/2] fp32 (computed in double exactly as llama3.py:31-38, then rounded)
//   workspace  h [T, D] residual stream, q [T, H*HD], attn [T, H*HD], hidden [T, FD],
//              logits [B, VS], ids [T], argmax [B]   (grown on demand, T = B*L)
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstddef>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <chrono>
#include <deque>
#include <vector>

#include "../../include/llama3hip.h"
#include "kernels.h"

using namespace l3;

static_assert(offsetof(DecState, pos) == 0, "captured kernels read &DecState::pos as pos_dev");

static thread_local std::string g_err;

static int fail(const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return 1;
}

#define HIP_TRY(expr)                                                                    \
    do {                                                                                 \
        hipError_t e_ = (expr);                                                          \
        if (e_ != hipSuccess)                                                            \
            return fail("%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, \
                        __LINE__);                                                       \
    } while (0)

#define NCCL_TRY(expr)                                                                         \
    do {                                                                                       \
        ncclResult_t r_ = (expr);                                                              \
        if (r_ != ncclSuccess) return fail("%s failed: %s", #expr, ncclGetErrorString(r_));    \
    } while (0)

#define CHECK_CTX(ctx) \
    if (!(ctx)) return fail("null context")

struct Layer {
    float* wqkv = nullptr;
    float* wo = nullptr;
    float* wgu = nullptr;
    float* wd = nullptr;
    float* n_attn = nullptr;
    float* n_ffn = nullptr;
    float* cache_k = nullptr;
    float* cache_v = nullptr;
    unsigned have = 0;  // bitmask of uploaded kinds
    // RMSNorm weight folded into the consuming GEMM's W columns at l3_finalize
    bool folded_qkv = false, folded_gu = false;
    // the opt-in x6 GEMM path (gemm_x6.h, l3_set_gemm_x6): each weight as three bf16 pieces
    // [N][3][K], made from the folded fp32 weight (null when the path is off)
    unsigned short *wqkv3 = nullptr, *wo3 = nullptr, *wgu3 = nullptr, *wd3 = nullptr;
};

struct Timer {
    hipEvent_t a, b;
    int kind;
};

struct l3_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    // batch split: a large prefill runs as two independent halves of the batch rows on stream
    // and aux (llama3.py:163-211 never mixes rows), so each half's kernels fill the other's
    // launch tails and boundaries; fork / join by events
    static constexpr int MAX_PARTS = 4;
    hipStream_t aux[MAX_PARTS - 1] = {};
    hipEvent_t fork_ev = nullptr, join_ev[MAX_PARTS - 1] = {};
    // host path: part p's last layers wait for part p - 1's same layer (forward_dev)
    hipEvent_t lag_ev[MAX_PARTS - 1] = {};
    int split = 2;                   // parts (1 = off); l3_set_batch_split, L3_BATCH_SPLIT
    bool gemm_x6 = false;            // prefill GEMMs on the x6 path (l3_set_gemm_x6, L3_GEMM_X6)
    bool prune_last = true;          // last layer: attention / O-proj / FFN on the last rows only
                                     // (l3_set_last_layer_rows, L3_LAST_LAYER_ALL_ROWS)
    int64_t split_min_tokens = 8192; // a part must hold at least this many tokens
    l3_dims d{};
    int HD = 0, qdim = 0, kvdim = 0, qkvn = 0;
    float* emb = nullptr;
    float* lm_head = nullptr;
    float* final_norm = nullptr;
    float* rope_cos = nullptr;
    float* rope_sin = nullptr;
    std::vector<Layer> layers;
    bool have_emb = false, have_lm = false, have_fnorm = false, finalized = false;
    bool folded_lm = false;
    // workspace
    int64_t ws_T = 0, ws_B = 0;
    float *h = nullptr, *q = nullptr, *attn = nullptr, *hid = nullptr, *logits = nullptr;
    float* oparts = nullptr;         // [8, H, D] per-head O-proj rows of the fused decode attention
    float* hsum = nullptr;           // [8, D] h + those rows (gate|up writes it for down's residual)
    float* skws = nullptr;           // split-K workspace of the layer GEMMs on `stream` (models
    int64_t skws_cap = 0;            //   with D or FD >= 2048; gemm.hip launch_split), floats
    ArgmaxPart* amax_part = nullptr; // batch-1 lm_head's per-block argmax partials
    int amax_n = 0;                  // partials the last lm_head wrote (0: none, use the logits)
    // captured batched decode steps: the tiled lm_head writes per-row argmax partials [B][ceil(VS/64)]
    // instead of the logits (GemmArgs::amax_rows), reduced by one B-row argmax launch
    ArgmaxPart* amax_rows = nullptr;
    int amax_rows_n = 0;             // partials per row the last lm_head wrote (0: none)
    bool rows_amax = false;          // capture_steps: the lm_head may leave partials only
    int32_t *ids = nullptr, *amax = nullptr;
    int32_t* ids_pin = nullptr;      // pinned host staging of the int32 ids (upload_ids)
    int64_t ids_pin_n = 0;
    // op scratch
    std::vector<void*> scratch;
    // timing (bit k of timing_mask: record HIP events around launches of kernel id k)
    bool timing = false;
    unsigned timing_mask = 0;
    std::vector<Timer> timers;
    size_t timer_used = 0;
    double tot_ms[L3_K_COUNT] = {0};
    int64_t cnt[L3_K_COUNT] = {0};
    // rccl
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0;
    bool comm_owned = true;          // false: the communicator belongs to an l3_group
    l3_group* group = nullptr;       // the group this context is a member of (l3_group_create)
    // logits gather form (l3_comm_set_overlap; env L3_COMM_MODE for A/B): 1 serialized on the
    // context stream (default), 3 the next forward's second batch part overlapping the gather,
    // 0 a comm stream ordered by events (measured slower)
    int comm_mode = 1;
    // comm stream of the A/B gather mode 0 (modes 1 and 3 gather on stream, see
    // l3_comm_gather_logits); the next lm_head (the writer of the gathered rows) waits for the
    // gather, every other entry point joins it first (set_dev)
    hipStream_t comm_stream = nullptr;
    int32_t* gather_ids = nullptr;   // [maxB] this rank's argmax ids (l3_comm_gather_argmax)
    hipEvent_t comm_fwd_ev = nullptr, comm_done_ev = nullptr;
    bool gather_pending = false;
    // mode 3 (l3_comm_set_overlap): the gather was the last work queued on stream, and comm_fwd_ev marks
    // the stream just before it — the next l3_forward_dev's second batch part starts from there,
    // so its layers overlap the transfer (only that entry point keeps the flag: set_dev clears it)
    bool gather_tail = false;
    // captured greedy decode step (llama3.py:316-320 as one hipGraph replay per token)
    int32_t* dec_ids = nullptr;      // [maxB] input ids of the next decode step (argmax output)
    DecState* dec_state = nullptr;   // device loop state: position, generate history
    int* dec_pos = nullptr;          // &dec_state->pos: start_pos of the next decode step
    int32_t* dec_host = nullptr;     // pinned [maxB] for the per-token ids copy-back
    hipGraph_t dec_graph = nullptr;
    hipGraphExec_t dec_exec = nullptr;
    int dec_B = 0;                   // batch the graph was captured for
    // the device loop (generate_all) replays dec_n steps per graph launch: one captured graph of
    // dec_n consecutive decode steps (the position and ids live on the device, so the steps
    // chain inside the graph), which removes the gap between graph launches
    hipGraph_t dec_graph_n = nullptr;
    hipGraphExec_t dec_exec_n = nullptr;
    int dec_n = 0, dec_n_B = 0;
    int64_t dec_pos_mirror = -1;     // host copy of *dec_pos; -1 = device decode state invalid
    std::vector<int64_t> dec_last;   // ids the device state holds (last returned)
    int64_t graph_steps = 0;         // decode steps served by graph replay (stats)
    // Run-ahead decode (lazy generate): when a step returns, up to SPEC_AHEAD further decode
    // steps are already queued as replays of the captured step graphs (the ids chain on the
    // device; each step's ids land in spec_hist by position), so the GPU keeps running while the
    // host yields.  Every captured QKV append first keeps the slot it overwrites in kv_bak; a call
    // that does not continue the schedule restores the slots of every step not yet handed out.
    // The queue is bounded by steps (SPEC_AHEAD) and by time: at most SPEC_BUDGET_US of queued
    // decode work, by the measured step time (step_us), so a caller that leaves the schedule
    // (EOS, an abandoned generator) waits at most about that long for work nobody asked for —
    // 16 steps at stories15M's 0.1 ms, none at the Llama-3-8B shape's 5 ms per step.
    static constexpr int SPEC_AHEAD = 16;
    static constexpr double SPEC_BUDGET_US = 4000.0;
    double step_us = 0.0;            // decode step time (EMA): graph replays (host wall clock of a
                                     // synced replay, HIP events around each queued run-ahead graph)
    bool step_us_seed = false;       // step_us is still the eager first step's (an upper bound):
                                     // the first replay's time replaces it
    float* kv_bak = nullptr;         // [n_layers][KV_BAK_SLOTS][2: k, v][8][KVH][HD]
    bool bak_capture = false;        // run_layer: QKV launches keep the overwritten slot
    // capture_steps, batch-1 argmax fold: the lm_head moves the position on (fold_adv), and the
    // layer-0 QKV of every step after a graph's first reduces the previous step's fold_n lm_head
    // partials itself (fold_in) instead of a separate argmax launch
    bool fold_in = false, fold_adv = false;
    int fold_n = 0;
    bool dec_bak = false;            // the captured single-step graph keeps it
    bool dec_n_bak = false;          // ... and the multi-step graph
    bool in_loop = false;            // generate_all drives the device state itself
    int32_t* spec_hist = nullptr;    // device [max_seq_len][8]: each run-ahead step's ids
    int32_t* spec_ids = nullptr;     // pinned mirror, copied chunk by chunk
    bool spec_hist_armed = false;    // DecState.hist points at spec_hist
    DecState* hist_host = nullptr;   // pinned staging of the DecState hist fields
    int spec_base = 0, spec_end = 0; // queued steps cover positions [spec_base, spec_end)
    int spec_B = 0;
    int spec_limit = 0x7fffffff;     // l3_set_decode_horizon: no step at or past this position
    // ev0 / ev1 bracket the chunk's graph launch (its device time keeps step_us current while
    // steps are served from the queue; ev0 after any wait for another context's decode graphs),
    // ev follows the ids copy (the chunk is ready)
    struct SpecChunk { int pos0, n; hipEvent_t ev0, ev1, ev; bool done; };
    std::deque<SpecChunk> spec_q;
    std::vector<hipEvent_t> spec_free;  // event pool (timing events)
    int64_t spec_hits = 0;
    // persistent batch-1 decode step (decode_persist.hip): a captured step is one launch of
    // decode_persist_kernel instead of 25 kernels (L3_DECODE_PERSIST; persist_setup)
    void* persist_mem = nullptr;     // per-layer pointer arrays, epoch word, granule slabs
    unsigned* persist_err = nullptr; // host-mapped error word (device writes it on a timeout)
    unsigned* persist_err_dev = nullptr;
    DecodePersistArgs persist{};
    bool persist_ready = false;
    bool persist_graph = false;      // the captured single-step graph runs the persistent step
    // graph-only for the rest of the context's life: a persistent step gave up on a hand-off
    // (persist_recover) or its launch was refused inside a capture (capture_steps)
    bool persist_off = false;
    // spec_resolve queued a guarded undo behind persistent steps without waiting for them: a
    // give-up among them is noticed (and the context turned graph-only) by persist_settle, at the
    // next decode entry point, before any further persistent step is launched
    bool persist_unsettled = false;
    int host_lag = 2;  // forward_dev: host-path lag of the later batch parts (layers; tools/host_path_probe.py)
    int64_t persist_recoveries = 0;  // steps recovered on the graph path (stats)
    hipEvent_t order_ev = nullptr;   // after this context's last decode graph (launch_decode_graph)
};

// ---------------------------------------------------------------------------------------
// join = the context stream waits for an in-flight logits gather: every entry point except
// l3_forward_dev (which waits only before its lm_head) and the gather itself
static int set_dev(l3_ctx* c, bool join = true) {
    HIP_TRY(hipSetDevice(c->device));
    if (join) c->gather_tail = false;
    if (join && c->gather_pending) {
        HIP_TRY(hipStreamWaitEvent(c->stream, c->comm_done_ev, 0));
        c->gather_pending = false;
    }
    return 0;
}

static int spec_resolve(l3_ctx* c);  // undo of a speculative decode step (below)

template <typename F>
static int timed_on(l3_ctx* c, int kind, hipStream_t s, F&& launch) {
    Timer* t = nullptr;
    if (c->timing && (c->timing_mask >> kind & 1u)) {
        if (c->timer_used == c->timers.size()) {
            Timer nt{};
            HIP_TRY(hipEventCreate(&nt.a));
            HIP_TRY(hipEventCreate(&nt.b));
            c->timers.push_back(nt);
        }
        t = &c->timers[c->timer_used++];
        t->kind = kind;
        HIP_TRY(hipEventRecord(t->a, s));
    }
    hipError_t e = launch();
    if (e != hipSuccess) return fail("kernel launch (kind %d) failed: %s", kind, hipGetErrorString(e));
    if (t) HIP_TRY(hipEventRecord(t->b, s));
    return 0;
}

template <typename F>
static int timed(l3_ctx* c, int kind, F&& launch) {
    return timed_on(c, kind, c->stream, launch);
}

static int harvest_timers(l3_ctx* c) {
    if (!c->timer_used) return 0;
    HIP_TRY(hipStreamSynchronize(c->stream));
    for (size_t i = 0; i < c->timer_used; ++i) {
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, c->timers[i].a, c->timers[i].b));
        c->tot_ms[c->timers[i].kind] += ms;
        c->cnt[c->timers[i].kind] += 1;
    }
    c->timer_used = 0;
    return 0;
}

static void dfree(void* p) {
    if (p) (void)hipFree(p);
}

static void drop_decode_graph(l3_ctx* c) {
    if (c->dec_exec) (void)hipGraphExecDestroy(c->dec_exec);
    if (c->dec_graph) (void)hipGraphDestroy(c->dec_graph);
    c->dec_exec = nullptr;
    c->dec_graph = nullptr;
    c->dec_B = 0;
    c->dec_bak = false;
    if (c->dec_exec_n) (void)hipGraphExecDestroy(c->dec_exec_n);
    if (c->dec_graph_n) (void)hipGraphDestroy(c->dec_graph_n);
    c->dec_exec_n = nullptr;
    c->dec_graph_n = nullptr;
    c->dec_n = c->dec_n_B = 0;
}

static int ensure_ws(l3_ctx* c, int64_t B, int64_t L) {
    const int64_t T = B * L;
    if (T <= c->ws_T && B <= c->ws_B) return 0;
    HIP_TRY(hipStreamSynchronize(c->stream));
    c->gather_tail = false;
    drop_decode_graph(c);  // the captured graph holds workspace pointers
    dfree(c->h); dfree(c->q); dfree(c->attn); dfree(c->hid); dfree(c->logits);
    dfree(c->ids); dfree(c->amax); dfree(c->oparts); dfree(c->amax_part); dfree(c->hsum); dfree(c->amax_rows);
    c->amax_rows = nullptr;
    c->oparts = nullptr;
    c->hsum = nullptr;
    c->amax_part = nullptr;
    const int64_t Tn = T > c->ws_T ? T : c->ws_T;
    const int64_t Bn = B > c->ws_B ? B : c->ws_B;
    const int64_t D = c->d.dim;
    HIP_TRY(hipMalloc(&c->h, Tn * D * 4));
    HIP_TRY(hipMalloc(&c->q, Tn * c->qdim * 4));
    HIP_TRY(hipMalloc(&c->attn, Tn * c->qdim * 4));
    HIP_TRY(hipMalloc(&c->hid, Tn * (int64_t)c->d.hidden_dim * 4));
    HIP_TRY(hipMalloc(&c->logits, Bn * (int64_t)c->d.vocab_size * 4));
    HIP_TRY(hipMalloc(&c->ids, Tn * 4));
    HIP_TRY(hipMalloc(&c->amax, Bn * 4));
    if (c->d.n_heads <= GEMV_MAXP && D <= 1024) {
        HIP_TRY(hipMalloc(&c->oparts, (int64_t)8 * c->d.n_heads * D * 4));
        HIP_TRY(hipMalloc(&c->hsum, (int64_t)8 * D * 4));
    }
    HIP_TRY(hipMalloc(&c->amax_part, ((int64_t)c->d.vocab_size / 4 + 64) * sizeof(ArgmaxPart)));
    HIP_TRY(hipMalloc(&c->amax_rows, Bn * (((int64_t)c->d.vocab_size + 63) / 64) * sizeof(ArgmaxPart)));
    if (!c->skws && (c->d.dim >= 2048 || c->d.hidden_dim >= 2048)) {
        c->skws_cap = (int64_t)16 << 20;  // 64 MB: gate|up at M = 256 in 2 slices fits
        HIP_TRY(hipMalloc(&c->skws, c->skws_cap * 4));
    }
    c->ws_T = Tn;
    c->ws_B = Bn;
    return 0;
}

// ---------------------------------------------------------------------------------------
extern "C" const char* l3_last_error(void) { return g_err.c_str(); }

extern "C" int l3_version(int32_t* major, int32_t* minor) {
    if (major) *major = 0;
    if (minor) *minor = 15;
    return 0;
}

#ifndef L3_SRC_HASH
#define L3_SRC_HASH "unknown"
#endif
// sha256 prefix of the sources this library was built from (Makefile SRC_HASH)
extern "C" const char* l3_source_hash(void) { return L3_SRC_HASH; }

extern "C" int l3_device_count(int32_t* n) {
    int k = 0;
    HIP_TRY(hipGetDeviceCount(&k));
    *n = k;
    return 0;
}

// Persistent decode steps need every CU of their device at once (decode_persist.hip): two running
// together — decode graphs of two contexts on one device, e.g. two models' lazy generators
// interleaved, each queued steps ahead — would each hold part of the CUs and wait for the rest
// until their bounded spins fail.  So the decode graphs of a device's contexts are ordered: each
// waits for the last one another context queued.
namespace {
struct DevOrder {
    std::mutex m;
    const l3_ctx* owner = nullptr;  // the context that queued the last decode graph
    hipEvent_t ev = nullptr;        // its order_ev, recorded after that graph
};
DevOrder g_order[64];
}  // namespace

// before (optional): recorded between that wait and the graph, so a timing pair around the graph
// does not count another context's queued decode work
static int launch_decode_graph(l3_ctx* c, hipGraphExec_t g, hipEvent_t before = nullptr) {
    DevOrder& d = g_order[c->device & 63];
    std::lock_guard<std::mutex> lk(d.m);
    if (d.ev && d.owner != c) HIP_TRY(hipStreamWaitEvent(c->stream, d.ev, 0));
    if (before) HIP_TRY(hipEventRecord(before, c->stream));
    HIP_TRY(hipGraphLaunch(g, c->stream));
    // recorded even while this is the device's only context: one created later must still wait
    // for the graphs this one has already queued (run-ahead)
    if (!c->order_ev) HIP_TRY(hipEventCreateWithFlags(&c->order_ev, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(c->order_ev, c->stream));
    d.ev = c->order_ev;
    d.owner = c;
    return 0;
}

extern "C" int l3_create(int32_t device, const l3_dims* dims, l3_ctx** out) {
    if (!dims || !out) return fail("l3_create: null argument");
    const l3_dims& d = *dims;
    if (d.dim <= 0 || d.n_heads <= 0 || d.n_kv_heads <= 0 || d.dim % d.n_heads)
        return fail("l3_create: bad dims (dim %d, heads %d)", d.dim, d.n_heads);
    if (d.n_heads % d.n_kv_heads) return fail("l3_create: n_heads %% n_kv_heads != 0");
    const int HD = d.dim / d.n_heads;
    if (d.n_layers > 0 && (HD % 16 || d.dim % 32 || d.hidden_dim % 32))
        return fail("l3_create: need head_dim %% 16 == 0, dim %% 32 == 0, hidden %% 32 == 0 "
                    "(got HD %d, D %d, FD %d)", HD, d.dim, d.hidden_dim);
    if (d.n_layers > 0 && !(HD == 16 || HD == 32 || HD == 48 || HD == 64 || HD == 96 || HD == 128))
        return fail("l3_create: head_dim %d has no attention instantiation (16, 32, 48, 64, 96, 128)", HD);
    if (d.n_layers > 0 && d.vocab_size % 4)  // logits rows leave the lm_head GEMM as 16-byte stores
        return fail("l3_create: vocab_size %d must be a multiple of 4", d.vocab_size);
    l3_ctx* c = new l3_ctx();
    c->device = device;
    c->d = d;
    c->prune_last = env_knob("L3_LAST_LAYER_ALL_ROWS", 0) == 0;
    c->gemm_x6 = env_knob("L3_GEMM_X6", 0) != 0;
    {  // batch-split default for new contexts
        const int n = env_knob("L3_BATCH_SPLIT", c->split);
        c->split = n < 1 ? 1 : n > l3_ctx::MAX_PARTS ? l3_ctx::MAX_PARTS : n;
    }
    c->HD = HD;
    c->qdim = d.n_heads * HD;
    c->kvdim = d.n_kv_heads * HD;
    c->qkvn = c->qdim + 2 * c->kvdim;
    auto bail = [&](int rc) { l3_destroy(c); return rc; };
    if (set_dev(c)) return bail(1);
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&c->fork_ev, hipEventDisableTiming) != hipSuccess)
        return bail(fail("hipStreamCreate / hipEventCreate failed"));
    for (int i = 0; i < l3_ctx::MAX_PARTS - 1; ++i)
        if (hipStreamCreateWithFlags(&c->aux[i], hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&c->join_ev[i], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&c->lag_ev[i], hipEventDisableTiming) != hipSuccess)
            return bail(fail("hipStreamCreate / hipEventCreate failed"));
    c->layers.resize(d.n_layers > 0 ? d.n_layers : 0);
    if (d.n_layers > 0) {
        const int64_t D = d.dim, FD = d.hidden_dim;
        const int64_t cache = (int64_t)d.max_batch_size * d.n_kv_heads * d.max_seq_len * HD * 4;
        for (auto& L : c->layers) {
            if (hipMalloc(&L.wqkv, c->qkvn * D * 4) || hipMalloc(&L.wo, D * c->qdim * 4) ||
                hipMalloc(&L.wgu, 2 * FD * D * 4) || hipMalloc(&L.wd, D * FD * 4) ||
                hipMalloc(&L.n_attn, D * 4) || hipMalloc(&L.n_ffn, D * 4) ||
                hipMalloc(&L.cache_k, cache) || hipMalloc(&L.cache_v, cache))
                return bail(fail("l3_create: out of device memory (layers)"));
            if (hipMemset(L.cache_k, 0, cache) || hipMemset(L.cache_v, 0, cache))
                return bail(fail("l3_create: memset failed"));
        }
        const int64_t VD = (int64_t)d.vocab_size * D;
        if (VD > 0 && (hipMalloc(&c->emb, VD * 4) || hipMalloc(&c->lm_head, VD * 4) ||
                       hipMalloc(&c->final_norm, D * 4)))
            return bail(fail("l3_create: out of device memory (embedding / lm_head)"));
        // RoPE tables: llama3.py:31-38 in double, then fp32
        const int half = HD / 2;
        std::vector<float> cs((size_t)d.max_seq_len * half), sn(cs.size());
        for (int t = 0; t < d.max_seq_len; ++t)
            for (int i = 0; i < half; ++i) {
                const double inv = 1.0 / std::pow(10000.0, (double)(2 * i) / (double)HD);
                const double a = (double)t * inv;
                cs[(size_t)t * half + i] = (float)std::cos(a);
                sn[(size_t)t * half + i] = (float)std::sin(a);
            }
        if (hipMalloc(&c->rope_cos, cs.size() * 4) || hipMalloc(&c->rope_sin, sn.size() * 4) ||
            hipMemcpy(c->rope_cos, cs.data(), cs.size() * 4, hipMemcpyHostToDevice) ||
            hipMemcpy(c->rope_sin, sn.data(), sn.size() * 4, hipMemcpyHostToDevice))
            return bail(fail("l3_create: rope table upload failed"));
    }
    *out = c;
    return 0;
}

extern "C" int l3_destroy(l3_ctx* c) {
    if (!c) return 0;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->comm_stream) (void)hipStreamSynchronize(c->comm_stream);
    if (c->comm && c->comm_owned) ncclCommDestroy(c->comm);
    if (c->comm_stream) (void)hipStreamDestroy(c->comm_stream);
    if (c->comm_fwd_ev) (void)hipEventDestroy(c->comm_fwd_ev);
    if (c->comm_done_ev) (void)hipEventDestroy(c->comm_done_ev);
    for (auto& L : c->layers) {
        dfree(L.wqkv); dfree(L.wo); dfree(L.wgu); dfree(L.wd); dfree(L.n_attn); dfree(L.n_ffn);
        dfree(L.cache_k); dfree(L.cache_v);
        dfree(L.wqkv3); dfree(L.wo3); dfree(L.wgu3); dfree(L.wd3);
    }
    dfree(c->emb); dfree(c->lm_head); dfree(c->final_norm); dfree(c->rope_cos); dfree(c->rope_sin);
    dfree(c->h); dfree(c->q); dfree(c->attn); dfree(c->hid); dfree(c->logits); dfree(c->ids);
    dfree(c->oparts); dfree(c->amax_part); dfree(c->hsum); dfree(c->skws); dfree(c->amax_rows);
    dfree(c->amax); dfree(c->gather_ids);
    if (c->ids_pin) (void)hipHostFree(c->ids_pin);
    for (void* p : c->scratch) dfree(p);
    for (auto& t : c->timers) { (void)hipEventDestroy(t.a); (void)hipEventDestroy(t.b); }
    drop_decode_graph(c);
    dfree(c->dec_ids); dfree(c->dec_state); dfree(c->kv_bak);
    if (c->dec_host) (void)hipHostFree(c->dec_host);
    for (auto& q : c->spec_q) { (void)hipEventDestroy(q.ev0); (void)hipEventDestroy(q.ev1); (void)hipEventDestroy(q.ev); }
    for (hipEvent_t e : c->spec_free) (void)hipEventDestroy(e);
    dfree(c->spec_hist);
    {
        DevOrder& o = g_order[c->device & 63];
        std::lock_guard<std::mutex> lk(o.m);
        if (o.owner == c) { o.owner = nullptr; o.ev = nullptr; }
    }
    if (c->order_ev) (void)hipEventDestroy(c->order_ev);
    dfree(c->persist_mem);
    dfree(c->persist.stamps);
    if (c->persist_err) (void)hipHostFree(c->persist_err);
    if (c->spec_ids) (void)hipHostFree(c->spec_ids);
    if (c->hist_host) (void)hipHostFree(c->hist_host);
    for (int i = 0; i < l3_ctx::MAX_PARTS - 1; ++i) {
        if (c->aux[i]) { (void)hipStreamSynchronize(c->aux[i]); (void)hipStreamDestroy(c->aux[i]); }
        if (c->join_ev[i]) (void)hipEventDestroy(c->join_ev[i]);
    }
    if (c->fork_ev) (void)hipEventDestroy(c->fork_ev);
    for (hipEvent_t e : c->lag_ev)
        if (e) (void)hipEventDestroy(e);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return 0;
}

static int expect_shape(int kind, int64_t rows, int64_t cols, int64_t er, int64_t ec) {
    if (rows != er || cols != ec)
        return fail("l3_upload_weight: kind %d has shape [%lld, %lld], expected [%lld, %lld]", kind,
                    (long long)rows, (long long)cols, (long long)er, (long long)ec);
    return 0;
}

extern "C" int l3_upload_weight(l3_ctx* c, int32_t layer, int32_t kind, const float* host,
                                int64_t rows, int64_t cols) {
    CHECK_CTX(c);
    if (!host) return fail("l3_upload_weight: null host pointer");
    if (c->finalized) return fail("l3_upload_weight: context already finalized");
    if (set_dev(c)) return 1;
    const int64_t D = c->d.dim, FD = c->d.hidden_dim, VS = c->d.vocab_size;
    if ((kind == L3_W_EMBED || kind == L3_W_LM_HEAD || kind == L3_W_FINAL_NORM) && VS == 0)
        return fail("l3_upload_weight: layer-only context (vocab_size 0) takes no kind %d", kind);
    const bool per_layer = kind >= L3_W_Q && kind <= L3_W_FFN_NORM;
    if (per_layer && (layer < 0 || layer >= (int)c->layers.size()))
        return fail("l3_upload_weight: layer %d out of range [0, %d)", layer, (int)c->layers.size());
    Layer* L = per_layer ? &c->layers[layer] : nullptr;
    auto h2d = [&](float* dst, int64_t n) -> int {
        HIP_TRY(hipMemcpy(dst, host, n * 4, hipMemcpyHostToDevice));
        return 0;
    };
    switch (kind) {
        case L3_W_EMBED:
            if (expect_shape(kind, rows, cols, VS, D) || h2d(c->emb, VS * D)) return 1;
            c->have_emb = true;
            return 0;
        case L3_W_LM_HEAD:
            if (expect_shape(kind, rows, cols, VS, D) || h2d(c->lm_head, VS * D)) return 1;
            c->have_lm = true;
            return 0;
        case L3_W_FINAL_NORM:
            if (expect_shape(kind, rows, cols, 1, D) || h2d(c->final_norm, D)) return 1;
            c->have_fnorm = true;
            return 0;
        case L3_W_Q:
            if (expect_shape(kind, rows, cols, c->qdim, D) || h2d(L->wqkv, c->qdim * D)) return 1;
            break;
        case L3_W_K:
            if (expect_shape(kind, rows, cols, c->kvdim, D) || h2d(L->wqkv + c->qdim * D, c->kvdim * D))
                return 1;
            break;
        case L3_W_V:
            if (expect_shape(kind, rows, cols, c->kvdim, D) ||
                h2d(L->wqkv + (c->qdim + c->kvdim) * D, c->kvdim * D))
                return 1;
            break;
        case L3_W_O:
            if (expect_shape(kind, rows, cols, D, c->qdim) || h2d(L->wo, D * c->qdim)) return 1;
            break;
        case L3_W_GATE:
        case L3_W_UP: {
            if (expect_shape(kind, rows, cols, FD, D)) return 1;
            // 16-row groups: fused row 32g + c <- gate row 16g + c, fused row 32g + 16 + c <- up
            float* dst = L->wgu + (kind == L3_W_UP ? 16 * D : 0);
            HIP_TRY(hipMemcpy2D(dst, 32 * D * 4, host, 16 * D * 4, 16 * D * 4, FD / 16,
                                hipMemcpyHostToDevice));
            break;
        }
        case L3_W_DOWN:
            if (expect_shape(kind, rows, cols, D, FD) || h2d(L->wd, D * FD)) return 1;
            break;
        case L3_W_ATTN_NORM:
            if (expect_shape(kind, rows, cols, 1, D) || h2d(L->n_attn, D)) return 1;
            break;
        case L3_W_FFN_NORM:
            if (expect_shape(kind, rows, cols, 1, D) || h2d(L->n_ffn, D)) return 1;
            break;
        default:
            return fail("l3_upload_weight: unknown kind %d", kind);
    }
    L->have |= 1u << kind;
    return 0;
}

// Weight kinds each entry point needs (bit = l3_weight_kind).
static const unsigned NEED_ATTN = (1u << L3_W_Q) | (1u << L3_W_K) | (1u << L3_W_V) | (1u << L3_W_O);
static const unsigned NEED_LAYER = NEED_ATTN | (1u << L3_W_GATE) | (1u << L3_W_UP) |
                                   (1u << L3_W_DOWN) | (1u << L3_W_ATTN_NORM) | (1u << L3_W_FFN_NORM);

// the x6 pieces of every layer weight (gemm_x6.h), from the weights as the GEMMs use them
// (after the RMSNorm fold); free_x6 drops them
static void free_x6(l3_ctx* c) {
    for (auto& L : c->layers) {
        dfree(L.wqkv3); dfree(L.wo3); dfree(L.wgu3); dfree(L.wd3);
        L.wqkv3 = L.wo3 = L.wgu3 = L.wd3 = nullptr;
    }
}

static int make_x6(l3_ctx* c) {
    const int64_t D = c->d.dim, FD = c->d.hidden_dim;
    hipError_t e = hipSuccess;
    for (auto& L : c->layers) {
        if (L.wqkv3) continue;
        if (hipMalloc(&L.wqkv3, c->qkvn * D * 6) || hipMalloc(&L.wo3, D * c->qdim * 6) ||
            hipMalloc(&L.wgu3, 2 * FD * D * 6) || hipMalloc(&L.wd3, D * FD * 6)) {
            free_x6(c);
            return fail("l3_set_gemm_x6: out of device memory (1.5x the layer weights)");
        }
        if (e == hipSuccess) e = launch_split_planes(L.wqkv, L.wqkv3, c->qkvn, (int)D, c->stream);
        if (e == hipSuccess) e = launch_split_planes(L.wo, L.wo3, D, c->qdim, c->stream);
        if (e == hipSuccess) e = launch_split_planes(L.wgu, L.wgu3, 2 * FD, (int)D, c->stream);
        if (e == hipSuccess) e = launch_split_planes(L.wd, L.wd3, D, (int)FD, c->stream);
    }
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) {  // no half-made pieces: the GEMMs run on them as soon as they exist
        (void)hipStreamSynchronize(c->stream);
        free_x6(c);
        return fail("l3_set_gemm_x6: making the weight pieces failed: %s", hipGetErrorString(e));
    }
    return 0;
}

// Switching the path: queued run-ahead decode steps are settled first and the captured decode
// graphs dropped (their launches hold the weight pointers, the pieces included), so no replay
// can read freed pieces or run the other arithmetic; a failure leaves the fp32 path on
extern "C" int l3_set_gemm_x6(l3_ctx* c, int32_t on) {
    CHECK_CTX(c);
    if (set_dev(c) || spec_resolve(c)) return 1;
    HIP_TRY(hipStreamSynchronize(c->stream));
    drop_decode_graph(c);
    if (!on) {
        c->gemm_x6 = false;
        free_x6(c);
        return 0;
    }
    c->gemm_x6 = true;
    if (c->finalized && make_x6(c)) {  // else l3_finalize makes them
        c->gemm_x6 = false;
        return 1;
    }
    return 0;
}

extern "C" int l3_finalize(l3_ctx* c) {
    CHECK_CTX(c);
    if (c->finalized) return 0;
    if (set_dev(c)) return 1;
    // Fold each RMSNorm weight into the columns of the GEMM that consumes the normalised rows
    // (attention norm -> wqkv, FFN norm -> wgu, final norm -> lm_head): the GEMMs then apply
    // only the per-row 1/rms factor.  Only where both were uploaded: a layer-only (attention)
    // context keeps its raw projections.
    const int D = c->d.dim;
    const unsigned QKV = (1u << L3_W_Q) | (1u << L3_W_K) | (1u << L3_W_V);
    const unsigned GU = (1u << L3_W_GATE) | (1u << L3_W_UP);
    for (auto& L : c->layers) {
        if ((L.have & QKV) == QKV && (L.have & (1u << L3_W_ATTN_NORM))) {
            HIP_TRY(launch_fold_cols(L.wqkv, c->qkvn, D, L.n_attn, c->stream));
            L.folded_qkv = true;
        }
        if ((L.have & GU) == GU && (L.have & (1u << L3_W_FFN_NORM))) {
            HIP_TRY(launch_fold_cols(L.wgu, 2 * (int64_t)c->d.hidden_dim, D, L.n_ffn, c->stream));
            L.folded_gu = true;
        }
    }
    if (c->have_lm && c->have_fnorm) {
        HIP_TRY(launch_fold_cols(c->lm_head, c->d.vocab_size, D, c->final_norm, c->stream));
        c->folded_lm = true;
    }
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (c->gemm_x6 && make_x6(c)) {  // asked for (L3_GEMM_X6) and not made: fail, pieces freed
        c->gemm_x6 = false;
        return 1;
    }
    c->finalized = true;
    return 0;
}

static int need_layer(l3_ctx* c, int li, unsigned mask) {
    const Layer& L = c->layers[li];
    if ((L.have & mask) != mask)
        return fail("layer %d is missing weights (have 0x%x, need 0x%x)", li, L.have, mask);
    if (mask == NEED_LAYER && !(L.folded_qkv && L.folded_gu))
        return fail("layer %d: norm weights not folded (l3_finalize before any forward)", li);
    return 0;
}

static int need_model(l3_ctx* c) {
    if (!c->have_emb || !c->have_lm || !c->have_fnorm)
        return fail("model forward needs embedding, lm_head and final norm uploaded");
    for (int i = 0; i < (int)c->layers.size(); ++i)
        if (need_layer(c, i, NEED_LAYER)) return 1;
    return 0;
}

extern "C" int l3_reset_cache(l3_ctx* c) {
    CHECK_CTX(c);
    if (set_dev(c)) return 1;
    for (auto& q : c->spec_q) c->spec_free.insert(c->spec_free.end(), {q.ev0, q.ev1, q.ev});  // cache cleared
    c->spec_q.clear();
    c->spec_base = c->spec_end = 0;
    c->dec_pos_mirror = -1;
    const int64_t cache = (int64_t)c->d.max_batch_size * c->d.n_kv_heads * c->d.max_seq_len * c->HD * 4;
    for (auto& L : c->layers) {
        HIP_TRY(hipMemsetAsync(L.cache_k, 0, cache, c->stream));
        HIP_TRY(hipMemsetAsync(L.cache_v, 0, cache, c->stream));
    }
    HIP_TRY(hipStreamSynchronize(c->stream));
    return 0;
}

// ---------------------------------------------------------------------------------------
static int check_call(l3_ctx* c, int B, int L, int start_pos) {
    if (!c->finalized) return fail("forward before l3_finalize");
    if (B <= 0 || L <= 0) return fail("empty input: B=%d L=%d", B, L);
    // the reference fails (broadcast error) in both cases: cache[:B] has max_batch_size rows
    // (llama3.py:184) and freqs/cache slices stop at max_seq_len (:184, :289)
    if (c->layers.empty()) return fail("op-only context has no layers");
    if (B > c->d.max_batch_size)
        return fail("batch %d exceeds max_batch_size %d", B, c->d.max_batch_size);
    if (start_pos < 0 || start_pos + L > c->d.max_seq_len)
        return fail("positions [%d, %d) exceed max_seq_len %d", start_pos, start_pos + L,
                    c->d.max_seq_len);
    return 0;
}

// one transformer block on the residual stream c->h [B*L, D] (llama3.py:239-261)
// emb_ids: layer 0 of a model forward reads its input rows straight from the embedding table
// (llama3.py:287 fused into the QKV GEMM's A gather and the O-proj's residual), so no embed
// kernel runs and h is first written by that O-proj
// last_rows (a model forward's last layer, L > 1): only the last position of each sequence
// reaches the output (llama3.py:304 keeps h[:, -1] of the last block), so after the QKV GEMM —
// which still appends every position's K / V to the cache, and past 256 rows computes q for the
// last rows only (a second, B-row QKV GEMM; the attention then runs the decode kernel, one
// query per sequence), else the last q-blocks of the prefill attention — and the O-proj, gate|up
// and down run on B rows instead of B*L: the logits and every cache slot are what the full
// layer gives (the other rows of h are never read again: the next forward starts from the
// embedding).  Those GEMMs always take the skinny MFMA kernel, whose rows round the same way
// at any M, so a batch split still gives bit-identical logits
static int run_layer(l3_ctx* c, int li, int B, int L, int start_pos, const int* pos_dev = nullptr,
                     const int32_t* emb_ids = nullptr, int b0 = 0, hipStream_t s = nullptr,
                     bool last_rows = false) {
    // rows [b0, b0 + B) of the batch on stream s: every buffer is offset to batch row b0
    if (!s) s = c->stream;
    Layer& Ly = c->layers[li];
    const int64_t T = (int64_t)B * L, r0 = (int64_t)b0 * L;
    const int D = c->d.dim, FD = c->d.hidden_dim;
    const int64_t cache0 = (int64_t)b0 * c->d.n_kv_heads * c->d.max_seq_len * c->HD;
    float* h = c->h + r0 * D;
    float* q = c->q + r0 * c->qdim;
    float* attn = c->attn + r0 * c->qdim;
    float* hid = c->hid + r0 * FD;
    if (emb_ids) emb_ids += r0;
    GemmArgs g{};
    g.eps = c->d.norm_eps;
    // rmsnorm -> QKV -> RoPE -> q + KV-cache append
    g.A = h; g.lda = D; g.W = Ly.wqkv; g.C = nullptr; g.ldc = 0;
    g.M = (int)T; g.N = c->qkvn; g.K = D; g.norm = true;  // n_attn folded into wqkv
    g.q_out = q; g.cache_k = Ly.cache_k + cache0; g.cache_v = Ly.cache_v + cache0;
    g.rope_cos = c->rope_cos; g.rope_sin = c->rope_sin;
    g.L = L; g.start_pos = start_pos; g.H = c->d.n_heads; g.KVH = c->d.n_kv_heads; g.HD = c->HD;
    g.Smax = c->d.max_seq_len;
    g.pos_dev = pos_dev;
    g.q_scale = (float)(1.4426950408889634 / std::sqrt((double)c->HD));
    if (emb_ids) { g.A = c->emb; g.a_rows = emb_ids; }
    if (emb_ids && c->fold_in) {  // the id comes from the previous step's lm_head partials
        g.a_rows = nullptr;
        g.amax_in = c->amax_part; g.amax_in_n = c->fold_n;
        g.amax_ids = c->dec_ids; g.amax_st = c->dec_state;  // read by gate|up / O-proj below
    }
    if (c->bak_capture) g.kv_bak = c->kv_bak + (int64_t)li * KV_BAK_SLOTS * 2 * 8 * c->d.n_kv_heads * c->HD;
    // split-K workspace: one, for the GEMMs on c->stream (a batch split's parts keep > 256 rows,
    // past launch_split's range, so no two streams ever share it)
    float* skws = s == c->stream ? c->skws : nullptr;
    g.ws = skws; g.ws_cap = c->skws_cap;
    const bool prune = last_rows && L > 1 && !emb_ids && !pos_dev;
    // a pruned block with more than 256 rows (the tiled QKV kernel): K / V for every row, q for
    // the last row of each sequence only (its RoPE at position start_pos + L - 1)
    const bool kv_only = prune && T > 256;
    g.W3 = Ly.wqkv3;  // null unless the x6 path is on (then launch_gemm takes it past 32 rows)
    if (kv_only) {
        g.W = Ly.wqkv + (int64_t)c->qdim * D; g.N = 2 * c->kvdim; g.col_base = c->qdim;
        if (g.W3) g.W3 += (int64_t)c->qdim * 3 * D;
    }
    if (timed_on(c, L3_K_QKV, s, [&] { return launch_gemm(EPI_QKV, g, s); })) return 1;
    if (prune) {
        const int D4 = D;
        float* hl = h + (int64_t)(L - 1) * D4;  // row b's last position: hl + b * L * D
        AttnArgs a{};
        a.cache_k = Ly.cache_k + cache0; a.cache_v = Ly.cache_v + cache0; a.out = attn;
        a.H = c->d.n_heads; a.KVH = c->d.n_kv_heads; a.HD = c->HD; a.Smax = c->d.max_seq_len;
        GemmArgs o{};  // O-proj + residual on the last rows, in place on h
        if (kv_only) {
            GemmArgs gq = g;  // q of the last rows: [B, qdim], compact
            gq.A = hl; gq.lda = (int64_t)L * D4; gq.W = Ly.wqkv; gq.W3 = nullptr; gq.N = c->qdim; gq.col_base = 0;
            gq.M = B; gq.L = 1; gq.start_pos = start_pos + L - 1; gq.force_skinny = true;
            gq.ws = nullptr;
            if (timed_on(c, L3_K_QKV, s, [&] { return launch_gemm(EPI_QKV, gq, s); })) return 1;
            a.q = q; a.B = B; a.L = 1; a.start_pos = start_pos + L - 1;  // one query per sequence
            if (timed_on(c, L3_K_ATTN, s, [&] { return launch_attention(a, s); })) return 1;
            o.A = attn; o.lda = c->qdim;
        } else {  // the last q-blocks of the full launch (same per-query arithmetic)
            a.q = q; a.B = B; a.L = L; a.start_pos = start_pos;
            if (timed_on(c, L3_K_ATTN, s, [&] { return launch_attention_last(a, s); })) return 1;
            o.A = attn + (int64_t)(L - 1) * c->qdim; o.lda = (int64_t)L * c->qdim;
        }
        o.W = Ly.wo; o.C = hl; o.ldc = (int64_t)L * D4;
        o.M = B; o.N = D4; o.K = c->qdim; o.norm = false; o.force_skinny = true;
        if (timed_on(c, L3_K_OPROJ, s, [&] { return launch_gemm(EPI_RESID, o, s); })) return 1;
        GemmArgs gl{};  // rmsnorm -> gate|up -> SwiGLU on the last rows
        gl.A = hl; gl.lda = (int64_t)L * D4; gl.W = Ly.wgu; gl.C = hid; gl.ldc = FD;
        gl.M = B; gl.N = 2 * FD; gl.K = D4; gl.norm = true; gl.eps = c->d.norm_eps; gl.force_skinny = true;
        if (timed_on(c, L3_K_GATEUP, s, [&] { return launch_gemm(EPI_SWIGLU, gl, s); })) return 1;
        GemmArgs dl{};  // down + residual on the last rows
        dl.A = hid; dl.lda = FD; dl.W = Ly.wd; dl.C = hl; dl.ldc = (int64_t)L * D4;
        dl.M = B; dl.N = D4; dl.K = FD; dl.norm = false; dl.force_skinny = true;
        return timed_on(c, L3_K_DOWN, s, [&] { return launch_gemm(EPI_RESID, dl, s); });
    }
    GemmArgs gu{};  // rmsnorm -> gate|up -> SwiGLU
    gu.A = h; gu.lda = D; gu.W = Ly.wgu; gu.W3 = Ly.wgu3; gu.C = hid; gu.ldc = FD;
    gu.M = (int)T; gu.N = 2 * FD; gu.K = D; gu.norm = true;  // n_ffn folded into wgu
    gu.eps = c->d.norm_eps;
    GemmArgs dn{};  // down + residual
    dn.A = hid; dn.lda = FD; dn.W = Ly.wd; dn.W3 = Ly.wd3; dn.C = h; dn.ldc = D;
    dn.M = (int)T; dn.N = D; dn.K = FD; dn.norm = false;
    gu.ws = dn.ws = skws; gu.ws_cap = dn.ws_cap = c->skws_cap;
    // Batch-1 decode: the O-proj rides in the attention launch as per-head partial rows, which
    // gate|up adds to its input and down to its residual (h + attn . Wo^T, llama3.py:211,253),
    // so a step runs one launch per layer fewer (device loop 0.104 -> 0.101 ms/step; at B = 8
    // the redundant attention of the z blocks costs more than the launch: 0.129 -> 0.134, so
    // B > 1 keeps the O-proj GEMV).  L3_DECODE_FUSE_O=0 keeps it at B = 1 too (A/B).
    static const bool fuse_env = env_knob("L3_DECODE_FUSE_O", 1) != 0;
    const bool fuse_o = fuse_env && L == 1 && c->oparts && c->hsum && b0 == 0 && T == 1 && D % 4 == 0 && c->HD % 16 == 0 &&
                        c->d.max_seq_len <= 8192 && gemv_direct(gu) && gemv_direct(dn);
    // causal attention over the cache
    AttnArgs a{};
    a.q = q; a.cache_k = Ly.cache_k + cache0; a.cache_v = Ly.cache_v + cache0; a.out = attn;
    a.B = B; a.L = L; a.start_pos = start_pos; a.H = c->d.n_heads; a.KVH = c->d.n_kv_heads;
    a.HD = c->HD; a.Smax = c->d.max_seq_len; a.pos_dev = pos_dev;
    if (fuse_o) { a.wo = Ly.wo; a.parts = c->oparts; a.D = D; }
    if (timed_on(c, L3_K_ATTN, s, [&] { return launch_attention(a, s); })) return 1;
    if (fuse_o) {
        gu.parts = c->oparts;
        gu.nparts = c->d.n_heads;
        gu.x_out = c->hsum;  // h + attention . Wo^T, summed once by gate|up for down's residual
        dn.res_src = c->hsum;
        if (emb_ids) { gu.A = c->emb; gu.a_rows = emb_ids; }  // layer 0: h is the embedding row
    } else {
        // O-proj + residual (in place on h)
        GemmArgs o{};
        o.A = attn; o.lda = c->qdim; o.W = Ly.wo; o.W3 = Ly.wo3; o.C = h; o.ldc = D;
        o.M = (int)T; o.N = D; o.K = c->qdim; o.norm = false;
        o.ws = skws; o.ws_cap = c->skws_cap;
        if (emb_ids) { o.res_src = c->emb; o.res_rows = emb_ids; }  // h = emb[ids] + attn . Wo^T
        if (timed_on(c, L3_K_OPROJ, s, [&] { return launch_gemm(EPI_RESID, o, s); })) return 1;
    }
    if (timed_on(c, L3_K_GATEUP, s, [&] { return launch_gemm(EPI_SWIGLU, gu, s); })) return 1;
    if (timed_on(c, L3_K_DOWN, s, [&] { return launch_gemm(EPI_RESID, dn, s); })) return 1;
    return 0;
}

// final RMSNorm + lm_head on the last position of rows [b0, b0 + B) (llama3.py:304-307)
static GemmArgs lm_head_args(l3_ctx* c, int B, int L, float* logits_dev, int b0) {
    const int64_t D = c->d.dim, VS = c->d.vocab_size;
    GemmArgs lm{};
    lm.A = c->h + ((int64_t)b0 * L + L - 1) * D; lm.lda = (int64_t)L * D; lm.W = c->lm_head;
    lm.C = logits_dev + (int64_t)b0 * VS; lm.ldc = VS;
    lm.M = B; lm.N = (int)VS; lm.K = (int)D; lm.norm = true;  // final norm folded
    lm.eps = c->d.norm_eps;
    return lm;
}

// batch 1 on the one-row GEMV: each lm_head block also leaves its (value, index) argmax, so a
// greedy step's argmax reads those partials instead of the whole logits row (L3_LM_AMAX=0: off)
static bool lm_amax_on() {
    static const bool on = env_knob("L3_LM_AMAX", 1) != 0;
    return on;
}

static int run_lm_head(l3_ctx* c, int B, int L, float* logits_dev, int b0, hipStream_t s) {
    GemmArgs lm = lm_head_args(c, B, L, logits_dev, b0);
    c->amax_n = lm_amax_on() && b0 == 0 ? gemv_store_blocks(lm) : 0;
    if (c->amax_n) lm.amax_part = c->amax_part;
    if (c->amax_n && c->fold_adv) lm.pos_adv = c->dec_state;
    // a captured batched decode step (ids only): argmax partials per row instead of the logits
    c->amax_rows_n = c->rows_amax && B > 1 && b0 == 0 && !c->amax_n && gemm_store_config(lm) != 0
                         ? (int)((c->d.vocab_size + 63) / 64) : 0;
    if (c->amax_rows_n) { lm.amax_rows = c->amax_rows; lm.amax_nct = c->amax_rows_n; }
    return timed_on(c, L3_K_LMHEAD, s, [&] { return launch_gemm(EPI_STORE, lm, s); });
}

// greedy argmax of the rows the last forward left in c->logits (llama3.py:320): from the
// lm_head's partials when it wrote them; hist_off 1 when that lm_head moved the position on
static hipError_t launch_greedy_argmax(l3_ctx* c, int B, DecState* st, int hist_off = 0) {
    if (c->amax_n && B == 1) return launch_argmax_parts(c->amax_part, c->amax_n, c->dec_ids, c->stream, st, hist_off);
    if (c->amax_rows_n) return launch_argmax_parts(c->amax_rows, c->amax_rows_n, c->dec_ids, c->stream, st, 0, B);
    return launch_argmax(c->logits, B, c->d.vocab_size, c->dec_ids, c->stream, st);
}

// partials the next step's layer-0 QKV reduces when a captured batch-1 step's argmax is folded
// into it (0: no fold).  Every QKV block reads all of them, so only a small vocabulary's
// (stories15M: 2000 partials, 16 KB; the Llama-3 shape's 32k keep the argmax launch).
// L3_DECODE_FOLD_ARGMAX=0: off (A/B)
static int fold_parts(l3_ctx* c, int B) {
    static const bool on = env_knob("L3_DECODE_FOLD_ARGMAX", 1) != 0;
    if (!on || B != 1 || !lm_amax_on() || !c->dec_state) return 0;
    const int n = gemv_store_blocks(lm_head_args(c, 1, 1, c->logits, 0));
    GemmArgs qkv{};
    qkv.M = 1;
    qkv.N = c->qkvn;
    qkv.K = c->d.dim;
    return n > 0 && n <= 4096 && gemv_direct(qkv) ? n : 0;
}


// Batch split of a prefill: rows are independent (llama3.py:163-211), so the layers run as
// c->split row ranges on their own streams and one range's kernels fill another's launch tails
// and kernel boundaries (C3: 7.31 -> 7.04 ms/step at 2 parts; 3 and 4 parts are slower).

// logits_host (optional): each part's rows are copied back on that part's own stream right
// after its lm_head, so part 0's D2H overlaps part 1's last layer and the parts' copies run
// concurrently (two DMA queues); the join below covers them
// host_pitch / host_off (a group member's rows): local row r lands in host row host_off +
// host_pitch * r (the group's interleave, one 2-D copy per part over this member's own link)
static int forward_dev(l3_ctx* c, const int32_t* ids_dev, int B, int L, int start_pos,
                       float* logits_dev, const int* pos_dev = nullptr, float* logits_host = nullptr,
                       int host_pitch = 1, int host_off = 0) {
    // roctx ranges (host-side launch spans; `rocprofv3 --marker-trace`) per block and lm_head
    static const char* names[] = {"l3.layer0", "l3.layer1", "l3.layer2", "l3.layer3", "l3.layer4",
                                  "l3.layer5", "l3.layer6", "l3.layer7", "l3.layerN"};
    // a part keeps more than 256 rows, so every layer GEMM runs the same M-independent MFMA
    // tiles as the unsplit batch (the row-blocked GEMV of short M rounds by row position)
    const int64_t min_part = c->split_min_tokens > 256 ? c->split_min_tokens : 257;
    // ... and only while a layer is short enough for launch tails to matter: past ~1 TFLOP per
    // layer (C5, Llama-3-8B shape: 57 TFLOP) the split measured -0.8 %, at C3 (0.12) +3.9 %
    const double D = c->d.dim, layer_flops = 2.0 * B * L *
        (D * c->qkvn + D * c->qdim + 3.0 * D * c->d.hidden_dim);
    int parts = pos_dev || layer_flops > 1e12 ? 1 : c->split;
    while (parts > 1 && (B < parts || (int64_t)(B / parts) * L < min_part)) --parts;
    int nb[l3_ctx::MAX_PARTS], b0[l3_ctx::MAX_PARTS];
    hipStream_t st[l3_ctx::MAX_PARTS];
    for (int p = 0; p < parts; ++p) {
        b0[p] = (int)((int64_t)B * p / parts);
        nb[p] = (int)((int64_t)B * (p + 1) / parts) - b0[p];
        st[p] = p ? c->aux[p - 1] : c->stream;
    }
    roctxRangePushA("l3.forward");
    // a logits gather queued last on stream (mode 3): the other parts start from the point just
    // before it, so their layers overlap the transfer; part 0 runs after it on stream, and every
    // part's lm_head (the writer of the rows it reads) waits for it below (gather_pending)
    const bool after_gather = c->gather_tail;
    c->gather_tail = false;
    if (parts > 1) {  // the aux streams join the work queued so far on stream
        if (!after_gather) HIP_TRY(hipEventRecord(c->fork_ev, c->stream));
        for (int p = 1; p < parts; ++p)
            HIP_TRY(hipStreamWaitEvent(st[p], after_gather ? c->comm_fwd_ev : c->fork_ev, 0));
    }
    // the lm_head too runs per part when every part picks the unsplit batch's tile (then each
    // part's lm_head overlaps the other parts' last layer); otherwise once after the join
    bool lm_parts = parts > 1;
    const int lm_cfg = gemm_store_config(lm_head_args(c, B, L, logits_dev, 0));
    for (int p = 0; p < parts && lm_parts; ++p)
        lm_parts = gemm_store_config(lm_head_args(c, nb[p], L, logits_dev, b0[p])) == lm_cfg;
    int rc = 0;
    const int nl = (int)c->layers.size();
    // host path (logits_host): the logits copy is PCIe-bound (32.8 MB at C3, ~0.59 ms at 56 GB/s)
    // and can start only once a part's logits exist; in lockstep both parts reach their lm_heads
    // together and the whole copy is exposed.  With lag k part p's last k layers each wait for
    // part p - 1's same layer (a staircase), so the earlier parts reach their lm_heads and start
    // their copies while the later ones still compute (L3_HOST_LAG; lockstep elsewhere:
    // desynchronised parts pack worse)
    const int host_lag_env = env_knob("L3_HOST_LAG", -1);
    const int lag = logits_host && parts > 1 ? (host_lag_env >= 0 ? host_lag_env : c->host_lag) : 0;
    for (int li = 0; li < nl && !rc; ++li) {
        roctxRangePushA(names[li < 8 ? li : 8]);
        for (int p = 0; p < parts && !rc; ++p) {
            if (p > 0 && li >= nl - lag) HIP_TRY(hipStreamWaitEvent(st[p], c->lag_ev[p - 1], 0));
            rc = run_layer(c, li, nb[p], L, start_pos, pos_dev, li == 0 ? ids_dev : nullptr, b0[p], st[p],
                           c->prune_last && li == nl - 1 && li > 0);
            if (!rc && p + 1 < parts && li >= nl - lag) HIP_TRY(hipEventRecord(c->lag_ev[p], st[p]));
        }
        roctxRangePop();
    }
    // the previous step's gather may still read the logits rows: the lm_head streams wait for
    // it (stream joins the parts below, so it has waited too once the forward returns)
    if (c->gather_pending && !rc) {
        for (int p = 0; p < (lm_parts ? parts : 1); ++p) HIP_TRY(hipStreamWaitEvent(st[p], c->comm_done_ev, 0));
        c->gather_pending = false;
    }
    const int64_t VS = c->d.vocab_size;
    auto d2h_rows = [&](int r0, int n, hipStream_t s) -> int {
        if (!logits_host || !n) return 0;
        if (host_pitch == 1) {
            HIP_TRY(hipMemcpyAsync(logits_host + ((int64_t)host_off + r0) * VS, logits_dev + (int64_t)r0 * VS,
                                   (size_t)n * VS * 4, hipMemcpyDeviceToHost, s));
        } else {
            const size_t w = (size_t)VS * 4;
            HIP_TRY(hipMemcpy2DAsync(logits_host + ((int64_t)host_off + (int64_t)host_pitch * r0) * VS,
                                     w * host_pitch, logits_dev + (int64_t)r0 * VS, w, w, (size_t)n,
                                     hipMemcpyDeviceToHost, s));
        }
        return 0;
    };
    roctxRangePushA("l3.lm_head");
    for (int p = 0; p < parts && lm_parts && !rc; ++p) {
        rc = run_lm_head(c, nb[p], L, logits_dev, b0[p], st[p]);
        if (!rc) rc = d2h_rows(b0[p], nb[p], st[p]);
    }
    roctxRangePop();
    for (int p = 1; p < parts; ++p) {  // stream waits for every part: later calls see all rows
        HIP_TRY(hipEventRecord(c->join_ev[p - 1], st[p]));
        HIP_TRY(hipStreamWaitEvent(c->stream, c->join_ev[p - 1], 0));
    }
    roctxRangePushA("l3.lm_head");
    if (!rc && !lm_parts) {
        rc = run_lm_head(c, B, L, logits_dev, 0, c->stream);
        // one lm_head for the batch: its rows still go back as two concurrent copies
        if (!rc && logits_host && B >= 2 && !pos_dev) {
            const int h = B / 2;
            HIP_TRY(hipEventRecord(c->fork_ev, c->stream));
            HIP_TRY(hipStreamWaitEvent(c->aux[0], c->fork_ev, 0));
            rc = d2h_rows(0, h, c->stream);
            if (!rc) rc = d2h_rows(h, B - h, c->aux[0]);
            HIP_TRY(hipEventRecord(c->join_ev[0], c->aux[0]));
            HIP_TRY(hipStreamWaitEvent(c->stream, c->join_ev[0], 0));
        } else if (!rc) {
            rc = d2h_rows(0, B, c->stream);
        }
    }
    roctxRangePop();
    roctxRangePop();
    return rc;
}

// int64 host ids -> int32 device ids through a pinned staging buffer (a DMA copy, no pageable
// bounce); the copy is ordered on stream before the forward, and the staging buffer is next
// rewritten only by a later call, after this call's closing synchronize
static int upload_ids(l3_ctx* c, const int64_t* ids_host, int64_t T) {
    if (T > c->ids_pin_n) {
        if (c->ids_pin) {
            HIP_TRY(hipStreamSynchronize(c->stream));
            HIP_TRY(hipHostFree(c->ids_pin));
            c->ids_pin = nullptr;
            c->ids_pin_n = 0;
        }
        HIP_TRY(hipHostMalloc(&c->ids_pin, (size_t)T * 4, hipHostMallocDefault));
        c->ids_pin_n = T;
    }
    const int64_t VS = c->d.vocab_size;
    // two branch-free passes (both vectorise): the range check, then the NumPy wrap of negatives
    int64_t lo = 0, hi = 0;
    for (int64_t i = 0; i < T; ++i) {
        lo = ids_host[i] < lo ? ids_host[i] : lo;
        hi = ids_host[i] > hi ? ids_host[i] : hi;
    }
    if (lo < -VS || hi >= VS) {  // NumPy fancy indexing raises IndexError here (llama3.py:287)
        for (int64_t i = 0; i < T; ++i)
            if (ids_host[i] < -VS || ids_host[i] >= VS)
                return fail("token id %lld out of range for vocab_size %lld", (long long)ids_host[i], (long long)VS);
    }
    int32_t* const dst = c->ids_pin;
    for (int64_t i = 0; i < T; ++i) {
        const int64_t v = ids_host[i];
        dst[i] = (int32_t)(v + (v < 0 ? VS : 0));  // ...and wraps negatives
    }
    HIP_TRY(hipMemcpyAsync(c->ids, c->ids_pin, T * 4, hipMemcpyHostToDevice, c->stream));
    return 0;
}

extern "C" int l3_set_batch_split(l3_ctx* c, int32_t parts, int64_t min_tokens) {
    CHECK_CTX(c);
    if (parts < 1 || parts > l3_ctx::MAX_PARTS)
        return fail("l3_set_batch_split: parts %d outside [1, %d]", parts, l3_ctx::MAX_PARTS);
    if (min_tokens < 1) return fail("l3_set_batch_split: min_tokens %lld < 1", (long long)min_tokens);
    c->split = parts;
    c->split_min_tokens = min_tokens;
    return 0;
}

extern "C" int l3_set_last_layer_rows(l3_ctx* c, int32_t all_rows) {
    CHECK_CTX(c);
    c->prune_last = all_rows == 0;
    return 0;
}

extern "C" int l3_forward_dev(l3_ctx* c, const int32_t* ids_dev, int32_t B, int32_t L,
                              int32_t start_pos, float* logits_dev) {
    CHECK_CTX(c);
    if (need_model(c) || check_call(c, B, L, start_pos) || set_dev(c, false) || spec_resolve(c) || ensure_ws(c, B, L))
        return 1;
    return forward_dev(c, ids_dev, B, L, start_pos, logits_dev);
}

extern "C" int l3_forward_host(l3_ctx* c, const int64_t* ids_host, int32_t B, int32_t L,
                               int32_t start_pos, float* logits_host) {
    CHECK_CTX(c);
    if (need_model(c) || check_call(c, B, L, start_pos) || set_dev(c) || spec_resolve(c) || ensure_ws(c, B, L))
        return 1;
    if (upload_ids(c, ids_host, (int64_t)B * L)) return 1;
    if (forward_dev(c, c->ids, B, L, start_pos, c->logits, nullptr, logits_host)) return 1;
    HIP_TRY(hipStreamSynchronize(c->stream));
    return 0;
}

// Persistent batch-1 decode step (decode_persist.hip; the default, L3_DECODE_PERSIST=0: the
// 25-kernel graph): the step's shape as the kernel sees it
static DecodePersistArgs persist_shape(const l3_ctx* c) {
    DecodePersistArgs a{};
    a.D = c->d.dim; a.H = c->d.n_heads; a.KVH = c->d.n_kv_heads; a.HD = c->HD; a.FD = c->d.hidden_dim;
    a.VS = c->d.vocab_size; a.n_layers = (int)c->layers.size(); a.Smax = c->d.max_seq_len; a.GL = 64;
    a.Dp = (a.D + 3) & ~3;
    int xp = c->qkvn > a.FD ? c->qkvn : a.FD;
    if (xp < 3 * a.HD) xp = 3 * a.HD;
    if (xp < 512) xp = 512;  // the final argmax's 2 x 256 partials
    a.Xp = (xp + 3) & ~3;
    a.fault_pos = -1;
    return a;
}

// Chosen at every capture (captures are rare, so a process can A/B the paths): the shape, and
// the launch conditions on THIS device — enough CUs for the layer and lm workgroups, every
// workgroup co-resident at the step's LDS (decode_persist_grid) — so a device the step cannot
// run on (e.g. a CPX partition's 32 CUs) captures the 25-kernel graph instead of failing
static bool persist_wanted(l3_ctx* c, int B) {
    const int mode = env_knob("L3_DECODE_PERSIST", 1);
    if (!mode || c->persist_off || B != 1 || c->layers.empty() || !c->dec_state) return false;
    return decode_persist_grid(persist_shape(c)) > 0;
}

// Its buffers, made once with the stream idle
static int persist_setup(l3_ctx* c) {
    if (c->persist_ready) return 0;
    DecodePersistArgs& a = c->persist;
    a = persist_shape(c);
    const int nl = (int)c->layers.size();
    a.eps = c->d.norm_eps;
    a.q_scale = (float)(1.4426950408889634 / std::sqrt((double)c->HD));
    a.emb = c->emb; a.lm_head = c->lm_head; a.rope_cos = c->rope_cos; a.rope_sin = c->rope_sin;
    a.bak_layer = (int64_t)KV_BAK_SLOTS * 2 * 8 * c->d.n_kv_heads * c->HD;
    const int64_t slab = decode_persist_slab(a.H, a.KVH, a.HD, a.D, a.FD);
    const size_t ptr_bytes = (size_t)6 * nl * sizeof(void*);
    const size_t gran_off = (ptr_bytes + 16 + 255) & ~(size_t)255;
    // per-layer slabs, the lm_head partials [2 x 256], the start marks [256], the write marks
    // [GL] (32-bit, in a 256-granule block)
    const size_t gran_bytes = (size_t)(slab * nl + 4 * 256) * 8;
    HIP_TRY(hipMalloc(&c->persist_mem, gran_off + gran_bytes));
    HIP_TRY(hipMemset(c->persist_mem, 0, gran_off + gran_bytes));
    std::vector<const void*> ptrs((size_t)6 * nl);
    for (int i = 0; i < nl; ++i) {
        const Layer& L = c->layers[(size_t)i];
        ptrs[(size_t)i] = L.wqkv; ptrs[(size_t)nl + i] = L.wo; ptrs[(size_t)2 * nl + i] = L.wgu;
        ptrs[(size_t)3 * nl + i] = L.wd; ptrs[(size_t)4 * nl + i] = L.cache_k; ptrs[(size_t)5 * nl + i] = L.cache_v;
    }
    HIP_TRY(hipMemcpy(c->persist_mem, ptrs.data(), ptr_bytes, hipMemcpyHostToDevice));
    char* base = static_cast<char*>(c->persist_mem);
    auto arr = [&](int k) { return reinterpret_cast<void* const*>(base) + (size_t)k * nl; };
    a.wqkv = reinterpret_cast<const float* const*>(arr(0));
    a.wo = reinterpret_cast<const float* const*>(arr(1));
    a.wgu = reinterpret_cast<const float* const*>(arr(2));
    a.wd = reinterpret_cast<const float* const*>(arr(3));
    a.cache_k = reinterpret_cast<float* const*>(arr(4));
    a.cache_v = reinterpret_cast<float* const*>(arr(5));
    a.epoch = reinterpret_cast<unsigned*>(base + ptr_bytes);  // [3] words (16 bytes reserved)
    const unsigned one = 1;  // tag 0 is what the zeroed slabs hold
    HIP_TRY(hipMemcpy(a.epoch, &one, sizeof one, hipMemcpyHostToDevice));
    a.gran = reinterpret_cast<unsigned long long*>(base + gran_off);
    HIP_TRY(hipHostMalloc(&c->persist_err, sizeof(unsigned), hipHostMallocMapped));
    *c->persist_err = 0;
    HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void**>(&c->persist_err_dev), c->persist_err, 0));
    a.err = c->persist_err_dev;
    // diagnostic timeline: L3_DECODE_PERSIST_STAMPS=<file> (tools/persist_stamps.py reads it; written
    // at the end of every l3_greedy_generate_host)
    if (getenv("L3_DECODE_PERSIST_STAMPS")) {
        HIP_TRY(hipMalloc(&a.stamps, (size_t)256 * 128 * 8));
        HIP_TRY(hipMemset(a.stamps, 0, (size_t)256 * 128 * 8));
    }
    c->persist_ready = true;
    return 0;
}

static void persist_dump_stamps(l3_ctx* c) {
    const char* path = getenv("L3_DECODE_PERSIST_STAMPS");
    if (!path || !c->persist.stamps) return;
    std::vector<unsigned long long> h((size_t)256 * 128);
    if (hipMemcpy(h.data(), c->persist.stamps, h.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) return;
    if (FILE* f = fopen(path, "wb")) {
        fwrite(h.data(), 8, h.size(), f);
        fclose(f);
    }
}

// after a synchronised replay / chunk: a persistent step gave up on a hand-off
static bool persist_failed(const l3_ctx* c) {
    return c->persist_err && *reinterpret_cast<volatile unsigned*>(c->persist_err) != 0u;
}

static void spec_drop_queue(l3_ctx* c) {
    for (auto& q : c->spec_q) c->spec_free.insert(c->spec_free.end(), {q.ev0, q.ev1, q.ev});
    c->spec_q.clear();
    c->spec_base = c->spec_end = 0;
}

// The undo's guard for one cache (sec 1: K, 2: V) of the persistent step (kv_restore_kernel)
static KvGuard persist_guard(const l3_ctx* c, int sec) {
    KvGuard g{};
    if (!c->persist_ready || c->spec_B != 1) return g;
    const DecodePersistArgs& a = c->persist;
    const int qdim = a.H * a.HD, kvdim = a.KVH * a.HD, qkvn = qdim + 2 * kvdim;
    g.err = c->persist_err_dev;
    g.epoch = a.epoch;
    g.wmarks = reinterpret_cast<const unsigned*>(a.gran + decode_persist_slab(a.H, a.KVH, a.HD, a.D, a.FD) * a.n_layers +
                                                 3 * 256);
    g.col_base = qdim + (sec - 1) * kvdim;
    g.per = (qkvn / 2 + a.GL - 1) / a.GL;
    return g;
}

// Queue the undo of every run-ahead step nobody has taken (stream-ordered after them): each
// step's K / V slot in every layer back from kv_bak.  Guarded on the device when persistent steps
// may be among them (a step that gave up: nothing from it on, and of it only what its workgroups
// wrote; KvGuard), so the host need not wait for the queue to drain first.
static int spec_undo(l3_ctx* c) {
    const int KVH = c->d.n_kv_heads, HD = c->HD, n = c->spec_B * KVH * HD;
    const bool guard = c->persist_ready && !c->persist_off;
    const KvGuard gk = guard ? persist_guard(c, 1) : KvGuard{}, gv = guard ? persist_guard(c, 2) : KvGuard{};
    for (int pos = c->spec_base; pos < c->spec_end; ++pos) {
        for (size_t li = 0; li < c->layers.size(); ++li) {
            const float* bak = c->kv_bak + (int64_t)li * KV_BAK_SLOTS * 2 * 8 * KVH * HD + (int64_t)(pos % KV_BAK_SLOTS) * 2 * n;
            HIP_TRY(launch_kv_restore(c->layers[li].cache_k, bak, c->spec_B, KVH, c->d.max_seq_len, HD, pos, c->stream, gk));
            HIP_TRY(launch_kv_restore(c->layers[li].cache_v, bak + n, c->spec_B, KVH, c->d.max_seq_len, HD, pos, c->stream, gv));
        }
    }
    spec_drop_queue(c);
    return 0;
}

// Recovery from a persistent step that gave up (decode_persist.hip: its position + 1 in the error
// word, its tag in epoch[2]; every launch queued after it returned at once, the sticky word set).
// With the stream drained: the run-ahead steps nobody has taken are undone (spec_undo: on the
// device, the failed step only where it wrote), the failure words are cleared, and the context
// turns graph-only: its decode graphs are dropped, so the caller's step runs eagerly and the next
// capture is the 25-kernel graph.  *failed_pos: the step to run again.
static int persist_recover(l3_ctx* c, int* failed_pos) {
    HIP_TRY(hipStreamSynchronize(c->stream));
    const int fp = (int)*c->persist_err - 1;
    unsigned w[3] = {0, 0, 0};
    HIP_TRY(hipMemcpy(w, c->persist.epoch, sizeof w, hipMemcpyDeviceToHost));
    if (spec_undo(c)) return 1;  // reads the error word: cleared only after these ran
    const unsigned fresh[3] = {w[0] + 1u, 0u, 0u};  // a tag no granule carries; sticky and failed-tag words cleared
    HIP_TRY(hipMemcpyAsync(c->persist.epoch, fresh, sizeof fresh, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    *c->persist_err = 0;
    c->persist_unsettled = false;
    c->persist_off = true;
    drop_decode_graph(c);
    c->persist_graph = false;
    c->dec_pos_mirror = -1;
    c->persist_recoveries++;
    if (failed_pos) *failed_pos = fp;
    return 0;
}

// A guarded undo was queued without waiting (spec_resolve): before anything launches another
// persistent step, see whether a step it undid had given up, and if so finish the recovery (the
// undo itself has run: nothing is left in the queue)
static int persist_settle(l3_ctx* c) {
    if (!c->persist_unsettled) return 0;
    HIP_TRY(hipStreamSynchronize(c->stream));
    c->persist_unsettled = false;
    return persist_failed(c) ? persist_recover(c, nullptr) : 0;
}

// Capture `steps` consecutive decode steps (B sequences, L = 1), each reading its position from
// dec_pos and its ids from dec_ids; each step's argmax writes the next ids back into dec_ids and
// advances dec_pos, so the steps chain on the device.
static int capture_steps(l3_ctx* c, int B, int steps, hipGraph_t* graph, hipGraphExec_t* exec) {
    const bool timing = c->timing;
    c->timing = false;  // no event records inside the graph
    bool persist = persist_wanted(c, B);
    if (persist && persist_setup(c)) { c->timing = timing; return 1; }
    const int pgrid = persist ? decode_persist_grid(c->persist) : 0;
    persist = pgrid > 0;
    int rc = 0;
    hipGraph_t g = nullptr;
    for (;;) {
        HIP_TRY(hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
        bool refused = false;
        for (int i = 0; i < steps && persist && !rc && !refused; ++i) {  // one launch per step
            DecodePersistArgs a = c->persist;
            a.ids = c->dec_ids;
            a.st = c->dec_state;
            a.kv_bak = c->bak_capture ? c->kv_bak : nullptr;
            a.from_parts = i > 0;            // the previous step in this graph left partials only
            a.write_id = i == steps - 1;     // the last one publishes the id for the host / next graph
            // test-only fault injection (kernels.h): honoured only together with
            // L3_TEST_FAULT_INJECTION=1, so a stray L3_DECODE_PERSIST_FAULT in a user's
            // environment cannot fail a step and switch the context to the graph path
            const bool inject_ok = env_knob("L3_TEST_FAULT_INJECTION", 0) == 1;
            a.fault_pos = inject_ok ? env_knob("L3_DECODE_PERSIST_FAULT", -1) : -1;
            a.fault_wg = env_knob("L3_DECODE_PERSIST_FAULT_WG", 1);
            a.fault_late = env_knob("L3_DECODE_PERSIST_FAULT_LATE", 0);
            refused = launch_decode_persist(a, pgrid, c->stream) != hipSuccess;
        }
        // batch 1 (graph path): each step's argmax folded into the next step's layer-0 QKV, one
        // argmax launch per graph (its last step); the lm_heads move the position on
        const int fold = persist ? 0 : fold_parts(c, B);
        // batched steps: the lm_head leaves per-row argmax partials, not logits (nobody reads a
        // captured step's logits); L3_DECODE_ROWS_AMAX=0 keeps the logits + full-row argmax (A/B)
        static const bool rows_amax = env_knob("L3_DECODE_ROWS_AMAX", 1) != 0;
        for (int i = 0; i < steps && !persist && !rc; ++i) {
            c->fold_in = fold && i > 0;
            c->fold_adv = fold > 0;
            c->fold_n = fold;
            c->rows_amax = rows_amax && B > 1;
            rc = forward_dev(c, c->dec_ids, B, 1, 0, c->logits, c->dec_pos);
            c->fold_in = c->fold_adv = false;
            c->rows_amax = false;
            if (!rc && fold && c->amax_n != fold) rc = fail("decode capture: lm_head partials %d, expected %d", c->amax_n, fold);
            if (!rc && (!fold || i == steps - 1)) {
                hipError_t e = launch_greedy_argmax(c, B, c->dec_state, fold ? 1 : 0);
                if (e != hipSuccess) rc = fail("argmax launch in capture failed: %s", hipGetErrorString(e));
            }
        }
        c->fold_in = c->fold_adv = false;
        c->rows_amax = false;
        g = nullptr;
        const hipError_t e = hipStreamEndCapture(c->stream, &g);
        if (refused) {
            // the persistent launch was refused inside the capture: this context captures the
            // 25-kernel graph from now on (the refusal left no work on the stream)
            if (g) (void)hipGraphDestroy(g);
            (void)hipGetLastError();
            c->persist_off = true;
            persist = false;
            continue;
        }
        if (rc) { if (g) (void)hipGraphDestroy(g); c->timing = timing; return rc; }
        if (e != hipSuccess) { c->timing = timing; return fail("hipStreamEndCapture failed: %s", hipGetErrorString(e)); }
        break;
    }
    c->timing = timing;
    hipError_t e = hipGraphInstantiate(exec, g, nullptr, nullptr, 0);
    if (e != hipSuccess) { (void)hipGraphDestroy(g); return fail("hipGraphInstantiate failed: %s", hipGetErrorString(e)); }
    *graph = g;
    return 0;
}

static bool speculation_on() {
    static const bool on = env_knob("L3_DECODE_SPECULATE", 1) != 0;
    return on;
}

// how many decode steps may be queued ahead: SPEC_AHEAD, fewer when that much work would
// exceed SPEC_BUDGET_US at the measured step time (0 before any step was timed)
static int spec_ahead(const l3_ctx* c) {
    if (c->step_us <= 0.0) return 0;
    const double n = l3_ctx::SPEC_BUDGET_US / c->step_us;
    return n >= l3_ctx::SPEC_AHEAD ? l3_ctx::SPEC_AHEAD : (int)n;
}

// replayed-step time: replaces the eager seed, then an EMA
static void note_step_time(l3_ctx* c, double us) {
    c->step_us = c->step_us > 0.0 && !c->step_us_seed ? 0.75 * c->step_us + 0.25 * us : us;
    c->step_us_seed = false;
}

// the eager first decode step (per-kernel launches, id upload: an upper bound of a replayed
// step) seeds step_us only while nothing better is known
static void seed_step_time(l3_ctx* c, double us) {
    if (c->step_us > 0.0) return;
    c->step_us = us;
    c->step_us_seed = true;
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// B <= 8 with run-ahead on: every QKV of a step runs on the GEMV, whose epilogue keeps the
// overwritten slot (GemmArgs::kv_bak)
static int bak_wanted(l3_ctx* c, int B, bool* bak) {
    GemmArgs qkv{};  // the shape of a decode step's QKV launch: only the GEMV keeps the slot
    qkv.M = B;
    qkv.N = c->qkvn;
    qkv.K = c->d.dim;
    *bak = speculation_on() && B <= 8 && gemm_is_gemv(qkv);
    if (*bak && !c->kv_bak)
        HIP_TRY(hipMalloc(&c->kv_bak, (size_t)c->layers.size() * KV_BAK_SLOTS * 2 * 8 * c->d.n_kv_heads * c->HD * 4));
    return 0;
}

static int capture_decode_graph(l3_ctx* c, int B) {
    drop_decode_graph(c);
    bool bak = false;
    if (bak_wanted(c, B, &bak)) return 1;
    c->bak_capture = bak;
    const int rc = capture_steps(c, B, 1, &c->dec_graph, &c->dec_exec);
    c->bak_capture = false;
    if (rc) return 1;
    c->dec_B = B;
    c->dec_bak = bak;
    c->persist_graph = persist_wanted(c, B);
    return 0;
}

// steps per graph launch in the device loop: L3_DECODE_GRAPH_STEPS (default 8; 1 = one replay
// of the single-step graph per token)
static int decode_graph_steps() {
    static const int n = [] {
        const int v = env_knob("L3_DECODE_GRAPH_STEPS", 8);
        return v < 1 ? 1 : v > 64 ? 64 : v;
    }();
    return n;
}

// the multi-step graph of decode_graph_steps() steps for batch B (device loop and run-ahead)
static int ensure_multi_graph(l3_ctx* c, int B) {
    const int n = decode_graph_steps();
    if (c->dec_n == n && c->dec_n_B == B) return 0;
    if (c->dec_exec_n) (void)hipGraphExecDestroy(c->dec_exec_n);
    if (c->dec_graph_n) (void)hipGraphDestroy(c->dec_graph_n);
    c->dec_exec_n = nullptr;
    c->dec_graph_n = nullptr;
    c->dec_n = c->dec_n_B = 0;
    bool bak = false;
    if (bak_wanted(c, B, &bak)) return 1;
    c->bak_capture = bak;
    const int rc = capture_steps(c, B, n, &c->dec_graph_n, &c->dec_exec_n);
    c->bak_capture = false;
    if (rc) return 1;
    c->dec_n = n;
    c->dec_n_B = B;
    c->dec_n_bak = bak;
    return 0;
}

// Queue decode steps ahead of the caller, from the position the device state will reach next,
// until SPEC_AHEAD are in flight or the horizon (l3_set_decode_horizon, max_seq_len) is reached:
// whole multi-step graphs where they fit, single steps otherwise; each chunk's ids are copied to
// spec_ids behind an event.  Only from a state a step just armed (dec_pos_mirror valid).
static int speculate(l3_ctx* c, int B) {
    if (!speculation_on() || c->in_loop || !c->dec_exec || !c->dec_bak || c->dec_B != B || c->timing ||
        c->dec_pos_mirror < 0)
        return 0;
    const int limit = c->spec_limit < c->d.max_seq_len ? c->spec_limit : c->d.max_seq_len;
    if (c->spec_q.empty()) {
        if (c->dec_pos_mirror >= limit) return 0;
        c->spec_base = c->spec_end = (int)c->dec_pos_mirror;
        c->spec_B = B;
        if (!c->spec_hist) {  // the stream is idle here (the step that armed the state synced)
            HIP_TRY(hipMalloc(&c->spec_hist, (size_t)c->d.max_seq_len * 8 * 4));
            HIP_TRY(hipHostMalloc(&c->spec_ids, (size_t)c->d.max_seq_len * 8 * 4, hipHostMallocDefault));
            HIP_TRY(hipHostMalloc(&c->hist_host, sizeof(DecState), hipHostMallocDefault));
        }
        if (ensure_multi_graph(c, B)) return 1;  // captured while the stream is idle
        if (!c->spec_hist_armed) {  // argmax records every step's ids at row pos of spec_hist
            c->hist_host->hist_base = 0;
            c->hist_host->hist_cap = c->d.max_seq_len;
            c->hist_host->arrive = 0;
            c->hist_host->hist = c->spec_hist;
            const size_t off = offsetof(DecState, hist_base);
            HIP_TRY(hipMemcpyAsync(reinterpret_cast<char*>(c->dec_state) + off,
                                   reinterpret_cast<char*>(c->hist_host) + off, sizeof(DecState) - off,
                                   hipMemcpyHostToDevice, c->stream));
            c->spec_hist_armed = true;
        }
    }
    const int ahead = spec_ahead(c);
    const int n = c->dec_n_bak && c->dec_n_B == B && c->dec_n <= ahead ? c->dec_n : 1;
    while (c->spec_end < limit) {
        // whole n-step graphs (the queue refills by n once n steps have been handed out, so it
        // holds ahead - n .. ahead steps); single steps for the tail before the horizon, or when
        // the time budget allows fewer than n
        const int k = n > 1 && limit - c->spec_end >= n ? n : 1;
        if (c->spec_end - c->spec_base + k > ahead) break;
        hipEvent_t ev[3];
        for (hipEvent_t& e : ev) {
            if (c->spec_free.empty()) {
                HIP_TRY(hipEventCreate(&e));
            } else {
                e = c->spec_free.back();
                c->spec_free.pop_back();
            }
        }
        if (launch_decode_graph(c, k > 1 ? c->dec_exec_n : c->dec_exec, ev[0])) return 1;
        HIP_TRY(hipEventRecord(ev[1], c->stream));
        HIP_TRY(hipMemcpyAsync(c->spec_ids + (size_t)c->spec_end * B, c->spec_hist + (size_t)c->spec_end * B,
                               (size_t)k * B * 4, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipEventRecord(ev[2], c->stream));
        c->spec_q.push_back({c->spec_end, k, ev[0], ev[1], ev[2], false});
        c->spec_end += k;
    }
    return 0;
}

// Undo the run-ahead steps nobody asked for: put back the K / V slot each appended in every
// layer (stream-ordered after them) and drop the device decode state (the next eager step
// re-arms it).  Every entry point that reads the cache calls this first, so the cache always
// holds what the reference's would.
static int spec_resolve(l3_ctx* c) {
    if (c->spec_q.empty()) return 0;
    HIP_TRY(hipSetDevice(c->device));
    c->gather_tail = false;  // the restores below are queued after the gather
    // persistent steps queued: one that gives up leaves its own slot partly or not at all written
    // and every later one unwritten; the guarded undo decides that on the device, after them, so
    // the caller does not wait here for the run-ahead to drain (persist_settle checks later)
    const bool persist = c->persist_ready && !c->persist_off;
    if (spec_undo(c)) return 1;
    if (persist) c->persist_unsettled = true;
    c->dec_pos_mirror = -1;
    return 0;
}

extern "C" int l3_greedy_step_host(l3_ctx* c, const int64_t* ids_host, int32_t B, int32_t L,
                                   int32_t start_pos, int64_t* next_ids_host, float* logits_host) {
    CHECK_CTX(c);
    if (need_model(c) || check_call(c, B, L, start_pos) || set_dev(c) || ensure_ws(c, B, L) || persist_settle(c))
        return 1;
    if (!c->dec_ids) {
        HIP_TRY(hipMalloc(&c->dec_ids, (size_t)c->d.max_batch_size * 4));
        HIP_TRY(hipMalloc(&c->dec_state, sizeof(DecState)));
        HIP_TRY(hipMemset(c->dec_state, 0, sizeof(DecState)));
        c->dec_pos = &c->dec_state->pos;
        HIP_TRY(hipHostMalloc(&c->dec_host, (size_t)c->d.max_batch_size * 4));
    }
    // A speculative step in flight serves this call when the call continues the schedule (the
    // position it ran at, fed the ids the previous call returned); otherwise it is undone.
    if (!c->spec_q.empty()) {
        bool hit = L == 1 && !logits_host && c->spec_B == B && c->spec_base == start_pos && !c->timing &&
                   (int)c->dec_last.size() == B;
        for (int i = 0; hit && i < B; ++i) hit = c->dec_last[(size_t)i] == ids_host[i];
        if (hit && !c->spec_q.front().done) {
            auto& q = c->spec_q.front();  // holds position spec_base
            HIP_TRY(hipEventSynchronize(q.ev));
            q.done = true;
            if (persist_failed(c)) {
                // a persistent step gave up: everything queued is undone, this step runs eagerly
                if (persist_recover(c, nullptr)) return 1;
                hit = false;
            } else {
                float ms = 0.f;  // the chunk's graph time on the device, per step
                if (hipEventElapsedTime(&ms, q.ev0, q.ev1) == hipSuccess && ms > 0.f)
                    note_step_time(c, 1e3 * (double)ms / q.n);
            }
        }
        if (hit) {
            auto& q = c->spec_q.front();
            for (int i = 0; i < B; ++i) next_ids_host[i] = c->spec_ids[(size_t)start_pos * B + i];
            if (++c->spec_base == q.pos0 + q.n) {
                c->spec_free.insert(c->spec_free.end(), {q.ev0, q.ev1, q.ev});
                c->spec_q.pop_front();
            }
            c->dec_last.assign(next_ids_host, next_ids_host + B);
            c->dec_pos_mirror = start_pos + 1;
            c->graph_steps++;
            c->spec_hits++;
            return speculate(c, B);
        }
        if (spec_resolve(c)) return 1;
    }
    // Graph replay when this call continues the device-resident decode state: one token per
    // sequence at the position the state expects, fed the ids the previous step returned.
    bool replay = L == 1 && !logits_host && c->dec_exec && c->dec_B == B &&
                  c->dec_pos_mirror == start_pos && (int)c->dec_last.size() == B && !c->timing;
    for (int i = 0; replay && i < B; ++i) replay = c->dec_last[(size_t)i] == ids_host[i];
    double t0_replay = 0.0;
    if (replay) {
        t0_replay = now_us();
        if (launch_decode_graph(c, c->dec_exec)) return 1;
        HIP_TRY(hipMemcpyAsync(c->dec_host, c->dec_ids, (size_t)B * 4, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        // a persistent step that gave up: recovered, then this step runs eagerly below
        if (persist_failed(c) && persist_recover(c, nullptr)) return 1;
        replay = c->dec_exec != nullptr;
    }
    if (replay) {
        note_step_time(c, now_us() - t0_replay);
        for (int i = 0; i < B; ++i) next_ids_host[i] = c->dec_host[i];
        c->dec_last.assign(next_ids_host, next_ids_host + B);
        c->dec_pos_mirror = start_pos + 1;
        c->graph_steps++;
        return speculate(c, B);
    }
    c->dec_pos_mirror = -1;
    const double t_eager = now_us();
    if (upload_ids(c, ids_host, (int64_t)B * L)) return 1;
    if (forward_dev(c, c->ids, B, L, start_pos, c->logits)) return 1;
    if (timed(c, L3_K_ARGMAX, [&] { return launch_greedy_argmax(c, B, nullptr); }))
        return 1;
    HIP_TRY(hipMemcpyAsync(c->dec_host, c->dec_ids, (size_t)B * 4, hipMemcpyDeviceToHost, c->stream));
    if (logits_host)
        HIP_TRY(hipMemcpyAsync(logits_host, c->logits, (int64_t)B * c->d.vocab_size * 4,
                               hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    // an eager decode step (per-kernel launches: an upper bound of the replayed step) seeds the
    // run-ahead budget's step time until a replay is timed; prefill calls (L > 1) do not
    if (L == 1) seed_step_time(c, now_us() - t_eager);
    for (int i = 0; i < B; ++i) next_ids_host[i] = c->dec_host[i];
    // L3_DECODE_GRAPH=0 keeps every step eager (rocprofv3 kernel tracing does not survive
    // stream capture in this ROCm build)
    static const bool graphs = env_knob("L3_DECODE_GRAPH", 1) != 0;
    if (graphs && L == 1 && start_pos + 1 < c->d.max_seq_len) {
        // arm the device state for the next decode step (one position later) and capture
        const int next = start_pos + 1;
        HIP_TRY(hipMemcpy(c->dec_pos, &next, sizeof(int), hipMemcpyHostToDevice));
        if (c->dec_B != B && capture_decode_graph(c, B)) return 1;
        c->dec_last.assign(next_ids_host, next_ids_host + B);
        c->dec_pos_mirror = next;
        return speculate(c, B);
    }
    return 0;
}

// Whole greedy loop on the device (the reference's schedule, llama3.py:310-321): prefill at 0,
// then decode step i >= 1 at pos = L + i, each step one replay of the captured decode graph;
// ids accumulate on the device and come back with one copy at the end.  Not lazy: all
// max_new_tokens - L steps run (Llama.generate keeps the reference's one-step-per-yield).
// out_vals (optional, [B, steps]): each step's winning logit, the value its argmax picked (the
// graph steps record it beside the id; the two eager steps read it from their logits rows).
static int greedy_generate(l3_ctx* c, const int64_t* ids_host, int B, int L, int max_new_tokens,
                           int64_t* out_ids_host, float* out_vals) {
    const int steps = max_new_tokens - L;
    if (steps <= 0) return 0;
    // the last decode step runs at position max_new_tokens - 1, which must be a cache slot
    // (the reference fails there with a broadcast error, llama3.py:184)
    if (max_new_tokens > c->d.max_seq_len)
        return fail("generate: last decode position %d exceeds max_seq_len %d", max_new_tokens - 1,
                    c->d.max_seq_len);
    if (spec_resolve(c)) return 1;
    c->spec_hist_armed = false;  // the loop points DecState.hist at its own history
    // the loop drives the device state itself: no run-ahead step between its own calls
    struct InLoop {
        l3_ctx* c;
        explicit InLoop(l3_ctx* x) : c(x) { c->in_loop = true; }
        ~InLoop() { c->in_loop = false; }
    } in_loop(c);
    const int64_t VS = c->d.vocab_size;
    std::vector<float> lg(out_vals ? (size_t)B * VS : 0);
    // an eager step's values: its logits row at the id it returned
    auto eager_vals = [&](const int64_t* ids, int row) {
        if (!out_vals) return;
        for (int b = 0; b < B; ++b) out_vals[(size_t)b * steps + row] = lg[(size_t)b * VS + ids[b]];
    };
    std::vector<int64_t> first((size_t)B);
    if (l3_greedy_step_host(c, ids_host, B, L, 0, first.data(), out_vals ? lg.data() : nullptr)) return 1;  // prefill
    eager_vals(first.data(), 0);
    if (steps == 1) {
        for (int b = 0; b < B; ++b) out_ids_host[(size_t)b * steps] = first[(size_t)b];
        return 0;
    }
    // decode step 1 at pos L + 1 runs eagerly and arms the graph (device ids, pos = L + 2)
    std::vector<int64_t> nxt((size_t)B);
    if (l3_greedy_step_host(c, first.data(), B, 1, L + 1, nxt.data(), out_vals ? lg.data() : nullptr)) return 1;
    eager_vals(nxt.data(), 1);
    int32_t* hist = nullptr;
    float* hval = nullptr;
    HIP_TRY(hipMalloc(&hist, (size_t)steps * B * 4));
    if (out_vals && hipMalloc(&hval, (size_t)steps * B * 4) != hipSuccess) {
        (void)hipFree(hist);
        return fail("generate: value history allocation failed");
    }
    // the captured argmax writes each replayed step's ids straight into hist (DecState: the
    // step at position L + i is row i), so the loop is graph launches only
    auto set_hist = [&](int32_t* ptr, float* vptr, int base, int cap) {
        DecState h{};
        h.hist_base = base;
        h.hist_cap = cap;
        h.hist = ptr;
        h.hist_val = vptr;
        const size_t off = offsetof(DecState, hist_base);
        if (hipMemcpyAsync(reinterpret_cast<char*>(c->dec_state) + off, reinterpret_cast<char*>(&h) + off,
                           sizeof(DecState) - off, hipMemcpyHostToDevice, c->stream) != hipSuccess)
            return false;
        return hipStreamSynchronize(c->stream) == hipSuccess;  // h is on this stack frame
    };
    auto done = [&](int rc) {
        (void)set_hist(nullptr, nullptr, 0, 0);
        (void)hipStreamSynchronize(c->stream);
        (void)hipFree(hist);
        if (hval) (void)hipFree(hval);
        return rc;
    };
    std::vector<int32_t> h32((size_t)B);
    for (int b = 0; b < B; ++b) h32[(size_t)b] = (int32_t)first[(size_t)b];
    if (hipMemcpy(hist, h32.data(), (size_t)B * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpyAsync(hist + B, c->dec_ids, (size_t)B * 4, hipMemcpyDeviceToDevice, c->stream) != hipSuccess)
        return done(fail("generate: history copy failed"));
    if (steps > 2 && !set_hist(hist, hval, L, steps)) return done(fail("generate: decode state update failed"));
    // the graph replays only from the state the eager step above armed (position L + 2)
    if (steps > 2 && (!c->dec_exec || c->dec_B != B || c->dec_pos_mirror != L + 2))
        return done(fail("generate: decode graph not armed"));
    // the remaining steps - 2 steps: whole dec_n-step graphs, then single-step replays
    const int n = decode_graph_steps();
    if (n > 1 && steps - 2 >= n && ensure_multi_graph(c, B)) return done(1);
    for (int i = 2; i < steps;) {
        const bool multi = n > 1 && steps - i >= n;
        if (launch_decode_graph(c, multi ? c->dec_exec_n : c->dec_exec)) return done(1);
        i += multi ? n : 1;
        c->graph_steps += multi ? n : 1;
    }
    std::vector<int32_t> all((size_t)steps * B);
    std::vector<float> vals(out_vals ? (size_t)steps * B : 0);
    if (hipMemcpyAsync(all.data(), hist, all.size() * 4, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
        (out_vals && hipMemcpyAsync(vals.data(), hval, vals.size() * 4, hipMemcpyDeviceToHost, c->stream) != hipSuccess) ||
        hipStreamSynchronize(c->stream) != hipSuccess)
        return done(fail("generate: copy-back failed"));
    int from = steps;  // rows [2, from) are the device loop's
    if (persist_failed(c)) {
        // a persistent step gave up at position fp = L + k: rows before k stand; the rest run on
        // the graph path, one call per step (the first eager at the failed position, then replays)
        int fp = 0;
        if (persist_recover(c, &fp)) return done(1);
        const int k = fp - L;
        if (k < 2 || k >= steps) return done(fail("generate: persistent step failed at position %d, outside [%d, %d)", fp, L + 2, L + steps));
        from = k;
        std::vector<int64_t> in((size_t)B), nx((size_t)B);
        for (int i = k; i < steps; ++i) {
            for (int b = 0; b < B; ++b) in[(size_t)b] = all[(size_t)(i - 1) * B + b];
            const bool eager = i == k;  // the replays record their values in hval, like the loop's
            if (l3_greedy_step_host(c, in.data(), B, 1, L + i, nx.data(), eager && out_vals ? lg.data() : nullptr))
                return done(1);
            if (eager) eager_vals(nx.data(), i);
            for (int b = 0; b < B; ++b) all[(size_t)i * B + b] = (int32_t)nx[(size_t)b];
        }
        if (out_vals && k + 1 < steps &&
            (hipMemcpyAsync(vals.data() + (size_t)(k + 1) * B, hval + (size_t)(k + 1) * B, (size_t)(steps - k - 1) * B * 4,
                            hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
             hipStreamSynchronize(c->stream) != hipSuccess))
            return done(fail("generate: copy-back failed"));
    }
    persist_dump_stamps(c);
    for (int i = 0; i < steps; ++i)
        for (int b = 0; b < B; ++b) out_ids_host[(size_t)b * steps + i] = all[(size_t)i * B + b];
    for (int i = 2; out_vals && i < steps; ++i) {
        if (i == from) continue;  // the eager step's own
        for (int b = 0; b < B; ++b) out_vals[(size_t)b * steps + i] = vals[(size_t)i * B + b];
    }
    c->dec_last.assign(B, 0);
    for (int b = 0; b < B; ++b) c->dec_last[(size_t)b] = all[(size_t)(steps - 1) * B + b];
    c->dec_pos_mirror = L + steps;  // the device state now expects position L + steps
    return done(0);
}

extern "C" int l3_greedy_generate_host(l3_ctx* c, const int64_t* ids_host, int32_t B, int32_t L,
                                       int32_t max_new_tokens, int64_t* out_ids_host) {
    CHECK_CTX(c);
    return greedy_generate(c, ids_host, B, L, max_new_tokens, out_ids_host, nullptr);
}

extern "C" int l3_greedy_generate_values_host(l3_ctx* c, const int64_t* ids_host, int32_t B, int32_t L,
                                              int32_t max_new_tokens, int64_t* out_ids_host, float* out_vals) {
    CHECK_CTX(c);
    if (!out_vals) return fail("l3_greedy_generate_values_host: null out_vals");
    return greedy_generate(c, ids_host, B, L, max_new_tokens, out_ids_host, out_vals);
}

extern "C" int l3_layer_forward_host(l3_ctx* c, int32_t layer, const float* x_host, int32_t B,
                                     int32_t L, int32_t start_pos, float* out_host) {
    CHECK_CTX(c);
    if (layer < 0 || layer >= (int)c->layers.size()) return fail("layer %d out of range", layer);
    if (need_layer(c, layer, NEED_LAYER) || check_call(c, B, L, start_pos) || set_dev(c) ||
        spec_resolve(c) || ensure_ws(c, B, L))
        return 1;
    const int64_t n = (int64_t)B * L * c->d.dim;
    HIP_TRY(hipMemcpyAsync(c->h, x_host, n * 4, hipMemcpyHostToDevice, c->stream));
    if (run_layer(c, layer, B, L, start_pos)) return 1;
    HIP_TRY(hipMemcpyAsync(out_host, c->h, n * 4, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return 0;
}

// Attention.__call__ (llama3.py:155-213): x is the already-normalised input; returns the
// O-projection output (no residual).  Uses and updates the layer's KV cache.
extern "C" int l3_attention_forward_host(l3_ctx* c, int32_t layer, const float* x_host, int32_t B,
                                         int32_t L, int32_t start_pos, float* out_host) {
    CHECK_CTX(c);
    if (layer < 0 || layer >= (int)c->layers.size()) return fail("layer %d out of range", layer);
    if (need_layer(c, layer, NEED_ATTN) || check_call(c, B, L, start_pos) || set_dev(c) ||
        spec_resolve(c) || ensure_ws(c, B, L))
        return 1;
    Layer& Ly = c->layers[layer];
    if (Ly.folded_qkv)  // this layer's wqkv carries its attention norm (full-layer context)
        return fail("l3_attention_forward: layer %d has the attention norm folded into its "
                    "projections; use a context holding only the attention weights", layer);
    const int64_t T = (int64_t)B * L;
    const int D = c->d.dim;
    HIP_TRY(hipMemcpyAsync(c->h, x_host, T * D * 4, hipMemcpyHostToDevice, c->stream));
    GemmArgs g{};
    g.A = c->h; g.lda = D; g.W = Ly.wqkv; g.M = (int)T; g.N = c->qkvn; g.K = D; g.norm = false;
    g.q_out = c->q; g.cache_k = Ly.cache_k; g.cache_v = Ly.cache_v;
    g.rope_cos = c->rope_cos; g.rope_sin = c->rope_sin;
    g.L = L; g.start_pos = start_pos; g.H = c->d.n_heads; g.KVH = c->d.n_kv_heads; g.HD = c->HD;
    g.Smax = c->d.max_seq_len;
    g.q_scale = (float)(1.4426950408889634 / std::sqrt((double)c->HD));
    if (timed(c, L3_K_QKV, [&] { return launch_gemm(EPI_QKV, g, c->stream); })) return 1;
    AttnArgs a{};
    a.q = c->q; a.cache_k = Ly.cache_k; a.cache_v = Ly.cache_v; a.out = c->attn;
    a.B = B; a.L = L; a.start_pos = start_pos; a.H = c->d.n_heads; a.KVH = c->d.n_kv_heads;
    a.HD = c->HD; a.Smax = c->d.max_seq_len;
    if (timed(c, L3_K_ATTN, [&] { return launch_attention(a, c->stream); })) return 1;
    GemmArgs o{};
    o.A = c->attn; o.lda = c->qdim; o.W = Ly.wo; o.C = c->h; o.ldc = D;
    o.M = (int)T; o.N = D; o.K = c->qdim; o.norm = false;
    if (timed(c, L3_K_OPROJ, [&] { return launch_gemm(EPI_STORE, o, c->stream); })) return 1;
    HIP_TRY(hipMemcpyAsync(out_host, c->h, T * D * 4, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return 0;
}

// ---------------------------------------------------------------------------------------
// op-level entry points: H2D -> kernel -> D2H on per-call scratch (not a hot path)
struct Scratch {
    l3_ctx* c;
    std::vector<void*> ptrs;
    ~Scratch() {
        for (void* p : ptrs) dfree(p);
    }
    float* get(int64_t n) {
        void* p = nullptr;
        if (hipMalloc(&p, (size_t)(n > 0 ? n : 1) * 4) != hipSuccess) return nullptr;
        ptrs.push_back(p);
        return (float*)p;
    }
};

#define SCRATCH(var, n)                                   \
    float* var = S.get(n);                                \
    if (!var) return fail("op scratch allocation failed")

#define H2D(dst, src, n) HIP_TRY(hipMemcpyAsync(dst, src, (size_t)(n) * 4, hipMemcpyHostToDevice, c->stream))
#define D2H(dst, src, n) HIP_TRY(hipMemcpyAsync(dst, src, (size_t)(n) * 4, hipMemcpyDeviceToHost, c->stream))

extern "C" int l3_op_softmax_host(l3_ctx* c, const float* x, int64_t rows, int64_t n, float* y) {
    CHECK_CTX(c);
    if (set_dev(c)) return 1;
    Scratch S{c};
    SCRATCH(dx, rows * n);
    SCRATCH(dy, rows * n);
    H2D(dx, x, rows * n);
    HIP_TRY(launch_softmax(dx, dy, rows, (int)n, c->stream));
    D2H(y, dy, rows * n);
    HIP_TRY(hipStreamSynchronize(c->stream));
    return 0;
}

extern "C" int l3_op_argmax_host(l3_ctx* c, const float* x, int64_t rows, int64_t n, int32_t* out) {
    CHECK_CTX(c);
    if (rows <= 0 || n <= 0 || n > INT32_MAX) return fail("argmax: bad shape %lld x %lld", (long long)rows, (long long)n);
    if (set_dev(c)) return 1;
    Scratch S{c};
    SCRATCH(dx, rows * n);
    SCRATCH(di, rows);
    H2D(dx, x, rows * n);
    HIP_TRY(launch_argmax(dx, rows, (int)n, reinterpret_cast<int32_t*>(di), c->stream));
    D2H(out, di, rows);
    HIP_TRY(hipStreamSynchronize(c->stream));
    return 0;
}

extern "C" int l3_op_silu_host(l3_ctx* c, const float* x, int64_t n, float* y) {
    CHECK_CTX(c);
    if (set_dev(c)) return 1;
    Scratch S{c};
    SCRATCH(dx, n);
    SCRATCH(dy, n);
    H2D(dx, x, n);
    HIP_TRY(launch_silu(dx, dy, n, c->stream));
    D2H(y, dy, n);
    HIP_TRY(hipStreamSynchronize(c->stream));
    return 0;
}

extern "C" int l3_op_rmsnorm_host(l3_ctx* c, const float* x, const float* w, int64_t rows,
                                  int64_t dim, float eps, float* y) {
    CHECK_CTX(c);
    if (set_dev(c)) return 1;
    Scratch S{c};
    SCRATCH(dx, rows * dim);
    SCRATCH(dw, dim);
    SCRATCH(dy, rows * dim);
    H2D(dx, x, rows * dim);
    H2D(dw, w, dim);
    HIP_TRY(launch_rmsnorm(dx, dw, dy, rows, (int)dim, eps, c->stream));
    D2H(y, dy, rows * dim);
    HIP_TRY(hipStreamSynchronize(c->stream));
    return 0;
}

extern "C" int l3_op_rope_host(l3_ctx* c, const float* x, int32_t B, int32_t L, int32_t nh,
                               int32_t hd, const float* cos_t, const float* sin_t, float* y) {
    CHECK_CTX(c);
    if (set_dev(c)) return 1;
    const int64_t n = (int64_t)B * L * nh * hd, nt = (int64_t)L * (hd / 2);
    Scratch S{c};
    SCRATCH(dx, n);
    SCRATCH(dy, n);
    SCRATCH(dc, nt);
    SCRATCH(ds, nt);
    H2D(dx, x, n);
    H2D(dc, cos_t, nt);
    H2D(ds, sin_t, nt);
    HIP_TRY(launch_rope(dx, dy, dc, ds, B, L, nh, hd, c->stream));
    D2H(y, dy, n);
    HIP_TRY(hipStreamSynchronize(c->stream));
    return 0;
}

static int op_linear(l3_ctx* c, int epi, const float* dA, int64_t rows, int K, int N,
                     const float* dW, float* dC, bool norm) {
    GemmArgs g{};
    g.A = dA; g.lda = K; g.W = dW; g.C = dC; g.ldc = (epi == EPI_SWIGLU) ? N / 2 : N;
    g.M = (int)rows; g.N = N; g.K = K; g.norm = norm;
    HIP_TRY(launch_gemm(epi, g, c->stream));
    return 0;
}

extern "C" int l3_op_linear_host(l3_ctx* c, const float* x, int64_t rows, int32_t K, int32_t N,
                                 const float* w, float* y) {
    CHECK_CTX(c);
    if (K % 32) return fail("l3_op_linear: K=%d must be a multiple of 32", K);
    if (set_dev(c)) return 1;
    Scratch S{c};
    SCRATCH(dx, rows * K);
    SCRATCH(dw, (int64_t)N * K);
    SCRATCH(dy, rows * N);
    H2D(dx, x, rows * K);
    H2D(dw, w, (int64_t)N * K);
    if (op_linear(c, EPI_STORE, dx, rows, K, N, dw, dy, false)) return 1;
    D2H(y, dy, rows * N);
    HIP_TRY(hipStreamSynchronize(c->stream));
    return 0;
}

extern "C" int l3_op_ffn_host(l3_ctx* c, const float* x, int64_t rows, int32_t dim, int32_t hidden,
                              const float* w_gate, const float* w_up, const float* w_down, float* y) {
    CHECK_CTX(c);
    if (dim % 32 || hidden % 32) return fail("l3_op_ffn: dim and hidden must be multiples of 32");
    if (set_dev(c)) return 1;
    Scratch S{c};
    SCRATCH(dx, rows * dim);
    SCRATCH(dgu, 2LL * hidden * dim);
    SCRATCH(dd, (int64_t)dim * hidden);
    SCRATCH(dh, rows * hidden);
    SCRATCH(dy, rows * dim);
    H2D(dx, x, rows * dim);
    HIP_TRY(hipMemcpy2DAsync(dgu, 32LL * dim * 4, w_gate, 16LL * dim * 4, 16LL * dim * 4, hidden / 16,
                             hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpy2DAsync(dgu + 16LL * dim, 32LL * dim * 4, w_up, 16LL * dim * 4, 16LL * dim * 4,
                             hidden / 16, hipMemcpyHostToDevice, c->stream));
    H2D(dd, w_down, (int64_t)dim * hidden);
    if (op_linear(c, EPI_SWIGLU, dx, rows, dim, 2 * hidden, dgu, dh, false)) return 1;
    HIP_TRY(hipMemsetAsync(dy, 0, rows * dim * 4, c->stream));
    if (op_linear(c, EPI_RESID, dh, rows, hidden, dim, dd, dy, false)) return 1;
    D2H(y, dy, rows * dim);
    HIP_TRY(hipStreamSynchronize(c->stream));
    return 0;
}

// ---------------------------------------------------------------------------------------
// pinned (page-locked) host memory: the copies of l3_forward_host / l3_d2h into it run as
// DMA at PCIe rate instead of through a pageable bounce (l3hip hands such buffers out as the
// NumPy arrays Llama.__call__ returns)
extern "C" int l3_host_alloc(size_t bytes, void** ptr) {
    if (!ptr) return fail("l3_host_alloc: null argument");
    HIP_TRY(hipHostMalloc(ptr, bytes ? bytes : 4, hipHostMallocPortable));
    return 0;
}
extern "C" int l3_host_free(void* ptr) {
    if (ptr) HIP_TRY(hipHostFree(ptr));
    return 0;
}

extern "C" int l3_dev_alloc(l3_ctx* c, size_t bytes, void** ptr) {
    CHECK_CTX(c);
    if (set_dev(c)) return 1;
    HIP_TRY(hipMalloc(ptr, bytes ? bytes : 4));
    return 0;
}
extern "C" int l3_dev_free(l3_ctx* c, void* ptr) {
    CHECK_CTX(c);
    if (set_dev(c)) return 1;
    HIP_TRY(hipStreamSynchronize(c->stream));
    HIP_TRY(hipFree(ptr));
    return 0;
}
extern "C" int l3_h2d(l3_ctx* c, void* dst, const void* src, size_t bytes) {
    CHECK_CTX(c);
    if (set_dev(c)) return 1;
    HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return 0;
}
extern "C" int l3_d2h(l3_ctx* c, void* dst, const void* src, size_t bytes) {
    CHECK_CTX(c);
    if (set_dev(c)) return 1;
    HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return 0;
}
extern "C" int l3_synchronize(l3_ctx* c) {
    CHECK_CTX(c);
    if (set_dev(c)) return 1;
    HIP_TRY(hipStreamSynchronize(c->stream));
    return 0;
}

extern "C" int l3_kernel_timing(l3_ctx* c, int32_t enable) {
    CHECK_CTX(c);
    if (set_dev(c)) return 1;
    HIP_TRY(hipStreamSynchronize(c->stream));
    c->timer_used = 0;
    for (int k = 0; k < L3_K_COUNT; ++k) { c->tot_ms[k] = 0; c->cnt[k] = 0; }
    c->timing = enable != 0;
    c->timing_mask = (unsigned)enable;
    return 0;
}

extern "C" int l3_set_decode_horizon(l3_ctx* c, int32_t end_pos) {
    CHECK_CTX(c);
    c->spec_limit = end_pos > 0 ? end_pos : 0x7fffffff;
    return 0;
}

extern "C" int l3_decode_persistent(l3_ctx* c, int32_t* active) {
    CHECK_CTX(c);
    if (active) *active = c->dec_exec && c->persist_graph ? 1 : 0;
    return 0;
}

extern "C" int l3_decode_recoveries(l3_ctx* c, int64_t* count) {
    CHECK_CTX(c);
    if (count) *count = c->persist_recoveries;
    return 0;
}

// device bounds checks (kernels.h L3_DCHECK): the counts every kernel of this library
// recorded on the context's device since the last call, then cleared (a check build only)
extern "C" int l3_device_check_counts(l3_ctx* c, uint32_t* counts, int32_t* enabled) {
    CHECK_CTX(c);
    if (enabled) *enabled = L3_DCHECK_ON;
    if (!counts) return 0;
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipDeviceSynchronize());
    unsigned n[CHK_N] = {};
    HIP_TRY(dcheck_collect_gemm(n));
    HIP_TRY(dcheck_collect_attention(n));
    HIP_TRY(dcheck_collect_misc(n));
    HIP_TRY(dcheck_collect_persist(n));
    for (int i = 0; i < CHK_N; ++i) counts[i] = n[i];
    return 0;
}

extern "C" int l3_device_check_selftest(l3_ctx* c) {
    CHECK_CTX(c);
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(launch_dcheck_selftest(c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return 0;
}

extern "C" int l3_decode_stats(l3_ctx* c, int64_t* graph_steps, int64_t* speculative_hits) {
    CHECK_CTX(c);
    if (graph_steps) *graph_steps = c->graph_steps;
    if (speculative_hits) *speculative_hits = c->spec_hits;
    return 0;
}

extern "C" int l3_kernel_stats(l3_ctx* c, double* total_ms, int64_t* count) {
    CHECK_CTX(c);
    if (set_dev(c) || harvest_timers(c)) return 1;
    for (int k = 0; k < L3_K_COUNT; ++k) {
        if (total_ms) total_ms[k] = c->tot_ms[k];
        if (count) count[k] = c->cnt[k];
    }
    return 0;
}

// ---------------------------------------------------------------------------------------
extern "C" int l3_comm_unique_id(uint8_t id_out[128]) {
    ncclUniqueId id;
    NCCL_TRY(ncclGetUniqueId(&id));
    static_assert(sizeof(ncclUniqueId) == 128, "unexpected ncclUniqueId size");
    memcpy(id_out, &id, 128);
    return 0;
}

// the comm stream / events a context's gathers use (before its communicator is set)
static int comm_prepare(l3_ctx* c) {
    if (!c->comm_stream) {
        // high priority: a queue apart from the (normal-priority) forward streams, so the
        // transfer does not serialize behind the next forward's kernels in a shared HW queue
        int least = 0, greatest = 0;
        HIP_TRY(hipDeviceGetStreamPriorityRange(&least, &greatest));
        // L3_COMM_PRIORITY=0: normal priority (A/B of the queue placement)
        const int prio = env_knob("L3_COMM_PRIORITY", 1) == 0 ? least : greatest;
        HIP_TRY(hipStreamCreateWithPriority(&c->comm_stream, hipStreamNonBlocking, prio));
        HIP_TRY(hipEventCreateWithFlags(&c->comm_fwd_ev, hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&c->comm_done_ev, hipEventDisableTiming));
    }
    const int mode = env_knob("L3_COMM_MODE", 1);
    c->comm_mode = mode == 0 || mode == 3 ? mode : 1;
    return 0;
}

extern "C" int l3_comm_init(l3_ctx* c, int32_t nranks, int32_t rank, const uint8_t id[128]) {
    CHECK_CTX(c);
    if (set_dev(c) || comm_prepare(c)) return 1;
    if (c->comm) return fail("l3_comm_init: communicator already initialised");
    if (nranks < 1 || rank < 0 || rank >= nranks)
        return fail("l3_comm_init: rank %d outside [0, %d)", rank, nranks);
    ncclUniqueId uid;
    memcpy(&uid, id, 128);
    NCCL_TRY(ncclCommInitRank(&c->comm, nranks, uid, rank));
    c->nranks = nranks;
    c->rank = rank;
    return 0;
}

extern "C" int l3_comm_set_overlap(l3_ctx* c, int32_t on) {
    CHECK_CTX(c);
    if (set_dev(c)) return 1;  // joins a gather in flight: the new form applies from the next one
    c->comm_mode = on ? 3 : 1;
    return 0;
}

static int group_busids(l3_group* g, char* busids, int64_t cap);  // (below)

// What RCCL itself reports for this rank (ncclCommCount / ncclCommUserRank / ncclCommCuDevice)
// and every rank's PCI bus id, all-gathered over the communicator (collective: every rank calls
// it), so a multi-GPU run can prove it ran N ranks on N distinct devices.
extern "C" int l3_comm_info(l3_ctx* c, int32_t* nranks, int32_t* rank, int32_t* device, char* busids,
                            int64_t busids_cap) {
    CHECK_CTX(c);
    if (set_dev(c)) return 1;
    char own[L3_BUSID_LEN] = {0};
    HIP_TRY(hipDeviceGetPCIBusId(own, L3_BUSID_LEN - 1, c->device));
    if (!c->comm) {
        if (nranks) *nranks = 1;
        if (rank) *rank = 0;
        if (device) *device = c->device;
        if (busids && busids_cap >= 1) memcpy(busids, own, L3_BUSID_LEN);
        return 0;
    }
    int n = 0, r = 0, dev = -1;
    NCCL_TRY(ncclCommCount(c->comm, &n));
    NCCL_TRY(ncclCommUserRank(c->comm, &r));
    NCCL_TRY(ncclCommCuDevice(c->comm, &dev));
    if (nranks) *nranks = n;
    if (rank) *rank = r;
    if (device) *device = dev;
    if (!busids) return 0;
    if (c->group) return group_busids(c->group, busids, busids_cap);  // one process: no collective
    if (busids_cap < n) return fail("l3_comm_info: room for %lld bus ids, the communicator has %d ranks",
                                    (long long)busids_cap, n);
    char* d = nullptr;
    HIP_TRY(hipMalloc(&d, (size_t)n * L3_BUSID_LEN));
    hipError_t e = hipMemcpyAsync(d + (size_t)r * L3_BUSID_LEN, own, L3_BUSID_LEN, hipMemcpyHostToDevice, c->stream);
    ncclResult_t nr = e == hipSuccess ? ncclAllGather(d + (size_t)r * L3_BUSID_LEN, d, L3_BUSID_LEN, ncclChar,
                                                      c->comm, c->stream)
                                      : ncclSuccess;
    if (e == hipSuccess && nr == ncclSuccess)
        e = hipMemcpyAsync(busids, d, (size_t)n * L3_BUSID_LEN, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    (void)hipFree(d);
    if (nr != ncclSuccess) return fail("ncclAllGather(bus ids) failed: %s", ncclGetErrorString(nr));
    if (e != hipSuccess) return fail("l3_comm_info copy failed: %s", hipGetErrorString(e));
    return 0;
}

// every rank's row count in [0, max_batch_size] (they size RCCL transfers and root offsets)
static int check_rows(l3_ctx* c, const char* who, const int64_t* rows_per_rank, int32_t root) {
    if (!rows_per_rank) return fail("%s: null rows_per_rank", who);
    if (root < 0 || root >= c->nranks) return fail("%s: root %d outside [0, %d)", who, root, c->nranks);
    const int64_t maxB = c->d.max_batch_size;
    for (int r = 0; r < c->nranks; ++r)
        if (rows_per_rank[r] < 0 || rows_per_rank[r] > maxB)
            return fail("%s: rank %d has %lld rows, outside [0, max_batch_size %lld]", who, r,
                        (long long)rows_per_rank[r], (long long)maxB);
    return 0;
}

extern "C" int l3_comm_gather_logits(l3_ctx* c, const float* src_dev, float* dst_dev,
                                     const int64_t* rows_per_rank, int32_t root) {
    CHECK_CTX(c);
    if (!c->comm) return fail("l3_comm_gather_logits: communicator not initialised");
    if (c->group) return fail("l3_comm_gather_logits: this context is a member of an l3_group (use l3_group_*)");
    if (check_rows(c, "l3_comm_gather_logits", rows_per_rank, root)) return 1;
    if (c->rank == root && !dst_dev) return fail("l3_comm_gather_logits: null destination on the root");
    if (set_dev(c, false)) return 1;
    const int64_t VS = c->d.vocab_size;
    // Mode 1 (default): on the context stream, after the forward that wrote src and before the next one —
    // no cross-stream events, the transfer fully serialized.  The overlapped form (mode 0: the
    // transfer on the high-priority comm stream, ordered by events, the next lm_head waiting for
    // it) measured 7.96 ms/step against 6.94 at world 1 on MI355X, and 7.97 still with the
    // comm stream left empty (mode 2: root's own rows on the context stream) — the event
    // hand-offs between the streams, not the transfer, cost the step (profiles/r02_comm_modes.md).
    //
    // Mode 3 (l3_comm_set_overlap): on the context stream as mode 1, but bracketed by events so that the
    // next l3_forward_dev's second batch part (aux stream) starts from the point before the
    // gather: its layers overlap the transfer, part 0 follows the gather on the context stream,
    // and both parts' lm_heads wait for its end (the rows it reads).  No comm stream; at world 1
    // (a self-copy) 6.038 / 6.051 ms/step against mode 1's 6.044 / 6.058, gathered rows
    // bit-exact (profiles/r03_comm_mode3_ab.log).  Not the default: at world 1 there is no
    // transfer to overlap, and the overlap has not yet run against a real RCCL peer
    const int mode = c->comm_mode;
    const bool on_ctx = mode == 1 || mode == 3;
    hipStream_t s = on_ctx ? c->stream : c->comm_stream;
    hipStream_t self_s = mode == 0 ? s : c->stream;
    if (mode != 1) HIP_TRY(hipEventRecord(c->comm_fwd_ev, c->stream));
    if (!on_ctx) HIP_TRY(hipStreamWaitEvent(c->comm_stream, c->comm_fwd_ev, 0));
    // RCCL has no native gather: root posts one recv per peer, peers one send, all in one
    // group so the point-to-point transfers run concurrently over the xGMI links.
    NCCL_TRY(ncclGroupStart());
    if (c->rank == root) {
        int64_t off = 0;
        for (int r = 0; r < c->nranks; ++r) {
            const int64_t n = rows_per_rank[r] * VS;
            if (r == root) {
                if (n && dst_dev + off * VS != src_dev) {
                    const hipError_t e = hipMemcpyAsync(dst_dev + off * VS, src_dev, n * 4,
                                                        hipMemcpyDeviceToDevice, self_s);
                    if (e != hipSuccess) {
                        (void)ncclGroupEnd();  // close the group before reporting
                        return fail("gather root copy: %s", hipGetErrorString(e));
                    }
                }
            } else if (n) {
                NCCL_TRY(ncclRecv(dst_dev + off * VS, (size_t)n, ncclFloat32, r, c->comm, s));
            }
            off += rows_per_rank[r];
        }
    } else if (rows_per_rank[c->rank]) {
        NCCL_TRY(ncclSend(src_dev, (size_t)(rows_per_rank[c->rank] * VS), ncclFloat32, root, c->comm, s));
    }
    NCCL_TRY(ncclGroupEnd());
    if (mode != 1) {
        HIP_TRY(hipEventRecord(c->comm_done_ev, s));
        c->gather_pending = true;
        c->gather_tail = mode == 3;
    }
    return 0;
}

// SURVEY 8(e) option: greedy ids only — each rank's argmax over its [rows_r, VS] logits
// (llama3.py:320: first index on ties, as the decode argmax) on the device, then the
// B x 4-byte ids gathered to the root instead of the B x VS x 4-byte logits.
extern "C" int l3_comm_gather_argmax(l3_ctx* c, const float* src_dev, int32_t* dst_dev,
                                     const int64_t* rows_per_rank, int32_t root) {
    CHECK_CTX(c);
    if (!c->comm) return fail("l3_comm_gather_argmax: communicator not initialised");
    if (c->group) return fail("l3_comm_gather_argmax: this context is a member of an l3_group (use l3_group_*)");
    if (check_rows(c, "l3_comm_gather_argmax", rows_per_rank, root)) return 1;
    if (c->rank == root && !dst_dev) return fail("l3_comm_gather_argmax: null destination on the root");
    if (set_dev(c)) return 1;
    const int64_t n = rows_per_rank[c->rank], maxB = c->d.max_batch_size;
    if (!c->gather_ids) HIP_TRY(hipMalloc(&c->gather_ids, (maxB > 0 ? maxB : 1) * 4));
    if (n) HIP_TRY(launch_argmax(src_dev, n, (int)c->d.vocab_size, c->gather_ids, c->stream));
    NCCL_TRY(ncclGroupStart());
    if (c->rank == root) {
        int64_t off = 0;
        for (int r = 0; r < c->nranks; ++r) {
            const int64_t m = rows_per_rank[r];
            if (r == root) {
                if (m) {
                    const hipError_t e = hipMemcpyAsync(dst_dev + off, c->gather_ids, m * 4,
                                                        hipMemcpyDeviceToDevice, c->stream);
                    if (e != hipSuccess) {
                        (void)ncclGroupEnd();
                        return fail("gather_argmax root copy: %s", hipGetErrorString(e));
                    }
                }
            } else if (m) {
                NCCL_TRY(ncclRecv(dst_dev + off, (size_t)m, ncclInt32, r, c->comm, c->stream));
            }
            off += m;
        }
    } else if (n) {
        NCCL_TRY(ncclSend(c->gather_ids, (size_t)n, ncclInt32, root, c->comm, c->stream));
    }
    NCCL_TRY(ncclGroupEnd());
    return 0;
}

extern "C" int l3_comm_allreduce_max(l3_ctx* c, double* value) {
    CHECK_CTX(c);
    if (!c->comm) return fail("l3_comm_allreduce_max: communicator not initialised");
    if (c->group) return fail("l3_comm_allreduce_max: this context is a member of an l3_group (use l3_group_*)");
    if (set_dev(c)) return 1;
    double* d = nullptr;
    HIP_TRY(hipMalloc(&d, sizeof(double)));
    hipError_t e = hipMemcpyAsync(d, value, sizeof(double), hipMemcpyHostToDevice, c->stream);
    ncclResult_t r = e == hipSuccess ? ncclAllReduce(d, d, 1, ncclFloat64, ncclMax, c->comm, c->stream)
                                     : ncclSuccess;
    if (e == hipSuccess && r == ncclSuccess)
        e = hipMemcpyAsync(value, d, sizeof(double), hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    (void)hipFree(d);
    if (r != ncclSuccess) return fail("ncclAllReduce(max) failed: %s", ncclGetErrorString(r));
    if (e != hipSuccess) return fail("allreduce_max copy failed: %s", hipGetErrorString(e));
    return 0;
}

extern "C" int l3_comm_barrier(l3_ctx* c) {
    CHECK_CTX(c);
    if (!c->comm) return fail("l3_comm_barrier: communicator not initialised");
    if (c->group) return fail("l3_comm_barrier: this context is a member of an l3_group (use l3_group_*)");
    if (set_dev(c)) return 1;
    float* one = nullptr;
    if (!c->scratch.empty()) one = (float*)c->scratch[0];
    else {
        HIP_TRY(hipMalloc(&one, 4));
        c->scratch.push_back(one);
        HIP_TRY(hipMemsetAsync(one, 0, 4, c->stream));  // the sum stays 0: no inf/NaN over time
    }
    NCCL_TRY(ncclAllReduce(one, one, 1, ncclFloat32, ncclSum, c->comm, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return 0;
}

// ---------------------------------------------------------------------------------------
// One process driving the N GPUs of a node (SURVEY 8(b) l3_group_*): the
// single-process drop-in of Llama.__call__ / generate (llama3.py:285-321).  One context per
// device; communicators from ncclCommInitAll; a call uploads and launches every member's rows
// without waiting (each member's work is asynchronous on its own streams), then one RCCL group
// of point-to-point transfers brings the other members' rows to member 0, then one sync.
// Batch row r is member r % n's local row r / n: the mapping does not depend on B, so a row's
// KV cache stays on one device whatever batch sizes later calls use (the reference's cache row r
// persists, llama3.py:138-153,184-187).
struct l3_group {
    int n = 0;
    // the multi-member path (per-member launches, the grouped gather, the row interleave):
    // n > 1, or n = 1 with L3_GROUP_MULTI_PATH=1 (tests: the 1-GPU box runs it against the
    // single-device path); otherwise every call is member 0's own
    bool multi = false;
    // L3_GROUP_VIRTUAL=1 (test knob): members may share a device, no communicators; the gather's
    // point-to-point transfers become device copies into the same member-0 buffers, ordered by
    // events, so the row split, the offsets and the interleave run for real on one GPU
    bool virt = false;
    std::vector<hipEvent_t> rows_ev; // virt: member i's rows written (recorded on its stream)
    hipEvent_t copied_ev = nullptr;  // virt: member 0 has copied every member's rows
    std::vector<l3_ctx*> m;
    std::vector<ncclComm_t> comms;
    std::vector<int> devs;
    l3_dims d{};                     // the model; max_batch_size the global batch
    float* gbuf = nullptr;           // member 0: the other members' logits rows, member order
    int64_t gbuf_rows = 0;
    int32_t* gids = nullptr;         // member 0: the other members' greedy ids
    int64_t gids_n = 0;
    std::vector<int64_t> tmp;        // host: one member's ids rows
};

static int group_rows(const l3_group* g, int B, int i) { return B > i ? (B - i + g->n - 1) / g->n : 0; }

static int group_busids(l3_group* g, char* busids, int64_t cap) {
    if (cap < g->n) return fail("l3_comm_info: room for %lld bus ids, the group has %d members", (long long)cap, g->n);
    for (int i = 0; i < g->n; ++i) {
        char b[L3_BUSID_LEN] = {0};
        HIP_TRY(hipDeviceGetPCIBusId(b, L3_BUSID_LEN - 1, g->devs[(size_t)i]));
        memcpy(busids + (size_t)i * L3_BUSID_LEN, b, L3_BUSID_LEN);
    }
    return 0;
}

extern "C" int l3_group_destroy(l3_group* g) {
    if (!g) return 0;
    for (l3_ctx* c : g->m)
        if (c) { (void)hipSetDevice(c->device); (void)hipStreamSynchronize(c->stream); }
    if (!g->m.empty() && g->m[0]) {
        (void)hipSetDevice(g->m[0]->device);
        dfree(g->gbuf); dfree(g->gids);
        for (hipEvent_t e : g->rows_ev) if (e) (void)hipEventDestroy(e);
        if (g->copied_ev) (void)hipEventDestroy(g->copied_ev);
    }
    for (size_t i = 0; i < g->comms.size(); ++i)
        if (g->comms[i]) { (void)hipSetDevice(g->devs[i]); ncclCommDestroy(g->comms[i]); }
    for (l3_ctx* c : g->m)
        if (c) { c->comm = nullptr; c->group = nullptr; l3_destroy(c); }
    delete g;
    return 0;
}

extern "C" int l3_group_create(int32_t ndev, const int32_t* devices, const l3_dims* dims, l3_group** out) {
    if (!devices || !dims || !out) return fail("l3_group_create: null argument");
    int have = 0;
    HIP_TRY(hipGetDeviceCount(&have));
    const bool virt = env_knob("L3_GROUP_VIRTUAL", 0) != 0;
    if (ndev < 1 || (ndev > have && !virt) || ndev > 64)
        return fail("l3_group_create: %d devices requested, %d present", ndev, have);
    for (int i = 0; i < ndev; ++i) {
        if (devices[i] < 0 || devices[i] >= have) return fail("l3_group_create: no device %d", devices[i]);
        for (int j = 0; j < i && !virt; ++j)
            if (devices[j] == devices[i]) return fail("l3_group_create: device %d listed twice", devices[i]);
    }
    if (dims->max_batch_size < 1) return fail("l3_group_create: max_batch_size %d < 1", dims->max_batch_size);
    l3_group* g = new l3_group();
    g->n = ndev;
    g->d = *dims;
    g->devs.assign(devices, devices + ndev);
    g->multi = ndev > 1 || env_knob("L3_GROUP_MULTI_PATH", 0) != 0;
    g->virt = virt;
    l3_dims local = *dims;  // each member holds the KV cache of its rows only
    local.max_batch_size = (dims->max_batch_size + ndev - 1) / ndev;
    g->m.assign((size_t)ndev, nullptr);
    for (int i = 0; i < ndev; ++i)
        if (l3_create(devices[i], &local, &g->m[(size_t)i])) {
            const std::string e = g_err;
            l3_group_destroy(g);
            return fail("l3_group_create: member %d (device %d): %s", i, devices[i], e.c_str());
        }
    g->comms.assign((size_t)ndev, nullptr);
    if (virt) {
        HIP_TRY(hipSetDevice(devices[0]));
        g->rows_ev.assign((size_t)ndev, nullptr);
        for (int i = 0; i < ndev; ++i) {
            HIP_TRY(hipSetDevice(devices[i]));
            HIP_TRY(hipEventCreateWithFlags(&g->rows_ev[(size_t)i], hipEventDisableTiming));
        }
        HIP_TRY(hipSetDevice(devices[0]));
        HIP_TRY(hipEventCreateWithFlags(&g->copied_ev, hipEventDisableTiming));
    }
    const ncclResult_t r = virt ? ncclSuccess : ncclCommInitAll(g->comms.data(), ndev, g->devs.data());
    if (r != ncclSuccess) {
        g->comms.assign((size_t)ndev, nullptr);
        l3_group_destroy(g);
        return fail("ncclCommInitAll over %d devices failed: %s", ndev, ncclGetErrorString(r));
    }
    for (int i = 0; i < ndev; ++i) {
        l3_ctx* c = g->m[(size_t)i];
        if (set_dev(c) || comm_prepare(c)) { const std::string e = g_err; l3_group_destroy(g); return fail("%s", e.c_str()); }
        c->comm = g->comms[(size_t)i];
        c->comm_owned = false;
        c->group = g;
        c->nranks = ndev;
        c->rank = i;
        c->comm_mode = 1;  // the group's gathers are always serialized on the member streams
    }
    *out = g;
    return 0;
}

extern "C" int l3_group_context(l3_group* g, int32_t i, l3_ctx** ctx) {
    if (!g || !ctx) return fail("l3_group_context: null argument");
    if (i < 0 || i >= g->n) return fail("l3_group_context: member %d outside [0, %d)", i, g->n);
    *ctx = g->m[(size_t)i];
    return 0;
}

extern "C" int l3_group_upload_weight(l3_group* g, int32_t layer, int32_t kind, const float* host,
                                      int64_t rows, int64_t cols) {
    if (!g) return fail("null group");
    for (l3_ctx* c : g->m)
        if (l3_upload_weight(c, layer, kind, host, rows, cols)) return 1;
    return 0;
}

extern "C" int l3_group_finalize(l3_group* g) {
    if (!g) return fail("null group");
    for (l3_ctx* c : g->m)
        if (l3_finalize(c)) return 1;
    return 0;
}

extern "C" int l3_group_synchronize(l3_group* g) {
    if (!g) return fail("null group");
    for (l3_ctx* c : g->m)
        if (l3_synchronize(c)) return 1;
    return 0;
}

// every member with rows: checks (all before any launch), then ids (host rows r = i + n*j, or
// the member's device block) and its forward into its own logits workspace, launched without
// waiting; each member's decode state is left (no graph replays in a multi-member call)
// logits_host: each member also copies its rows straight into the caller's array (row i + n*j),
// over its own PCIe link, right after each of its parts' lm_head (forward_dev host_pitch)
static int group_launch(l3_group* g, const int64_t* ids_host, const int32_t* const* ids_dev, int B, int L,
                        int start_pos, float* logits_host = nullptr) {
    if (B > g->d.max_batch_size) return fail("batch %d exceeds max_batch_size %d", B, g->d.max_batch_size);
    if (B <= 0 || L <= 0) return fail("empty input: B=%d L=%d", B, L);
    for (int i = 0; i < g->n; ++i) {
        const int nb = group_rows(g, B, i);
        l3_ctx* c = g->m[(size_t)i];
        if (!nb) continue;
        if (need_model(c) || check_call(c, nb, L, start_pos) || set_dev(c) || spec_resolve(c) || ensure_ws(c, nb, L))
            return 1;
        c->dec_pos_mirror = -1;
    }
    for (int i = 0; i < g->n; ++i) {
        const int nb = group_rows(g, B, i);
        l3_ctx* c = g->m[(size_t)i];
        if (!nb) continue;
        if (set_dev(c)) return 1;
        const int32_t* ids = ids_dev ? ids_dev[i] : c->ids;
        if (ids_host) {
            g->tmp.resize((size_t)nb * L);
            for (int j = 0; j < nb; ++j)
                memcpy(&g->tmp[(size_t)j * L], ids_host + ((int64_t)i + (int64_t)g->n * j) * L, (size_t)L * 8);
            if (upload_ids(c, g->tmp.data(), (int64_t)nb * L)) return 1;
        }
        if (forward_dev(c, ids, nb, L, start_pos, c->logits, nullptr, logits_host, g->n, i)) return 1;
    }
    return 0;
}

// rows of `each` floats per row: member i's nb_i rows (src_i) to member 0, interleaved into
// dst [B, each] in row order (row i + n*j <- member i's row j).  src_0 goes straight into dst.
template <typename T>
static int group_gather(l3_group* g, int B, int64_t each, T** src, T* peer_buf, T* dst, ncclDataType_t type) {
    l3_ctx* c0 = g->m[0];
    if (g->virt) {
        // the same transfers as device copies on member 0's stream: after each member's rows are
        // written (its event), into the same peer_buf offsets; the members' next writes of their
        // rows wait for the copies (RCCL's send completes on the sender's stream the same way)
        int64_t voff = 0;
        for (int i = 1; i < g->n; ++i) {
            const int64_t nb = group_rows(g, B, i);
            if (!nb) continue;
            l3_ctx* ci = g->m[(size_t)i];
            HIP_TRY(hipSetDevice(ci->device));
            HIP_TRY(hipEventRecord(g->rows_ev[(size_t)i], ci->stream));
            HIP_TRY(hipSetDevice(c0->device));
            HIP_TRY(hipStreamWaitEvent(c0->stream, g->rows_ev[(size_t)i], 0));
            HIP_TRY(hipMemcpyAsync(peer_buf + voff * each, src[i], (size_t)(nb * each) * sizeof(T), hipMemcpyDeviceToDevice,
                                   c0->stream));
            voff += nb;
        }
        HIP_TRY(hipEventRecord(g->copied_ev, c0->stream));
        for (int i = 1; i < g->n; ++i) {
            if (!group_rows(g, B, i)) continue;
            HIP_TRY(hipSetDevice(g->m[(size_t)i]->device));
            HIP_TRY(hipStreamWaitEvent(g->m[(size_t)i]->stream, g->copied_ev, 0));
        }
    } else {
        NCCL_TRY(ncclGroupStart());
        int64_t off = 0;
        for (int i = 1; i < g->n; ++i) {
            const int64_t nb = group_rows(g, B, i);
            if (!nb) continue;
            ncclResult_t r = ncclRecv(peer_buf + off * each, (size_t)(nb * each), type, i, g->comms[0], c0->stream);
            if (r == ncclSuccess)
                r = ncclSend(src[i], (size_t)(nb * each), type, 0, g->comms[(size_t)i], g->m[(size_t)i]->stream);
            if (r != ncclSuccess) {
                (void)ncclGroupEnd();
                return fail("group gather (member %d): %s", i, ncclGetErrorString(r));
            }
            off += nb;
        }
        NCCL_TRY(ncclGroupEnd());
    }
    HIP_TRY(hipSetDevice(c0->device));
    const size_t pitch = (size_t)g->n * each * sizeof(T), w = (size_t)each * sizeof(T);
    HIP_TRY(hipMemcpy2DAsync(dst, pitch, src[0], w, w, (size_t)group_rows(g, B, 0), hipMemcpyDeviceToDevice,
                             c0->stream));
    int64_t off = 0;
    for (int i = 1; i < g->n; ++i) {
        const int64_t nb = group_rows(g, B, i);
        if (!nb) continue;
        HIP_TRY(hipMemcpy2DAsync(dst + (size_t)i * each, pitch, peer_buf + off * each, w, w, (size_t)nb,
                                 hipMemcpyDeviceToDevice, c0->stream));
        off += nb;
    }
    return 0;
}

// member-0 buffer of at least `rows` rows of `each` elements (grown; the stream is idle when
// it grows: callers grow before launching)
template <typename T>
static int group_buf(l3_group* g, T** p, int64_t* have, int64_t rows, int64_t each) {
    if (rows <= *have) return 0;
    HIP_TRY(hipSetDevice(g->m[0]->device));
    HIP_TRY(hipStreamSynchronize(g->m[0]->stream));
    dfree(*p);
    *p = nullptr;
    *have = 0;
    HIP_TRY(hipMalloc(p, (size_t)rows * each * sizeof(T)));
    *have = rows;
    return 0;
}

extern "C" int l3_group_forward_dev(l3_group* g, const int32_t* const* ids_dev, int32_t B, int32_t L,
                                    int32_t start_pos, float* logits_dev) {
    if (!g || !ids_dev || !logits_dev) return fail("l3_group_forward_dev: null argument");
    if (!g->multi || B == 1) return l3_forward_dev(g->m[0], ids_dev[0], B, L, start_pos, logits_dev);
    const int64_t VS = g->d.vocab_size;
    if (group_buf(g, &g->gbuf, &g->gbuf_rows, B - group_rows(g, B, 0), VS)) return 1;
    if (group_launch(g, nullptr, ids_dev, B, L, start_pos)) return 1;
    std::vector<float*> src((size_t)g->n);
    for (int i = 0; i < g->n; ++i) src[(size_t)i] = g->m[(size_t)i]->logits;
    return group_gather(g, B, VS, src.data(), g->gbuf, logits_dev, ncclFloat32);
}

extern "C" int l3_group_forward_host(l3_group* g, const int64_t* ids_host, int32_t B, int32_t L,
                                     int32_t start_pos, float* logits_host) {
    if (!g || !ids_host || !logits_host) return fail("l3_group_forward_host: null argument");
    // rows on member 0 only: its own single-device host path (pinned per-part copies)
    if (!g->multi || B == 1) return l3_forward_host(g->m[0], ids_host, B, L, start_pos, logits_host);
    // no gather: every member copies its own rows into the caller's (page-locked, portable) array
    // over its own link, each batch part right after its lm_head — at C4 on 8 GPUs 32.8 MB per
    // link in parallel (~0.6 ms) instead of 262 MB through member 0's one link (~4.7 ms).  The
    // RCCL gather stays for l3_group_forward_dev (device-resident logits, north_star's gather)
    if (group_launch(g, ids_host, nullptr, B, L, start_pos, logits_host)) return 1;
    return l3_group_synchronize(g);
}

extern "C" int l3_group_greedy_step_host(l3_group* g, const int64_t* ids_host, int32_t B, int32_t L,
                                         int32_t start_pos, int64_t* next_ids_host) {
    if (!g || !ids_host || !next_ids_host) return fail("l3_group_greedy_step_host: null argument");
    // single-prompt greedy decode stays on one GPU (member 0: graph-replayed steps, run-ahead)
    if (!g->multi || B == 1) return l3_greedy_step_host(g->m[0], ids_host, B, L, start_pos, next_ids_host, nullptr);
    // gids: [0, B) the ids in row order, [B, 2B) the other members' ids as received
    if (group_buf(g, &g->gids, &g->gids_n, 2 * (int64_t)B, 1)) return 1;
    if (group_launch(g, ids_host, nullptr, B, L, start_pos)) return 1;
    std::vector<int32_t*> src((size_t)g->n);
    for (int i = 0; i < g->n; ++i) {
        l3_ctx* c = g->m[(size_t)i];
        const int nb = group_rows(g, B, i);
        src[(size_t)i] = c->amax;
        if (!nb) continue;
        if (set_dev(c)) return 1;
        // np.argmax over the member's rows (llama3.py:320: first index on ties)
        if (timed(c, L3_K_ARGMAX, [&] { return launch_argmax(c->logits, nb, (int)c->d.vocab_size, c->amax, c->stream); }))
            return 1;
    }
    if (group_gather(g, B, 1, src.data(), g->gids + B, g->gids, ncclInt32)) return 1;
    std::vector<int32_t> ids32((size_t)B);
    HIP_TRY(hipMemcpyAsync(ids32.data(), g->gids, (size_t)B * 4, hipMemcpyDeviceToHost, g->m[0]->stream));
    if (l3_group_synchronize(g)) return 1;
    for (int b = 0; b < B; ++b) next_ids_host[b] = ids32[(size_t)b];
    return 0;
}
