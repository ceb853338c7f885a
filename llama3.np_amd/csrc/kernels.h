// Internal kernel interface of libllama3hip (not part of the C ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

namespace l3 {

// A/B knobs: environment variables read once per process; every default is the measured best
// (DESIGN.md decisions table) and the knobs exist only to re-run those A/B measurements.
//   runtime.hip  L3_BATCH_SPLIT (2), L3_LAST_LAYER_ALL_ROWS (0), L3_DECODE_FUSE_O (1),
//                L3_LM_AMAX (1), L3_DECODE_FOLD_ARGMAX (1), L3_DECODE_SPECULATE (1), L3_DECODE_GRAPH_STEPS (8),
//                L3_DECODE_GRAPH (1), L3_COMM_MODE (1), L3_COMM_PRIORITY (1), L3_GROUP_MULTI_PATH (0),
//                L3_DECODE_PERSIST (1 persistent step; 0 graph), L3_DECODE_ROWS_AMAX (1)
//   test knobs   L3_DECODE_PERSIST_MAX_CUS (cap the CUs the persistent step sees), L3_DECODE_PERSIST_FAULT
//                (a workgroup gives up in the step at that position; L3_DECODE_PERSIST_FAULT_WG which),
//                L3_GROUP_VIRTUAL (a group's members may share one device; D2D copies for the gather),
//                L3_DECODE_PERSIST_STAMPS=<file> (diagnostic timeline, tools/persist_stamps.py)
//   gemm.hip     L3_SPLITK (1), L3_SPLITK_CFG (0), L3_SPLITK_BLOCKS (1024), L3_SPLITK_MINKT (8),
//                L3_GEMV_NT (1), L3_GEMV_LPU (0 = by shape), L3_GEMV_MR (by shape), L3_SKINNY (1),
//                L3_SKINNY_MIN (9), L3_SKINNY_CH (2), L3_SKINNY_TN2_MIN (256), L3_GEMM_GROUP_M (8)
inline int env_knob(const char* name, int def) {
    const char* e = getenv(name);
    return e && *e ? atoi(e) : def;
}

// Device bounds checks (SURVEY §5 "device bounds asserts in a debug build"): built with
// -DL3_DEVICE_CHECKS (libllama3hip_check.so, `make check-lib`), the kernels count, per class,
// every index that leaves the buffer it addresses — in counters, not traps, so a violation is
// reported by l3_device_check_counts instead of faulting the device.  The release library
// compiles them away.  Classes: a K / V cache slot (position outside [0, Smax)), an attention
// launch's key range (start_pos + L > Smax), a token id out of [0, n) (argmax results, the
// embedding rows the lm_head partials select).
enum CheckClass : int { CHK_KV_SLOT = 0, CHK_ATTN_KEYS = 1, CHK_TOKEN_ID = 2, CHK_N = 4 };
#ifdef L3_DEVICE_CHECKS
static __device__ unsigned l3_dcheck_counts[CHK_N];  // one set per translation unit
#define L3_DCHECK(cond, cls)                                                      \
    do {                                                                          \
        if (!(cond)) atomicAdd(&::l3::l3_dcheck_counts[(cls)], 1u);               \
    } while (0)
// this translation unit's counters, added into out[CHK_N], then cleared
static inline hipError_t dcheck_collect(unsigned* out) {
    unsigned h[CHK_N] = {};
    hipError_t e = hipMemcpyFromSymbol(h, HIP_SYMBOL(l3_dcheck_counts), sizeof h, 0, hipMemcpyDeviceToHost);
    if (e != hipSuccess) return e;
    for (int i = 0; i < CHK_N; ++i) out[i] += h[i];
    const unsigned z[CHK_N] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(l3_dcheck_counts), z, sizeof z, 0, hipMemcpyHostToDevice);
}
#define L3_DCHECK_ON 1
#else
#define L3_DCHECK(cond, cls) ((void)0)
static inline hipError_t dcheck_collect(unsigned*) { return hipSuccess; }
#define L3_DCHECK_ON 0
#endif

// Epilogues of the NT GEMM  C[M,N] = A[M,K] * W[N,K]^T  (see gemm.hip).
enum Epilogue : int {
    EPI_STORE = 0,   // C = s_row * acc
    EPI_RESID = 1,   // C += acc                        (O-proj / down-proj + residual)
    EPI_SWIGLU = 2,  // C[:, j] = silu(s*g_j) * (s*u_j) (gate/up interleaved by 16 rows)
    EPI_QKV = 3,     // s_row * acc -> RoPE(q,k) -> q buffer + KV cache append
};

struct ArgmaxPart {
    float v;
    int i;
};

// Device-resident state of the greedy decode loop (graph replay).  pos is first, so &st->pos
// is the pos_dev the captured kernels read.
struct DecState {
    int pos;           // start_pos of the next decode step; the argmax advances it
    int hist_base;     // generate loop: the ids of the step at position q go to
    int hist_cap;      //   hist[(q - hist_base) * B + b] while 0 <= q - hist_base < hist_cap
    unsigned arrive;   // argmax_kernel's block arrival count (0 between launches)
    int32_t* hist;     // null: no history
    float* hist_val;   // null, or beside hist: each step's winning logit (the value argmax picked)
};

struct GemmArgs {
    const float* A; int64_t lda;   // A rows, row stride (floats)
    const float* W;                // [N, K] row-major
    const unsigned short* W3;      // opt-in x6 path (gemm_x6.h): W as three bf16 pieces
                                   // [N][3][K] (null: the fp32 MFMA kernels)
    float* C; int64_t ldc;         // output (EPI_QKV: unused)
    int M, N, K;
    bool norm;                     // RMSNorm on A: rows scaled by 1/sqrt(mean(A^2)+eps); the norm
                                   // weight is folded into W's columns (launch_fold_cols)
    float eps;
    // EPI_QKV
    float* q_out;                  // [M, H*HD], pre-scaled by q_scale
    float* cache_k; float* cache_v;// [maxB, KVH, Smax, HD]
    const float* rope_cos; const float* rope_sin;  // [Smax, HD/2]
    int L, start_pos, H, KVH, HD, Smax;
    const int* pos_dev;            // if set, start_pos is read from device memory (graph replay)
    float q_scale;
    // EPI_QKV on the tiled kernel: the division-free full-tile epilogue may run (set by the
    // launcher when HD % 16 == 0 and L >= the tile's wave rows; gemm_kernel.h qkv_epilogue_full)
    bool qkv_fast;
    // gemm_skinny_kernel: tiles dealt to the XCDs in contiguous runs walked column-major, so one
    // XCD's blocks share a few W column tiles in its L2 instead of every XCD pulling all of W
    bool skinny_xcd;
    int col_base;                  // EPI_QKV on the tiled / skinny kernels: index of output column 0
                                   // in the [q | k | v] layout (W starts at that row of wqkv): a
                                   // pruned last block appends K / V for every row without q
    // EPI_QKV on the GEMV (captured batch-1..8 decode steps): before appending K / V at pos, keep
    // the slot's previous contents in kv_bak [pos % KV_BAK_SLOTS][2: k, v][M][KVH][HD], so decode
    // steps run ahead of the caller can be undone (runtime.hip, speculate / spec_resolve)
    float* kv_bak;
    unsigned long long* stamps;    // diagnostic builds only (STAMP template flag): 10 per block
    // Embedding fused into layer 0 (llama3.py:287): when set, A row r is A + a_rows[r] * lda
    // (the token's embedding row) and EPI_RESID adds res_src[res_rows[r] * ldc + col] instead
    // of reading C, so the residual stream h is first written by layer 0's O-proj
    const int32_t* a_rows;
    const float* res_src; const int32_t* res_rows;
    // Decode with the O-proj fused into attention (attn_decode_kernel<HD, true>): the O-proj
    // arrives as nparts (= n_heads, <= GEMV_MAXP) per-head partial rows [M][nparts][D] that the
    // GEMV adds to its A row (EPI_SWIGLU) or to its residual (EPI_RESID) in head order
    const float* parts; int nparts;
    float* x_out;                  // EPI_SWIGLU with parts: the summed input row (A row + parts),
                                   // [M][K], for the down-proj's residual (written by block 0)
    // EPI_STORE on the one-row GEMV (batch-1 lm_head): also the block's (value, index) argmax
    // over its columns -> amax_part[blockIdx.x], reduced by launch_argmax_parts
    ArgmaxPart* amax_part;
    // EPI_STORE on the tiled kernel (a captured batched decode step's lm_head): instead of the
    // logits, each wave's (value, index) argmax over its 64 columns of every row ->
    // amax_rows[row][column tile], amax_nct tiles per row (C is not written)
    ArgmaxPart* amax_rows; int amax_nct;
    DecState* pos_adv;             // ... and block 0 moves the decode position on (a captured step
                                   // whose argmax the next step's layer-0 QKV folds in)
    // EPI_QKV on the one-row GEMV (a captured batch-1 decode step after the first of a graph): the
    // A row is the embedding row of the previous step's greedy id, reduced by every block from
    // that step's lm_head partials (amax_in, amax_in_n); block 0 also stores the id to amax_ids[0]
    // (the layer-0 gate|up's embedding row) and to the generate history of amax_st at pos - 1
    const ArgmaxPart* amax_in; int amax_in_n;
    int32_t* amax_ids;
    DecState* amax_st;
    // Split-K (short M against a long K, gemm.hip launch_split): the caller's workspace of ws_cap
    // floats (null: no split); the k-slices leave raw partial tiles [splits][M][N] and partial
    // row sums of squares [splits][M] there, and splitk_finish_kernel applies the epilogue
    float* ws; int64_t ws_cap;
    int splits;                    // set by launch_gemm
    // the skinny MFMA kernel whatever M and W (a pruned last layer: every row rounds the same
    // way for any batch split, runtime.hip run_layer last_rows)
    bool force_skinny;
    // tiled kernel: tile order within each XCD's run of tiles — 0 row-major (n fastest), g > 0
    // groups of g row tiles walked column by column, so a k-step's concurrent blocks share g A
    // slices and ~blocks / g W slices in L2 (set by launch_gemm for long K; results identical)
    int group_m;
};
constexpr int GEMV_MAXP = 8;
constexpr int KV_BAK_SLOTS = 32;  // > the decode steps ever run ahead (runtime.hip SPEC_AHEAD)


// Exchange with lane ^ 16 and lane ^ 32 through v_permlane16_swap / v_permlane32_swap (VALU)
// rather than ds_bpermute: a bpermute is an LDS-pipe round trip whose lgkmcnt wait also
// drains the wave's outstanding LDS fragment reads.  With both operands the same register,
// lane i of the pair returned holds {v[i], v[i ^ 16]} (resp. ^ 32) in some order.
__device__ __forceinline__ float max_xor16_32(float v) {
    const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
    const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
__device__ __forceinline__ float sum_xor16_32(float v) {
    const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
    const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

// Reductions over aligned groups of LANES = 16, 32 or 64 lanes, every lane of a group left
// with its result, all on the VALU: DPP quad_perm (lane ^ 1, lane ^ 2), row_half_mirror and
// row_mirror complete 16-lane rows (each step pairs lanes whose partial sums cover disjoint
// halves), then the permlane swaps above.  Each step adds the same two values on both lanes of
// a pair, so all lanes agree bit for bit.
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <int LANES>
__device__ __forceinline__ float group_sum(float v) {
    static_assert(LANES == 16 || LANES == 32 || LANES == 64, "16, 32 or 64 lanes");
    v += dpp_mov<0xB1>(v);   // quad_perm [1,0,3,2]
    v += dpp_mov<0x4E>(v);   // quad_perm [2,3,0,1]
    v += dpp_mov<0x141>(v);  // row_half_mirror
    v += dpp_mov<0x140>(v);  // row_mirror
    if constexpr (LANES >= 32) {
        const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
        v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
    }
    if constexpr (LANES >= 64) {
        const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
        v = __uint_as_float(b[0]) + __uint_as_float(b[1]);
    }
    return v;
}
template <int LANES>
__device__ __forceinline__ float group_max(float v) {
    static_assert(LANES == 16 || LANES == 32 || LANES == 64, "16, 32 or 64 lanes");
    v = fmaxf(v, dpp_mov<0xB1>(v));
    v = fmaxf(v, dpp_mov<0x4E>(v));
    v = fmaxf(v, dpp_mov<0x141>(v));
    v = fmaxf(v, dpp_mov<0x140>(v));
    if constexpr (LANES >= 32) {
        const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
        v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
    }
    if constexpr (LANES >= 64) {
        const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
        v = fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
    }
    return v;
}

// np.argmax order (llama3.py:320): larger value first, ties to the lower index, a NaN beats any
// number and the first NaN wins (a strict total order, so any reduction tree gives the same id)
__device__ __forceinline__ bool argmax_better(float v, int i, float bv, int bi) {
    const bool vn = v != v, bn = bv != bv, lo = i < bi;
    // one boolean expression (selects, no branches): the same order as
    //   vn || bn ? vn && (!bn || lo) : v > bv || (v == bv && lo)
    return (vn & (!bn | lo)) | (!vn & !bn & ((v > bv) | ((v == bv) & lo)));
}

// (value, index) argmax over aligned groups of LANES lanes on the VALU (the group_sum pattern of
// kernels.h: DPP quad_perm / row mirrors, then permlane swaps); argmax_better is a strict total
// order, so the winner does not depend on the pairing
template <int CTRL>
__device__ __forceinline__ int dpp_mov_i(int v) {
    return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}
// the argmax of lanes l and l ^ 16 (X16), then of l and l ^ 32 (X32): lane i of a swapped pair
// holds {own, lane ^ 16} with the partner second in rows 0, 2
template <bool X16, bool X32>
__device__ __forceinline__ void argmax_xor16_32(float& best, int& bi, int lane) {
    auto step = [&](float ov, int oi) {
        const bool t = argmax_better(ov, oi, best, bi);
        best = t ? ov : best;
        bi = t ? oi : bi;
    };
    if constexpr (X16) {
        const auto v = __builtin_amdgcn_permlane16_swap(__float_as_uint(best), __float_as_uint(best), false, false);
        const auto x = __builtin_amdgcn_permlane16_swap((unsigned)bi, (unsigned)bi, false, false);
        const bool hi = lane & 16;
        step(__uint_as_float(hi ? v[0] : v[1]), (int)(hi ? x[0] : x[1]));
    }
    if constexpr (X32) {
        const auto v = __builtin_amdgcn_permlane32_swap(__float_as_uint(best), __float_as_uint(best), false, false);
        const auto x = __builtin_amdgcn_permlane32_swap((unsigned)bi, (unsigned)bi, false, false);
        const bool hi = lane & 32;
        step(__uint_as_float(hi ? v[0] : v[1]), (int)(hi ? x[0] : x[1]));
    }
}
template <int LANES>
__device__ __forceinline__ void group_argmax(float& best, int& bi, int lane) {
    auto step = [&](float ov, int oi) {
        const bool t = argmax_better(ov, oi, best, bi);
        best = t ? ov : best;
        bi = t ? oi : bi;
    };
    step(__int_as_float(dpp_mov_i<0xB1>(__float_as_int(best))), dpp_mov_i<0xB1>(bi));
    step(__int_as_float(dpp_mov_i<0x4E>(__float_as_int(best))), dpp_mov_i<0x4E>(bi));
    step(__int_as_float(dpp_mov_i<0x141>(__float_as_int(best))), dpp_mov_i<0x141>(bi));
    step(__int_as_float(dpp_mov_i<0x140>(__float_as_int(best))), dpp_mov_i<0x140>(bi));
    argmax_xor16_32<LANES >= 32, LANES >= 64>(best, bi, lane);
}

// row r of A (identity, or the gathered embedding row)
__device__ __forceinline__ const float* a_row(const GemmArgs& p, int64_t r) {
    return p.A + (p.a_rows ? (int64_t)p.a_rows[r] : r) * p.lda;
}
// residual operand of EPI_RESID at (row, col): C itself, or the gathered embedding row
__device__ __forceinline__ const float* res_row(const GemmArgs& p, int64_t row) {
    return p.res_src ? p.res_src + (p.res_rows ? (int64_t)p.res_rows[row] : row) * p.ldc
                     : p.C + row * p.ldc;
}
__device__ __forceinline__ const float* res_at(const GemmArgs& p, int64_t row, int col) {
    return res_row(p, row) + col;
}

struct AttnArgs {
    const float* q;       // [B*L, H*HD], pre-scaled by log2(e)/sqrt(HD)
    int q_first;          // prefill: first query row of the launch (grid.x covers [q_first, L));
                          // a pruned last block runs only the last query rows of each sequence
    const float* cache_k; // [maxB, KVH, Smax, HD]
    const float* cache_v;
    float* out;           // [B*L, H*HD]
    int B, L, start_pos, H, KVH, HD, Smax;
    const int* pos_dev;   // if set, start_pos is read from device memory (graph replay)
    // decode only: when wo is set the launch also applies the O-proj (llama3.py:211) per head:
    // parts[b][h][0:D] = Wo[:, h*HD:(h+1)*HD] . out[b][h] (out itself is not written); the
    // residual add and the sum over heads happen in the consumers (GemmArgs::parts)
    const float* wo;      // [D, H*HD]
    float* parts;         // [B, H, D]
    int D;
};

// start position of a launch: the argument, or the device word a captured decode graph reads
template <typename Args>
__device__ __forceinline__ int start_of(const Args& p) {
    return p.pos_dev ? *p.pos_dev : p.start_pos;
}

// Persistent batch-1 decode step (decode_persist.hip): one launch runs a whole greedy step —
// every layer, the lm_head and the argmax — with in-launch hand-offs between the stages
struct DecodePersistArgs {
    int D, H, KVH, HD, FD, VS, n_layers, Smax;
    int GL;                        // workgroups that run the layer stages (the others: the lm_head)
    int Dp, Xp;                    // LDS floats: per D-vector, per stage-input vector (multiples of 4)
    float eps, q_scale;
    const float* emb;              // [VS, D]
    const float* lm_head;          // [VS, D], final norm folded
    const float* const* wqkv;      // per layer (device arrays of device pointers); norms folded
    const float* const* wo;
    const float* const* wgu;
    const float* const* wd;
    float* const* cache_k;         // per layer [maxB, KVH, Smax, HD]; batch row 0
    float* const* cache_v;
    const float* rope_cos; const float* rope_sin;
    float* kv_bak;                 // null, or the run-ahead undo slots (GemmArgs::kv_bak layout, B = 1)
    int64_t bak_layer;             // floats per layer of kv_bak
    int32_t* ids;                  // [1]: this step's token id in, the next step's out
    int from_parts;                // 1: the token id is the argmax of the previous launch's lm partials
    int write_id;                  // 1: reduce this launch's partials to ids[0] / history (last step
                                   //    of a graph); 0: leave them for the next launch
    DecState* st;                  // pos (read; +1), generate history
    unsigned long long* gran;      // granule slabs (decode_persist.hip), zeroed at allocation
    unsigned* epoch;               // [0] granule tag of the next launch (starts at 1); [1] sticky failure;
                                   // [2] pos + 1 of the last step that wrote its K / V rows to the caches
    unsigned* err;                 // host-mapped: pos + 1 of the step in which a workgroup gave up
    unsigned long long* stamps;    // diagnostic (null): [workgroup][128] s_memrealtime at stage points
    int fault_pos, fault_wg;       // test knob: workgroup fault_wg gives up in the step at fault_pos (-1: none)
    int fault_late;                // ... at its last wait of the step instead of its first (a layer workgroup)
};
// granules per layer of the persistent step: [qkv | o | h1 | hid | h2]
__host__ __device__ inline int64_t decode_persist_slab(int H, int KVH, int HD, int D, int FD) {
    return (int64_t)(H + 2 * KVH) * HD + (int64_t)H * HD + D + FD + D;
}
bool decode_persist_ok(const DecodePersistArgs& a);
// the launch's grid on the current device, 0 when the step cannot run there (shape, CU count,
// co-residency by the occupancy query at its LDS)
int decode_persist_grid(const DecodePersistArgs& a);
// grid: decode_persist_grid's, taken before a stream capture (no device queries inside one)
hipError_t launch_decode_persist(const DecodePersistArgs& a, int grid, hipStream_t s);

hipError_t launch_gemm(int epi, const GemmArgs& a, hipStream_t s);
// W [rows][K] fp32 -> W3 [rows][3][K] bf16 pieces for the x6 path (gemm_x6.h)
hipError_t launch_split_planes(const float* w, unsigned short* w3, int64_t rows, int K, hipStream_t s);
hipError_t launch_attention(const AttnArgs& a, hipStream_t s);
hipError_t launch_attention_last(const AttnArgs& a, hipStream_t s);
hipError_t launch_argmax(const float* logits, int64_t rows, int n, int32_t* out, hipStream_t s,
                         DecState* st = nullptr);
// the same result from the lm_head's partials: rows x nparts (GemmArgs::amax_part, one row;
// GemmArgs::amax_rows, a batch)
hipError_t launch_argmax_parts(const ArgmaxPart* parts, int nparts, int32_t* out, hipStream_t s,
                               DecState* st = nullptr, int hist_off = 0, int rows = 1);
// blocks of the one-row lm_head GEMV (= its partial count when amax_part is set), 0 otherwise
int gemv_store_blocks(const GemmArgs& a);
// true when launch_gemm runs this shape on the row-blocked GEMV (short M)
bool gemm_is_gemv(const GemmArgs& a);
// true when that GEMV runs one row per block with the input row read per lane (the only form
// that takes GemmArgs::parts)
bool gemv_direct(const GemmArgs& a);
// which EPI_STORE kernel launch_gemm picks (0 = GEMV): launches of equal id round identically
// row by row, whatever their M
int gemm_store_config(const GemmArgs& a);
hipError_t launch_softmax(const float* x, float* y, int64_t rows, int n, hipStream_t s);
hipError_t launch_silu(const float* x, float* y, int64_t n, hipStream_t s);
hipError_t launch_rmsnorm(const float* x, const float* w, float* y, int64_t rows, int dim,
                          float eps, hipStream_t s);
hipError_t launch_fold_cols(float* W, int64_t rows, int K, const float* w, hipStream_t s);
// cache[b][h][pos][:] = bak[b][h][:] for b < B, h < KVH (undo of a speculative decode step)
// the persistent step's failure words, read by the undo on the device (kv_restore_kernel); err
// null: restore unconditionally (the graph path's steps cannot fail)
struct KvGuard {
    const unsigned* err;     // host-mapped error word: failed position + 1, or 0
    const unsigned* epoch;   // [3]; epoch[2]: the tag of the launch that gave up
    const unsigned* wmarks;  // [GL] each layer workgroup's write mark (the tag of its last write)
    int col_base;            // QKV column of this cache's first element (qdim, or qdim + kvdim)
    int per;                 // RoPE-pair units per layer workgroup (stage_unit: ceil(qkvn / 2 / GL))
};
hipError_t launch_kv_restore(float* cache, const float* bak, int B, int KVH, int Smax, int HD, int pos,
                             hipStream_t s, KvGuard g = KvGuard{});
// device bounds-check counters of each translation unit (L3_DEVICE_CHECKS builds; else no-ops)
hipError_t dcheck_collect_gemm(unsigned* out);
hipError_t dcheck_collect_attention(unsigned* out);
hipError_t dcheck_collect_misc(unsigned* out);
hipError_t dcheck_collect_persist(unsigned* out);
hipError_t launch_dcheck_selftest(hipStream_t s);
hipError_t launch_rope(const float* x, float* y, const float* cos_t, const float* sin_t, int B,
                       int L, int nh, int hd, hipStream_t s);

}  // namespace l3
