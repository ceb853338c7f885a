/*
 * llama3hip.h — C ABI of the MI355X (gfx950) forward pass for llama3.np.
 *
 * The reference (swap357/llama3.np) is pure NumPy and has no FFI; this ABI is
 * what its Python classes bind to through ctypes (llama3.np_amd/l3hip.py).
 * Each entry point names the reference interface it replaces (file:line in
 * the reference repo).  Plain pointers and sizes only: no C++ or torch types.
 *
 * Conventions
 *   - Every function returns 0 on success, non-zero on failure; the message is
 *     in l3_last_error() (thread-local).  Nothing throws across the ABI.
 *   - "_host" pointers are caller-owned host memory (C-contiguous); those
 *     calls are synchronous.  "_dev" pointers are device memory from
 *     l3_dev_alloc; those calls are asynchronous on the context's stream
 *     (l3_synchronize waits).
 *   - One context per device; a context is not re-entrant.
 *   - All arithmetic is fp32 (the reference promotes to f64 after RoPE; parity
 *     is to tolerance).
 */
#ifndef LLAMA3HIP_H
#define LLAMA3HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct l3_ctx l3_ctx;

/* Model shape; mirrors config.ModelArgs (reference config.py:5-19) plus the
 * FeedForward hidden size, which the reference infers from the weights
 * (llama3.py:89-95). */
/* vocab_size 0 makes a layer-only context (standalone TransformerBlock /
 * Attention); n_layers 0 makes an op-only context. */
typedef struct l3_dims {
    int32_t dim;            /* D */
    int32_t n_layers;
    int32_t n_heads;        /* H */
    int32_t n_kv_heads;     /* KVH (already resolved: never "None") */
    int32_t vocab_size;     /* VS */
    int32_t hidden_dim;     /* FD */
    int32_t max_seq_len;    /* M: KV-cache positions and RoPE table rows */
    int32_t max_batch_size; /* KV-cache batch rows */
    float norm_eps;
} l3_dims;

/* Weight kinds for l3_upload_weight; names follow the .npz keys the reference
 * reads (llama3.py:219-237, 269, 280-281).  Shapes are the stored [out, in]. */
enum l3_weight_kind {
    L3_W_EMBED = 0,      /* model.embed_tokens.weight            [VS, D]        */
    L3_W_Q = 1,          /* model.layers.i.self_attn.q_proj      [H*HD, D]      */
    L3_W_K = 2,          /* ...k_proj                            [KVH*HD, D]    */
    L3_W_V = 3,          /* ...v_proj                            [KVH*HD, D]    */
    L3_W_O = 4,          /* ...o_proj                            [D, H*HD]      */
    L3_W_GATE = 5,       /* model.layers.i.mlp.gate_proj         [FD, D]        */
    L3_W_UP = 6,         /* ...up_proj                           [FD, D]        */
    L3_W_DOWN = 7,       /* ...down_proj                         [D, FD]        */
    L3_W_ATTN_NORM = 8,  /* model.layers.i.input_layernorm       [D]            */
    L3_W_FFN_NORM = 9,   /* ...post_attention_layernorm          [D]            */
    L3_W_FINAL_NORM = 10,/* model.norm.weight                    [D]            */
    L3_W_LM_HEAD = 11    /* lm_head.weight                       [VS, D]        */
};

/* Kernel ids for l3_kernel_stats (per-kind HIP-event timing).  L3_K_EMBED counts nothing
 * since layer 0 gathers its input rows from the embedding table (llama3.py:287 fused into
 * its QKV and O-proj launches); the id is kept so the numbering stays stable. */
enum l3_kernel_id {
    L3_K_EMBED = 0, L3_K_QKV = 1, L3_K_ATTN = 2, L3_K_OPROJ = 3, L3_K_GATEUP = 4,
    L3_K_DOWN = 5, L3_K_LMHEAD = 6, L3_K_ARGMAX = 7, L3_K_GATHER = 8, L3_K_COUNT = 9
};

/* ---- errors / devices ---------------------------------------------------- */
const char* l3_last_error(void);
int l3_device_count(int32_t* n);
int l3_version(int32_t* major, int32_t* minor);
/* sha256 prefix of the sources the library was built from (kernels, runtime, this header,
 * the Makefile); bench lines and profile artefacts are keyed to it. */
const char* l3_source_hash(void);

/* ---- context (replaces Llama.__init__, llama3.py:265-283) ---------------- */
/* n_layers may be 0 (op-only context); ctx owns all device memory. */
int l3_create(int32_t device, const l3_dims* dims, l3_ctx** out);
int l3_destroy(l3_ctx* ctx);
/* Upload one tensor (host fp32, [rows, cols] row-major).  layer is ignored for
 * EMBED/FINAL_NORM/LM_HEAD.  Replaces the weight.get(...) calls of
 * TransformerBlock.__init__ (llama3.py:217-237) and Llama.__init__ (:269-281). */
int l3_upload_weight(l3_ctx* ctx, int32_t layer, int32_t kind, const float* host,
                     int64_t rows, int64_t cols);
/* Mark the upload phase complete (QKV and gate/up are fused at upload time:
 * q|k|v rows stacked, gate/up interleaved in 16-row groups).  Folds each
 * RMSNorm weight into the columns of the GEMM that consumes the normalised
 * rows (attention norm -> QKV, FFN norm -> gate/up, final norm -> lm_head)
 * where both were uploaded.  Must be called once after the uploads, before
 * any forward; entry points check that the tensors they need were uploaded. */
int l3_finalize(l3_ctx* ctx);
/* Zero every KV cache (the reference never does this; provided for reuse). */
int l3_reset_cache(l3_ctx* ctx);

/* ---- forward (replaces Llama.__call__, llama3.py:285-308) ----------------- */
/* ids [B, L] int64 (host); logits_host [B, VS] fp32 = the reference's
 * logits[:, 0, :].  Caches persist across calls, exactly as the reference's. */
int l3_forward_host(l3_ctx* ctx, const int64_t* ids_host, int32_t B, int32_t L,
                    int32_t start_pos, float* logits_host);
/* Batch split of a model forward (extension; default 2 parts, env L3_BATCH_SPLIT): the layers
 * run on `parts` contiguous ranges of the B rows, each on its own HIP stream, joined on the
 * context stream before the call returns; the lm_head runs per part when every part picks the
 * batch's lm_head tile, else once after the join.  Rows never interact (llama3.py:163-211) and
 * every part keeps the unsplit batch's kernels, so the results are bit-identical for any split;
 * one part's kernels fill another's launch tails.  A forward uses fewer parts when a part would hold fewer
 * than max(min_tokens, 257) tokens (B*L/parts), one part when a layer exceeds 1 TFLOP (long
 * kernels: no tails to fill) and one part for graph-captured decode steps.
 * parts in [1, 4], min_tokens >= 1 (default 8192). */
int l3_set_batch_split(l3_ctx* ctx, int32_t parts, int64_t min_tokens);
/* Last layer of a model forward (extension; default on, env L3_LAST_LAYER_ALL_ROWS=1 turns it
 * off): only each sequence's last position reaches the logits (llama3.py:304), so the last
 * block runs its QKV GEMM on every position (the KV cache gets every slot, as the reference's)
 * and its attention, O-proj and FFN on the last position only.  The caches are the full
 * block's, bit for bit.  The logits equal the all-rows forward's to fp32 rounding, not bit for
 * bit: past 256 rows (B*L) the pruned row's attention runs on the decode kernel (K / V-only QKV
 * for every row plus a B-row q GEMM), at <= 256 rows on the prefill kernel over each sequence's
 * last q-blocks; the small GEMMs after it take the skinny MFMA kernel at M = B either way
 * (tests: <= 1e-5 against the all-rows logits, C smoke 1e-4).  all_rows != 0: every position
 * through the whole block. */
int l3_set_last_layer_rows(l3_ctx* ctx, int32_t all_rows);
/* GEMM arithmetic of the prefill projections (extension; default off, env L3_GEMM_X6=1 turns it
 * on for new contexts).  on != 0: the QKV / O-proj / gate|up / down GEMMs past 32 rows run on the
 * x6 kernel — each fp32 operand cut exactly into three bf16 pieces and the product summed from
 * the six largest piece products on bf16 MFMAs (gemm_x6.h; error against an fp64 product at or
 * below the fp32 MFMA kernel's, tools/gemm_tune x6acc) — with 1.5x the layer weights' memory for
 * the pieces, made now (or at l3_finalize).  Results round differently from the fp32 MFMA path
 * (not bit-identical to it); batch-1 / batched decode (<= 256 rows), the lm_head and the
 * attention keep their fp32 kernels.  on == 0 frees the pieces. */
int l3_set_gemm_x6(l3_ctx* ctx, int32_t on);
/* Same with device-resident ids (int32 [B, L]) and logits ([B, VS]); async. */
int l3_forward_dev(l3_ctx* ctx, const int32_t* ids_dev, int32_t B, int32_t L,
                   int32_t start_pos, float* logits_dev);
/* One greedy step (Llama.generate body, llama3.py:313-320): forward + argmax
 * (lowest index on ties, as np.argmax).  next_ids_host [B] int64;
 * logits_host may be NULL. */
int l3_greedy_step_host(l3_ctx* ctx, const int64_t* ids_host, int32_t B, int32_t L,
                        int32_t start_pos, int64_t* next_ids_host, float* logits_host);

/* The whole greedy loop on the device (same schedule and ids as Llama.generate,
 * llama3.py:310-321, but not lazy: all max_new_tokens - L steps run, each one
 * hipGraph replay, one copy-back at the end).  out_ids_host [B, max_new_tokens - L]. */
int l3_greedy_generate_host(l3_ctx* ctx, const int64_t* ids_host, int32_t B, int32_t L,
                            int32_t max_new_tokens, int64_t* out_ids_host);
/* The same loop, also returning each step's winning logit (the value np.argmax picked at
 * llama3.py:320, i.e. logits[b, -1, id]) in out_vals [B, max_new_tokens - L] fp32: the replayed
 * steps record it beside the id on the device, the eager steps read it from their logits rows.
 * Pins a decode path's values, not only its ids, against the reference (extension). */
int l3_greedy_generate_values_host(l3_ctx* ctx, const int64_t* ids_host, int32_t B, int32_t L,
                                   int32_t max_new_tokens, int64_t* out_ids_host, float* out_vals);

/* ---- one block (replaces TransformerBlock.__call__, llama3.py:239-261) --- */
/* x [B, L, D] fp32 host -> out [B, L, D]; uses and updates layer's KV cache. */
int l3_layer_forward_host(l3_ctx* ctx, int32_t layer, const float* x_host, int32_t B,
                          int32_t L, int32_t start_pos, float* out_host);

/* ---- one attention (replaces Attention.__call__, llama3.py:155-213) ------ */
/* x [B, L, D] = the already-normalised block input; out [B, L, D] = O-projection
 * output without residual.  Uses and updates the layer's KV cache.  Needs a
 * context whose layer holds only attention weights (no attention norm: a
 * folded layer is refused). */
int l3_attention_forward_host(l3_ctx* ctx, int32_t layer, const float* x_host, int32_t B,
                              int32_t L, int32_t start_pos, float* out_host);

/* ---- op-level entry points (reference module functions and classes) ------ */
/* softmax over the last axis (llama3.py:22-24); rows x n. */
int l3_op_softmax_host(l3_ctx* ctx, const float* x, int64_t rows, int64_t n, float* y);
/* argmax over the last axis with np.argmax's tie-break: first index of the maximum, the first
 * NaN if any (llama3.py:320); rows x n -> rows int32. */
int l3_op_argmax_host(l3_ctx* ctx, const float* x, int64_t rows, int64_t n, int32_t* out);
/* silu (llama3.py:27-28); n elements. */
int l3_op_silu_host(l3_ctx* ctx, const float* x, int64_t n, float* y);
/* RMSNorm (llama3.py:111-114); rows x dim. */
int l3_op_rmsnorm_host(l3_ctx* ctx, const float* x, const float* w, int64_t rows,
                       int64_t dim, float eps, float* y);
/* apply_rotary_emb (llama3.py:41-76) on one tensor x [B, L, nh, HD] with fp32
 * cos/sin tables [L, HD/2]. */
int l3_op_rope_host(l3_ctx* ctx, const float* x, int32_t B, int32_t L, int32_t nh,
                    int32_t hd, const float* cos_t, const float* sin_t, float* y);
/* FeedForward.__call__ (llama3.py:97-103): x [rows, D], W as stored. */
int l3_op_ffn_host(l3_ctx* ctx, const float* x, int64_t rows, int32_t dim, int32_t hidden,
                   const float* w_gate, const float* w_up, const float* w_down, float* y);
/* y [rows, N] = x [rows, K] @ W[N, K]^T (the reference's `x @ W.T`). */
int l3_op_linear_host(l3_ctx* ctx, const float* x, int64_t rows, int32_t K, int32_t N,
                      const float* w, float* y);

/* ---- pinned host memory (fast host-buffer path) ------------------------------ */
/* Page-locked host allocation: l3_forward_host / l3_greedy_step_host / l3_d2h copying into
 * it run as DMA at PCIe rate (the reference returns host logits, llama3.py:307-308; the
 * Python binding hands these buffers out as the returned NumPy arrays).  Device-independent. */
int l3_host_alloc(size_t bytes, void** ptr);
int l3_host_free(void* ptr);

/* ---- device memory helpers (bench: inputs resident in HBM) --------------- */
int l3_dev_alloc(l3_ctx* ctx, size_t bytes, void** ptr);
int l3_dev_free(l3_ctx* ctx, void* ptr);
int l3_h2d(l3_ctx* ctx, void* dst_dev, const void* src_host, size_t bytes);
int l3_d2h(l3_ctx* ctx, void* dst_host, const void* src_dev, size_t bytes);
int l3_synchronize(l3_ctx* ctx);

/* ---- kernel timing (HIP events on the context stream) -------------------- */
/* mask: bit k = record HIP events around launches of l3_kernel_id k (0 = off);
 * also resets the stats */
int l3_kernel_timing(l3_ctx* ctx, int32_t mask);
/* total milliseconds and launch count per l3_kernel_id since last reset */
int l3_kernel_stats(l3_ctx* ctx, double* total_ms, int64_t* count);
/* Greedy-decode counters (extension; llama3.py:310-321 has no counterpart): decode steps
 * served by a captured-graph replay, and of those the ones a speculative step (launched when
 * the previous l3_greedy_step_host returned) answered. */
int l3_decode_stats(l3_ctx* ctx, int64_t* graph_steps, int64_t* speculative_hits);
/* Whether the captured batch-1 decode step is the persistent kernel (one launch per greedy step,
 * decode_persist.hip: every layer, the lm_head and the argmax with in-launch hand-offs) rather
 * than the 25-kernel graph.  The persistent step is the default for shapes it takes (HD <= 64,
 * decode_persist_ok) on devices it can run on (every one of its workgroups resident: enough CUs,
 * checked at capture; otherwise the graph is captured); env L3_DECODE_PERSIST (read at capture):
 * 1 default, 0 the graph.  A persistent step that gives up on an in-launch hand-off is recovered,
 * not reported: the steps queued ahead are undone, the step runs again on the graph path with
 * the same result, and the context stays on the graph path (l3_decode_recoveries counts this). */
int l3_decode_persistent(l3_ctx* ctx, int32_t* active);
/* Persistent decode steps recovered on the graph path over the context's life (see above). */
int l3_decode_recoveries(l3_ctx* ctx, int64_t* count);
/* Device bounds checks (no reference counterpart; SURVEY.md §5 "device bounds asserts in a debug
 * build"): in the check build (libllama3hip_check.so, `make -C llama3.np_amd/csrc check-lib`;
 * load it with L3_LIB_PATH) every kernel counts the indices that leave their buffers —
 * counts[0] K / V cache slots outside [0, max_seq_len), counts[1] attention launches whose keys
 * pass max_seq_len, counts[2] token ids outside the vocabulary, counts[3] reserved — and this
 * returns the counts of the context's device since the last call (then clears them);
 * *enabled = 1 in the check build, 0 in the release library (whose counts stay 0).
 * l3_device_check_selftest records one of each of the first three classes (plumbing check). */
int l3_device_check_counts(l3_ctx* ctx, uint32_t* counts, int32_t* enabled);
int l3_device_check_selftest(l3_ctx* ctx);
/* Lazy greedy decode runs up to 16 steps ahead of the caller on the device (undone if the
 * caller leaves the schedule, so results are unchanged), and at most ~4 ms of decode work by
 * the measured step time: a caller that stops early (EOS, an abandoned generator) or makes any
 * other call first waits for at most that much queued work plus one step (stories15M: 16 steps
 * ≈ 1.6 ms; Llama-3-8B shape at ~5 ms per step: no run-ahead).  No step at position >= end_pos
 * is run ahead (Llama.generate passes its max_new_tokens, llama3.py:312).  end_pos <= 0: no
 * horizon.  Env L3_DECODE_SPECULATE=0 turns run-ahead off. */
int l3_set_decode_horizon(l3_ctx* ctx, int32_t end_pos);

/* ---- multi-GPU: batch-sharded prefill + RCCL logits gather (xGMI) -------- */
/* The reference never mixes batch rows (llama3.py:163-211), so the batch axis shards with no
 * exchange until the last-position logits (llama3.py:304-307), which one RCCL gather brings to
 * the root.  Two ways to drive it: one process per GPU (l3_comm_*, what torch.distributed.run
 * launches) or one process driving N devices (l3_group_*, below). */
#define L3_BUSID_LEN 16  /* PCI bus id "dddd:bb:dd.f" + NUL, as hipDeviceGetPCIBusId writes it */
/* 128-byte RCCL unique id (rank 0 creates, every rank receives it). */
int l3_comm_unique_id(uint8_t id_out[128]);
int l3_comm_init(l3_ctx* ctx, int32_t nranks, int32_t rank, const uint8_t id[128]);
/* What RCCL reports for this rank — ncclCommCount (nranks), ncclCommUserRank (rank),
 * ncclCommCuDevice (device) — and every rank's PCI bus id, all-gathered over the communicator
 * into busids [nranks][L3_BUSID_LEN] (busids_cap entries of room; NULL: skip the gather).
 * Collective when busids is given: every rank calls it.  Without a communicator: 1 rank, this
 * device.  Lets a multi-GPU run prove it ran N ranks on N distinct devices. */
int l3_comm_info(l3_ctx* ctx, int32_t* nranks, int32_t* rank, int32_t* device, char* busids,
                 int64_t busids_cap);
/* on != 0: the overlapped gather form below (default off: serialized). */
int l3_comm_set_overlap(l3_ctx* ctx, int32_t on);
/* Gather each rank's logits rows [rows_r, VS] (device) into root's dst_dev
 * [sum rows, VS] in rank order; rows_per_rank has nranks entries.  Async, on
 * the context stream, after the forward that wrote src; any later call runs
 * after it.  An l3_d2h of dst_dev or l3_synchronize sees the gathered rows.
 * Calls of one step must be made in the same order on every rank (RCCL
 * point-to-point: one grouped ncclRecv per peer on the root, one ncclSend per
 * non-root rank).  Only for contexts with their own communicator (l3_comm_init):
 * a group's members gather through l3_group_* (one thread, all ranks in one
 * RCCL group).  l3_comm_set_overlap(ctx, 1) takes the overlapped form: when
 * the next call is l3_forward_dev with its batch split, that forward's second
 * part starts from the point before the gather (its layers overlap the
 * transfer), its first part runs after the gather, and every part's lm_head
 * waits for it (it reads the rows the lm_head rewrites).  Env L3_COMM_MODE (A/B
 * only): 1 serialized (default), 3 overlapped, 0 a comm stream ordered by events
 * (measured slower, DESIGN.md Multi-GPU). */
int l3_comm_gather_logits(l3_ctx* ctx, const float* src_dev, float* dst_dev,
                          const int64_t* rows_per_rank, int32_t root);
/* Greedy ids only (SURVEY 8(e) option): argmax of each rank's logits rows
 * [rows_r, VS] (device; first index on ties, llama3.py:320) gathered as int32
 * into root's ids_dst_dev [sum rows] in rank order — B x 4 bytes over xGMI
 * instead of B x VS x 4.  Ordered on the context stream.  Replaces the host
 * np.argmax of llama3.py:320 over the gathered logits. */
int l3_comm_gather_argmax(l3_ctx* ctx, const float* logits_dev, int32_t* ids_dst_dev,
                          const int64_t* rows_per_rank, int32_t root);
int l3_comm_barrier(l3_ctx* ctx);
/* max over ranks of one host double (in place; synchronous) — e.g. step time */
int l3_comm_allreduce_max(l3_ctx* ctx, double* value);

/* ---- one process, N devices (SURVEY 8(b) l3_group_*) -------------------
 * The single-process drop-in of Llama.__call__ / Llama.generate (llama3.py:285-321) over the
 * GPUs of a node: one context per device, communicators from ncclCommInitAll, every call
 * launched asynchronously on all devices from one thread, one grouped RCCL gather, one sync.
 * Batch row r lives on member r % n as its local row r / n (a mapping that does not depend on B,
 * so each row's KV cache stays on one device across calls of any batch size, exactly as the
 * reference's cache row r persists, llama3.py:138-153,184-187); each member's max_batch_size is
 * ceil(max_batch_size / n).  Rows on one device only (B = 1: single-prompt greedy decode) run
 * that member's own single-device path (graph-replayed decode steps).  Results are the
 * single-device forward's: every member runs the same kernels on its rows (rows never interact);
 * each row's logits are bit-identical to a single-device run of the same rows whenever both
 * pick the same kernels for their row counts (every prefill of more than 256 tokens per part). */
typedef struct l3_group l3_group;
/* devices: n device ordinals (distinct); dims: the model, max_batch_size the global batch. */
int l3_group_create(int32_t ndev, const int32_t* devices, const l3_dims* dims, l3_group** out);
int l3_group_destroy(l3_group* g);
/* member i's context (owned by the group: never l3_destroy it); for per-device buffers,
 * timing and settings (l3_set_batch_split, l3_kernel_timing, ...). */
int l3_group_context(l3_group* g, int32_t i, l3_ctx** ctx);
/* l3_upload_weight / l3_finalize on every member. */
int l3_group_upload_weight(l3_group* g, int32_t layer, int32_t kind, const float* host, int64_t rows,
                           int64_t cols);
int l3_group_finalize(l3_group* g);
/* Llama.__call__ (llama3.py:285-308): ids [B, L] int64 host -> logits_host [B, VS] fp32 in
 * row order.  Each member uploads and runs its rows, the root (member 0) receives the others'
 * rows over RCCL and copies the assembled rows back. */
int l3_group_forward_host(l3_group* g, const int64_t* ids_host, int32_t B, int32_t L,
                          int32_t start_pos, float* logits_host);
/* Device-resident form (bench): ids_dev[i] = member i's rows (int32 [B_i, L], rows i, i + n, ...,
 * on device i), logits_dev = [B, VS] on member 0 in row order.  Async; l3_group_synchronize. */
int l3_group_forward_dev(l3_group* g, const int32_t* const* ids_dev, int32_t B, int32_t L,
                         int32_t start_pos, float* logits_dev);
/* One greedy step (llama3.py:313-320): forward + argmax per member (first index on ties),
 * only the B int32 ids gathered.  next_ids_host [B] int64. */
int l3_group_greedy_step_host(l3_group* g, const int64_t* ids_host, int32_t B, int32_t L,
                              int32_t start_pos, int64_t* next_ids_host);
int l3_group_synchronize(l3_group* g);

#ifdef __cplusplus
}
#endif
#endif /* LLAMA3HIP_H */
