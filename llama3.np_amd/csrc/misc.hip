// Bandwidth-bound helper kernels for gfx950: greedy argmax and the
// op-level kernels behind the reference's module functions.  Loads are 16 B per lane where the layout allows (rows are multiples of 4 floats), one wavefront-wide
// reduction per row for the row ops.
#include "kernels.h"

namespace l3 {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
    return v;
}

// argmax over each row with np.argmax's first-index tie-break (llama3.py:320); a NaN wins
// (np.argmax returns the first NaN).  One 1024-thread block per row: each thread has all of
// its float4 loads in flight at once (8 per thread at the 32000-wide vocab), then a wavefront
// butterfly and a 16-way LDS step — a decode step waits on one memory round trip, not on a
// serial walk of the row.
// block-wide finish of a row argmax (1024 threads, every thread's candidate in best / bi): the
// id to out[blockIdx.x]; in a captured decode step also the generate history and the position
// advance (last-arriving row)
// hist_off 1: the step's lm_head has already moved the position on (GemmArgs::pos_adv), so the
// id belongs at pos - 1 and the position stays
__device__ __forceinline__ void argmax_finish(float best, int bi, int32_t* __restrict__ out,
                                              DecState* __restrict__ st, int hist_off = 0, int n_ids = 0) {
    constexpr int NT = 1024;
    const int tid = threadIdx.x;
    group_argmax<64>(best, bi, tid & 63);
    __shared__ float sv[NT / 64];
    __shared__ int si[NT / 64];
    if ((tid & 63) == 0) { sv[tid >> 6] = best; si[tid >> 6] = bi; }
    __syncthreads();
    if (tid < 64) {
        best = tid < NT / 64 ? sv[tid] : -INFINITY;
        bi = tid < NT / 64 ? si[tid] : 0x7fffffff;
        group_argmax<16>(best, bi, tid);  // the NT / 64 = 16 wave results in lanes 0-15
        if (tid == 0) {
            if (n_ids > 0) L3_DCHECK(bi >= 0 && bi < n_ids, CHK_TOKEN_ID);
            out[blockIdx.x] = bi;
            if (st) {
                // captured decode step: record the id in the generate history, and the last row
                // to arrive moves the loop one position on (llama3.py:312-318).  Every block
                // reads pos before its arrival (the fence orders the read and the history store
                // before the atomic), so none sees the advanced value.
                const int pos = st->pos - hist_off, q = pos - st->hist_base;
                if (st->hist && q >= 0 && q < st->hist_cap) st->hist[(int64_t)q * gridDim.x + blockIdx.x] = bi;
                if (st->hist_val && q >= 0 && q < st->hist_cap) st->hist_val[(int64_t)q * gridDim.x + blockIdx.x] = best;
                if (hist_off) {
                    // the lm_head of this step already moved the position on
                } else if (gridDim.x == 1) {
                    // one row (batch-1 decode): this thread is the only reader of pos in this
                    // launch, so it advances it directly — no agent-scope fence (≈1-3 µs of the
                    // step) and no arrival count
                    st->pos = pos + 1;
                } else {
                    __threadfence();
                    if (atomicAdd(&st->arrive, 1u) == gridDim.x - 1) {
                        st->arrive = 0u;
                        st->pos = pos + 1;
                    }
                }
            }
        }
    }
}

__global__ void __launch_bounds__(1024) argmax_kernel(const float* __restrict__ x, int n,
                                                      int32_t* __restrict__ out,
                                                      DecState* __restrict__ st) {
    constexpr int NT = 1024, U = 8;
    const float* row = x + (int64_t)blockIdx.x * n;
    const int tid = threadIdx.x;
    float best = -INFINITY;
    int bi = 0x7fffffff;
    if ((n & 3) == 0) {  // 16-byte rows
        const int n4 = n >> 2;
        for (int base = 0; base < n4; base += NT * U) {
            f32x4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int f = base + u * NT + tid;
                v[u] = f < n4 ? reinterpret_cast<const f32x4*>(row)[f] : f32x4{0.f, 0.f, 0.f, 0.f};
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int f = base + u * NT + tid;
                if (f < n4)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        if (argmax_better(v[u][r], 4 * f + r, best, bi)) { best = v[u][r]; bi = 4 * f + r; }
            }
        }
    } else {
        for (int i = tid; i < n; i += NT)
            if (argmax_better(row[i], i, best, bi)) { best = row[i]; bi = i; }
    }
    argmax_finish(best, bi, out, st, 0, n);
}

// one row from the batch-1 lm_head's per-block (value, index) partials (GemmArgs::amax_part):
// 16 KB instead of the 128 KB logits row for one block to read
__global__ void __launch_bounds__(1024) argmax_parts_kernel(const ArgmaxPart* __restrict__ parts, int n,
                                                            int32_t* __restrict__ out,
                                                            DecState* __restrict__ st, int hist_off) {
    constexpr int NT = 1024, U = 4;
    const int tid = threadIdx.x;
    parts += (int64_t)blockIdx.x * n;  // row blockIdx.x
    float best = -INFINITY;
    int bi = 0x7fffffff;
    for (int base = 0; base < n; base += NT * U) {
        ArgmaxPart q[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int f = base + u * NT + tid;
            q[u] = f < n ? parts[f] : ArgmaxPart{-INFINITY, 0x7fffffff};
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (argmax_better(q[u].v, q[u].i, best, bi)) { best = q[u].v; bi = q[u].i; }
    }
    argmax_finish(best, bi, out, st, hist_off);
}

// row softmax (llama3.py:22-24): one wavefront per row, three passes over the row
// (max, sum of exp, normalise); -inf entries give exact zeros.
__global__ void softmax_kernel(const float* __restrict__ x, float* __restrict__ y, int64_t rows,
                               int n) {
    const int lane = threadIdx.x & 63;
    const int64_t row = blockIdx.x * (int64_t)(blockDim.x >> 6) + (threadIdx.x >> 6);
    if (row >= rows) return;
    const float* xr = x + row * n;
    float* yr = y + row * n;
    float m = -INFINITY;
    for (int i = lane; i < n; i += 64) m = fmaxf(m, xr[i]);
    m = wave_max(m);
    float s = 0.f;
    for (int i = lane; i < n; i += 64) s += __expf(xr[i] - m);
    s = wave_sum(s);
    const float inv = 1.0f / s;
    for (int i = lane; i < n; i += 64) yr[i] = __expf(xr[i] - m) * inv;
}

__global__ void silu_kernel(const float* __restrict__ x, float* __restrict__ y, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const float v = x[i];
        y[i] = v * (1.0f / (1.0f + __expf(-v)));
    }
}

// RMSNorm (llama3.py:111-114): one wavefront per row.
__global__ void rmsnorm_kernel(const float* __restrict__ x, const float* __restrict__ w,
                               float* __restrict__ y, int64_t rows, int dim, float eps) {
    const int lane = threadIdx.x & 63;
    const int64_t row = blockIdx.x * (int64_t)(blockDim.x >> 6) + (threadIdx.x >> 6);
    if (row >= rows) return;
    const float* xr = x + row * dim;
    float s = 0.f;
    for (int i = lane; i < dim; i += 64) s += xr[i] * xr[i];
    s = wave_sum(s);
    const float inv = 1.0f / sqrtf(s / (float)dim + eps);
    for (int i = lane; i < dim; i += 64) y[row * dim + i] = xr[i] * inv * w[i];
}

// interleaved-pair RoPE (llama3.py:41-76) on x [B, L, nh, hd] with tables [L, hd/2].
__global__ void rope_kernel(const float* __restrict__ x, float* __restrict__ y,
                            const float* __restrict__ cs, const float* __restrict__ sn, int B,
                            int L, int nh, int hd) {
    const int half = hd >> 1;
    const int64_t pairs = (int64_t)B * L * nh * half;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < pairs;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int k = (int)(i % half);
        const int64_t bl = i / ((int64_t)half * nh);
        const int l = (int)(bl % L);
        const float re = x[2 * i], im = x[2 * i + 1];
        const float c = cs[l * half + k], s = sn[l * half + k];
        y[2 * i] = re * c - im * s;
        y[2 * i + 1] = re * s + im * c;
    }
}

static inline unsigned grid_for(int64_t n, int block) {
    int64_t g = (n + block - 1) / block;
    if (g > 4096) g = 4096;
    return (unsigned)(g < 1 ? 1 : g);
}

hipError_t launch_argmax(const float* logits, int64_t rows, int n, int32_t* out, hipStream_t s,
                         DecState* st) {
    hipLaunchKernelGGL(argmax_kernel, dim3((unsigned)rows), dim3(1024), 0, s, logits, n, out, st);
    return hipGetLastError();
}
hipError_t launch_argmax_parts(const ArgmaxPart* parts, int nparts, int32_t* out, hipStream_t s,
                               DecState* st, int hist_off, int rows) {
    hipLaunchKernelGGL(argmax_parts_kernel, dim3(rows), dim3(1024), 0, s, parts, nparts, out, st, hist_off);
    return hipGetLastError();
}
hipError_t launch_softmax(const float* x, float* y, int64_t rows, int n, hipStream_t s) {
    hipLaunchKernelGGL(softmax_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s, x, y, rows,
                       n);
    return hipGetLastError();
}

hipError_t launch_silu(const float* x, float* y, int64_t n, hipStream_t s) {
    hipLaunchKernelGGL(silu_kernel, dim3(grid_for(n, 256)), dim3(256), 0, s, x, y, n);
    return hipGetLastError();
}

hipError_t launch_rmsnorm(const float* x, const float* w, float* y, int64_t rows, int dim,
                          float eps, hipStream_t s) {
    hipLaunchKernelGGL(rmsnorm_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s, x, w, y,
                       rows, dim, eps);
    return hipGetLastError();
}

hipError_t launch_rope(const float* x, float* y, const float* cos_t, const float* sin_t, int B,
                       int L, int nh, int hd, hipStream_t s) {
    if (hd % 2) return hipErrorInvalidValue;
    hipLaunchKernelGGL(rope_kernel, dim3(grid_for((int64_t)B * L * nh * (hd / 2), 256)), dim3(256),
                       0, s, x, y, cos_t, sin_t, B, L, nh, hd);
    return hipGetLastError();
}

// W[r][k] *= w[k]: folds an RMSNorm weight into the K columns of the matrix that consumes the
// normalised activations (rmsnorm(x) @ W^T = diag(1/rms(x)) * x @ (W * w)^T), once at
// l3_finalize.  HBM-bound, float4 per thread.
__global__ void fold_cols_kernel(float* W, int64_t n4, int K4, const float* w) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n4) return;
    f32x4 v = reinterpret_cast<f32x4*>(W)[i];
    v *= reinterpret_cast<const f32x4*>(w)[i % K4];
    reinterpret_cast<f32x4*>(W)[i] = v;
}

hipError_t launch_fold_cols(float* W, int64_t rows, int K, const float* w, hipStream_t s) {
    if (K % 4) return hipErrorInvalidValue;
    const int64_t n4 = rows * (K / 4);
    if (n4 == 0) return hipSuccess;
    hipLaunchKernelGGL(fold_cols_kernel, dim3(grid_for(n4, 256)), dim3(256), 0, s, W, n4, K / 4, w);
    return hipGetLastError();
}

// undo of a speculative decode step's K / V append (runtime.hip, l3_greedy_step_host)
// Put back one cache slot from kv_bak (the run-ahead undo).  With a guard (the persistent batch-1
// step, B = 1), what to put back is decided on the device when the restore runs, stream-ordered
// after the steps it undoes: nothing if no step gave up; else nothing past the failed position,
// everything before it, and at it only the units whose layer workgroup stored its write mark under
// the failing launch's tag (decode_persist.hip: it wrote those slots and their kv_bak entries)
__global__ void kv_restore_kernel(float* cache, const float* bak, int B, int KVH, int Smax, int HD, int pos,
                                  KvGuard g) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= B * KVH * HD) return;
    const int d = i % HD, bh = i / HD;  // bh = b * KVH + h
    if (g.err) {
        const unsigned e = __hip_atomic_load(g.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (e) {
            const int fp = (int)e - 1;
            if (pos > fp) return;  // never ran
            if (pos == fp) {       // ran up to its give-up: the units its workgroups wrote
                const int wg = ((g.col_base + i) >> 1) / g.per;
                if (g.wmarks[wg] != g.epoch[2]) return;
            }
        }
    }
    if (i == 0) L3_DCHECK(pos >= 0 && pos < Smax, CHK_KV_SLOT);
    cache[((int64_t)bh * Smax + pos) * HD + d] = bak[i];
}

hipError_t launch_kv_restore(float* cache, const float* bak, int B, int KVH, int Smax, int HD, int pos,
                             hipStream_t s, KvGuard g) {
    const int n = B * KVH * HD;
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(kv_restore_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, cache, bak, B, KVH,
                       Smax, HD, pos, g);
    return hipGetLastError();
}

// device bounds checks (kernels.h): a check build's self-test — one violation of each class
// recorded, so a caller can see the counters reach the host
__global__ void dcheck_selftest_kernel(int n) {
    if (threadIdx.x == 0 && blockIdx.x == 0)
        for (int c = 0; c < n; ++c) L3_DCHECK(false, c);
}

hipError_t launch_dcheck_selftest(hipStream_t s) {
    hipLaunchKernelGGL(dcheck_selftest_kernel, dim3(1), dim3(64), 0, s, (int)CHK_TOKEN_ID + 1);
    return hipGetLastError();
}

hipError_t dcheck_collect_misc(unsigned* out) { return dcheck_collect(out); }

}  // namespace l3
