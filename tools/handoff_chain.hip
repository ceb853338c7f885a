// Feasibility probe for a persistent batch-1 decode step: what one
// all-to-all edge costs inside a launch on MI355X.  E edges, each: every workgroup publishes its
// share of a V-value vector as 8-byte {tag = edge + 1, value} granules (one agent-scope relaxed
// atomic store each, R2 of cdna_hip_programming.md Guideline 16), then every workgroup reads all
// V granules (agent-scope relaxed loads, re-read until every tag matches) and sums them; the sum
// feeds the next edge's values, so the edges are a dependent chain — a decode step's
// stage-to-stage hand-off (every output of a stage needs the whole input vector).
// Compared with the graph launch floor (tools/launch_floor: 1.77 us per dependent empty kernel).
// Spins are bounded: a workgroup that waits too long sets *tmo and leaves (no hang).
//   Build: make -C tools handoff_chain ; run: tools/handoff_chain
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e = (x);                                                                \
        if (e != hipSuccess) {                                                             \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                         \
            exit(2);                                                                       \
        }                                                                                  \
    } while (0)

typedef unsigned long long u64;

__device__ __forceinline__ void put(u64* g, unsigned tag, float v) {
    __hip_atomic_store(g, ((u64)tag << 32) | __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int PER>  // granules per thread (V <= 256 * PER)
__global__ void __launch_bounds__(256) chain_kernel(u64* buf, int E, int V, float* out, unsigned* tmo) {
    __shared__ float red[4];
    __shared__ int bad;
    const int tid = threadIdx.x, G = gridDim.x, wg = blockIdx.x;
    const int per_wg = (V + G - 1) / G;
    float carry = 1.0f + wg * 1e-3f;
    if (tid == 0) bad = 0;
    __syncthreads();
    for (int e = 0; e < E; ++e) {
        u64* g = buf + (size_t)e * V;
        const unsigned tag = e + 1;
        // publish this workgroup's share
        for (int i = tid; i < per_wg; i += 256) {
            const int idx = wg * per_wg + i;
            if (idx < V) put(g + idx, tag, carry + idx * 1e-6f);
        }
        // read every granule until all tags match (one pass = PER loads per thread in flight)
        float v[PER];
        bool ok = false;
        for (unsigned spin = 0; !ok; ++spin) {
            ok = true;
#pragma unroll
            for (int k = 0; k < PER; ++k) {
                const int idx = tid + 256 * k;
                if (idx < V) {
                    const u64 x = __hip_atomic_load(g + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    v[k] = __uint_as_float((unsigned)x);
                    ok &= (unsigned)(x >> 32) == tag;
                } else {
                    v[k] = 0.f;
                }
            }
            ok = __all(ok);
            if (!ok && spin > (1u << 20)) {
                atomicOr(tmo, 1u);
                bad = 1;
                break;
            }
            if (!ok) __builtin_amdgcn_s_sleep(1);
        }
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < PER; ++k) s += v[k];
        for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
        if ((tid & 63) == 0) red[tid >> 6] = s;
        __syncthreads();
        if (bad) return;
        carry = (red[0] + red[1] + red[2] + red[3]) * 1e-6f + 1.0f;
        __syncthreads();
    }
    if (tid == 0) out[wg] = carry;
}

int main() {
    const int E = 26, Vs[] = {288, 768, 1728}, Gs[] = {64, 128, 256};
    u64* buf;
    float* out;
    unsigned* tmo;
    CK(hipMalloc(&buf, (size_t)E * 2048 * 8));
    CK(hipMalloc(&out, 256 * 4));
    CK(hipMalloc(&tmo, 4));
    CK(hipMemset(tmo, 0, 4));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int G : Gs)
        for (int V : Vs) {
            double us[2];
            for (int which = 0; which < 2; ++which) {
                const int edges = which ? E : 0;
                auto launch = [&]() {
                    CK(hipMemsetAsync(buf, 0, (size_t)E * V * 8, s));
                    if (V <= 512)
                        hipLaunchKernelGGL(chain_kernel<2>, dim3(G), dim3(256), 0, s, buf, edges, V, out, tmo);
                    else
                        hipLaunchKernelGGL(chain_kernel<7>, dim3(G), dim3(256), 0, s, buf, edges, V, out, tmo);
                };
                for (int r = 0; r < 20; ++r) launch();
                CK(hipStreamSynchronize(s));
                const int reps = 200;
                CK(hipEventRecord(e0, s));
                for (int r = 0; r < reps; ++r) launch();
                CK(hipEventRecord(e1, s));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                us[which] = ms * 1e3 / reps;
            }
            unsigned t = 0;
            CK(hipMemcpy(&t, tmo, 4, hipMemcpyDeviceToHost));
            printf("G=%3d V=%4d: launch+memset %.2f us, %d edges %.2f us -> %.3f us per edge%s\n", G, V, us[0], E,
                   us[1], (us[1] - us[0]) / E, t ? "  (TIMEOUT seen)" : "");
        }
    return 0;
}
