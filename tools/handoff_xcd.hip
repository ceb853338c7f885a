// Probe: what an all-to-all hand-off costs when every participant sits on ONE XCD (shared L2)
// against the same chain spread over all 8 XCDs (tools/handoff_chain.hip).
// E dependent edges; per edge every active workgroup publishes its share of V {tag, value}
// granules and re-reads all V until every tag matches (bounded spins, *tmo on timeout).
//   mode 0 (agent): agent-scope relaxed atomic stores / loads (sc1: through L2 to the MALL),
//                   participants = every workgroup (stride 1) or wg % 8 == 0 (stride 8)
//   modes 1-4 (below): store / load pairs for participants wg % 8 == 0, which round-robin
//                   dispatch puts on one XCD — each participant records HW_REG_XCC_ID
// The grid is 256 workgroups (one per CU); non-participants leave at once.
//   Build: make -C tools handoff_xcd ; run: tools/handoff_xcd
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

// MODE 0: agent-scope store + agent-scope load (sc1 both)
// MODE 1: workgroup-scope store (lands in the XCD's L2) + sc0 buffer load (found NOT to see it:
//         timeout — a group-scope load may hit the CU's L1)
// MODE 2: workgroup-scope store + L1 invalidate (buffer_inv sc0) + plain load per poll round
// MODE 3: workgroup-scope store + agent-scope load
// MODE 4: agent-scope store + L1 invalidate + plain load
// MODE 5: non-temporal store (nt) + agent-scope load
template <int MODE>
__device__ __forceinline__ void put(u64* g, unsigned tag, float v) {
    const u64 x = ((u64)tag << 32) | __float_as_uint(v);
    if (MODE == 0 || MODE == 4) __hip_atomic_store(g, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else if (MODE == 5) __builtin_nontemporal_store(x, g);
    else __hip_atomic_store(g, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

template <int MODE>
__device__ __forceinline__ u64 get(u64* base, __amdgpu_buffer_rsrc_t r, int idx) {
    if (MODE == 0 || MODE == 3 || MODE == 5) return __hip_atomic_load(base + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (MODE == 2 || MODE == 4) return __hip_atomic_load(base + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(r, idx * 8, 0, 1);  // sc0: miss L1
    return (u64)(unsigned)v[0] | ((u64)(unsigned)v[1] << 32);
}

template <int PER, int MODE>
__global__ void __launch_bounds__(256) chain_kernel(u64* buf, int E, int V, int stride, float* out,
                                                    unsigned* tmo, unsigned* xcc) {
    __shared__ float red[4];
    __shared__ int bad;
    const int tid = threadIdx.x, wg0 = blockIdx.x;
    if (wg0 % stride) return;
    const int G = gridDim.x / stride, wg = wg0 / stride;
    if (tid == 0) xcc[wg] = __builtin_amdgcn_s_getreg((20) | (0 << 6) | ((16 - 1) << 11)) + 1;
    const int per_wg = (V + G - 1) / G;
    float carry = 1.0f + wg * 1e-3f;
    if (tid == 0) bad = 0;
    __syncthreads();
    for (int e = 0; e < E; ++e) {
        u64* g = buf + (size_t)e * V;
        const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(g, 0, V * 8, 0x00020000);
        const unsigned tag = e + 1;
        for (int i = tid; i < per_wg; i += 256) {
            const int idx = wg * per_wg + i;
            if (idx < V) put<MODE>(g + idx, tag, carry + idx * 1e-6f);
        }
        float v[PER];
        bool ok = false;
        for (unsigned spin = 0; !ok; ++spin) {
            ok = true;
            u64 x[PER];
            if (MODE == 2 || MODE == 4) asm volatile("buffer_inv sc0" ::: "memory");  // drop this CU's L1 lines
#pragma unroll
            for (int k = 0; k < PER; ++k) x[k] = get<MODE>(g, r, min(tid + 256 * k, V - 1));
#pragma unroll
            for (int k = 0; k < PER; ++k) {
                v[k] = tid + 256 * k < V ? __uint_as_float((unsigned)x[k]) : 0.f;
                ok &= (unsigned)(x[k] >> 32) == tag;
            }
            ok = __all(ok);
            if (!ok && spin > (1u << 16)) {
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
    const int E = 26, Vs[] = {288, 768};
    u64* buf;
    float* out;
    unsigned *tmo, *xcc;
    CK(hipMalloc(&buf, (size_t)E * 2048 * 8));
    CK(hipMalloc(&out, 256 * 4));
    CK(hipMalloc(&tmo, 4));
    CK(hipMalloc(&xcc, 256 * 4));
    CK(hipMemset(tmo, 0, 4));
    int dev = 0, cus = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const int grid = cus < 256 ? cus : 256;
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    struct Cfg { int mode, stride; const char* name; } cfgs[] = {
        {0, 1, "agent, all 256 wgs"}, {0, 8, "agent, wg%8==0 (32)"}, {2, 8, "wg st, inv+ld (32)"},
        {3, 8, "wg st, agent ld (32)"}, {4, 8, "agent st, inv+ld (32)"}, {1, 8, "wg st, sc0 ld (32)"},
        {5, 1, "nt st, agent ld, all 256"}, {5, 4, "nt st, agent ld (64)"}, {0, 4, "agent, wg%4==0 (64)"}};
    for (const Cfg& cf : cfgs)
        for (int V : Vs) {
            double us[2];
            for (int which = 0; which < 2; ++which) {
                const int edges = which ? E : 0;
                auto launch = [&]() {
                    CK(hipMemsetAsync(buf, 0, (size_t)E * V * 8, s));
                    switch (cf.mode) {
#define CASE(M) case M: hipLaunchKernelGGL((chain_kernel<4, M>), dim3(grid), dim3(256), 0, s, buf, edges, V, cf.stride, out, tmo, xcc); break;
                        CASE(0) CASE(1) CASE(2) CASE(3) CASE(4) CASE(5)
#undef CASE
                    }
                };
                CK(hipMemset(xcc, 0, 256 * 4));
                for (int r = 0; r < 20; ++r) launch();
                CK(hipStreamSynchronize(s));
                unsigned t0 = 0;
                CK(hipMemcpy(&t0, tmo, 4, hipMemcpyDeviceToHost));
                if (t0) {  // the hand-off never completed: the next configs still run
                    printf("%-22s V=%4d: TIMEOUT in warm-up, not timed\n", cf.name, V);
                    CK(hipMemset(tmo, 0, 4));
                    us[0] = us[1] = -1;
                    break;
                }
                const int reps = 200;
                CK(hipEventRecord(e0, s));
                for (int r = 0; r < reps; ++r) launch();
                CK(hipEventRecord(e1, s));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                us[which] = ms * 1e3 / reps;
            }
            if (us[0] < 0) continue;
            unsigned t = 0, x[256];
            CK(hipMemcpy(&t, tmo, 4, hipMemcpyDeviceToHost));
            CK(hipMemcpy(x, xcc, sizeof x, hipMemcpyDeviceToHost));
            const int n = grid / cf.stride;
            int distinct = 0;
            unsigned seen[16] = {0};
            for (int i = 0; i < n; ++i)
                if (x[i] && x[i] <= 16 && !seen[x[i] - 1]++) ++distinct;
            printf("%-22s V=%4d: %.2f us base, %d edges %.2f us -> %.3f us per edge; participants on %d XCD(s)%s\n",
                   cf.name, V, us[0], E, us[1], (us[1] - us[0]) / E, distinct, t ? "  (TIMEOUT seen)" : "");
        }
    return 0;
}
