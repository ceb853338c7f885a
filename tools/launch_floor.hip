// Launch floor of a graph-replayed chain of dependent small kernels on MI355X: what a decode
// step of 32 launches costs before any kernel does work.  Build: hipcc --offload-arch=gfx950 -O3
// tools/launch_floor.hip -o tools/launch_floor ; run: tools/launch_floor
//   empty   : 32 empty kernels (1 block)
//   touch   : 32 kernels, 48 blocks x 256 threads, each lane loads 16 B of the previous
//             kernel's output and stores 16 B (a dependent round trip per kernel)
//   gemv-ish: 32 kernels, 48 blocks, each lane loads 10 x 16 B from a 2 MB weight buffer
//             (L2/MALL resident) plus 16 B of the previous output, reduces, stores
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

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void k_empty() {}

__global__ void k_touch(const f32x4* in, f32x4* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    out[i] = in[i] + 1.0f;
}

__global__ void k_gemv(const f32x4* w, const f32x4* in, f32x4* out, int nw) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    f32x4 acc = in[i];
#pragma unroll
    for (int t = 0; t < 10; ++t) acc += w[(i * 10 + t) % nw];
    out[i] = acc;
}

int main() {
    const int N = 32, BLK = 48, THR = 256, n = BLK * THR;
    f32x4 *a, *b, *w;
    const int nw = (2 << 20) / 16;
    CK(hipMalloc(&a, n * 16));
    CK(hipMalloc(&b, n * 16));
    CK(hipMalloc(&w, nw * 16));
    CK(hipMemset(a, 0, n * 16));
    CK(hipMemset(b, 0, n * 16));
    CK(hipMemset(w, 0, nw * 16));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    for (int mode = 0; mode < 3; ++mode) {
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        for (int k = 0; k < N; ++k) {
            const f32x4* in = (k & 1) ? b : a;
            f32x4* out = (k & 1) ? a : b;
            if (mode == 0) hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s);
            else if (mode == 1) hipLaunchKernelGGL(k_touch, dim3(BLK), dim3(THR), 0, s, in, out);
            else hipLaunchKernelGGL(k_gemv, dim3(BLK), dim3(THR), 0, s, w, in, out, nw);
        }
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        for (int r = 0; r < 50; ++r) CK(hipGraphLaunch(ge, s));
        CK(hipStreamSynchronize(s));
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        const int reps = 500;
        CK(hipEventRecord(e0, s));
        for (int r = 0; r < reps; ++r) CK(hipGraphLaunch(ge, s));
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const char* name[] = {"empty", "touch", "gemv-ish"};
        printf("%-9s %d kernels per graph: %.2f us per graph, %.3f us per kernel\n", name[mode], N,
               ms * 1e3 / reps, ms * 1e3 / reps / N);
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
    }
    return 0;
}
