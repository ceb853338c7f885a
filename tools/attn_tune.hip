// Attention variant tuner: times attn_fwd_kernel configurations interleaved in one process
// and checks each against the first.  Build: make -C tools attn_tune ; run: tools/attn_tune
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#include "../llama3.np_amd/csrc/attn_kernel.h"
#include "attn_research.h"

using namespace l3;

#define CK(x)                                                                                 \
    do {                                                                                      \
        hipError_t e = (x);                                                                   \
        if (e != hipSuccess) {                                                                \
            fprintf(stderr, "%s: %s (%s:%d)\n", #x, hipGetErrorString(e), __FILE__, __LINE__); \
            exit(2);                                                                          \
        }                                                                                     \
    } while (0)

struct Variant {
    std::string name;
    std::function<void(const AttnArgs&, hipStream_t)> run;
};

#define AVAR(HD, QBW, G, KT)                                                                  \
    Variant{"attn<" #HD ",q" #QBW ",g" #G ",kt" #KT ">", [](const AttnArgs& a, hipStream_t s) { \
                constexpr int QW = 16 * QBW * (4 / G);                                        \
                dim3 grid((a.L + QW - 1) / QW, a.H / G, a.B);                                 \
                hipLaunchKernelGGL((attn_fwd_kernel<HD, QBW, G, KT>), grid, dim3(256), 0, s, a); \
            }}

#define AVARPK(HD, QBW, G, KT)                                                                \
    Variant{"attn<" #HD ",q" #QBW ",g" #G ",kt" #KT "> pk", [](const AttnArgs& a, hipStream_t s) { \
                constexpr int QW = 16 * QBW * (4 / G);                                        \
                dim3 grid((a.L + QW - 1) / QW, a.H / G, a.B);                                 \
                hipLaunchKernelGGL((attn_fwd_kernel<HD, QBW, G, KT, true>), grid, dim3(256), 0, s, a); \
            }}

#define ADEF(HD, QBW, G, KT)                                                                  \
    Variant{"defer<" #HD ",q" #QBW ",g" #G ",kt" #KT ">", [](const AttnArgs& a, hipStream_t s) { \
                constexpr int QW = 16 * QBW * (4 / G);                                        \
                dim3 grid((a.L + QW - 1) / QW, a.H / G, a.B);                                 \
                hipLaunchKernelGGL((attn_research_kernel<HD, QBW, G, KT, 0, true>), grid, dim3(256), 0, s, a); \
            }}

#define AABL(ABL)                                                                             \
    Variant{"v1<48,q4,kt64> abl" #ABL, [](const AttnArgs& a, hipStream_t s) {                  \
                dim3 grid((a.L + 255) / 256, a.H, a.B);                                        \
                hipLaunchKernelGGL((attn_research_kernel<48, 4, 1, 64, ABL>), grid, dim3(256), 0, s, a); \
            }}

static void fill(std::vector<float>& v, float lo, float hi, unsigned seed) {
    srand(seed);
    for (auto& x : v) x = lo + (hi - lo) * (float)rand() / (float)RAND_MAX;
}

static void run(const char* label, int B, int L, int H, int KVH, int HD, std::vector<Variant> vars,
                int rounds, int iters, int start_pos = 0) {
    const int Smax = start_pos + L;
    const size_t nq = (size_t)B * L * H * HD, nkv = (size_t)B * KVH * Smax * HD;
    std::vector<float> hq(nq), hk(nkv), hv(nkv);
    fill(hq, -1.f, 1.f, 1);
    fill(hk, -1.f, 1.f, 2);
    fill(hv, -1.f, 1.f, 3);
    float *q, *k, *v, *o;
    CK(hipMalloc(&q, nq * 4)); CK(hipMalloc(&k, nkv * 4)); CK(hipMalloc(&v, nkv * 4)); CK(hipMalloc(&o, nq * 4));
    CK(hipMemcpy(q, hq.data(), nq * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(k, hk.data(), nkv * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(v, hv.data(), nkv * 4, hipMemcpyHostToDevice));
    AttnArgs a{};
    a.q = q; a.cache_k = k; a.cache_v = v; a.out = o;
    a.B = B; a.L = L; a.start_pos = start_pos; a.H = H; a.KVH = KVH; a.HD = HD; a.Smax = Smax;
    const double flops = 4.0 * HD * H * (double)B * L * ((L + 1) / 2.0 + start_pos);  // causal useful part
    printf("\n== %s B=%d L=%d H=%d KVH=%d HD=%d (%.2f GFLOP useful)\n", label, B, L, H, KVH, HD, flops / 1e9);
    std::vector<float> ref(nq), got(nq);
    for (size_t i = 0; i < vars.size(); ++i) {
        CK(hipMemset(o, 0, nq * 4));
        vars[i].run(a, 0);
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(i ? got.data() : ref.data(), o, nq * 4, hipMemcpyDeviceToHost));
        if (i) {
            double md = 0;
            for (size_t t = 0; t < nq; ++t) md = std::max(md, (double)std::fabs(got[t] - ref[t]));
            printf("   check %-20s max|diff| %.3e%s\n", vars[i].name.c_str(), md, md < 1e-4 ? "" : "  <-- MISMATCH");
        }
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    std::vector<std::vector<double>> tf(vars.size());
    for (int r = 0; r <= rounds; ++r)
        for (size_t i = 0; i < vars.size(); ++i) {
            CK(hipEventRecord(e0, 0));
            for (int it = 0; it < iters; ++it) vars[i].run(a, 0);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r) tf[i].push_back(flops * iters / (ms * 1e-3) / 1e12);
        }
    for (size_t i = 0; i < vars.size(); ++i) {
        auto x = tf[i];
        std::sort(x.begin(), x.end());
        const double med = x[x.size() / 2];
        printf("   %-22s median %7.2f TF/s (%5.1f%%)  us/launch %8.1f\n", vars[i].name.c_str(), med,
               med / 157.3 * 100, flops / (med * 1e12) * 1e6);
    }
    CK(hipFree(q)); CK(hipFree(k)); CK(hipFree(v)); CK(hipFree(o));
}

// Per-wave s_memtime stamps of the C3 launch (research kernel with ABL 512: same code as the
// product kernel plus the stamps), after `warm` warm-up launches; raw dump for
// tools/attn_stamps.py: [n_waves][16] uint64 (layout in attn_research.h)
static void stamps(const char* path, int warm) {
    const int B = 256, L = 256, H = 6, HD = 48;
    const size_t nq = (size_t)B * L * H * HD;
    std::vector<float> hq(nq);
    fill(hq, -1.f, 1.f, 1);
    float *q, *k, *v, *o;
    CK(hipMalloc(&q, nq * 4)); CK(hipMalloc(&k, nq * 4)); CK(hipMalloc(&v, nq * 4)); CK(hipMalloc(&o, nq * 4));
    CK(hipMemcpy(q, hq.data(), nq * 4, hipMemcpyHostToDevice));
    fill(hq, -1.f, 1.f, 2);
    CK(hipMemcpy(k, hq.data(), nq * 4, hipMemcpyHostToDevice));
    fill(hq, -1.f, 1.f, 3);
    CK(hipMemcpy(v, hq.data(), nq * 4, hipMemcpyHostToDevice));
    AttnArgs a{};
    a.q = q; a.cache_k = k; a.cache_v = v; a.out = o;
    a.B = B; a.L = L; a.start_pos = 0; a.H = H; a.KVH = H; a.HD = HD; a.Smax = L;
    dim3 grid(1, H, B);
    const size_t nst = (size_t)B * H * 4 * 16;
    unsigned long long* st;
    CK(hipMalloc(&st, nst * 8));
    CK(hipMemset(st, 0, nst * 8));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_attn_stamps), &st, sizeof(st)));
    for (int i = 0; i <= warm; ++i)
        hipLaunchKernelGGL((attn_research_kernel<48, 4, 1, 64, 512>), grid, dim3(256), 0, 0, a);
    CK(hipDeviceSynchronize());
    std::vector<unsigned long long> h(nst);
    CK(hipMemcpy(h.data(), st, nst * 8, hipMemcpyDeviceToHost));
    FILE* f = fopen(path, "wb");
    fwrite(h.data(), 8, nst, f);
    fclose(f);
    printf("stamps: %zu waves -> %s\n", nst / 16, path);
    CK(hipFree(q)); CK(hipFree(k)); CK(hipFree(v)); CK(hipFree(o)); CK(hipFree(st));
}

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 5, iters = argc > 2 ? atoi(argv[2]) : 10;
    if (argc > 3 && std::string(argv[3]) == "early") {  // K/V tile 0 before q, raw prologue barrier
        std::vector<Variant> v = {AVAR(48, 4, 1, 64), AABL(0), AABL(1024), AVAR(48, 4, 1, 64), AABL(1024)};
        run("stories15M C3", 256, 256, 6, 6, 48, v, rounds, iters);
        run("stories15M C3 half batch (one part of the split)", 128, 256, 6, 6, 48, v, rounds, iters);
        run("stories15M chunk L=200 at start_pos 37", 64, 200, 6, 6, 48, v, 1, 1, 37);
        run("stories15M L=100", 16, 100, 6, 6, 48, v, 1, 1);
        return 0;
    }
    if (argc > 3 && std::string(argv[3]) == "stamps") {
        stamps(argc > 4 ? argv[4] : "gpurun_out/attn_stamps.bin", rounds);
        return 0;
    }
    if (argc > 3 && std::string(argv[3]) == "pk") {  // round 6: packed softmax + interleaved score chains
        std::vector<Variant> v = {AVAR(48, 4, 1, 64), AVARPK(48, 4, 1, 64), AVAR(48, 4, 1, 64), AVARPK(48, 4, 1, 64)};
        run("stories15M C3", 256, 256, 6, 6, 48, v, rounds, iters);
        run("stories15M C3 half batch (one part of the split)", 128, 256, 6, 6, 48, v, rounds, iters);
        run("Llama-3 shape B=2 L=2048 HD 128 GQA 4", 2, 2048, 32, 8, 128,
            {AVAR(128, 1, 4, 32), AVARPK(128, 1, 4, 32)}, rounds, 3);
        return 0;
    }
    if (argc > 3 && std::string(argv[3]) == "c3") {  // the product C3 kernel alone (PMC passes)
        run("stories15M C3", 256, 256, 6, 6, 48, {AVAR(48, 4, 1, 64)}, rounds, iters);
        return 0;
    }
    if (argc > 3 && std::string(argv[3]) == "pf2") {
        run("stories15M C3", 256, 256, 6, 6, 48, {AVAR(48, 4, 1, 64), AABL(32)}, rounds, iters);
        run("stories15M chunk L=200 at start_pos 37", 64, 200, 6, 6, 48, {AVAR(48, 4, 1, 64), AABL(32)}, 1, 1, 37);
        return 0;
    }
    if (argc > 3 && std::string(argv[3]) == "defer") {  // 3 slots, even tiles' diagonal units deferred
        std::vector<Variant> v = {AVAR(48, 4, 1, 64), ADEF(48, 4, 1, 64), AVAR(48, 4, 1, 64), ADEF(48, 4, 1, 64)};
        run("stories15M C3", 256, 256, 6, 6, 48, v, rounds, iters);
        run("stories15M chunk L=200 at start_pos 37", 64, 200, 6, 6, 48, v, 1, 1, 37);
        run("stories15M L=100", 16, 100, 6, 6, 48, {AVAR(48, 4, 1, 64), ADEF(48, 4, 1, 64)}, 1, 1);
        run("stories15M L=333 at 5", 4, 333, 6, 6, 48, {AVAR(48, 4, 1, 64), ADEF(48, 4, 1, 64)}, 1, 1, 5);
        run("GQA n_rep 2, L=77 at 19", 8, 77, 6, 3, 48, {AVAR(48, 4, 2, 64), ADEF(48, 4, 2, 64)}, 1, 1, 19);
        run("GQA n_rep 4, L=300 at 3", 2, 300, 8, 2, 48, {AVAR(48, 4, 4, 64), ADEF(48, 4, 4, 64)}, 1, 1, 3);
        return 0;
    }
    if (argc > 3 && std::string(argv[3]) == "abl") {  // ablations of v1 (timing only)
        run("stories15M C3 ablations", 256, 256, 6, 6, 48,
            {AVAR(48, 4, 1, 64), AABL(32), AABL(1), AABL(2), AABL(4), AABL(8), AABL(16), AABL(18), AABL(12),
             AABL(1 | 8), AABL(1 | 4 | 8), AABL(1 | 4 | 8 | 16)},
            rounds, iters);
        return 0;
    }
    if (argc > 3 && std::string(argv[3]) == "sched") {  // hand-ordered score / P.V phases
        std::vector<Variant> v = {AVAR(48, 4, 1, 64), AABL(2048), AABL(4096), AABL(2048 | 4096), AVAR(48, 4, 1, 64)};
        run("stories15M C3", 256, 256, 6, 6, 48, v, rounds, iters);
        run("stories15M chunk L=200 at start_pos 37", 64, 200, 6, 6, 48, v, 1, 1, 37);
        return 0;
    }
    if (argc > 3 && std::string(argv[3]) == "prio") {  // s_setprio around the MFMA clusters
        std::vector<Variant> v = {AVAR(48, 4, 1, 64), AABL(64), AABL(128), AABL(256), AVAR(48, 4, 1, 64)};
        run("stories15M C3", 256, 256, 6, 6, 48, v, rounds, iters);
        run("stories15M chunk L=200 at start_pos 37", 64, 200, 6, 6, 48, v, 1, 1, 37);
        return 0;
    }
    run("stories15M C3", 256, 256, 6, 6, 48,
        {AVAR(48, 4, 1, 64), AVAR(48, 4, 1, 32), AVAR(48, 2, 1, 64), AVAR(48, 2, 1, 32),
         AVAR(48, 1, 1, 32), AVAR(48, 1, 1, 64)}, rounds, iters);
    run("Llama-3 shape (C5 slice)", 4, 2048, 32, 8, 128,
        {AVAR(128, 1, 4, 32), AVAR(128, 2, 4, 32)}, rounds, 3);
    return 0;
}
