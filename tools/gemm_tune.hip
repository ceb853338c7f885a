// GEMM variant tuner: times kernel configurations on the stories15M prefill shapes,
// interleaved in one process (rounds x variants), and checks every variant's output against
// the first one.  Build: make -C tools gemm_tune ; run on the GPU box: tools/gemm_tune
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#include "../llama3.np_amd/csrc/gemm_kernel.h"
#include "../llama3.np_amd/csrc/gemm_x6.h"

using namespace l3;

#define CK(x)                                                                           \
    do {                                                                                \
        hipError_t e = (x);                                                             \
        if (e != hipSuccess) {                                                          \
            fprintf(stderr, "%s: %s (%s:%d)\n", #x, hipGetErrorString(e), __FILE__, __LINE__); \
            exit(2);                                                                    \
        }                                                                               \
    } while (0)

struct Variant {
    std::string name;
    std::function<void(const GemmArgs&, hipStream_t)> run;
};

// RVAR: k-tiles by register staging + ds_write_b128; GVAR: by global_load_lds (product path)
#define TVAR(TAG, GL, WM, WN, TM, TN, EPI, WPE, BK)                                                   \
    Variant{TAG "<" #WM "," #WN "," #TM "," #TN ",wpe" #WPE ",bk" #BK ">", [](const GemmArgs& a, hipStream_t s) { \
                constexpr int BM = WM * TM * 16, BN = WN * TN * 16;                                  \
                const int64_t tiles = (int64_t)((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);        \
                hipLaunchKernelGGL((gemm_lds_kernel<WM, WN, TM, TN, EPI, WPE, false, BK, GL>), dim3((unsigned)tiles), dim3(64 * WM * WN), 0, s, a); \
            }}
// NS-deep LDS ring (counted vmcnt, NS - 1 k-tiles in flight)
#define GVARN(WM, WN, TM, TN, EPI, WPE, BK, NS)                                                      \
    Variant{"ring<" #WM "," #WN "," #TM "," #TN ",wpe" #WPE ",bk" #BK ",ns" #NS ">", [](const GemmArgs& a, hipStream_t s) { \
                constexpr int BM = WM * TM * 16, BN = WN * TN * 16;                                  \
                const int64_t tiles = (int64_t)((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);        \
                hipLaunchKernelGGL((gemm_lds_kernel<WM, WN, TM, TN, EPI, WPE, false, BK, true, NS>), dim3((unsigned)tiles), dim3(64 * WM * WN), 0, s, a); \
            }}
// the skinny MFMA kernel (9-256 rows): a block per 16-row x 16*TN-column tile, 4 waves split K
#define SVAR(EPI, TN, CH)                                                                             \
    Variant{"skinny<tn" #TN ",ch" #CH ">", [](const GemmArgs& a, hipStream_t s) {                      \
                const int64_t blocks = (int64_t)((a.M + 15) / 16) * ((a.N + 16 * TN - 1) / (16 * TN)); \
                hipLaunchKernelGGL((gemm_skinny_kernel<EPI, TN, CH>), dim3((unsigned)blocks), dim3(256), 0, s, a); \
            }}
#define SVARW(EPI, TN, CH, NW)                                                                        \
    Variant{"skinny<tn" #TN ",ch" #CH ",nw" #NW ">", [](const GemmArgs& a, hipStream_t s) {            \
                const int64_t blocks = (int64_t)((a.M + 15) / 16) * ((a.N + 16 * TN - 1) / (16 * TN)); \
                hipLaunchKernelGGL((gemm_skinny_kernel<EPI, TN, CH, NW>), dim3((unsigned)blocks), dim3(64 * NW), 0, s, a); \
            }}
// the product tile with GemmArgs::group_m = G (grouped tile order inside each XCD's run)
#define GVARG(WM, WN, TM, TN, EPI, WPE, BK, G)                                                       \
    Variant{"glds<" #WM "," #WN "," #TM "," #TN ",wpe" #WPE ",bk" #BK ",gm" #G ">", [](const GemmArgs& a0, hipStream_t s) { \
                constexpr int BM = WM * TM * 16, BN = WN * TN * 16;                                  \
                GemmArgs a = a0;                                                                     \
                a.group_m = G;                                                                       \
                const int64_t tiles = (int64_t)((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);        \
                hipLaunchKernelGGL((gemm_lds_kernel<WM, WN, TM, TN, EPI, WPE, false, BK, true>), dim3((unsigned)tiles), dim3(64 * WM * WN), 0, s, a); \
            }}
#define RVAR(WM, WN, TM, TN, EPI, WPE, BK) TVAR("regs", false, WM, WN, TM, TN, EPI, WPE, BK)
#define GVAR(WM, WN, TM, TN, EPI, WPE, BK) TVAR("glds", true, WM, WN, TM, TN, EPI, WPE, BK)

static void fill(std::vector<float>& v, float lo, float hi, unsigned seed) {
    srand(seed);
    for (auto& x : v) x = lo + (hi - lo) * (float)rand() / (float)RAND_MAX;
}

// cold mode (g_cold): every launch follows a kernel that reads 96 MB, so the weights and inputs
// come from the MALL / HBM as in the batched decode loop (each XCD's 4 MB L2 evicted); per-launch
// time = (flush + launch) - flush alone, both timed over the same iterations
static bool g_cold = false;
static int g_planes_gen = 0;
static int g_repeat_check = 0;  // run_shape: each variant this many more times, outputs compared bit for bit  // x6 planes cache epoch, bumped by every run_shape: a freed buffer's address comes back
static bool g_qkv_fast = false;  // stamp_report: EPI_QKV with the division-free epilogue
static bool g_qkv_fast_run = false;  // run_shape: EPI_QKV with the division-free epilogue
__global__ void flush_kernel(const f32x4* buf, int64_t n, float* sink) {
    f32x4 a = {0.f, 0.f, 0.f, 0.f};
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) a += buf[i];
    if (a.x + a.y + a.z + a.w == 12345.f) sink[0] = a.x;
}
static f32x4* g_flush = nullptr;
static float* g_sink = nullptr;
static const int64_t FLUSH_N = (96ll << 20) / 16;
static void flush(hipStream_t s) {
    if (!g_flush) {
        CK(hipMalloc(&g_flush, FLUSH_N * 16));
        CK(hipMemset(g_flush, 0, FLUSH_N * 16));
        CK(hipMalloc(&g_sink, 4));
    }
    hipLaunchKernelGGL(flush_kernel, dim3(2048), dim3(256), 0, s, g_flush, FLUSH_N, g_sink);
}

static void run_shape(const char* label, int epi, int M, int K, int N, bool norm,
                      std::vector<Variant> vars, int rounds, int iters) {
    const int outN = epi == EPI_SWIGLU ? N / 2 : (epi == EPI_QKV ? 288 : N);
    ++g_planes_gen;
    std::vector<float> hA((size_t)M * K), hW((size_t)N * K), hw(K);
    fill(hA, -1.f, 1.f, 1);
    fill(hW, -0.05f, 0.05f, 2);
    fill(hw, 0.5f, 1.5f, 3);
    float *A, *W, *w, *C;
    CK(hipMalloc(&A, hA.size() * 4));
    CK(hipMalloc(&W, hW.size() * 4));
    CK(hipMalloc(&w, hw.size() * 4));
    CK(hipMalloc(&C, (size_t)M * outN * 4));
    CK(hipMemcpy(A, hA.data(), hA.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(W, hW.data(), hW.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(w, hw.data(), hw.size() * 4, hipMemcpyHostToDevice));
    GemmArgs g{};
    g.A = A; g.lda = K; g.W = W; g.C = C; g.ldc = outN; g.M = M; g.N = N; g.K = K;
    g.norm = norm; g.eps = 1e-6f;
    float *qo = nullptr, *ck = nullptr, *cv = nullptr, *rc = nullptr, *rsn = nullptr;
    if (epi == EPI_QKV) {  // stories15M attention geometry: H = KVH = 6, HD = 48, L = 256
        g.H = 6; g.KVH = 6; g.HD = 48; g.L = 256; g.Smax = 256; g.start_pos = 0;
        g.q_scale = 0.2f;
        const size_t cache = (size_t)((M + 255) / 256) * 6 * 256 * 48;  // whole sequences of L = 256
        CK(hipMalloc(&qo, (size_t)M * 288 * 4)); CK(hipMalloc(&ck, cache * 4)); CK(hipMalloc(&cv, cache * 4));
        std::vector<float> tc(256 * 24), ts(256 * 24);
        fill(tc, -1.f, 1.f, 4); fill(ts, -1.f, 1.f, 5);
        CK(hipMalloc(&rc, tc.size() * 4)); CK(hipMalloc(&rsn, ts.size() * 4));
        CK(hipMemcpy(rc, tc.data(), tc.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(rsn, ts.data(), ts.size() * 4, hipMemcpyHostToDevice));
        g.q_out = qo; g.cache_k = ck; g.cache_v = cv; g.rope_cos = rc; g.rope_sin = rsn;
        g.qkv_fast = g_qkv_fast_run;  // x6 mode: the product's division-free epilogue
        g.C = qo;  // the correctness check reads the q section
        g.ldc = 288;
    }
    // W with the RMSNorm weight folded into its columns (as l3_finalize does)
    if (norm) {
        std::vector<float> hWf(hW);
        for (size_t n = 0; n < (size_t)N; ++n)
            for (size_t k = 0; k < (size_t)K; ++k) hWf[n * K + k] *= hw[k];
        CK(hipMemcpy(W, hWf.data(), hWf.size() * 4, hipMemcpyHostToDevice));
    }
    hipStream_t s;
    CK(hipStreamCreate(&s));
    const double flops = 2.0 * M * N * K;
    printf("\n== %s  M=%d K=%d N=%d epi=%d norm=%d  (%.2f GFLOP/launch)\n", label, M, K, N, epi,
           (int)norm, flops / 1e9);
    // correctness vs variant 0 (RESID: start from zero output each time)
    std::vector<float> ref((size_t)M * outN), got((size_t)M * outN);
    const size_t cache_n = epi == EPI_QKV ? (size_t)((M + 255) / 256) * 6 * 256 * 48 : 0;
    std::vector<float> refk(cache_n), refv(cache_n), gotk(cache_n), gotv(cache_n);
    for (size_t v = 0; v < vars.size(); ++v) {
        CK(hipMemsetAsync(g.C, 0, (size_t)M * outN * 4, s));
        if (cache_n) { CK(hipMemsetAsync(ck, 0, cache_n * 4, s)); CK(hipMemsetAsync(cv, 0, cache_n * 4, s)); }
        vars[v].run(g, s);
        CK(hipGetLastError());
        CK(hipStreamSynchronize(s));
        CK(hipMemcpy(v ? got.data() : ref.data(), g.C, got.size() * 4, hipMemcpyDeviceToHost));
        if (cache_n) {  // EPI_QKV: the K / V cache slots too, bit for bit
            CK(hipMemcpy(v ? gotk.data() : refk.data(), ck, cache_n * 4, hipMemcpyDeviceToHost));
            CK(hipMemcpy(v ? gotv.data() : refv.data(), cv, cache_n * 4, hipMemcpyDeviceToHost));
            if (v) printf("   check %-40s K cache %s, V cache %s\n", vars[v].name.c_str(),
                          gotk == refk ? "bit-identical" : "DIFFERS", gotv == refv ? "bit-identical" : "DIFFERS");
        }
        if (v) {
            double md = 0, mr = 0;
            for (size_t i = 0; i < got.size(); ++i) {
                md = std::max(md, (double)std::fabs(got[i] - ref[i]));
                mr = std::max(mr, (double)std::fabs(ref[i]));
            }
            printf("   check %-40s max|diff| %.3e (max|ref| %.3e)%s\n", vars[v].name.c_str(), md, mr,
                   md <= 1e-4 * std::max(1.0, mr) ? "" : "  <-- MISMATCH");
        }
    }
    for (size_t v = 0; v < vars.size() && g_repeat_check; ++v) {  // run-to-run determinism
        std::vector<float> first(got.size()), again(got.size());
        int bad = 0;
        for (int r = 0; r <= g_repeat_check; ++r) {
            CK(hipMemsetAsync(g.C, 0, (size_t)M * outN * 4, s));
            vars[v].run(g, s);
            CK(hipStreamSynchronize(s));
            CK(hipMemcpy(r ? again.data() : first.data(), g.C, got.size() * 4, hipMemcpyDeviceToHost));
            if (r && again != first) {
                ++bad;
                // where: count, max |diff|, the first differing element's row / column and tile
                size_t n = 0, i0 = SIZE_MAX;
                double md = 0;
                for (size_t i = 0; i < again.size(); ++i)
                    if (again[i] != first[i]) {
                        ++n;
                        md = std::max(md, (double)std::fabs(again[i] - first[i]));
                        if (i0 == SIZE_MAX) i0 = i;
                    }
                if (bad <= 5)
                    printf("      run %d: %zu elements differ, max %.3e, first at row %zu col %zu\n", r, n, md,
                           i0 / outN, i0 % outN);
                if (bad == 1 && getenv("X6_DUMP")) {  // where: per 128-row block and per column, samples
                    std::vector<int> rb(M / 128 + 1), cc(outN);
                    int shown = 0;
                    for (size_t i = 0; i < again.size(); ++i)
                        if (again[i] != first[i]) {
                            rb[(i / outN) / 128]++;
                            cc[i % outN]++;
                            if (shown++ < 24)
                                printf("        row %zu (seq %zu pos %zu) col %zu: %.6f vs %.6f\n", i / outN, i / outN / 256,
                                       (i / outN) % 256, i % outN, first[i], again[i]);
                        }
                    printf("        row blocks hit:");
                    int nb = 0;
                    for (size_t b = 0; b < rb.size(); ++b)
                        if (rb[b]) { if (nb++ < 40) printf(" %zu:%d", b, rb[b]); }
                    printf(" (%d blocks)\n        cols hit:", nb);
                    for (int c = 0; c < outN; ++c)
                        if (cc[c]) printf(" %d", c);
                    printf("\n");
                }
            }
        }
        printf("   repeat %-39s %d of %d runs differ from the first\n", vars[v].name.c_str(), bad, g_repeat_check);
    }
    std::vector<std::vector<double>> tf(vars.size());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int r = 0; r < rounds + 1; ++r) {
        float fl_ms = 0;
        if (g_cold) {  // the flushes alone
            CK(hipEventRecord(e0, s));
            for (int i = 0; i < iters; ++i) flush(s);
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&fl_ms, e0, e1));
        }
        for (size_t v = 0; v < vars.size(); ++v) {
            CK(hipEventRecord(e0, s));
            for (int i = 0; i < iters; ++i) {
                if (g_cold) flush(s);
                vars[v].run(g, s);
            }
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            ms -= fl_ms;
            if (r) tf[v].push_back(flops * iters / (ms * 1e-3) / 1e12);  // round 0 = warm-up
        }
    }
    for (size_t v = 0; v < vars.size(); ++v) {
        auto x = tf[v];
        std::sort(x.begin(), x.end());
        const double med = x[x.size() / 2];
        printf("   %-44s median %7.2f TF/s (%5.1f%% of 157.3)  min %7.2f  max %7.2f  us/launch %8.1f\n",
               vars[v].name.c_str(), med, med / 157.3 * 100, x.front(), x.back(), flops / (med * 1e12) * 1e6);
    }
    CK(hipFree(A)); CK(hipFree(W)); CK(hipFree(w)); CK(hipFree(C));
    if (qo) { CK(hipFree(qo)); CK(hipFree(ck)); CK(hipFree(cv)); CK(hipFree(rc)); CK(hipFree(rsn)); }
    CK(hipStreamDestroy(s));
}

// Diagnostic: cycle split per block from in-kernel stamps (STAMP build): shader-counter
// (s_memtime) and 100 MHz real-time stamps at start, after the first k-tile is staged
// (prologue), after the main loop, and after the epilogue.  Residency = sum of block lifetimes
// / (launch span x 256 CUs): the average number of blocks a CU holds.
template <int WM, int WN, int TM, int TN, int EPI, int WPE, int BK>
static void stamp_report(const char* label, int M, int K, int N, bool norm) {
    const int outN = EPI == EPI_SWIGLU ? N / 2 : N;
    float *A, *W, *C;
    CK(hipMalloc(&A, (size_t)M * K * 4)); CK(hipMalloc(&W, (size_t)N * K * 4));
    CK(hipMalloc(&C, (size_t)M * outN * 4));
    // EPI_QKV: the stories15M attention geometry (as run_shape), q / cache / RoPE tables
    float *qo = nullptr, *ck = nullptr, *cv = nullptr, *rc = nullptr, *rsn = nullptr;
    if (EPI == EPI_QKV) {
        const size_t cache = (size_t)((M + 255) / 256) * 6 * 256 * 48;
        CK(hipMalloc(&qo, (size_t)M * 288 * 4)); CK(hipMalloc(&ck, cache * 4)); CK(hipMalloc(&cv, cache * 4));
        std::vector<float> tc(256 * 24), ts(256 * 24);
        fill(tc, -1.f, 1.f, 4); fill(ts, -1.f, 1.f, 5);
        CK(hipMalloc(&rc, tc.size() * 4)); CK(hipMalloc(&rsn, ts.size() * 4));
        CK(hipMemcpy(rc, tc.data(), tc.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(rsn, ts.data(), ts.size() * 4, hipMemcpyHostToDevice));
    }
    std::vector<float> hA((size_t)M * K), hW((size_t)N * K);
    fill(hA, -1.f, 1.f, 1); fill(hW, -0.05f, 0.05f, 2);
    CK(hipMemcpy(A, hA.data(), hA.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(W, hW.data(), hW.size() * 4, hipMemcpyHostToDevice));
    constexpr int BM = WM * TM * 16, BN = WN * TN * 16;
    const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
    unsigned long long* st;
    CK(hipMalloc(&st, (size_t)tiles * 10 * 8));
    GemmArgs g{};
    g.A = A; g.lda = K; g.W = W; g.C = C; g.ldc = outN; g.M = M; g.N = N; g.K = K;
    g.norm = norm; g.eps = 1e-6f; g.stamps = st;
    if (EPI == EPI_QKV) {
        g.H = 6; g.KVH = 6; g.HD = 48; g.L = 256; g.Smax = 256; g.start_pos = 0; g.q_scale = 0.2f;
        g.q_out = qo; g.cache_k = ck; g.cache_v = cv; g.rope_cos = rc; g.rope_sin = rsn; g.C = qo; g.ldc = 288;
        g.qkv_fast = g_qkv_fast;
    }
    for (int it = 0; it < 20; ++it)  // back-to-back launches so the clock settles; last one kept
        hipLaunchKernelGGL((gemm_lds_kernel<WM, WN, TM, TN, EPI, WPE, true, BK>), dim3(tiles), dim3(256), 0, 0, g);
    CK(hipDeviceSynchronize());
    std::vector<unsigned long long> h((size_t)tiles * 10);
    CK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
    std::vector<double> ratio, pro, loop, epi;
    unsigned long long t0 = ~0ull, t1 = 0;
    double life = 0;
    for (int b = 0; b < tiles; ++b) {
        const unsigned long long* d = &h[(size_t)b * 10];
        if (d[7] > d[1]) ratio.push_back((double)(d[6] - d[0]) / (double)(d[7] - d[1]) * 100.0);
        pro.push_back((double)(d[2] - d[0]));
        loop.push_back((double)(d[4] - d[2]));
        epi.push_back((double)(d[6] - d[4]));
        life += (double)(d[7] - d[1]);
        t0 = std::min(t0, d[1]); t1 = std::max(t1, d[7]);
    }
    auto med = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
    const double mfma_cycles = (double)K / 4 * TM * TN * 32;  // per wave, 16x16x4 f32 at 32 cyc
    const double span = (double)(t1 - t0);
    printf("\n== stamps %s wpe%d bk%d: blocks %d, s_memtime rate %.0f MHz, prologue median %.0f, "
           "main loop median %.0f (MFMA-only %.0f per wave), epilogue median %.0f counts; "
           "launch span %.1f us, residency %.2f blocks/CU\n",
           label, WPE, BK, tiles, med(ratio), med(pro), med(loop), mfma_cycles, med(epi), span / 100.0,
           life / (span * 256.0));
    // MFMA share of a CU's cycles: blocks x 4 waves x MFMA cycles / (4 SIMDs x 256 CUs x span
    // in shader cycles), the span converted at the blocks' median clock
    const double clk = med(ratio) * 1e6;  // Hz (s_memtime counts per 100 MHz realtime tick x 1e6)
    const double occ = (double)tiles * 4.0 * mfma_cycles / (1024.0 * span / 1e8 * clk);
    printf("   MFMA occupancy over the launch %.3f; at this clock the peak is %.1f TF/s (%.1f%% of 157.3)\n",
           occ, 157.3 * clk / 2.4e9, 100.0 * clk / 2.4e9);
    CK(hipFree(A)); CK(hipFree(W)); CK(hipFree(C)); CK(hipFree(st));
    if (qo) { CK(hipFree(qo)); CK(hipFree(ck)); CK(hipFree(cv)); CK(hipFree(rc)); CK(hipFree(rsn)); }
}

// Round 6 (verdict r05 item 4): where a batched-decode skinny launch's time goes.  A decode-like
// chain at M = B rows — per layer the QKV, O-proj, gate|up and down skinny GEMMs (TN and tiles of
// the product at B = 256, own weights per layer: 6 layers, 24 MB), back to back on one stream,
// STAMP build — and per launch: the gap from the previous launch's last block exit to this
// launch's first block entry, the span from first entry to last exit, and per block (medians)
// the first fragments' round trip, the rest of the k-loop, the wait at the partials' barrier,
// the epilogue and its stores' acknowledgement.  All in 10 ns ticks of s_memrealtime.
static int g_sk_ch = 2;
static int g_sk_nw = 4;  // waves per block (the K split)
template <int EPI, int TN>
static void skinny_stamp_launch(GemmArgs g, hipStream_t s) {
    const int blocks = ((g.M + 15) / 16) * ((g.N + 16 * TN - 1) / (16 * TN));
    if (g_sk_nw == 8) hipLaunchKernelGGL((gemm_skinny_kernel<EPI, TN, 2, 8, true>), dim3(blocks), dim3(512), 0, s, g);
    else if (g_sk_nw == 16) hipLaunchKernelGGL((gemm_skinny_kernel<EPI, TN, 2, 16, true>), dim3(blocks), dim3(1024), 0, s, g);
    else if (g_sk_ch >= 6) hipLaunchKernelGGL((gemm_skinny_kernel<EPI, TN, 6, 4, true>), dim3(blocks), dim3(256), 0, s, g);
    else if (g_sk_ch >= 3) hipLaunchKernelGGL((gemm_skinny_kernel<EPI, TN, 3, 4, true>), dim3(blocks), dim3(256), 0, s, g);
    else hipLaunchKernelGGL((gemm_skinny_kernel<EPI, TN, 2, 4, true>), dim3(blocks), dim3(256), 0, s, g);
}
static bool g_sk_xcd = false;
static void skinny_stamps(int M, int reps) {
    const int D = 288, FD = 768, NL = 6;
    struct Sh { const char* name; int epi, K, N, TN; };
    const Sh sh[4] = {{"QKV", EPI_QKV, D, 864, 1}, {"O-proj", EPI_RESID, D, D, 1},
                      {"gate|up", EPI_SWIGLU, D, 2 * FD, 2}, {"down", EPI_RESID, FD, D, 1}};
    std::vector<float*> W(4 * NL);
    for (int l = 0; l < NL; ++l)
        for (int k = 0; k < 4; ++k) {
            std::vector<float> h((size_t)sh[k].N * sh[k].K);
            fill(h, -0.05f, 0.05f, 10 + 4 * l + k);
            CK(hipMalloc(&W[4 * l + k], h.size() * 4));
            CK(hipMemcpy(W[4 * l + k], h.data(), h.size() * 4, hipMemcpyHostToDevice));
        }
    float *x, *q, *hid, *ck, *cv, *rc, *rsn;
    std::vector<float> hx((size_t)M * D);
    fill(hx, -1.f, 1.f, 1);
    CK(hipMalloc(&x, hx.size() * 4)); CK(hipMemcpy(x, hx.data(), hx.size() * 4, hipMemcpyHostToDevice));
    CK(hipMalloc(&q, (size_t)M * D * 4)); CK(hipMalloc(&hid, (size_t)M * FD * 4));
    CK(hipMalloc(&ck, (size_t)M * 6 * 256 * 48 * 4)); CK(hipMalloc(&cv, (size_t)M * 6 * 256 * 48 * 4));
    std::vector<float> tc(256 * 24), ts(256 * 24);
    fill(tc, -1.f, 1.f, 4); fill(ts, -1.f, 1.f, 5);
    CK(hipMalloc(&rc, tc.size() * 4)); CK(hipMalloc(&rsn, ts.size() * 4));
    CK(hipMemcpy(rc, tc.data(), tc.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(rsn, ts.data(), ts.size() * 4, hipMemcpyHostToDevice));
    const int nl = 4 * NL;
    int blk[4];
    for (int k = 0; k < 4; ++k) blk[k] = ((M + 15) / 16) * ((sh[k].N + 16 * sh[k].TN - 1) / (16 * sh[k].TN));
    std::vector<unsigned long long*> st(nl);
    for (int i = 0; i < nl; ++i) {
        CK(hipMalloc(&st[i], (size_t)blk[i % 4] * 8 * 8));
        CK(hipMemset(st[i], 0, (size_t)blk[i % 4] * 8 * 8));
    }
    hipStream_t s;
    CK(hipStreamCreate(&s));
    auto chain = [&]() {
        for (int l = 0; l < NL; ++l)
            for (int k = 0; k < 4; ++k) {
                GemmArgs g{};
                g.M = M; g.K = sh[k].K; g.N = sh[k].N; g.W = W[4 * l + k]; g.eps = 1e-6f; g.stamps = st[4 * l + k];
                g.skinny_xcd = g_sk_xcd;
                if (k == 0) {  // QKV, decode geometry: one row per sequence at position 100
                    g.A = x; g.lda = D; g.norm = true; g.H = 6; g.KVH = 6; g.HD = 48; g.L = 1; g.Smax = 256;
                    g.start_pos = 100; g.q_scale = 0.2f; g.q_out = q; g.cache_k = ck; g.cache_v = cv;
                    g.rope_cos = rc; g.rope_sin = rsn;
                    skinny_stamp_launch<EPI_QKV, 1>(g, s);
                } else if (k == 1) {  // O-proj on q as the attention output, residual in place on x
                    g.A = q; g.lda = D; g.C = x; g.ldc = D;
                    skinny_stamp_launch<EPI_RESID, 1>(g, s);
                } else if (k == 2) {
                    g.A = x; g.lda = D; g.norm = true; g.C = hid; g.ldc = FD;
                    skinny_stamp_launch<EPI_SWIGLU, 2>(g, s);
                } else {
                    g.A = hid; g.lda = FD; g.C = x; g.ldc = D;
                    skinny_stamp_launch<EPI_RESID, 1>(g, s);
                }
            }
    };
    for (int r = 0; r < reps; ++r) chain();  // back to back; the last chain's stamps are read
    CK(hipStreamSynchronize(s));
    auto med = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v.empty() ? 0.0 : v[v.size() / 2]; };
    std::vector<std::vector<double>> gap(4), span(4), first(4), loop(4), red(4), epi(4), ack(4), life(4);
    unsigned long long prev_exit = 0;
    for (int i = 0; i < nl; ++i) {
        std::vector<unsigned long long> h((size_t)blk[i % 4] * 8);
        CK(hipMemcpy(h.data(), st[i], h.size() * 8, hipMemcpyDeviceToHost));
        unsigned long long t0 = ~0ull, t1 = 0;
        for (int b = 0; b < blk[i % 4]; ++b) {
            const unsigned long long* d = &h[(size_t)b * 8];
            t0 = std::min(t0, d[0]); t1 = std::max(t1, d[5]);
            first[i % 4].push_back((double)(d[1] - d[0]));
            loop[i % 4].push_back((double)(d[2] - d[1]));
            red[i % 4].push_back((double)(d[3] - d[2]));
            epi[i % 4].push_back((double)(d[4] - d[3]));
            ack[i % 4].push_back((double)(d[5] - d[4]));
            life[i % 4].push_back((double)(d[5] - d[0]));
        }
        if (prev_exit) gap[i % 4].push_back((double)t0 - (double)prev_exit);
        span[i % 4].push_back((double)(t1 - t0));
        prev_exit = t1;
    }
    double tot = 0;
    for (int k = 0; k < 4; ++k) tot += (med(gap[k]) + med(span[k])) / 100;
    printf("\n== skinny stamps M=%d CH=%d NW=%d xcd-runs=%d: one layer's four launches %.2f us (us; medians over 6 layers' launches / their blocks; 10 ns ticks)\n",
           M, g_sk_ch, g_sk_nw, (int)g_sk_xcd, tot);
    for (int k = 0; k < 4; ++k)
        printf("   %-8s blocks %4d  gap from previous launch %.2f  span %.2f | per block: life %.2f = first fragments %.2f "
               "+ rest of k-loop %.2f + partials barrier %.2f + epilogue %.2f + stores acked %.2f\n",
               sh[k].name, blk[k], med(gap[k]) / 100, med(span[k]) / 100, med(life[k]) / 100, med(first[k]) / 100,
               med(loop[k]) / 100, med(red[k]) / 100, med(epi[k]) / 100, med(ack[k]) / 100);
}

// x6 (research, gemm_x6.h): the weight (and, for A3, the activation) split into bf16 planes once
// per buffer on first use, outside the timed launches
static unsigned short* planes_of(const float* src, int rows, int K, hipStream_t s) {
    struct Ent { const float* p; int gen; unsigned short* d; };
    static std::vector<Ent> cache;
    for (auto& c : cache)
        if (c.p == src && c.gen == g_planes_gen) return c.d;
    unsigned short* d;
    CK(hipMalloc(&d, (size_t)rows * 3 * K * 2));
    const int64_t n = (int64_t)rows * K;
    hipLaunchKernelGGL(split_planes_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, src, d, (int64_t)rows, K);
    CK(hipStreamSynchronize(s));
    cache.push_back({src, g_planes_gen, d});
    return d;
}
#define X6VAR(WM, WN, TM, TN, EPI, WPE)                                                                \
    Variant{"x6<" #WM "," #WN "," #TM "," #TN ",wpe" #WPE ">", [](const GemmArgs& a0, hipStream_t s) {       \
                constexpr int BM = WM * TM * 16, BN = WN * TN * 16;                                    \
                GemmArgs a = a0;                                                                       \
                a.W3 = planes_of(a.W, a.N, a.K, s);                                                    \
                const int64_t tiles = (int64_t)((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);          \
                hipLaunchKernelGGL((gemm_x6_kernel<WM, WN, TM, TN, EPI, WPE>), dim3((unsigned)tiles),  \
                                   dim3(64 * WM * WN), 0, s, a);                                       \
            }}

// x6acc: C = A W^T (plain store, no norm) from the fp32 MFMA kernel and from the six-product
// bf16 kernel, each against an fp64 host product on every row: max and rms absolute error
static void x6_accuracy(int M, int K, int N) {
    std::vector<float> hA((size_t)M * K), hW((size_t)N * K);
    fill(hA, -1.f, 1.f, 11);
    fill(hW, -0.05f, 0.05f, 12);
    float *A, *W, *C;
    CK(hipMalloc(&A, hA.size() * 4)); CK(hipMalloc(&W, hW.size() * 4)); CK(hipMalloc(&C, (size_t)M * N * 4));
    CK(hipMemcpy(A, hA.data(), hA.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(W, hW.data(), hW.size() * 4, hipMemcpyHostToDevice));
    ++g_planes_gen;
    GemmArgs g{};
    g.A = A; g.lda = K; g.W = W; g.C = C; g.ldc = N; g.M = M; g.N = N; g.K = K; g.norm = false;
    hipStream_t s;
    CK(hipStreamCreate(&s));
    std::vector<double> ref((size_t)M * N);
    for (int m = 0; m < M; ++m)
        for (int n = 0; n < N; ++n) {
            double a = 0;
            for (int k = 0; k < K; ++k) a += (double)hA[(size_t)m * K + k] * hW[(size_t)n * K + k];
            ref[(size_t)m * N + n] = a;
        }
    std::vector<Variant> vars = {GVAR(2, 2, 4, 4, EPI_STORE, 3, 32), X6VAR(4, 1, 2, 8, EPI_STORE, 2)};
    std::vector<float> got((size_t)M * N);
    printf("\n== accuracy against fp64  M=%d K=%d N=%d (A in [-1,1], W in [-0.05,0.05])\n", M, K, N);
    for (auto& v : vars) {
        CK(hipMemsetAsync(C, 0, got.size() * 4, s));
        v.run(g, s);
        CK(hipStreamSynchronize(s));
        CK(hipMemcpy(got.data(), C, got.size() * 4, hipMemcpyDeviceToHost));
        double mx = 0, se = 0, mr = 0;
        for (size_t i = 0; i < got.size(); ++i) {
            const double e = std::fabs((double)got[i] - ref[i]);
            mx = std::max(mx, e);
            se += e * e;
            mr = std::max(mr, std::fabs(ref[i]));
        }
        printf("   %-40s max|err| %.3e  rms err %.3e  (max|ref| %.3f)\n", v.name.c_str(), mx,
               std::sqrt(se / got.size()), mr);
    }
    CK(hipFree(A)); CK(hipFree(W)); CK(hipFree(C));
    CK(hipStreamDestroy(s));
}

int main(int argc, char** argv) {
    if (argc > 3 && std::string(argv[3]) == "x6acc") {  // error against fp64, both paths
        x6_accuracy(4096, 288, 1536);
        x6_accuracy(4096, 768, 288);
        x6_accuracy(1024, 4096, 4096);
        return 0;
    }
    if (argc > 3 && std::string(argv[3]) == "x6detq") {  // QKV only: epilogue forms, tile heights
        g_repeat_check = argc > 4 ? atoi(argv[4]) : 20;
        for (int fast = 1; fast >= 0; --fast) {
            g_qkv_fast_run = fast;
            printf("\n### qkv_fast %d\n", fast);
            run_shape("QKV (+RoPE, KV append)", EPI_QKV, 65536, 288, 864, true,
                      {GVAR(2, 2, 4, 3, EPI_QKV, 4, 16), GVAR(2, 2, 2, 3, EPI_QKV, 4, 16), X6VAR(4, 1, 2, 6, EPI_QKV, 2),
                       X6VAR(2, 2, 4, 3, EPI_QKV, 2)}, 1, 1);
        }
        run_shape("QKV shape, plain store", EPI_STORE, 65536, 288, 864, true,
                  {GVAR(2, 2, 4, 3, EPI_STORE, 4, 16), X6VAR(4, 1, 2, 6, EPI_STORE, 2)}, 1, 1);
        return 0;
    }
    if (argc > 3 && std::string(argv[3]) == "x6big") {  // 8-wave x6 blocks (one per CU by LDS)
        const int rounds = atoi(argv[1]), iters = atoi(argv[2]);
        g_qkv_fast_run = true;
        run_shape("gate|up (SwiGLU)", EPI_SWIGLU, 65536, 288, 1536, true,
                  {X6VAR(4, 1, 2, 8, EPI_SWIGLU, 2), X6VAR(8, 1, 2, 8, EPI_SWIGLU, 1), X6VAR(4, 2, 2, 8, EPI_SWIGLU, 1),
                   X6VAR(4, 2, 2, 4, EPI_SWIGLU, 2), X6VAR(8, 1, 1, 8, EPI_SWIGLU, 2)},
                  rounds, iters);
        run_shape("down (+resid)", EPI_RESID, 65536, 768, 288, false,
                  {X6VAR(4, 1, 2, 6, EPI_RESID, 2), X6VAR(8, 1, 2, 6, EPI_RESID, 1), X6VAR(4, 2, 2, 6, EPI_RESID, 1)},
                  rounds, iters);
        run_shape("QKV (+RoPE, KV append)", EPI_QKV, 65536, 288, 864, true,
                  {X6VAR(4, 1, 2, 8, EPI_QKV, 2), X6VAR(8, 1, 2, 8, EPI_QKV, 1), X6VAR(8, 1, 2, 6, EPI_QKV, 1)},
                  rounds, iters);
        return 0;
    }
    if (argc > 3 && std::string(argv[3]) == "x6det") {  // run-to-run determinism of the x6 tiles
        g_repeat_check = argc > 4 ? atoi(argv[4]) : 20;
        g_qkv_fast_run = true;
        run_shape("QKV (+RoPE, KV append)", EPI_QKV, 65536, 288, 864, true,
                  {GVAR(2, 2, 4, 3, EPI_QKV, 4, 16), X6VAR(4, 1, 2, 6, EPI_QKV, 2), X6VAR(4, 1, 2, 8, EPI_QKV, 2)}, 1, 1);
        run_shape("down (+resid)", EPI_RESID, 65536, 768, 288, false,
                  {GVAR(2, 2, 4, 3, EPI_RESID, 2, 32), X6VAR(4, 1, 2, 6, EPI_RESID, 2), X6VAR(4, 1, 2, 8, EPI_RESID, 2)}, 1, 1);
        run_shape("O-proj (+resid)", EPI_RESID, 65536, 288, 288, false,
                  {GVAR(2, 2, 2, 3, EPI_RESID, 3, 32), X6VAR(4, 2, 2, 3, EPI_RESID, 2), X6VAR(4, 1, 2, 6, EPI_RESID, 2)}, 1, 1);
        run_shape("gate|up (SwiGLU)", EPI_SWIGLU, 65536, 288, 1536, true,
                  {GVAR(2, 2, 4, 4, EPI_SWIGLU, 3, 16), X6VAR(8, 1, 1, 8, EPI_SWIGLU, 2), X6VAR(4, 1, 2, 8, EPI_SWIGLU, 2)}, 1, 1);
        return 0;
    }
    if (argc > 3 && std::string(argv[3]) == "x6") {  // fp32 from six bf16 MFMA products (gemm_x6.h)
        const int rounds = atoi(argv[1]), iters = atoi(argv[2]);
        g_qkv_fast_run = true;
        run_shape("gate|up (SwiGLU)", EPI_SWIGLU, 65536, 288, 1536, true,
                  {GVAR(2, 2, 4, 4, EPI_SWIGLU, 3, 16), X6VAR(4, 1, 2, 8, EPI_SWIGLU, 2),
                   X6VAR(4, 1, 2, 6, EPI_SWIGLU, 2), X6VAR(4, 2, 2, 4, EPI_SWIGLU, 2),
                   X6VAR(4, 1, 1, 8, EPI_SWIGLU, 2)},
                  rounds, iters);
        run_shape("QKV (+RoPE, KV append)", EPI_QKV, 65536, 288, 864, true,
                  {GVAR(2, 2, 4, 3, EPI_QKV, 4, 16), X6VAR(4, 1, 2, 6, EPI_QKV, 2),
                   X6VAR(4, 2, 2, 3, EPI_QKV, 2), X6VAR(2, 1, 2, 6, EPI_QKV, 2), X6VAR(4, 1, 2, 8, EPI_QKV, 2)},
                  rounds, iters);
        run_shape("down (+resid)", EPI_RESID, 65536, 768, 288, false,
                  {GVAR(2, 2, 4, 3, EPI_RESID, 2, 32), X6VAR(4, 1, 2, 6, EPI_RESID, 2),
                   X6VAR(4, 1, 2, 9, EPI_RESID, 2), X6VAR(4, 2, 2, 3, EPI_RESID, 2)},
                  rounds, iters);
        run_shape("O-proj (+resid)", EPI_RESID, 65536, 288, 288, false,
                  {GVAR(2, 2, 2, 3, EPI_RESID, 3, 32), X6VAR(4, 1, 2, 6, EPI_RESID, 2),
                   X6VAR(4, 2, 2, 3, EPI_RESID, 2), X6VAR(2, 1, 2, 6, EPI_RESID, 2), X6VAR(2, 2, 2, 3, EPI_RESID, 2)},
                  rounds, iters);
        return 0;
    }
    if (argc > 3 && std::string(argv[3]) == "skinnynw") {  // the K split over 4 / 8 / 16 waves
        for (int r = 0; r < 2; ++r)
            for (int nw : {4, 8, 16}) {
                g_sk_nw = nw;
                skinny_stamps(256, 20);
            }
        return 0;
    }
    if (argc > 3 && std::string(argv[3]) == "skinnystamps") {
        for (int r = 0; r < 2; ++r)
            for (int ch : {2, 3, 6})
                for (int x : {0, 1}) {
                    g_sk_ch = ch;
                    g_sk_xcd = x;
                    skinny_stamps(256, 20);
                }
        g_sk_ch = 2;
        g_sk_xcd = false;
        skinny_stamps(64, 20);
        g_sk_xcd = true;
        skinny_stamps(64, 20);
        return 0;
    }
    if (argc > 3 && std::string(argv[3]) == "qkvstamps") {  // round 6: the real QKV epilogue
        for (int r = 0; r < 2; ++r) {
            stamp_report<2, 2, 4, 3, EPI_QKV, 4, 16>("QKV 128x96 (+RoPE, KV append)", 65536, 288, 864, true);
            g_qkv_fast = true;
            stamp_report<2, 2, 4, 3, EPI_QKV, 4, 16>("QKV 128x96 fast epilogue", 65536, 288, 864, true);
            g_qkv_fast = false;
            stamp_report<2, 2, 4, 3, EPI_STORE, 4, 16>("QKV-shape 128x96 plain store", 65536, 288, 864, true);
            stamp_report<2, 2, 4, 4, EPI_QKV, 3, 16>("QKV 128x128 (+RoPE, KV append)", 65536, 288, 864, true);
            stamp_report<2, 2, 4, 4, EPI_SWIGLU, 3, 16>("gate|up 128x128", 65536, 288, 1536, true);
        }
        return 0;
    }
    if (argc > 3 && std::string(argv[3]) == "stamps") {
        stamp_report<2, 2, 4, 4, EPI_SWIGLU, 3, 16>("gate|up 128x128", 65536, 288, 1536, true);
        stamp_report<2, 2, 4, 3, EPI_STORE, 4, 16>("QKV-shape 128x96", 65536, 288, 864, true);
        stamp_report<2, 2, 4, 3, EPI_RESID, 2, 32>("down 128x96", 65536, 768, 288, false);
        stamp_report<2, 2, 2, 3, EPI_RESID, 3, 32>("O-proj 64x96", 65536, 288, 288, false);
        return 0;
    }
    const int rounds = argc > 1 ? atoi(argv[1]) : 5;
    const int iters = argc > 2 ? atoi(argv[2]) : 10;
    const int M = 65536;
    const bool c5 = argc > 3 && std::string(argv[3]) == "c5";
    if (argc > 3 && std::string(argv[3]) == "qkvq") {  // QKV tiles by whole block rounds
        // 128x96: 4608 blocks = 4.5 rounds at 4 blocks/CU; 128x144: 3072 = 3 (4/CU) or 4 (3/CU);
        // 64x96: 9216 = 9 rounds at 4/CU
        run_shape("QKV (+RoPE, KV append)", EPI_QKV, M, 288, 864, true,
                  {GVAR(2, 2, 4, 3, EPI_QKV, 4, 16), GVAR(4, 1, 2, 9, EPI_QKV, 3, 16),
                   GVAR(4, 1, 2, 9, EPI_QKV, 4, 16), GVAR(2, 2, 2, 3, EPI_QKV, 4, 16),
                   GVAR(2, 2, 2, 3, EPI_QKV, 5, 16), GVAR(4, 1, 2, 9, EPI_QKV, 3, 32)}, rounds, iters);
        return 0;
    }
    if (argc > 3 && std::string(argv[3]) == "resq") {  // O-proj / down tiles by block rounds
        // N = 288: 128x144 (4x1 waves of 32x144) = 1024 blocks, one round at 4 blocks/CU
        run_shape("O-proj (+resid)", EPI_RESID, M, 288, 288, false,
                  {GVAR(2, 2, 2, 3, EPI_RESID, 3, 32), GVAR(4, 1, 2, 9, EPI_RESID, 4, 16),
                   GVAR(4, 1, 2, 9, EPI_RESID, 3, 16), GVAR(2, 2, 2, 3, EPI_RESID, 4, 16),
                   GVAR(4, 1, 1, 9, EPI_RESID, 4, 16)}, rounds, iters);
        run_shape("down (+resid)", EPI_RESID, M, 768, 288, false,
                  {GVAR(2, 2, 4, 3, EPI_RESID, 2, 32), GVAR(4, 1, 2, 9, EPI_RESID, 4, 16),
                   GVAR(4, 1, 2, 9, EPI_RESID, 3, 16), GVAR(4, 1, 2, 9, EPI_RESID, 2, 32),
                   GVAR(2, 2, 4, 3, EPI_RESID, 3, 16)}, rounds, iters);
        return 0;
    }
    if (argc > 3 && std::string(argv[3]) == "ring") {  // deeper k-tile prefetch on the short-K GEMMs
        run_shape("O-proj (+resid)", EPI_RESID, M, 288, 288, false,
                  {GVAR(2, 2, 2, 3, EPI_RESID, 3, 32), GVARN(2, 2, 2, 3, EPI_RESID, 3, 16, 3),
                   GVARN(2, 2, 2, 3, EPI_RESID, 4, 16, 3), GVARN(2, 2, 2, 3, EPI_RESID, 3, 32, 3),
                   GVARN(2, 2, 4, 3, EPI_RESID, 3, 16, 3), GVARN(2, 2, 2, 3, EPI_RESID, 4, 16, 4),
                   GVAR(2, 2, 2, 3, EPI_RESID, 3, 32)}, rounds, iters);
        run_shape("QKV (+RoPE, KV append)", EPI_QKV, M, 288, 864, true,
                  {GVAR(2, 2, 4, 3, EPI_QKV, 4, 16), GVARN(2, 2, 4, 3, EPI_QKV, 3, 16, 3),
                   GVARN(2, 2, 4, 3, EPI_QKV, 4, 16, 3), GVARN(2, 2, 4, 3, EPI_QKV, 3, 16, 4),
                   GVAR(2, 2, 4, 3, EPI_QKV, 4, 16)}, rounds, iters);
        run_shape("down (+resid)", EPI_RESID, M, 768, 288, false,
                  {GVAR(2, 2, 4, 3, EPI_RESID, 2, 32), GVARN(2, 2, 4, 3, EPI_RESID, 3, 16, 3),
                   GVARN(2, 2, 4, 3, EPI_RESID, 2, 32, 3)}, rounds, iters);
        return 0;
    }
    if (argc > 3 && std::string(argv[3]) == "rows") {  // 6-wave blocks: 128 x 288 (whole O-proj rows)
        run_shape("QKV (+RoPE, KV append)", EPI_QKV, M, 288, 864, true,
                  {GVAR(2, 2, 4, 3, EPI_QKV, 4, 16), GVAR(2, 3, 4, 6, EPI_QKV, 3, 16),
                   GVAR(2, 3, 2, 6, EPI_QKV, 4, 16), GVAR(2, 3, 4, 6, EPI_QKV, 2, 16),
                   GVAR(2, 3, 4, 3, EPI_QKV, 4, 16)}, rounds, iters);
        run_shape("O-proj (+resid)", EPI_RESID, M, 288, 288, false,
                  {GVAR(2, 2, 2, 3, EPI_RESID, 3, 32), GVAR(2, 3, 4, 6, EPI_RESID, 3, 16),
                   GVAR(2, 3, 2, 6, EPI_RESID, 4, 32), GVAR(2, 3, 4, 6, EPI_RESID, 2, 32),
                   GVAR(2, 3, 2, 6, EPI_RESID, 4, 16)}, rounds, iters);
        run_shape("down (+resid)", EPI_RESID, M, 768, 288, false,
                  {GVAR(2, 2, 4, 3, EPI_RESID, 2, 32), GVAR(2, 3, 4, 6, EPI_RESID, 3, 16),
                   GVAR(2, 3, 2, 6, EPI_RESID, 4, 32), GVAR(2, 3, 4, 6, EPI_RESID, 2, 32)}, rounds, iters);
        run_shape("gate|up (SwiGLU)", EPI_SWIGLU, M, 288, 1536, true,
                  {GVAR(2, 2, 4, 4, EPI_SWIGLU, 3, 16), GVAR(2, 3, 4, 4, EPI_SWIGLU, 3, 16),
                   GVAR(2, 3, 4, 4, EPI_SWIGLU, 2, 16)}, rounds, iters);
        return 0;
    }
    if (argc > 3 && std::string(argv[3]) == "skinnycold") {  // batched decode GEMMs, each launch after an L2 flush
        g_cold = true;
        for (int Ms : {64, 256}) {
            char l[64];
            snprintf(l, sizeof l, "M=%d QKV", Ms);
            run_shape(l, EPI_QKV, Ms, 288, 864, true,
                      {SVAR(EPI_QKV, 1, 2), SVAR(EPI_QKV, 1, 3), SVAR(EPI_QKV, 1, 4), SVAR(EPI_QKV, 1, 6)}, rounds, iters);
            snprintf(l, sizeof l, "M=%d gate|up", Ms);
            run_shape(l, EPI_SWIGLU, Ms, 288, 1536, true,
                      {SVAR(EPI_SWIGLU, 2, 2), SVAR(EPI_SWIGLU, 2, 3), SVAR(EPI_SWIGLU, 2, 4)}, rounds, iters);
            snprintf(l, sizeof l, "M=%d O-proj", Ms);
            run_shape(l, EPI_RESID, Ms, 288, 288, false,
                      {SVAR(EPI_RESID, 1, 2), SVAR(EPI_RESID, 1, 3), SVAR(EPI_RESID, 1, 4)}, rounds, iters);
            snprintf(l, sizeof l, "M=%d down", Ms);
            run_shape(l, EPI_RESID, Ms, 768, 288, false,
                      {SVAR(EPI_RESID, 1, 2), SVAR(EPI_RESID, 1, 3), SVAR(EPI_RESID, 1, 4), SVAR(EPI_RESID, 1, 6)}, rounds, iters);
        }
        return 0;
    }
    if (argc > 3 && std::string(argv[3]) == "skinny") {  // batched decode: the layer GEMMs at M = B
        // waves per block (the K split): 4 (product) against 2 and 8 at the product's TN / CH;
        // NW changes the partial sums, so the checks show rounding-level differences
        for (int Ms : {64, 128, 256}) {
            char l[64];
            const bool wide = Ms > 128;
            snprintf(l, sizeof l, "M=%d QKV", Ms);
            run_shape(l, EPI_QKV, Ms, 288, 864, true,
                      wide ? std::vector<Variant>{SVARW(EPI_QKV, 2, 2, 4), SVARW(EPI_QKV, 2, 2, 2), SVARW(EPI_QKV, 2, 2, 8), SVARW(EPI_QKV, 2, 1, 8)}
                           : std::vector<Variant>{SVARW(EPI_QKV, 1, 2, 4), SVARW(EPI_QKV, 1, 2, 2), SVARW(EPI_QKV, 1, 2, 8), SVARW(EPI_QKV, 1, 1, 8)},
                      rounds, iters);
            snprintf(l, sizeof l, "M=%d gate|up", Ms);
            run_shape(l, EPI_SWIGLU, Ms, 288, 1536, true,
                      {SVARW(EPI_SWIGLU, 2, 2, 4), SVARW(EPI_SWIGLU, 2, 2, 2), SVARW(EPI_SWIGLU, 2, 2, 8), SVARW(EPI_SWIGLU, 2, 1, 8)},
                      rounds, iters);
            snprintf(l, sizeof l, "M=%d O-proj", Ms);
            run_shape(l, EPI_RESID, Ms, 288, 288, false,
                      wide ? std::vector<Variant>{SVARW(EPI_RESID, 2, 2, 4), SVARW(EPI_RESID, 2, 2, 2), SVARW(EPI_RESID, 2, 2, 8), SVARW(EPI_RESID, 2, 1, 8)}
                           : std::vector<Variant>{SVARW(EPI_RESID, 1, 2, 4), SVARW(EPI_RESID, 1, 2, 2), SVARW(EPI_RESID, 1, 2, 8), SVARW(EPI_RESID, 1, 1, 8)},
                      rounds, iters);
            snprintf(l, sizeof l, "M=%d down", Ms);
            run_shape(l, EPI_RESID, Ms, 768, 288, false,
                      wide ? std::vector<Variant>{SVARW(EPI_RESID, 2, 2, 4), SVARW(EPI_RESID, 2, 2, 2), SVARW(EPI_RESID, 2, 2, 8), SVARW(EPI_RESID, 2, 1, 8)}
                           : std::vector<Variant>{SVARW(EPI_RESID, 1, 2, 4), SVARW(EPI_RESID, 1, 2, 2), SVARW(EPI_RESID, 1, 2, 8), SVARW(EPI_RESID, 1, 1, 8)},
                      rounds, iters);
        }
        return 0;
    }
    if (argc > 3 && std::string(argv[3]) == "group") {  // round 5: grouped tile order, C5 and C3 shapes
        const int Mc = 16384;
        run_shape("C5 gate|up", EPI_SWIGLU, Mc, 4096, 28672, true,
                  {GVAR(2, 2, 4, 4, EPI_SWIGLU, 3, 16), GVARG(2, 2, 4, 4, EPI_SWIGLU, 3, 16, 4),
                   GVARG(2, 2, 4, 4, EPI_SWIGLU, 3, 16, 8), GVARG(2, 2, 4, 4, EPI_SWIGLU, 3, 16, 16)}, rounds, 3);
        run_shape("C5 QKV-shape (store)", EPI_STORE, Mc, 4096, 6144, true,
                  {GVAR(2, 2, 4, 4, EPI_STORE, 3, 16), GVARG(2, 2, 4, 4, EPI_STORE, 3, 16, 8)}, rounds, 3);
        run_shape("C5 O-proj", EPI_RESID, Mc, 4096, 4096, false,
                  {GVAR(2, 2, 4, 4, EPI_RESID, 2, 32), GVARG(2, 2, 4, 4, EPI_RESID, 2, 32, 8)}, rounds, 3);
        run_shape("C5 down", EPI_RESID, Mc, 14336, 4096, false,
                  {GVAR(2, 2, 4, 4, EPI_RESID, 2, 32), GVARG(2, 2, 4, 4, EPI_RESID, 2, 32, 8)}, rounds, 3);
        run_shape("C3 gate|up (SwiGLU)", EPI_SWIGLU, M, 288, 1536, true,
                  {GVAR(2, 2, 4, 4, EPI_SWIGLU, 3, 16), GVARG(2, 2, 4, 4, EPI_SWIGLU, 3, 16, 8)}, rounds, iters);
        return 0;
    }
    if (argc > 3 && std::string(argv[3]) == "big8") {  // round 5: 8-wave blocks at the C3 shapes
        // the product's 64 x 64 / 64 x 48 wave tiles in 256 x 128 (4 x 2 waves) and 128 x 256
        // (2 x 4) blocks: a staged A / W piece feeds twice the MFMAs of the 4-wave block's
        run_shape("gate|up (SwiGLU)", EPI_SWIGLU, M, 288, 1536, true,
                  {GVAR(2, 2, 4, 4, EPI_SWIGLU, 3, 16), GVAR(4, 2, 4, 4, EPI_SWIGLU, 2, 16),
                   GVAR(4, 2, 4, 4, EPI_SWIGLU, 1, 16), GVAR(2, 4, 4, 4, EPI_SWIGLU, 2, 16),
                   GVAR(4, 2, 4, 4, EPI_SWIGLU, 2, 32)}, rounds, iters);
        run_shape("QKV (+RoPE, KV append)", EPI_QKV, M, 288, 864, true,
                  {GVAR(2, 2, 4, 3, EPI_QKV, 4, 16), GVAR(4, 2, 4, 3, EPI_QKV, 2, 16),
                   GVAR(2, 4, 4, 3, EPI_QKV, 2, 16)}, rounds, iters);
        run_shape("down (+resid)", EPI_RESID, M, 768, 288, false,
                  {GVAR(2, 2, 4, 3, EPI_RESID, 2, 32), GVAR(4, 2, 4, 3, EPI_RESID, 2, 32),
                   GVAR(4, 2, 4, 3, EPI_RESID, 2, 16)}, rounds, iters);
        run_shape("O-proj (+resid)", EPI_RESID, M, 288, 288, false,
                  {GVAR(2, 2, 2, 3, EPI_RESID, 3, 32), GVAR(4, 2, 2, 3, EPI_RESID, 2, 32),
                   GVAR(4, 2, 2, 3, EPI_RESID, 3, 32)}, rounds, iters);
        return 0;
    }
    if (argc > 3 && std::string(argv[3]) == "wide") {  // 64 x 96 wave tiles: 24 MFMAs per 4-deep k-step
        run_shape("QKV (+RoPE, KV append)", EPI_QKV, M, 288, 864, true,
                  {GVAR(2, 2, 4, 3, EPI_QKV, 4, 16), GVAR(2, 1, 4, 6, EPI_QKV, 4, 16),
                   GVAR(2, 1, 4, 6, EPI_QKV, 3, 16), GVAR(4, 1, 4, 6, EPI_QKV, 2, 16),
                   GVAR(2, 1, 4, 6, EPI_QKV, 4, 32), GVAR(1, 1, 4, 6, EPI_QKV, 4, 16)}, rounds, iters);
        run_shape("O-proj (+resid)", EPI_RESID, M, 288, 288, false,
                  {GVAR(2, 2, 2, 3, EPI_RESID, 3, 32), GVAR(2, 1, 2, 6, EPI_RESID, 4, 32),
                   GVAR(2, 1, 4, 6, EPI_RESID, 4, 32), GVAR(2, 1, 4, 6, EPI_RESID, 3, 16),
                   GVAR(1, 1, 4, 6, EPI_RESID, 4, 32)}, rounds, iters);
        run_shape("down (+resid)", EPI_RESID, M, 768, 288, false,
                  {GVAR(2, 2, 4, 3, EPI_RESID, 2, 32), GVAR(2, 1, 4, 6, EPI_RESID, 3, 32),
                   GVAR(2, 1, 4, 6, EPI_RESID, 2, 32), GVAR(4, 1, 4, 6, EPI_RESID, 2, 16)}, rounds, iters);
        run_shape("gate|up (SwiGLU)", EPI_SWIGLU, M, 288, 1536, true,
                  {GVAR(2, 2, 4, 4, EPI_SWIGLU, 3, 16), GVAR(2, 1, 4, 8, EPI_SWIGLU, 3, 16),
                   GVAR(2, 1, 4, 8, EPI_SWIGLU, 2, 16)}, rounds, iters);
        return 0;
    }
    if (argc > 3 && std::string(argv[3]) == "qkv18") {  // QKV wave tiles with more MFMAs per k-step
        // 64 x 48 wave tiles issue 12 MFMAs per 4-deep k-step; 96 x 48 (192 x 96 blocks) 18 and
        // 128 x 32 (3-wave 128 x 96 blocks) 16, both dividing N = 864 without padding
        run_shape("QKV (+RoPE, KV append)", EPI_QKV, M, 288, 864, true,
                  {GVAR(2, 2, 4, 3, EPI_QKV, 4, 16), GVAR(2, 2, 6, 3, EPI_QKV, 3, 16),
                   GVAR(2, 2, 6, 3, EPI_QKV, 2, 16), GVAR(1, 3, 8, 2, EPI_QKV, 4, 16),
                   GVAR(1, 3, 8, 2, EPI_QKV, 3, 16)}, rounds, iters);
        run_shape("QKV shape, plain store", EPI_STORE, M, 288, 864, true,
                  {GVAR(2, 2, 4, 3, EPI_STORE, 4, 16), GVAR(2, 2, 6, 3, EPI_STORE, 3, 16),
                   GVAR(1, 3, 8, 2, EPI_STORE, 4, 16)}, rounds, iters);
        return 0;
    }
    if (argc > 3 && std::string(argv[3]) == "lmcold") {  // round 6: batched-decode lm_head, L2 flushed per launch
        g_cold = true;
        run_shape("lm_head M=256 (cold)", EPI_STORE, 256, 288, 32000, true,
                  {GVARN(4, 1, 4, 4, EPI_STORE, 2, 16, 3), GVARN(4, 1, 4, 2, EPI_STORE, 2, 16, 3),
                   GVARN(4, 1, 4, 2, EPI_STORE, 2, 16, 4), GVARN(4, 1, 4, 1, EPI_STORE, 2, 16, 4),
                   GVARN(2, 2, 4, 2, EPI_STORE, 2, 16, 4), GVARN(4, 1, 2, 4, EPI_STORE, 2, 16, 4),
                   GVARN(2, 2, 4, 4, EPI_STORE, 2, 16, 4), GVARN(4, 1, 2, 2, EPI_STORE, 2, 16, 4)},
                  rounds, iters);
        return 0;
    }
    if (argc > 3 && std::string(argv[3]) == "lmhead") {  // last-position lm_head tiles (C3 part / batched decode)
        // M = 128 (a C3 batch-split part) and 256 (the batch, batched decode B = 256): one block
        // per CU at the product tiles (250 / 500 blocks); smaller tiles put several on each CU
        for (int m : {128, 256})
            run_shape(m == 128 ? "lm_head M=128" : "lm_head M=256", EPI_STORE, m, 288, 32000, true,
                      {m == 128 ? GVARN(2, 2, 4, 4, EPI_STORE, 2, 16, 4) : GVARN(4, 1, 4, 4, EPI_STORE, 2, 16, 3),
                       GVARN(2, 2, 4, 2, EPI_STORE, 2, 16, 4), GVARN(2, 2, 2, 4, EPI_STORE, 2, 16, 4),
                       GVARN(2, 2, 2, 4, EPI_STORE, 2, 16, 6), GVARN(2, 2, 2, 2, EPI_STORE, 4, 16, 4),
                       GVARN(2, 2, 4, 2, EPI_STORE, 3, 16, 3), GVARN(1, 4, 4, 2, EPI_STORE, 2, 16, 4),
                       GVARN(2, 2, 1, 4, EPI_STORE, 2, 16, 6)},
                      rounds, iters);
        return 0;
    }
    if (argc > 3 && std::string(argv[3]) == "qkvfast") {  // round 6: the division-free QKV epilogue
        Variant fast{"glds<2,2,4,3,wpe4,bk16> fast epilogue", [](const GemmArgs& a0, hipStream_t s) {
            GemmArgs a = a0;
            a.qkv_fast = true;
            hipLaunchKernelGGL((gemm_lds_kernel<2, 2, 4, 3, EPI_QKV, 4, false, 16, true>), dim3(512 * 9), dim3(256), 0, s, a);
        }};
        Variant fast128{"glds<2,2,4,4,wpe3,bk16> fast epilogue", [](const GemmArgs& a0, hipStream_t s) {
            GemmArgs a = a0;
            a.qkv_fast = true;
            hipLaunchKernelGGL((gemm_lds_kernel<2, 2, 4, 4, EPI_QKV, 3, false, 16, true>), dim3(512 * 7), dim3(256), 0, s, a);
        }};
        for (int r = 0; r < 2; ++r) {
            run_shape("QKV (+RoPE, KV append)", EPI_QKV, M, 288, 864, true,
                      {GVAR(2, 2, 4, 3, EPI_QKV, 4, 16), fast, fast128}, rounds, iters);
            run_shape("QKV shape, plain store", EPI_STORE, M, 288, 864, true,
                      {GVAR(2, 2, 4, 3, EPI_STORE, 4, 16)}, rounds, iters);
        }
        return 0;
    }
    if (argc > 3 && std::string(argv[3]) == "normab") {  // the two norm-fused C3 GEMMs (run by gemm_tune and gemm_tune_ssh)
        Variant fast{"QKV glds<2,2,4,3,wpe4,bk16> fast epilogue", [](const GemmArgs& a0, hipStream_t s) {
            GemmArgs a = a0;
            a.qkv_fast = true;
            hipLaunchKernelGGL((gemm_lds_kernel<2, 2, 4, 3, EPI_QKV, 4, false, 16, true>), dim3(512 * 9), dim3(256), 0, s, a);
        }};
        for (int r = 0; r < 2; ++r) {
            run_shape("QKV (+RoPE, KV append)", EPI_QKV, M, 288, 864, true, {fast}, rounds, iters);
            run_shape("gate|up (SwiGLU)", EPI_SWIGLU, M, 288, 1536, true, {GVAR(2, 2, 4, 4, EPI_SWIGLU, 3, 16)}, rounds, iters);
        }
        return 0;
    }
    if (argc > 3 && std::string(argv[3]) == "qkvsplit") {  // round 6: QKV columns by two tiles
        // columns [0, 768) on the 128 x 128 tile (16 MFMAs per 4-deep k-step, the gate|up tile:
        // 6 column tiles, no padding) and [768, 864) on 128 x 96, as two launches
        Variant two{"two launches 128x128 [0,768) + 128x96 [768,864)", [](const GemmArgs& a0, hipStream_t s) {
            GemmArgs a = a0;
            a.N = 768;
            hipLaunchKernelGGL((gemm_lds_kernel<2, 2, 4, 4, EPI_QKV, 3, false, 16, true>), dim3(512 * 6), dim3(256), 0, s, a);
            GemmArgs b = a0;
            b.W = a0.W + (int64_t)768 * a0.K; b.N = 96; b.col_base = 768;
            hipLaunchKernelGGL((gemm_lds_kernel<2, 2, 4, 3, EPI_QKV, 4, false, 16, true>), dim3(512), dim3(256), 0, s, b);
        }};
        Variant two4{"two launches 128x128 wpe4 + 128x96", [](const GemmArgs& a0, hipStream_t s) {
            GemmArgs a = a0;
            a.N = 768;
            hipLaunchKernelGGL((gemm_lds_kernel<2, 2, 4, 4, EPI_QKV, 4, false, 16, true>), dim3(512 * 6), dim3(256), 0, s, a);
            GemmArgs b = a0;
            b.W = a0.W + (int64_t)768 * a0.K; b.N = 96; b.col_base = 768;
            hipLaunchKernelGGL((gemm_lds_kernel<2, 2, 4, 3, EPI_QKV, 4, false, 16, true>), dim3(512), dim3(256), 0, s, b);
        }};
        for (int r = 0; r < 2; ++r)
            run_shape("QKV (+RoPE, KV append)", EPI_QKV, M, 288, 864, true,
                      {GVAR(2, 2, 4, 3, EPI_QKV, 4, 16), two, two4, GVAR(2, 2, 4, 4, EPI_QKV, 3, 16)}, rounds, iters);
        return 0;
    }
    if (argc > 3 && std::string(argv[3]) == "qkvepi") {  // what the QKV epilogue costs
        run_shape("QKV (+RoPE, KV append)", EPI_QKV, M, 288, 864, true,
                  {GVAR(2, 2, 4, 3, EPI_QKV, 4, 16), GVAR(4, 1, 4, 6, EPI_QKV, 3, 16),
                   GVAR(4, 1, 4, 6, EPI_QKV, 2, 16), GVAR(2, 2, 4, 6, EPI_QKV, 2, 16)}, rounds, iters);
        run_shape("QKV shape, plain store", EPI_STORE, M, 288, 864, true,
                  {GVAR(2, 2, 4, 3, EPI_STORE, 4, 16), GVAR(4, 1, 4, 6, EPI_STORE, 3, 16)}, rounds, iters);
        run_shape("gate|up shape, plain store", EPI_STORE, M, 288, 1536, true,
                  {GVAR(2, 2, 4, 4, EPI_STORE, 3, 16)}, rounds, iters);
        return 0;
    }
    if (!c5) {
    run_shape("gate|up (SwiGLU)", EPI_SWIGLU, M, 288, 1536, true,
              {RVAR(2, 2, 4, 4, EPI_SWIGLU, 3, 16), GVAR(2, 2, 4, 4, EPI_SWIGLU, 3, 16),
               GVAR(2, 2, 4, 4, EPI_SWIGLU, 2, 32)}, rounds, iters);
    run_shape("QKV (+RoPE, KV append)", EPI_QKV, M, 288, 864, true,
              {RVAR(2, 2, 4, 4, EPI_QKV, 3, 16), GVAR(2, 2, 4, 4, EPI_QKV, 3, 16),
               GVAR(2, 2, 4, 3, EPI_QKV, 3, 16), GVAR(2, 2, 4, 3, EPI_QKV, 4, 16)}, rounds, iters);
    run_shape("down (+resid)", EPI_RESID, M, 768, 288, false,
              {RVAR(2, 2, 4, 3, EPI_RESID, 2, 32), GVAR(2, 2, 4, 3, EPI_RESID, 2, 32),
               GVAR(2, 2, 4, 3, EPI_RESID, 3, 16)}, rounds, iters);
    run_shape("O-proj (+resid)", EPI_RESID, M, 288, 288, false,
              {RVAR(2, 2, 2, 3, EPI_RESID, 2, 32), GVAR(2, 2, 2, 3, EPI_RESID, 3, 32),
               GVAR(2, 2, 2, 3, EPI_RESID, 3, 16), GVAR(2, 2, 4, 3, EPI_RESID, 3, 16)}, rounds, iters);
    } else {
    // Llama-3-8B shapes (C5) at M = 16384 rows (tuning size)
    const int Mc = 16384;
    // round 5: + 8-wave 256 x 128 / 128 x 256 blocks (half the LDS fragment traffic per MFMA of
    // the 128 x 128 block) and deeper k-tile rings, for the long-K (4096) shapes
    run_shape("C5 gate|up", EPI_SWIGLU, Mc, 4096, 28672, true,
              {GVAR(2, 2, 4, 4, EPI_SWIGLU, 3, 16), GVAR(2, 2, 4, 4, EPI_SWIGLU, 2, 32),
               GVARN(2, 2, 4, 4, EPI_SWIGLU, 3, 16, 3), GVAR(4, 2, 4, 4, EPI_SWIGLU, 2, 16),
               GVAR(4, 2, 4, 4, EPI_SWIGLU, 1, 32), GVAR(2, 4, 4, 4, EPI_SWIGLU, 2, 16)}, rounds, 3);
    run_shape("C5 QKV-shape (store)", EPI_STORE, Mc, 4096, 6144, true,
              {GVAR(2, 2, 4, 4, EPI_STORE, 3, 16), GVAR(2, 2, 4, 3, EPI_STORE, 4, 16),
               GVAR(2, 2, 4, 4, EPI_STORE, 2, 32), GVAR(4, 2, 4, 4, EPI_STORE, 2, 16),
               GVAR(2, 4, 4, 4, EPI_STORE, 2, 16)}, rounds, 3);
    run_shape("C5 O-proj", EPI_RESID, Mc, 4096, 4096, false,
              {GVAR(2, 2, 4, 4, EPI_RESID, 3, 16), GVAR(2, 2, 4, 4, EPI_RESID, 2, 32)}, rounds, 3);
    run_shape("C5 down", EPI_RESID, Mc, 14336, 4096, false,
              {GVAR(2, 2, 4, 4, EPI_RESID, 3, 16), GVAR(2, 2, 4, 4, EPI_RESID, 2, 32)}, rounds, 3);
    }
    return 0;
}
