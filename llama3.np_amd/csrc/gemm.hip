// fp32 MFMA GEMM dispatch (kernel templates and design notes: gemm_kernel.h).
// Only the (tile, epilogue) pairs used below are instantiated.
#include <cstdlib>

#include "gemm_kernel.h"
#include "gemm_x6.h"

namespace l3 {

// Product kernels: k-tiles filled by global_load_lds (GLDS) and the register-direct epilogue
// (DIRECT): RMSNorm weights are folded into W at l3_finalize, the row factor comes from the A
// fragments, the tile leaves from registers.
template <int EPI, int WM, int WN, int TM, int TN, int WPE, int BK, int NS = 2>
static hipError_t launch(const GemmArgs& a, hipStream_t s) {
    constexpr int BM = WM * TM * 16, BN = WN * TN * 16;
    const int64_t tiles = (int64_t)((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
    hipLaunchKernelGGL((gemm_lds_kernel<WM, WN, TM, TN, EPI, WPE, false, BK, true, NS>),
                       dim3((unsigned)tiles), dim3(64 * WM * WN), 0, s, a);
    return hipGetLastError();
}

// the opt-in x6 path (gemm_x6.h): six bf16 MFMA products per fp32 product, W3 pieces from
// l3_finalize; WM*TM*16 x WN*TN*16 tiles (BK 32, 2 blocks per CU by LDS)
template <int EPI, int WM, int WN, int TM, int TN>
static hipError_t launch_x6(const GemmArgs& a, hipStream_t s) {
    constexpr int BM = WM * TM * 16, BN = WN * TN * 16;
    const int64_t tiles = (int64_t)((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
    hipLaunchKernelGGL((gemm_x6_kernel<WM, WN, TM, TN, EPI, 2>), dim3((unsigned)tiles), dim3(64 * WM * WN), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_split_planes(const float* w, unsigned short* w3, int64_t rows, int K, hipStream_t s) {
    const int64_t n = rows * K;
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(split_planes_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, w, w3, rows, K);
    return hipGetLastError();
}

// Split-K for short M against a long K (batched decode and short prompts at Llama-3 sizes):
// a 64-row x 4096-deep O-proj is 32 tiles of 128 columns, so 32 blocks would each stream a
// 2 MB weight panel (C5 64-token prefill: 0.59 ms per O-proj / down launch).  The k-slices run
// as tiles x S blocks (S a power of two up to 16, >= 8 k-tiles per slice, about 1024 blocks in
// all) and splitk_finish_kernel sums them in slice order and applies the epilogue.
template <int WM, int WN, int TM, int TN, int BK, int NS>
static hipError_t launch_split_cfg(int epi, GemmArgs a, hipStream_t s) {
    constexpr int BM = WM * TM * 16, BN = WN * TN * 16;
    const int64_t tiles = (int64_t)((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
    const int nk = a.K / BK;
    const int64_t need_per = (int64_t)a.M * a.N + a.M;  // floats per slice
    static const int target = env_knob("L3_SPLITK_BLOCKS", 1024);
    static const int min_kt = env_knob("L3_SPLITK_MINKT", 8);
    int S = 1;
    while (S < 16 && tiles * S < target && nk % (2 * S) == 0 && nk / (2 * S) >= min_kt &&
           2 * S * need_per <= a.ws_cap)
        S *= 2;
    if (S == 1) return hipErrorNotReady;  // not worth it: the caller runs the unsplit tiles
    a.splits = S;
    hipLaunchKernelGGL((gemm_lds_kernel<WM, WN, TM, TN, EPI_STORE, 2, false, BK, true, NS, true>),
                       dim3((unsigned)(tiles * S)), dim3(64 * WM * WN), 0, s, a);
    if (const hipError_t e = hipGetLastError(); e != hipSuccess) return e;
    const int64_t outs = (int64_t)a.M * (epi == EPI_SWIGLU ? a.N / 2 : a.N) / 4;
    const dim3 grid((unsigned)((outs + 255) / 256));
    switch (epi) {
        case EPI_SWIGLU: hipLaunchKernelGGL(splitk_finish_kernel<EPI_SWIGLU>, grid, dim3(256), 0, s, a); break;
        case EPI_QKV: hipLaunchKernelGGL(splitk_finish_kernel<EPI_QKV>, grid, dim3(256), 0, s, a); break;
        case EPI_RESID: hipLaunchKernelGGL(splitk_finish_kernel<EPI_RESID>, grid, dim3(256), 0, s, a); break;
        default: hipLaunchKernelGGL(splitk_finish_kernel<EPI_STORE>, grid, dim3(256), 0, s, a); break;
    }
    return hipGetLastError();
}

// L3_SPLITK=0: off (A/B); L3_SPLITK_CFG picks the slice tile (tuning)
static hipError_t launch_split(int epi, const GemmArgs& a, hipStream_t s) {
    static const int on = env_knob("L3_SPLITK", 1);
    static const int cfg = env_knob("L3_SPLITK_CFG", 0);
    if (!on || !a.ws || a.M <= 8 || a.M > 256 || a.K < 2048 || a.K % 32 != 0) return hipErrorNotReady;
    switch (cfg) {
        case 1: return launch_split_cfg<2, 2, 4, 4, 16, 2>(epi, a, s);
        case 2: return launch_split_cfg<2, 2, 2, 4, 32, 2>(epi, a, s);
        case 3: return launch_split_cfg<2, 2, 2, 4, 16, 4>(epi, a, s);
        case 4: return launch_split_cfg<1, 4, 1, 2, 32, 2>(epi, a, s);
        default:
            if (a.M <= 16) return launch_split_cfg<1, 4, 1, 2, 32, 2>(epi, a, s);  // 16 x 128
            if (a.M <= 64) return launch_split_cfg<2, 2, 2, 4, 32, 2>(epi, a, s);  // 64 x 128
            return launch_split_cfg<2, 2, 4, 4, 32, 2>(epi, a, s);                 // 128 x 128
    }
}

template <int EPI, int MR, int LPU, bool PARTS = false, bool NT = false, bool FOLD = false>
static hipError_t launch_gemv_lpu(const GemmArgs& a, hipStream_t s) {
    const int units = (EPI == EPI_SWIGLU || EPI == EPI_QKV) ? a.N / 2 : a.N;
    const int per_block = 4 * (64 / LPU);
    const dim3 grid((unsigned)((units + per_block - 1) / per_block), (unsigned)((a.M + MR - 1) / MR)),
        block(256);
    hipLaunchKernelGGL((gemv_kernel<EPI, MR, LPU, PARTS, NT, FOLD>), grid, block, MR == 1 ? 0 : (size_t)MR * a.K * 4, s, a);
    return hipGetLastError();
}

// non-temporal W loads for the one-row GEMV over a weight larger than the caches would keep
// (>= 64 MB: the Llama-3-shape decode; gemv_kernel NT); L3_GEMV_NT=0 turns them off (A/B)
static bool gemv_nt(const GemmArgs& a) {
    static const int on = env_knob("L3_GEMV_NT", 1);
    return on && (int64_t)a.N * a.K * 4 >= ((int64_t)64 << 20);
}

// the O-proj partial rows of the fused decode attention (GemmArgs::parts): EPI_SWIGLU carries
// GEMV_MAXP partial loads per piece, so its lanes take fewer pieces (<= 4 up to K = 1024)
template <int EPI>
static hipError_t launch_gemv_parts(const GemmArgs& a, hipStream_t s) {
    if (a.nparts < 1 || a.nparts > GEMV_MAXP || !gemv_direct(a)) return hipErrorInvalidValue;
    const int k4 = a.K / 4;
    if constexpr (EPI == EPI_SWIGLU) {
        if (k4 <= 128) return launch_gemv_lpu<EPI, 1, 32, true>(a, s);
    } else {
        if (k4 <= 128) return launch_gemv_lpu<EPI, 1, 16, true>(a, s);
        if (k4 <= 256) return launch_gemv_lpu<EPI, 1, 32, true>(a, s);
    }
    if (gemv_nt(a)) return launch_gemv_lpu<EPI, 1, 64, true, true>(a, s);
    return launch_gemv_lpu<EPI, 1, 64, true>(a, s);
}

// lanes per unit from K: ~5-8 float4 per lane per W row in one chunk at the stories15M sizes;
// L3_GEMV_LPU=16/32/64 forces it (A/B tuning of the decode GEMVs)
static int gemv_lpu(const GemmArgs& a) {
    static const int force = env_knob("L3_GEMV_LPU", 0);
    if (force == 16 || force == 32 || force == 64) return force;
    const int k4 = a.K / 4;
    return k4 <= 128 ? 16 : k4 <= 256 ? 32 : 64;
}

template <int EPI, int MR>
static hipError_t launch_gemv_mr(const GemmArgs& a, hipStream_t s) {
    if constexpr (MR == 1) {
        if (gemv_lpu(a) == 64 && gemv_nt(a)) return launch_gemv_lpu<EPI, 1, 64, false, true>(a, s);
    }
    switch (gemv_lpu(a)) {
        case 16: return launch_gemv_lpu<EPI, MR, 16>(a, s);
        case 32: return launch_gemv_lpu<EPI, MR, 32>(a, s);
        default: return launch_gemv_lpu<EPI, MR, 64>(a, s);
    }
}

int gemv_store_blocks(const GemmArgs& a) {
    if (a.M != 1 || !gemv_direct(a)) return 0;
    const int per_block = 4 * (64 / gemv_lpu(a));
    return (a.N + per_block - 1) / per_block;
}

template <int EPI>
static hipError_t launch_gemv(const GemmArgs& a, hipStream_t s) {
    // Rows per block: up to M = 8, a layer weight (<= 16 MB, L2-resident) runs one row per
    // block and re-reads W through L2 (B = 8 decode: QKV 13.7 -> 6.1 us, gate|up 12.3 -> 5.5
    // against 8-row blocks); the lm_head streams once with all rows per block (25 vs 37 us);
    // past M = 8, 4-row blocks: twice the blocks of 8-row ones hide more of each block's round
    // trips (batched decode B = 64 0.355 -> 0.316, B = 256 0.548 -> 0.530 ms per step; 2-row
    // blocks 0.310 / 0.591; where the skinny MFMA kernel does not take them); a weight past the
    // caches keeps one block row up to M = 8 so it streams once.  L3_GEMV_MR caps it (tuning).
    static const int env_cap = env_knob("L3_GEMV_MR", 0);
    const bool small_w = (int64_t)a.N * a.K <= (int64_t)4 << 20;
    const int cap = env_cap ? env_cap : small_w ? 4 : 8;
    if (a.M <= 1 || cap == 1 || (small_w && a.M <= 8)) return launch_gemv_mr<EPI, 1>(a, s);
    if (a.M <= 2 || cap == 2) return launch_gemv_mr<EPI, 2>(a, s);
    if (a.M <= 4 || cap == 4) return launch_gemv_mr<EPI, 4>(a, s);
    return launch_gemv_mr<EPI, 8>(a, s);
}

bool gemv_direct(const GemmArgs& a) {
    static const int cap = env_knob("L3_GEMV_MR", 4);
    const bool small_w = (int64_t)a.N * a.K <= (int64_t)4 << 20;
    return gemm_is_gemv(a) && (a.M <= 1 || cap == 1 || (small_w && a.M <= 8));
}

// 9..256 rows against a small weight on the skinny MFMA kernel (gemm_kernel.h); L3_SKINNY=0
// keeps them on the GEMV (A/B)
// CH = 2 k-blocks per round trip, TN = 2 column tiles only for SwiGLU (the gate / up pair); TN and
// CH leave every element's K order as it is, so all of them round identically
// (tools/gemm_tune 5 50 skinny: at M = 64 / 128 / 256 CH 2 beat the earlier CH 6 by 10-30 %)
template <int EPI, int TN>
static hipError_t launch_skinny(const GemmArgs& a, hipStream_t s) {
    constexpr int WN = 16 * TN;
    const int64_t blocks = (int64_t)((a.M + 15) / 16) * ((a.N + WN - 1) / WN);
    // k-blocks per round trip: 2.  In the batched decode loop (weights from MALL, not the L2-hot
    // loop of tools/gemm_tune) CH 6 / 12 measured 0.333 / 0.408 ms per B = 256 step against 0.313
    // (profiles/r05_skinny_ab.txt); L3_SKINNY_CH re-runs that A/B
    static const int ch = env_knob("L3_SKINNY_CH", 2);
    // tile order (GemmArgs::skinny_xcd, bit-identical either way): L3_SKINNY_XCD
    static const bool xcd = env_knob("L3_SKINNY_XCD", 0) != 0;
    GemmArgs g = a;
    g.skinny_xcd = xcd;
    if (ch >= 12)
        hipLaunchKernelGGL((gemm_skinny_kernel<EPI, TN, 12>), dim3((unsigned)blocks), dim3(256), 0, s, g);
    else if (ch >= 6)
        hipLaunchKernelGGL((gemm_skinny_kernel<EPI, TN, 6>), dim3((unsigned)blocks), dim3(256), 0, s, g);
    else
        hipLaunchKernelGGL((gemm_skinny_kernel<EPI, TN, 2>), dim3((unsigned)blocks), dim3(256), 0, s, g);
    return hipGetLastError();
}

// rows past which QKV / O-proj / down take 2-tile columns: none up to 256 (one-tile columns give
// the 256-row launches twice the blocks: B = 256 decode 0.308-0.309 against 0.313-0.315 ms per step,
// profiles/r05_skinny_ab.txt; the column tiling leaves each element's K order, so results are
// bit-identical); L3_SKINNY_TN2_MIN re-runs that A/B
static int skinny_tn2() {
    static const int m = env_knob("L3_SKINNY_TN2_MIN", 256);
    return m;
}

static bool use_skinny(const GemmArgs& a) {
    static const int on = env_knob("L3_SKINNY", 1);
    static const int lo = env_knob("L3_SKINNY_MIN", 9);
    return on && a.M >= lo && a.M <= 256 && !a.kv_bak && !a.parts && !a.amax_part && a.K % 16 == 0;
}

bool gemm_is_gemv(const GemmArgs& a) {
    const int mr = a.M <= 1 ? 1 : a.M <= 2 ? 2 : a.M <= 4 ? 4 : 8;
    const bool short_m = a.M <= 8 || (a.M <= 256 && (int64_t)a.N * a.K <= (int64_t)4 << 20);
    return short_m && (size_t)mr * a.K <= 16384;  // A rows fit 64 KB of LDS (QKV: N even)
}

// ids compare rounding: 3 and 4 (128 x 128 vs 256 x 64 tiles) visit K in the same order per
// element (BK 16, one MFMA chain per accumulator), so they round identically
int gemm_store_config(const GemmArgs& a) {
    if (gemm_is_gemv(a)) return 0;
    return a.M <= 32 ? 1 : a.M <= 64 ? 2 : 3;
}

hipError_t launch_gemm(int epi, const GemmArgs& a, hipStream_t s) {
    if (a.M <= 0 || a.N <= 0) return hipSuccess;
    if (a.K % 32 != 0 || a.K <= 0) return hipErrorInvalidValue;  // whole 32-deep k-tiles
    if (epi == EPI_SWIGLU && a.N % 32 != 0) return hipErrorInvalidValue;
    if (a.N % 4 != 0 || a.ldc % 4 != 0 || a.lda % 4 != 0) return hipErrorInvalidValue;  // 16-B rows
    // Short M (decode, batched decode, short prompts): weight-streaming GEMV with the same
    // epilogues, 8-row blocks beyond M = 8 re-reading W through L2 — for the layer weights up
    // to M = 256 (a 128-row MFMA tile there is one k-loop of memory round trips on a handful of
    // blocks); the 37 MB lm_head keeps the MFMA tiles past M = 8
    if (a.parts) {
        switch (epi) {
            case EPI_SWIGLU: return launch_gemv_parts<EPI_SWIGLU>(a, s);
            case EPI_RESID: return launch_gemv_parts<EPI_RESID>(a, s);
            default: return hipErrorInvalidValue;
        }
    }
    if (a.amax_part && (epi != EPI_STORE || !gemv_store_blocks(a))) return hipErrorInvalidValue;
    // amax_rows: the tiled EPI_STORE kernels only (16 * TN = 64-column wave tiles, no split-K)
    if (a.amax_rows && (epi != EPI_STORE || gemm_store_config(a) == 0 || a.ws || a.amax_nct != (a.N + 63) / 64))
        return hipErrorInvalidValue;
    if (a.pos_adv && !a.amax_part) return hipErrorInvalidValue;
    if (a.amax_in) {  // layer-0 QKV of a captured batch-1 decode step with the previous argmax folded in
        if (epi != EPI_QKV || a.M != 1 || !gemv_direct(a) || a.col_base || a.a_rows || a.amax_in_n < 1 ||
            !a.amax_ids || !a.amax_st)
            return hipErrorInvalidValue;
        switch (gemv_lpu(a)) {
            case 16: return launch_gemv_lpu<EPI_QKV, 1, 16, false, false, true>(a, s);
            case 32: return launch_gemv_lpu<EPI_QKV, 1, 32, false, false, true>(a, s);
            default: return launch_gemv_lpu<EPI_QKV, 1, 64, false, false, true>(a, s);
        }
    }
    if (a.force_skinny || (gemm_is_gemv(a) && use_skinny(a))) {
        switch (epi) {
            case EPI_SWIGLU: return launch_skinny<EPI_SWIGLU, 2>(a, s);
            case EPI_QKV: return a.M > skinny_tn2() ? launch_skinny<EPI_QKV, 2>(a, s) : launch_skinny<EPI_QKV, 1>(a, s);
            case EPI_RESID: return a.M > skinny_tn2() ? launch_skinny<EPI_RESID, 2>(a, s) : launch_skinny<EPI_RESID, 1>(a, s);
            case EPI_STORE: return launch_skinny<EPI_STORE, 1>(a, s);
            default: return hipErrorInvalidValue;
        }
    }
    if (gemm_is_gemv(a)) {
        // GemmArgs::col_base (a K / V-only QKV) is honoured by the skinny and tiled epilogues
        // only: the GEMV would write the K / V columns as q
        if (a.col_base) return hipErrorInvalidValue;
        switch (epi) {
            case EPI_SWIGLU: return launch_gemv<EPI_SWIGLU>(a, s);
            case EPI_QKV: return launch_gemv<EPI_QKV>(a, s);
            case EPI_RESID: return launch_gemv<EPI_RESID>(a, s);
            case EPI_STORE: return launch_gemv<EPI_STORE>(a, s);
            default: return hipErrorInvalidValue;
        }
    }
    if (a.ws && !a.col_base) {  // splitk_finish_kernel's QKV epilogue has no col_base either
        const hipError_t e = launch_split(epi, a, s);
        if (e != hipErrorNotReady) return e;
    }
    // Configurations chosen with tools/gemm_tune (interleaved A/B on MI355X).
    // 128 x 128 BK16: 120 VGPRs + 32 KB LDS -> 4 blocks per CU.
    const bool small_m = a.M <= 32;  // tiny M: 16 x 128 tile
    // long K (the Llama-3 shape's gate|up): tiles in groups of 4 row tiles walked column by
    // column, so a k-step's concurrent blocks on an XCD share a few A and W slices in L2 instead
    // of one A slice and ~96 W slices (round 5, groups of 8: C5 gate|up 134.7 -> 135.8 TF/s,
    // profiles/r05_gemm_group_ab.txt; round 6 sweep, profiles/r06_c5_group_pmc.txt: 4 / 8 / 16 /
    // 32 rows per group 136.6 / 135.9 / 134.6 / 128.6 TF/s and 222 / 261 / 264 / 474 GB of L2-miss
    // traffic per launch; bit-identical; QKV and C3's K = 288 keep the row-major order);
    // L3_GEMM_GROUP_M=0 turns it off (A/B)
    static const int group_env = env_knob("L3_GEMM_GROUP_M", 4);
    GemmArgs ag = a;
    ag.group_m = a.K >= 1024 && !small_m ? group_env : 0;
    // EPI_QKV: the division-free full-tile epilogue (gemm_kernel.h qkv_epilogue_full) where its
    // shape conditions hold — heads in whole 16-column groups, every wave's 64 rows within two
    // sequences; L3_QKV_FAST_EPI=0 keeps the generic epilogue (A/B; both round identically)
    static const bool qkv_fast_env = env_knob("L3_QKV_FAST_EPI", 1) != 0;
    ag.qkv_fast = epi == EPI_QKV && qkv_fast_env && a.HD % 16 == 0 && a.L >= 64;
    // x6 (opt-in): 128-row tiles, four waves (eight for gate|up and the O-proj); tools/gemm_tune x6 at C3
    // (profiles/r06_x6_tiles*.txt, final build r06_x6_tiles_final.txt): gate|up 128 x 128 195.0
    // fp32-equivalent TF/s against 119.7 for the fp32 kernel on the same box, QKV 128 x 128 162.0
    // (128 x 96 158.1), down 128 x 96 178.7, O-proj 128 x 96 of 8 waves 151.8 (4 waves 145.4);
    // gate|up on 8 waves of 16 x 128 193.9 vs 186.2 for 4 of 32 x 128 (r06_x6_big.txt), C3 x6
    // step 4.505-4.509 vs 4.552-4.569 ms (r06_x6_gateup8_ab.txt)
    if (a.W3 && !small_m && epi != EPI_STORE) {
        switch (epi) {
            case EPI_SWIGLU: return launch_x6<EPI_SWIGLU, 8, 1, 1, 8>(ag, s);   // 128 x 128, 8 waves
            case EPI_QKV:  // 128 x 128 (C3's 864 columns: 6 3/4 tiles, the last on the generic epilogue)
                return launch_x6<EPI_QKV, 4, 1, 2, 8>(ag, s);
            case EPI_RESID:  // O-proj (short K): 8 waves of 32 x 48; down: 4 waves of 32 x 96
                if (a.N % 96 == 0) {
                    static const bool w8 = env_knob("L3_X6_OPROJ_W8", 1) != 0;  // A/B: 0 = 4 waves
                    return a.K <= 512 && w8 ? launch_x6<EPI_RESID, 4, 2, 2, 3>(ag, s) : launch_x6<EPI_RESID, 4, 1, 2, 6>(ag, s);
                }
                return launch_x6<EPI_RESID, 4, 1, 2, 8>(ag, s);
            default: return hipErrorInvalidValue;
        }
    }
    switch (epi) {
        case EPI_SWIGLU:  // 128 x 128, BK 16
            if (small_m) return launch<EPI_SWIGLU, 1, 4, 1, 2, 2, 32>(a, s);
            return launch<EPI_SWIGLU, 2, 2, 4, 4, 3, 16>(ag, s);
        case EPI_QKV:     // 128 x 96 at short K (stories15M), else 128 x 128; BK 16
            if (small_m) return launch<EPI_QKV, 1, 4, 1, 2, 2, 32>(ag, s);
            if (a.N % 96 == 0 && a.K <= 1024) return launch<EPI_QKV, 2, 2, 4, 3, 4, 16>(ag, s);
            return launch<EPI_QKV, 2, 2, 4, 4, 3, 16>(ag, s);
        case EPI_RESID:   // O-proj / down
            if (small_m) return launch<EPI_RESID, 1, 4, 1, 2, 2, 32>(a, s);
            if (a.N % 96 == 0)
                return a.K <= 512 ? launch<EPI_RESID, 2, 2, 2, 3, 3, 32>(a, s)   // 64 x 96
                                  : launch<EPI_RESID, 2, 2, 4, 3, 2, 32>(a, s);  // 128 x 96
            return launch<EPI_RESID, 2, 2, 4, 4, 2, 32>(a, s);                   // 128 x 128
        case EPI_STORE:   // lm_head (the 37 MB W streams from HBM past few blocks: deep
                          // LDS rings, B = 64 lm_head 30.3 -> 18.4 us), op-level linear
            switch (gemm_store_config(a)) {
                case 1: return launch<EPI_STORE, 2, 2, 1, 4, 2, 16, 6>(a, s);
                case 2: return launch<EPI_STORE, 2, 2, 2, 4, 2, 16, 6>(a, s);
                default:
                    // 129-256 rows: one 256-row panel per column tile, so the weight streams from
                    // HBM once per launch (two 128-row tiles read it twice: 1.54x the algorithmic
                    // bytes at B = 256, profiles/pmc_gateup.json r01)
                    if (a.M > 128 && a.M <= 256) return launch<EPI_STORE, 4, 1, 4, 4, 2, 16, 3>(a, s);
                    return launch<EPI_STORE, 2, 2, 4, 4, 2, 16, 4>(a, s);
            }
        default:
            return hipErrorInvalidValue;
    }
}

hipError_t dcheck_collect_gemm(unsigned* out) { return dcheck_collect(out); }

}  // namespace l3
