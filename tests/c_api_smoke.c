/*
 * c_api_smoke.c — the C ABI (include/llama3hip.h) driven from plain C, no Python: a small
 * random GQA model (D 64, 2 layers, H 4 / KVH 2, VS 512, FD 192) through create -> upload ->
 * finalize -> prefill -> greedy steps -> device-side greedy loop -> destroy, plus the error
 * paths the reference fails on (llama3.py:184, :287, :289).
 *
 * Built twice by llama3.np_amd/csrc/Makefile: `c_smoke` against libllama3hip.so and
 * `c_smoke_asan`, whose library and host program are compiled with host-side
 * AddressSanitizer (`-Xarch_host -fsanitize=address`: host code only, the gfx950 code objects
 * are unchanged).  tests/test_c_abi_gpu.py runs both on the GPU.  Exit status 0 = pass.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "llama3hip.h"

enum { D = 64, NL = 2, H = 4, KVH = 2, VS = 512, FD = 192, MS = 64, MB = 2, HD = D / H };

static uint32_t seed = 12345u;
static float frand(float scale) {  // xorshift32, uniform in [-scale, scale)
    seed ^= seed << 13;
    seed ^= seed >> 17;
    seed ^= seed << 5;
    return scale * ((float)(seed >> 8) / 8388608.0f - 1.0f);
}

static float* tensor(int64_t n, float scale) {
    float* t = (float*)malloc((size_t)n * sizeof(float));
    for (int64_t i = 0; i < n; ++i) t[i] = frand(scale);
    return t;
}

#define CHECK(call)                                                                  \
    do {                                                                             \
        if ((call) != 0) {                                                           \
            fprintf(stderr, "FAIL %s:%d %s: %s\n", __FILE__, __LINE__, #call, l3_last_error()); \
            return 1;                                                                \
        }                                                                            \
    } while (0)

#define EXPECT_FAIL(call)                                                            \
    do {                                                                             \
        if ((call) == 0) {                                                           \
            fprintf(stderr, "FAIL %s:%d %s succeeded\n", __FILE__, __LINE__, #call); \
            return 1;                                                                \
        }                                                                            \
        if (!l3_last_error() || !l3_last_error()[0]) {                               \
            fprintf(stderr, "FAIL %s:%d %s: no error message\n", __FILE__, __LINE__, #call); \
            return 1;                                                                \
        }                                                                            \
    } while (0)

static int upload(l3_ctx* c, int layer, int kind, int64_t rows, int64_t cols, float scale) {
    float* t = tensor(rows * cols, scale);
    if (kind == L3_W_ATTN_NORM || kind == L3_W_FFN_NORM || kind == L3_W_FINAL_NORM)
        for (int64_t i = 0; i < rows * cols; ++i) t[i] = 1.0f + 0.5f * t[i];
    const int rc = l3_upload_weight(c, layer, kind, t, rows, cols);
    free(t);
    return rc;
}

static int argmax_row(const float* x, int n) {
    int b = 0;
    for (int i = 1; i < n; ++i)
        if (x[i] > x[b]) b = i;
    return b;
}

int main(void) {
    int32_t ndev = 0;
    CHECK(l3_device_count(&ndev));
    if (ndev < 1) {
        fprintf(stderr, "FAIL no HIP device\n");
        return 1;
    }
    const l3_dims dims = {D, NL, H, KVH, VS, FD, MS, MB, 1e-6f};
    l3_ctx* c = NULL;
    CHECK(l3_create(0, &dims, &c));
    CHECK(upload(c, 0, L3_W_EMBED, VS, D, 1.0f));
    for (int l = 0; l < NL; ++l) {
        CHECK(upload(c, l, L3_W_Q, H * HD, D, 0.1f));
        CHECK(upload(c, l, L3_W_K, KVH * HD, D, 0.1f));
        CHECK(upload(c, l, L3_W_V, KVH * HD, D, 0.1f));
        CHECK(upload(c, l, L3_W_O, D, H * HD, 0.1f));
        CHECK(upload(c, l, L3_W_GATE, FD, D, 0.1f));
        CHECK(upload(c, l, L3_W_UP, FD, D, 0.1f));
        CHECK(upload(c, l, L3_W_DOWN, D, FD, 0.1f));
        CHECK(upload(c, l, L3_W_ATTN_NORM, 1, D, 1.0f));
        CHECK(upload(c, l, L3_W_FFN_NORM, 1, D, 1.0f));
    }
    CHECK(upload(c, 0, L3_W_FINAL_NORM, 1, D, 1.0f));
    CHECK(upload(c, 0, L3_W_LM_HEAD, VS, D, 0.3f));
    EXPECT_FAIL(upload(c, NL, L3_W_Q, H * HD, D, 0.1f));  // layer out of range
    CHECK(l3_finalize(c));

    // prefill B = 2, L = 9: finite logits; the greedy step on the same inputs and positions
    // (the KV cache is rewritten identically) returns their argmax
    enum { B = 2, L = 9 };
    int64_t ids[B * L];
    for (int i = 0; i < B * L; ++i) ids[i] = (int64_t)((seed = seed * 1664525u + 1013904223u) >> 8) % VS;
    float* logits = (float*)malloc(sizeof(float) * B * VS);
    CHECK(l3_forward_host(c, ids, B, L, 0, logits));
    for (int i = 0; i < B * VS; ++i)
        if (!isfinite(logits[i])) {
            fprintf(stderr, "FAIL non-finite logit at %d\n", i);
            return 1;
        }
    // batch split API (parts of 9 tokens stay unsplit: a part needs > 256 rows)
    float* logits2 = (float*)malloc(sizeof(float) * B * VS);
    EXPECT_FAIL(l3_set_batch_split(c, 0, 1));
    CHECK(l3_set_batch_split(c, 2, 1));
    CHECK(l3_forward_host(c, ids, B, L, 0, logits2));
    if (memcmp(logits, logits2, sizeof(float) * B * VS) != 0) {
        fprintf(stderr, "FAIL batch split changed the logits\n");
        return 1;
    }
    // last block on every position (extension): the same logits within fp32 rounding
    CHECK(l3_set_last_layer_rows(c, 1));
    CHECK(l3_forward_host(c, ids, B, L, 0, logits2));
    for (int i = 0; i < B * VS; ++i)
        if (fabsf(logits[i] - logits2[i]) > 1e-4f) {
            fprintf(stderr, "FAIL all-rows last layer differs at %d: %g vs %g\n", i, logits[i], logits2[i]);
            return 1;
        }
    CHECK(l3_set_last_layer_rows(c, 0));
    free(logits2);
    CHECK(l3_set_batch_split(c, 1, 1));
    int64_t nxt[B];
    CHECK(l3_greedy_step_host(c, ids, B, L, 0, nxt, NULL));
    for (int b = 0; b < B; ++b)
        if (nxt[b] != argmax_row(logits + b * VS, VS)) {
            fprintf(stderr, "FAIL greedy id %lld != argmax %d (row %d)\n", (long long)nxt[b],
                    argmax_row(logits + b * VS, VS), b);
            return 1;
        }
    // decode steps at the reference's schedule (pos L + i), then the device-side loop
    for (int i = 1; i < 6; ++i) CHECK(l3_greedy_step_host(c, nxt, B, 1, L + i, nxt, NULL));
    int64_t out[B * 20];
    CHECK(l3_greedy_generate_host(c, ids, B, 5, 25, out));
    for (int i = 0; i < B * 20; ++i)
        if (out[i] < 0 || out[i] >= VS) {
            fprintf(stderr, "FAIL generated id %lld out of range\n", (long long)out[i]);
            return 1;
        }
    // the same schedule one step per call (the reference's lazy generator: prefill, then decode
    // at pos 5 + i, i >= 1) with the device running ahead: the device loop's ids, step for step
    CHECK(l3_set_decode_horizon(c, 25));
    int64_t lz[B];
    CHECK(l3_greedy_step_host(c, ids, B, 5, 0, lz, NULL));
    for (int i = 0; i < 20; ++i) {
        if (i) CHECK(l3_greedy_step_host(c, lz, B, 1, 5 + i, lz, NULL));
        for (int b = 0; b < B; ++b)
            if (lz[b] != out[b * 20 + i]) {
                fprintf(stderr, "FAIL lazy step %d row %d: %lld != device loop %lld\n", i, b,
                        (long long)lz[b], (long long)out[b * 20 + i]);
                return 1;
            }
    }
    int64_t replayed = 0, ahead = 0;
    CHECK(l3_decode_stats(c, &replayed, &ahead));
    if (ahead < 10) {
        fprintf(stderr, "FAIL only %lld of the lazy steps were run ahead\n", (long long)ahead);
        return 1;
    }

    // the reference's failure modes become error returns with a message
    EXPECT_FAIL(l3_forward_host(c, ids, MB + 1, 1, 0, logits));  // batch > max_batch_size
    EXPECT_FAIL(l3_forward_host(c, ids, B, L, MS - 4, logits));  // positions past max_seq_len
    ids[3] = VS;                                                  // token id out of range
    EXPECT_FAIL(l3_forward_host(c, ids, B, L, 0, logits));
    EXPECT_FAIL(l3_forward_host(c, ids, 0, L, 0, logits));        // empty batch

    free(logits);
    CHECK(l3_destroy(c));
    printf("c_api_smoke ok\n");
    return 0;
}
