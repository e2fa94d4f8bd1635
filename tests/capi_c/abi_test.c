/*
 * abi_test.c -- a native C caller of the engine's C ABI, compiled against include/tfhe_mi355.h
 * alone (gcc -std=c11, no C++ and no torch), the way a Rust `extern "C"` binding would use it
 * (INTEGRATION.md).  Driven by tests/test_capi_c_gpu.py; built by tfhe-rs-odd_amd/Makefile.
 *
 *   abi_test contract   every device scratch is sized by its *_scratch query only; the async PBS,
 *                       the async KS->PBS and submit/wait are bit-exact against the synchronous
 *                       host-pointer calls at a persistent-grid classic shape (N = 2048, the 2_2
 *                       shape), a split-CMUX shape (N = 4096, chunk scratch) and multi-bit
 *                       (N = 2048, g = 3, no scratch); an async PBS given a NULL or a short
 *                       scratch fails with rc = 1 instead of running a fallback.
 *   abi_test multi      a context over devices {0, 0} (tfhe_mi355_context_create_devices: two
 *                       shards on the box's one GPU) against a single-device context with the same
 *                       keys: batched PBS / KS->PBS / PBS->KS / KS (split over the shards), count-1
 *                       calls and submit/wait (spread over the shards' coalescers) bit-identical.
 *   abi_test destroy    (run with TFHE_MI355_COALESCE_WINDOW_US / _GAP_US = 2 s so that the
 *                       request is still queued) destroying a context with an unwaited request
 *                       returns 1, and that request's wait returns 1 with a message.
 *
 * Error convention under test: 0 = ok, 1 = failure + tfhe_mi355_last_error() (c_api/utils.rs:3-73).
 * Keys come from the engine's client helpers with a reduced LWE dimension (fast keygen; the
 * checks are engine-vs-engine, so the dimension does not matter to them).
 */
#define __HIP_PLATFORM_AMD__ 1
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "tfhe_mi355.h"

static int failures = 0;

#define CHECK(cond, ...)                                  \
    do {                                                  \
        if (!(cond)) {                                    \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);                 \
            fprintf(stderr, "\n");                        \
            failures++;                                   \
        }                                                 \
    } while (0)
#define ABI(call)                                                                                     \
    do {                                                                                              \
        if ((call) != TFHE_MI355_OK) {                                                                \
            fprintf(stderr, "FAIL %s:%d: %s -> %s\n", __FILE__, __LINE__, #call, tfhe_mi355_last_error()); \
            exit(2);                                                                                  \
        }                                                                                             \
    } while (0)
#define HIP(call)                                                                               \
    do {                                                                                        \
        if ((call) != hipSuccess) {                                                             \
            fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #call);                     \
            exit(2);                                                                            \
        }                                                                                       \
    } while (0)

static uint64_t *xalloc(size_t words) {
    uint64_t *p = (uint64_t *)calloc(words ? words : 1, 8);
    if (!p) {
        fprintf(stderr, "out of memory\n");
        exit(2);
    }
    return p;
}

static void *dalloc(size_t bytes) {
    void *p = NULL;
    if (bytes) HIP(hipMalloc(&p, bytes));
    return p;
}

typedef struct {
    const char *name;
    TfheMi355Parameters p;
    double lwe_std, glwe_std;
    size_t count;  /* batch of the async / sync comparison */
} Case;

typedef struct {
    TfheMi355Context *ctx;
    uint64_t *lwe_sk, *glwe_sk;
    uint64_t *bsk, *ksk;  /* kept for a second context (multi mode) */
    size_t bsk_len, ksk_len;
    uint64_t *lut;   /* 2 LUTs */
    size_t n, big, glwe;
} Keys;

static uint64_t delta_of(const TfheMi355Parameters *p) {
    return (1ULL << 63) / ((uint64_t)p->message_modulus * p->carry_modulus);
}

static void setup(const Case *c, Keys *k) {
    const TfheMi355Parameters *p = &c->p;
    k->n = p->lwe_dimension;
    k->big = (size_t)p->glwe_dimension * p->polynomial_size;
    k->glwe = k->big + p->polynomial_size;
    ABI(tfhe_mi355_context_create(p, 0, &k->ctx));
    k->lwe_sk = xalloc(k->n);
    k->glwe_sk = xalloc(k->big);
    ABI(tfhe_mi355_client_gen_binary_key(7, 1, k->lwe_sk, k->n));
    ABI(tfhe_mi355_client_gen_binary_key(7, 2, k->glwe_sk, k->big));
    const size_t ggsw = p->grouping_factor ? (k->n / p->grouping_factor) << p->grouping_factor : k->n;
    const size_t bsk_len = ggsw * p->pbs_level * (p->glwe_dimension + 1) * (p->glwe_dimension + 1) * p->polynomial_size;
    uint64_t *bsk = xalloc(bsk_len);
    if (p->grouping_factor)
        ABI(tfhe_mi355_client_gen_multi_bit_bootstrap_key(8, k->lwe_sk, (uint32_t)k->n, k->glwe_sk, p->glwe_dimension,
                                                          p->polynomial_size, p->pbs_base_log, p->pbs_level,
                                                          p->grouping_factor, c->glwe_std, bsk, 8));
    else
        ABI(tfhe_mi355_client_gen_bootstrap_key(8, k->lwe_sk, (uint32_t)k->n, k->glwe_sk, p->glwe_dimension,
                                                p->polynomial_size, p->pbs_base_log, p->pbs_level, c->glwe_std, bsk, 8));
    ABI(tfhe_mi355_bootstrap_key_upload(k->ctx, bsk, bsk_len));
    const size_t ksk_len = k->big * p->ks_level * (k->n + 1);
    uint64_t *ksk = xalloc(ksk_len);
    ABI(tfhe_mi355_client_gen_keyswitch_key(9, k->glwe_sk, (uint32_t)k->big, k->lwe_sk, (uint32_t)k->n, p->ks_base_log,
                                            p->ks_level, c->lwe_std, ksk));
    ABI(tfhe_mi355_keyswitch_key_upload(k->ctx, ksk, ksk_len));
    k->bsk = bsk;
    k->ksk = ksk;
    k->bsk_len = bsk_len;
    k->ksk_len = ksk_len;
    /* two LUTs: identity and x -> 3x + 1 (shortint fill_accumulator) */
    const uint64_t msg = (uint64_t)p->message_modulus * p->carry_modulus;
    uint64_t *f = xalloc(msg);
    k->lut = xalloc(2 * k->glwe);
    for (uint64_t i = 0; i < msg; i++) f[i] = i;
    ABI(tfhe_mi355_fill_accumulator(p, f, k->lut));
    for (uint64_t i = 0; i < msg; i++) f[i] = (3 * i + 1) % msg;
    ABI(tfhe_mi355_fill_accumulator(p, f, k->lut + k->glwe));
    free(f);
}

static void teardown(Keys *k) {
    int rc = tfhe_mi355_context_destroy(k->ctx);
    CHECK(rc == TFHE_MI355_OK, "destroy: %s", tfhe_mi355_last_error());
    free(k->bsk);
    free(k->ksk);
    free(k->lwe_sk);
    free(k->glwe_sk);
    free(k->lut);
}

/* `count` ciphertexts of message i % msg under key sk (dimension dim) */
static uint64_t *encrypt(const Case *c, const uint64_t *sk, size_t dim, size_t count, double std, uint64_t seed) {
    const uint64_t msg = (uint64_t)c->p.message_modulus * c->p.carry_modulus;
    uint64_t *pt = xalloc(count), *ct = xalloc(count * (dim + 1));
    for (size_t i = 0; i < count; i++) pt[i] = (i % msg) * delta_of(&c->p);
    ABI(tfhe_mi355_client_lwe_encrypt(seed, sk, (uint32_t)dim, pt, count, std, ct));
    free(pt);
    return ct;
}

static uint32_t *lut_indexes(size_t count) {
    uint32_t *x = (uint32_t *)calloc(count, 4);
    for (size_t i = 0; i < count; i++) x[i] = (uint32_t)(i % 3 == 0);
    return x;
}

/* decrypt and check against the LUT each row used */
static void check_decrypt(const Case *c, const Keys *k, const uint64_t *out, size_t count, const uint32_t *idx,
                          const char *what) {
    const uint64_t msg = (uint64_t)c->p.message_modulus * c->p.carry_modulus, delta = delta_of(&c->p);
    uint64_t *pt = xalloc(count);
    ABI(tfhe_mi355_client_lwe_decrypt(k->glwe_sk, (uint32_t)k->big, out, count, pt));
    size_t bad = 0;
    for (size_t i = 0; i < count; i++) {
        const uint64_t m = i % msg, want = idx && idx[i] ? (3 * m + 1) % msg : m;
        const uint64_t d = pt[i] + (delta >> 1);
        if ((d / delta) % msg != want) bad++;
    }
    CHECK(bad == 0, "%s %s: %zu of %zu outputs decrypt wrong", c->name, what, bad, count);
    free(pt);
}

static int same(const uint64_t *a, const uint64_t *b, size_t words) { return memcmp(a, b, words * 8) == 0; }

static void run_contract(const Case *c) {
    Keys k;
    setup(c, &k);
    const size_t B = c->count, small_w = k.n + 1, big_w = k.big + 1;
    uint32_t *idx = lut_indexes(B);
    uint64_t *ct_small = encrypt(c, k.lwe_sk, k.n, B, c->lwe_std, 11);
    uint64_t *ct_big = encrypt(c, k.glwe_sk, k.big, B, c->glwe_std, 12);

    /* reference: the synchronous host-pointer calls */
    uint64_t *pbs_sync = xalloc(B * big_w), *kspbs_sync = xalloc(B * big_w);
    ABI(tfhe_mi355_programmable_bootstrap(k.ctx, ct_small, pbs_sync, k.lut, 2, idx, B));
    ABI(tfhe_mi355_keyswitch_programmable_bootstrap(k.ctx, ct_big, kspbs_sync, k.lut, 2, idx, B));
    check_decrypt(c, &k, pbs_sync, B, idx, "sync PBS");
    check_decrypt(c, &k, kspbs_sync, B, idx, "sync KS->PBS");

    /* async: device buffers, scratch sized ONLY by the queries */
    hipStream_t s;
    HIP(hipStreamCreate(&s));
    uint64_t *d_small = (uint64_t *)dalloc(B * small_w * 8), *d_big = (uint64_t *)dalloc(B * big_w * 8);
    uint64_t *d_out = (uint64_t *)dalloc(B * big_w * 8), *d_lut = (uint64_t *)dalloc(2 * k.glwe * 8);
    uint32_t *d_idx = (uint32_t *)dalloc(B * 4);
    HIP(hipMemcpy(d_small, ct_small, B * small_w * 8, hipMemcpyHostToDevice));
    HIP(hipMemcpy(d_big, ct_big, B * big_w * 8, hipMemcpyHostToDevice));
    HIP(hipMemcpy(d_lut, k.lut, 2 * k.glwe * 8, hipMemcpyHostToDevice));
    HIP(hipMemcpy(d_idx, idx, B * 4, hipMemcpyHostToDevice));
    uint64_t *got = xalloc(B * big_w);

    size_t pbs_scratch = 0, kspbs_scratch = 0, ks_scratch = 0;
    ABI(tfhe_mi355_programmable_bootstrap_scratch(k.ctx, B, &pbs_scratch));
    ABI(tfhe_mi355_keyswitch_programmable_bootstrap_scratch(k.ctx, B, &kspbs_scratch));
    ABI(tfhe_mi355_keyswitch_scratch(k.ctx, B, &ks_scratch));
    printf("%s: scratch bytes pbs %zu ks_pbs %zu ks %zu\n", c->name, pbs_scratch, kspbs_scratch, ks_scratch);
    void *d_scratch = dalloc(pbs_scratch);
    ABI(tfhe_mi355_programmable_bootstrap_async(k.ctx, d_small, d_out, d_lut, 2, d_idx, B, d_scratch, pbs_scratch, s));
    HIP(hipStreamSynchronize(s));
    HIP(hipMemcpy(got, d_out, B * big_w * 8, hipMemcpyDeviceToHost));
    CHECK(same(got, pbs_sync, B * big_w), "%s: async PBS differs from the sync call", c->name);
    if (pbs_scratch) {  /* the query is the contract: less scratch is an error, never a fallback */
        int rc = tfhe_mi355_programmable_bootstrap_async(k.ctx, d_small, d_out, d_lut, 2, d_idx, B, NULL, 0, s);
        CHECK(rc == TFHE_MI355_ERROR && strstr(tfhe_mi355_last_error(), "scratch"),
              "%s: async PBS with NULL scratch returned %d (%s)", c->name, rc, tfhe_mi355_last_error());
        if (c->p.polynomial_size <= 2048) {
            rc = tfhe_mi355_programmable_bootstrap_async(k.ctx, d_small, d_out, d_lut, 2, d_idx, B, d_scratch,
                                                         pbs_scratch - 1, s);
            CHECK(rc == TFHE_MI355_ERROR, "%s: async PBS with a short scratch returned %d", c->name, rc);
        }
    }
    HIP(hipFree(d_scratch));

    d_scratch = dalloc(kspbs_scratch);
    HIP(hipMemset(d_out, 0, B * big_w * 8));
    ABI(tfhe_mi355_keyswitch_programmable_bootstrap_async(k.ctx, d_big, d_out, d_lut, 2, d_idx, B, d_scratch,
                                                          kspbs_scratch, s));
    HIP(hipStreamSynchronize(s));
    HIP(hipMemcpy(got, d_out, B * big_w * 8, hipMemcpyDeviceToHost));
    CHECK(same(got, kspbs_sync, B * big_w), "%s: async KS->PBS differs from the sync call", c->name);
    HIP(hipFree(d_scratch));

    /* submit / wait: one request per row (count = 1, the reference's per-block calls), all four
     * ops in flight together, then every wait; each row equal to the batched sync result */
    const size_t R = B < 48 ? B : 48;
    uint64_t *ks_sync = xalloc(B * small_w), *pbsks_sync = xalloc(B * small_w);
    ABI(tfhe_mi355_keyswitch(k.ctx, ct_big, ks_sync, B));
    ABI(tfhe_mi355_programmable_bootstrap_keyswitch(k.ctx, ct_small, pbsks_sync, k.lut, 2, idx, B));
    uint64_t *o_pbs = xalloc(R * big_w), *o_kspbs = xalloc(R * big_w), *o_pbsks = xalloc(R * small_w),
             *o_ks = xalloc(R * small_w);
    TfheMi355Request **req = (TfheMi355Request **)calloc(4 * R, sizeof(*req));
    for (size_t i = 0; i < R; i++) {
        ABI(tfhe_mi355_submit(k.ctx, 0, ct_small + i * small_w, o_pbs + i * big_w, k.lut, 2, idx + i, 1, &req[4 * i]));
        ABI(tfhe_mi355_submit(k.ctx, 1, ct_big + i * big_w, o_kspbs + i * big_w, k.lut, 2, idx + i, 1,
                              &req[4 * i + 1]));
        ABI(tfhe_mi355_submit(k.ctx, 2, ct_small + i * small_w, o_pbsks + i * small_w, k.lut, 2, idx + i, 1,
                              &req[4 * i + 2]));
        ABI(tfhe_mi355_submit(k.ctx, 3, ct_big + i * big_w, o_ks + i * small_w, NULL, 0, NULL, 1, &req[4 * i + 3]));
    }
    for (size_t i = 0; i < 4 * R; i++) ABI(tfhe_mi355_wait(req[i]));
    CHECK(same(o_pbs, pbs_sync, R * big_w), "%s: submit/wait PBS differs", c->name);
    CHECK(same(o_kspbs, kspbs_sync, R * big_w), "%s: submit/wait KS->PBS differs", c->name);
    CHECK(same(o_pbsks, pbsks_sync, R * small_w), "%s: submit/wait PBS->KS differs", c->name);
    CHECK(same(o_ks, ks_sync, R * small_w), "%s: submit/wait KS differs", c->name);

    /* bad arguments fail with rc = 1 and a message, out-handles nulled */
    TfheMi355Request *r = (TfheMi355Request *)&r;
    int rc = tfhe_mi355_submit(k.ctx, 9, ct_small, o_pbs, k.lut, 2, NULL, 1, &r);
    CHECK(rc == TFHE_MI355_ERROR && r == NULL && strlen(tfhe_mi355_last_error()) > 0, "%s: bad op accepted", c->name);

    free(req);
    free(o_pbs);
    free(o_kspbs);
    free(o_pbsks);
    free(o_ks);
    free(ks_sync);
    free(pbsks_sync);
    HIP(hipFree(d_small));
    HIP(hipFree(d_big));
    HIP(hipFree(d_out));
    HIP(hipFree(d_lut));
    HIP(hipFree(d_idx));
    HIP(hipStreamDestroy(s));
    free(got);
    free(pbs_sync);
    free(kspbs_sync);
    free(ct_small);
    free(ct_big);
    free(idx);
    teardown(&k);
    printf("%s: %s\n", c->name, failures ? "FAILED" : "ok");
}

/* 2_2 (shortint/parameters/mod.rs, PARAM_MESSAGE_2_CARRY_2_KS_PBS) with n reduced to 64 */
static const Case CASE_2_2 = {"2_2", {64, 1, 2048, 23, 1, 3, 5, 4, 4, 0}, 7.069849454709433e-06, 2.9403601535432533e-16, 1000};
/* PARAM_MESSAGE_2_CARRY_3_KS_PBS (N = 4096, split CMUX, chunk scratch), n = 64; noise of the real set */
static const Case CASE_2_3 = {"2_3", {64, 1, 4096, 22, 1, 3, 6, 4, 8, 0}, 8.775214009854235e-07, 2.168404344971009e-19, 150};
/* PARAM_MULTI_BIT_MESSAGE_2_CARRY_2_GROUP_3_KS_PBS (N = 2048, g = 3), n = 66 */
static const Case CASE_MB3 = {"mb3", {66, 1, 2048, 21, 1, 7, 2, 4, 4, 3}, 6.125031601933181e-07, 3.152931493498455e-16, 200};

/* multi mode: the same calls on a {0, 0} context and a single-device one, compared row for row */
static void run_multi(const Case *c) {
    Keys k;
    setup(c, &k);
    const int devs[2] = {0, 0};
    TfheMi355Context *m = NULL;
    ABI(tfhe_mi355_context_create_devices(&c->p, devs, 2, &m));
    size_t nd = 0;
    ABI(tfhe_mi355_context_devices(m, &nd));
    CHECK(nd == 2, "%s: %zu devices reported", c->name, nd);
    TfheMi355Context *shard = NULL;
    int dev = -1;
    ABI(tfhe_mi355_context_device_context(m, 1, &shard, &dev));
    CHECK(shard != NULL && dev == 0, "%s: shard 1 on device %d", c->name, dev);
    CHECK(tfhe_mi355_context_destroy(shard) == TFHE_MI355_ERROR, "%s: a shard could be destroyed directly", c->name);
    ABI(tfhe_mi355_bootstrap_key_upload(m, k.bsk, k.bsk_len));
    ABI(tfhe_mi355_keyswitch_key_upload(m, k.ksk, k.ksk_len));
    const size_t B = c->count, small_w = k.n + 1, big_w = k.big + 1;
    uint32_t *idx = lut_indexes(B);
    uint64_t *ct_small = encrypt(c, k.lwe_sk, k.n, B, c->lwe_std, 21);
    uint64_t *ct_big = encrypt(c, k.glwe_sk, k.big, B, c->glwe_std, 22);
    uint64_t *a = xalloc(B * big_w), *b = xalloc(B * big_w);
    ABI(tfhe_mi355_programmable_bootstrap(k.ctx, ct_small, a, k.lut, 2, idx, B));
    ABI(tfhe_mi355_programmable_bootstrap(m, ct_small, b, k.lut, 2, idx, B));
    CHECK(same(a, b, B * big_w), "%s: multi-device PBS differs", c->name);
    check_decrypt(c, &k, b, B, idx, "multi-device PBS");
    ABI(tfhe_mi355_keyswitch_programmable_bootstrap(k.ctx, ct_big, a, k.lut, 2, idx, B));
    ABI(tfhe_mi355_keyswitch_programmable_bootstrap(m, ct_big, b, k.lut, 2, idx, B));
    CHECK(same(a, b, B * big_w), "%s: multi-device KS->PBS differs", c->name);
    ABI(tfhe_mi355_keyswitch(k.ctx, ct_big, a, B));
    ABI(tfhe_mi355_keyswitch(m, ct_big, b, B));
    CHECK(same(a, b, B * small_w), "%s: multi-device KS differs", c->name);
    ABI(tfhe_mi355_programmable_bootstrap_keyswitch(k.ctx, ct_small, a, k.lut, 2, idx, B));
    ABI(tfhe_mi355_programmable_bootstrap_keyswitch(m, ct_small, b, k.lut, 2, idx, B));
    CHECK(same(a, b, B * small_w), "%s: multi-device PBS->KS differs", c->name);
    /* count-1 calls and submitted requests: spread over the shards' coalescers */
    ABI(tfhe_mi355_programmable_bootstrap(k.ctx, ct_small, a, k.lut, 2, idx, B));
    const size_t R = B < 40 ? B : 40;
    TfheMi355Request **req = (TfheMi355Request **)calloc(R, sizeof(*req));
    for (size_t i = 0; i < R; i++)
        ABI(tfhe_mi355_submit(m, 0, ct_small + i * small_w, b + i * big_w, k.lut, 2, idx + i, 1, &req[i]));
    for (size_t i = 0; i < R; i++) ABI(tfhe_mi355_wait(req[i]));
    CHECK(same(a, b, R * big_w), "%s: multi-device submit/wait differs", c->name);
    ABI(tfhe_mi355_programmable_bootstrap(m, ct_small + 5 * small_w, b, k.lut, 2, idx + 5, 1));
    CHECK(same(a + 5 * big_w, b, big_w), "%s: multi-device count-1 call differs", c->name);
    uint64_t batches = 0, rows = 0, inflight = 0;
    double secs = 0;
    ABI(tfhe_mi355_coalesce_stats(m, 0, &batches, &rows, &inflight, &secs));
    CHECK(rows == R + 1, "%s: coalesced rows %llu, expected %zu", c->name, (unsigned long long)rows, R + 1);
    free(req);
    free(a);
    free(b);
    free(ct_small);
    free(ct_big);
    free(idx);
    CHECK(tfhe_mi355_context_destroy(m) == TFHE_MI355_OK, "multi destroy: %s", tfhe_mi355_last_error());
    teardown(&k);
    printf("%s multi: %s\n", c->name, failures ? "FAILED" : "ok");
}

static int run_destroy(void) {
    Keys k;
    Case c = CASE_2_2;
    c.count = 4;
    setup(&c, &k);
    uint64_t *ct = encrypt(&c, k.lwe_sk, k.n, 1, c.lwe_std, 13);
    uint64_t *out = xalloc(k.big + 1);
    TfheMi355Request *req = NULL;
    ABI(tfhe_mi355_submit(k.ctx, 0, ct, out, k.lut, 2, NULL, 1, &req));
    /* the coalescer's window (2 s in this run) keeps the request queued: destroy must fail it */
    int rc = tfhe_mi355_context_destroy(k.ctx);
    CHECK(rc == TFHE_MI355_ERROR && strstr(tfhe_mi355_last_error(), "still queued"),
          "destroy with a queued request returned %d (%s)", rc, tfhe_mi355_last_error());
    printf("destroy: rc %d: %s\n", rc, tfhe_mi355_last_error());
    rc = tfhe_mi355_wait(req);
    CHECK(rc == TFHE_MI355_ERROR && strstr(tfhe_mi355_last_error(), "destroyed"),
          "wait on the failed request returned %d (%s)", rc, tfhe_mi355_last_error());
    printf("wait: rc %d: %s\n", rc, tfhe_mi355_last_error());
    free(ct);
    free(out);
    free(k.bsk);
    free(k.ksk);
    free(k.lwe_sk);
    free(k.glwe_sk);
    free(k.lut);
    return failures;
}

int main(int argc, char **argv) {
    const char *mode = argc > 1 ? argv[1] : "contract";
    int devices = 0;
    ABI(tfhe_mi355_device_count(&devices));
    if (devices < 1) {
        fprintf(stderr, "no GPU\n");
        return 2;
    }
    if (!strcmp(mode, "destroy")) return run_destroy() ? 1 : 0;
    if (!strcmp(mode, "multi")) {
        run_multi(&CASE_2_2);
        run_multi(&CASE_2_3);
        run_multi(&CASE_MB3);
        printf("%s\n", failures ? "FAILED" : "ALL OK");
        return failures ? 1 : 0;
    }
    if (strcmp(mode, "contract")) {
        fprintf(stderr, "usage: abi_test contract|multi|destroy\n");
        return 2;
    }
    run_contract(&CASE_2_2);
    run_contract(&CASE_2_3);
    run_contract(&CASE_MB3);
    printf("%s\n", failures ? "FAILED" : "ALL OK");
    return failures ? 1 : 0;
}
