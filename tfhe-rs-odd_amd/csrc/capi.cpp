// capi.cpp -- C ABI implementation (include/tfhe_mi355.h).  Host-side runtime of the engine:
// context = device + parameter set + key material + FFT tables, guarded by a mutex so that
// concurrent callers (the reference's rayon workers, shortint/engine/mod.rs:23-25) can share one
// key.  Error convention: 0/1 return + thread-local message (tfhe/src/c_api/utils.rs:3-73).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/tfhe_mi355.h"
#include "engine.h"
#include "errors.h"

using namespace tfhe_mi355;

namespace {

struct Failure : std::runtime_error {
    using std::runtime_error::runtime_error;
};

[[noreturn]] void fail(const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    throw Failure(buf);
}

void check(hipError_t e, const char *what) {
    if (e != hipSuccess) fail("%s: %s", what, hipGetErrorString(e));
}

template <class F>
int guarded(F &&f) {
    try {
        f();
        last_error_text().clear();
        return TFHE_MI355_OK;
    } catch (const std::exception &ex) {
        last_error_text() = ex.what();
        return TFHE_MI355_ERROR;
    } catch (...) {
        last_error_text() = "unknown failure";
        return TFHE_MI355_ERROR;
    }
}

struct DeviceBuffer {
    void *ptr = nullptr;
    size_t bytes = 0;
    void reserve(size_t b) {
        if (b <= bytes) return;
        if (ptr) check(hipFree(ptr), "hipFree");
        ptr = nullptr;
        bytes = 0;
        check(hipMalloc(&ptr, b), "hipMalloc");
        bytes = b;
    }
    void release() {
        if (ptr) (void)hipFree(ptr);
        ptr = nullptr;
        bytes = 0;
    }
};

bool is_pow2(uint32_t x) { return x && !(x & (x - 1)); }
}  // namespace

struct TfheMi355Context {
    TfheMi355Parameters p{};
    int device = 0;
    std::mutex mu;
    hipStream_t stream = nullptr;
    FftTables tables;
    DeviceBuffer fbsk, ksk, std_staging;
    DeviceBuffer io_in, io_out, io_luts, io_idx, io_tmp;
    DeviceBuffer pbs_scratch;  // N = 32768: accumulators + spectra of one chunk of ciphertexts
    DeviceBuffer ksk_planes;   // int8 byte planes of the KSK for the MFMA keyswitch
    DeviceBuffer ks_scratch;   // MFMA keyswitch digits
    bool ksk_planes_ready = false;
    bool fbsk_ready = false, ksk_ready = false;
    // LWE -> GLWE packing keyswitching key of the gadget layer (big LWE key -> GLWE key)
    DeviceBuffer pksk, pksk_planes;
    uint32_t pks_base_log = 0, pks_level = 0;
    bool pksk_ready = false, pksk_planes_ready = false;

    size_t n() const { return p.lwe_dimension; }
    size_t k() const { return p.glwe_dimension; }
    size_t N() const { return p.polynomial_size; }
    size_t big_dim() const { return k() * N(); }
    size_t glwe_len() const { return (k() + 1) * N(); }
    // GGSWs in the key: n (classic) or (n/g) 2^g (multi-bit, lwe_multi_bit_bootstrap_key.rs:40-55)
    size_t ggsw_count() const {
        return p.grouping_factor ? (n() / p.grouping_factor) << p.grouping_factor : n();
    }
    size_t std_bsk_len() const {
        return ggsw_count() * p.pbs_level * (k() + 1) * (k() + 1) * N();
    }
    size_t fourier_bsk_bytes() const {
        return ggsw_count() * p.pbs_level * (k() + 1) * (k() + 1) * (N() / 2) * sizeof(double2);
    }
    size_t ksk_len() const { return big_dim() * p.ks_level * (n() + 1); }
    size_t pksk_len(uint32_t level) const { return big_dim() * level * glwe_len(); }
};

namespace {

// cos and sin called separately through opaque pointers (no compiler fusion into sincos, whose
// last bits can differ): the same tables as the oracle's fft_init, bit for bit.
double (*volatile host_cos)(double) = static_cast<double (*)(double)>(std::cos);
double (*volatile host_sin)(double) = static_cast<double (*)(double)>(std::sin);

void build_tables(TfheMi355Context *c) {
    const int N = c->p.polynomial_size, M = N / 2;
    // W[t] = exp(-2 pi i t / M); twist w_j = exp(i pi j / N) as fft/mod.rs:58-69
    std::vector<double2> W(M), tw(M);
    for (int t = 0; t < M; t++) {
        double ang = 2.0 * M_PI * (double)t / (double)M;
        W[t] = make_double2(host_cos(ang), -host_sin(ang));
    }
    double unit = M_PI / (2.0 * (double)M);
    for (int j = 0; j < M; j++) {
        double a = (double)j * unit;
        tw[j] = make_double2(host_cos(a), host_sin(a));
    }
    size_t bytes = sizeof(double2) * M;
    check(hipMalloc(&c->tables.W, bytes), "hipMalloc(W)");
    check(hipMalloc(&c->tables.twist, bytes), "hipMalloc(twist)");
    check(hipMemcpy(c->tables.W, W.data(), bytes, hipMemcpyHostToDevice), "upload W");
    check(hipMemcpy(c->tables.twist, tw.data(), bytes, hipMemcpyHostToDevice), "upload twist");
    if (M >= 16 * 1024) {
        // the large-N top radix-16 stage reads W[a c] for a < M/16: laid out [c-1][a] so that a
        // wave's 64 consecutive butterflies read 1 KiB contiguously instead of 64 scattered lines
        const int A = M / 16;
        std::vector<double2> top((size_t)15 * A);
        for (int c = 1; c < 16; c++)
            for (int a = 0; a < A; a++) top[(size_t)(c - 1) * A + a] = W[(size_t)a * c];
        const size_t tb = sizeof(double2) * top.size();
        check(hipMalloc(&c->tables.wtop, tb), "hipMalloc(wtop)");
        check(hipMemcpy(c->tables.wtop, top.data(), tb, hipMemcpyHostToDevice), "upload wtop");
    }
    c->tables.N = N;
}

void require_fbsk(TfheMi355Context *c) {
    if (!c->fbsk_ready) fail("bootstrapping key not uploaded");
}
void require_ksk(TfheMi355Context *c) {
    if (!c->ksk_ready) fail("keyswitching key not uploaded");
}

hipError_t convert_bsk(TfheMi355Context *c, const uint64_t *d_std, size_t npoly, hipStream_t s) {
    if (large_pbs_supported((int)c->N(), (int)c->k(), (int)c->p.pbs_level))
        return launch_large_bsk_to_fourier(d_std, (double2 *)c->fbsk.ptr, npoly, c->tables, s);
    return launch_bsk_to_fourier((int)c->N(), d_std, (double2 *)c->fbsk.ptr, npoly, c->tables, s);
}

void launch_pbs_dev(TfheMi355Context *c, const uint64_t *d_in, uint64_t *d_out, const uint64_t *d_luts,
                    size_t lut_count, const uint32_t *d_idx, size_t count, hipStream_t s, bool glwe_out = false) {
    require_fbsk(c);
    if (lut_count == 0) fail("lut_count must be >= 1");
    if (count > 0x7fffffff) fail("batch too large");
    if (c->p.grouping_factor) {
        MultiBitPbsLaunch a;
        a.lwe_in = d_in;
        a.lwe_out = d_out;
        a.luts = d_luts;
        a.lut_indexes = d_idx;
        a.fbsk = reinterpret_cast<const double2 *>(c->fbsk.ptr);
        a.W = c->tables.W;
        a.twist = c->tables.twist;
        a.n = (int)c->n();
        a.base_log = (int)c->p.pbs_base_log;
        a.count = (int)count;
        a.glwe_out = glwe_out;
        check(launch_multibit_pbs((int)c->N(), (int)c->k(), (int)c->p.pbs_level, (int)c->p.grouping_factor, a, s),
              "launch multi-bit pbs");
        return;
    }
    if (large_pbs_supported((int)c->N(), (int)c->k(), (int)c->p.pbs_level)) {
        if (glwe_out) fail("blind rotation without sample extraction is not available at N = %zu", c->N());
        // ciphertexts per pass: the chunk's accumulators + spectra (1.5 MiB per ciphertext at 4_4)
        // should stay resident in the 256 MiB Infinity Cache across the three launches of a CMUX
        static const size_t kChunk = [] {
            const char *e = std::getenv("TFHE_MI355_LARGE_CHUNK");
            const long v = e ? std::atol(e) : 0;
            return v > 0 ? (size_t)v : (size_t)128;  // 128: best of 64..1024 at 4_4 (profiles)
        }();
        const size_t per_ct = large_pbs_scratch_per_ct((int)c->N(), (int)c->k(), (int)c->p.pbs_level);
        c->pbs_scratch.reserve(per_ct * std::max<size_t>(1, std::min(count, kChunk)));
        LargePbsLaunch a{};
        a.lwe_in = d_in;
        a.lwe_out = d_out;
        a.luts = d_luts;
        a.lut_indexes = d_idx;
        a.fbsk = reinterpret_cast<const double2 *>(c->fbsk.ptr);
        a.W = c->tables.W;
        a.twist = c->tables.twist;
        a.wtop = c->tables.wtop;
        a.n = (int)c->n();
        a.base_log = (int)c->p.pbs_base_log;
        a.count = (int)count;
        a.scratch = c->pbs_scratch.ptr;
        a.scratch_bytes = c->pbs_scratch.bytes;
        check(launch_large_pbs((int)c->N(), (int)c->k(), (int)c->p.pbs_level, a, s), "launch large pbs");
        return;
    }
    ClassicPbsLaunch a;
    a.lwe_in = d_in;
    a.lwe_out = d_out;
    a.luts = d_luts;
    a.lut_indexes = d_idx;
    a.fbsk = reinterpret_cast<const double2 *>(c->fbsk.ptr);
    a.W = c->tables.W;
    a.twist = c->tables.twist;
    a.n = (int)c->n();
    a.base_log = (int)c->p.pbs_base_log;
    a.count = (int)count;
    a.glwe_out = glwe_out;
    check(launch_classic_pbs((int)c->N(), (int)c->k(), (int)c->p.pbs_level, a, s), "launch pbs");
}

bool ks_use_mfma(TfheMi355Context *c) {
    static const bool disabled = std::getenv("TFHE_MI355_KS_NO_MFMA") != nullptr;
    return !disabled && ks_mfma_supported((int)c->big_dim(), (int)c->p.ks_level, (int)c->p.ks_base_log);
}

// KSK -> int8 byte planes (once per key, after the u64 KSK is on the device)
void repack_ksk(TfheMi355Context *c, hipStream_t s) {
    c->ksk_planes_ready = false;
    if (!ks_use_mfma(c)) return;
    const size_t bytes = 8 * ks_mfma_rows((int)c->big_dim(), (int)c->p.ks_level) * ks_mfma_cols((int)c->n());
    c->ksk_planes.reserve(bytes);
    check(launch_ksk_repack((const uint64_t *)c->ksk.ptr, (int8_t *)c->ksk_planes.ptr, (int)c->big_dim(),
                            (int)c->p.ks_level, (int)c->n(), s),
          "ksk repack");
    c->ksk_planes_ready = true;
}

void launch_ks_dev(TfheMi355Context *c, const uint64_t *d_in, uint64_t *d_out, size_t count, hipStream_t s) {
    require_ksk(c);
    if (c->ksk_planes_ready && count > 0) {
        KeyswitchLaunch a;
        a.lwe_in = d_in;
        a.lwe_out = d_out;
        a.ksk = reinterpret_cast<const uint64_t *>(c->ksk.ptr);
        a.in_dim = (int)c->big_dim();
        a.out_dim = (int)c->n();
        a.base_log = (int)c->p.ks_base_log;
        a.level = (int)c->p.ks_level;
        a.count = (int)count;
        c->ks_scratch.reserve(ks_mfma_scratch_bytes(a.in_dim, a.level, a.count));
        check(launch_keyswitch_mfma(a, (const int8_t *)c->ksk_planes.ptr, c->ks_scratch.ptr, s), "launch mfma keyswitch");
        return;
    }
    KeyswitchLaunch a;
    a.lwe_in = d_in;
    a.lwe_out = d_out;
    a.ksk = reinterpret_cast<const uint64_t *>(c->ksk.ptr);
    a.in_dim = (int)c->big_dim();
    a.out_dim = (int)c->n();
    a.base_log = (int)c->p.ks_base_log;
    a.level = (int)c->p.ks_level;
    a.count = (int)count;
    check(launch_keyswitch(a, s), "launch keyswitch");
}

// LWE -> GLWE packing keyswitch (lwe_packing_keyswitch.rs:102-186): the LWE keyswitch GEMM with
// (k+1)N-word GLWE rows and the input body landing on the GLWE body's constant term
KeyswitchLaunch packing_ks_args(TfheMi355Context *c, const uint64_t *d_in, uint64_t *d_out, size_t count) {
    KeyswitchLaunch a;
    a.lwe_in = d_in;
    a.lwe_out = d_out;
    a.ksk = reinterpret_cast<const uint64_t *>(c->pksk.ptr);
    a.in_dim = (int)c->big_dim();
    a.out_dim = (int)c->glwe_len() - 1;
    a.body_col = (int)c->big_dim();
    a.base_log = (int)c->pks_base_log;
    a.level = (int)c->pks_level;
    a.count = (int)count;
    return a;
}

void launch_packing_ks_dev(TfheMi355Context *c, const uint64_t *d_in, uint64_t *d_out, size_t count, hipStream_t s) {
    if (!c->pksk_ready) fail("packing keyswitching key not uploaded");
    if (count == 0) return;
    if (count > 0x7fffffffu) fail("count too large");
    KeyswitchLaunch a = packing_ks_args(c, d_in, d_out, count);
    if (c->pksk_planes_ready) {
        c->ks_scratch.reserve(ks_mfma_scratch_bytes(a.in_dim, a.level, a.count));
        check(launch_keyswitch_mfma(a, (const int8_t *)c->pksk_planes.ptr, c->ks_scratch.ptr, s),
              "launch mfma packing keyswitch");
    } else {
        check(launch_keyswitch(a, s), "launch packing keyswitch");
    }
}

void launch_glwe_poly_mul_dev(TfheMi355Context *c, const uint64_t *d_glwe, size_t glwe_per_item,
                              const uint64_t *d_polys, size_t npoly, size_t count, bool extract, uint64_t *d_out,
                              hipStream_t s) {
    if (glwe_per_item == 0 || glwe_per_item > 0xffff) fail("glwe_per_item out of range");
    if (npoly > 0x7fffffffu) fail("npoly too large");
    GlwePolyMulLaunch a;
    a.glwe_in = d_glwe;
    a.polys = d_polys;
    a.out = d_out;
    a.k = (int)c->k();
    a.N = (int)c->N();
    a.J = (int)glwe_per_item;
    a.npoly = (int)npoly;
    a.count = count;
    a.extract = extract;
    check(launch_glwe_poly_mul(a, s), "launch glwe poly mul");
}

void validate_lut_indexes(const uint32_t *idx, size_t count, size_t lut_count) {
    if (!idx) return;
    for (size_t i = 0; i < count; i++)
        if (idx[i] >= lut_count) fail("lut_indexes[%zu] = %u out of range (lut_count %zu)", i, idx[i], lut_count);
}

}  // namespace

extern "C" {

const char *tfhe_mi355_last_error(void) { return last_error_text().c_str(); }

int tfhe_mi355_device_count(int *out_count) {
    return guarded([&] {
        if (!out_count) fail("null out_count");
        *out_count = 0;
        int n = 0;
        check(hipGetDeviceCount(&n), "hipGetDeviceCount");
        *out_count = n;
    });
}

int tfhe_mi355_context_create(const TfheMi355Parameters *params, int device, TfheMi355Context **out_ctx) {
    return guarded([&] {
        if (!out_ctx) fail("null out_ctx");
        *out_ctx = nullptr;
        if (!params) fail("null params");
        const TfheMi355Parameters &p = *params;
        if (!is_pow2(p.polynomial_size)) fail("polynomial_size must be a power of two");
        if (p.grouping_factor != 0) {
            if (!multibit_pbs_supported((int)p.polynomial_size, (int)p.glwe_dimension, (int)p.pbs_level,
                                        (int)p.grouping_factor))
                fail("no multi-bit kernel for N=%u k=%u pbs_level=%u grouping_factor=%u", p.polynomial_size,
                     p.glwe_dimension, p.pbs_level, p.grouping_factor);
            if (p.lwe_dimension % p.grouping_factor)
                fail("lwe_dimension %u is not a multiple of grouping_factor %u", p.lwe_dimension, p.grouping_factor);
        } else if (!classic_pbs_supported((int)p.polynomial_size, (int)p.glwe_dimension, (int)p.pbs_level) &&
                   !large_pbs_supported((int)p.polynomial_size, (int)p.glwe_dimension, (int)p.pbs_level)) {
            fail("no kernel for N=%u k=%u pbs_level=%u", p.polynomial_size, p.glwe_dimension, p.pbs_level);
        }
        if (p.pbs_base_log < 2 || p.pbs_base_log * p.pbs_level > 30)
            fail("pbs decomposition base_log*level must be in [2, 30] (got %u x %u)", p.pbs_base_log, p.pbs_level);
        if (p.ks_level && (p.ks_base_log == 0 || p.ks_base_log * p.ks_level >= 64)) fail("invalid ks decomposition");
        if (p.lwe_dimension == 0) fail("lwe_dimension must be > 0");
        check(hipSetDevice(device), "hipSetDevice");
        auto *c = new TfheMi355Context();
        c->p = p;
        c->device = device;
        try {
            check(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking), "hipStreamCreate");
            build_tables(c);
        } catch (...) {
            tfhe_mi355_context_destroy(c);
            throw;
        }
        *out_ctx = c;
    });
}

int tfhe_mi355_context_destroy(TfheMi355Context *ctx) {
    return guarded([&] {
        if (!ctx) return;
        (void)hipSetDevice(ctx->device);
        if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
        for (DeviceBuffer *b : {&ctx->fbsk, &ctx->ksk, &ctx->std_staging, &ctx->io_in, &ctx->io_out,
                                &ctx->io_luts, &ctx->io_idx, &ctx->io_tmp, &ctx->pbs_scratch,
                                &ctx->ksk_planes, &ctx->ks_scratch, &ctx->pksk, &ctx->pksk_planes})
            b->release();
        if (ctx->tables.W) (void)hipFree(ctx->tables.W);
        if (ctx->tables.twist) (void)hipFree(ctx->tables.twist);
        if (ctx->tables.wtop) (void)hipFree(ctx->tables.wtop);
        if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
        delete ctx;
    });
}

int tfhe_mi355_bootstrap_key_upload(TfheMi355Context *ctx, const uint64_t *bsk, size_t len) {
    return guarded([&] {
        if (!ctx || !bsk) fail("null argument");
        std::lock_guard<std::mutex> g(ctx->mu);
        check(hipSetDevice(ctx->device), "hipSetDevice");
        if (len != ctx->std_bsk_len()) fail("bootstrapping key has %zu words, expected %zu", len, ctx->std_bsk_len());
        ctx->std_staging.reserve(len * sizeof(uint64_t));
        check(hipMemcpyAsync(ctx->std_staging.ptr, bsk, len * sizeof(uint64_t), hipMemcpyHostToDevice,
                             ctx->stream), "upload bsk");
        ctx->fbsk.reserve(ctx->fourier_bsk_bytes());
        check(convert_bsk(ctx, (const uint64_t *)ctx->std_staging.ptr, len / ctx->N(), ctx->stream),
              "bsk conversion");
        check(hipStreamSynchronize(ctx->stream), "bsk conversion sync");
        ctx->std_staging.release();
        ctx->fbsk_ready = true;
    });
}

namespace {
// AES tables of a compression seed on the device (a few KiB, one per call)
void upload_aes_tables(TfheMi355Context *c, uint64_t seed_lo, uint64_t seed_hi, DeviceBuffer &d) {
    std::vector<unsigned char> host(aes_tables_bytes());
    aes_tables_build(seed_lo, seed_hi, host.data());
    d.reserve(host.size());
    check(hipMemcpyAsync(d.ptr, host.data(), host.size(), hipMemcpyHostToDevice, c->stream), "upload aes tables");
    check(hipStreamSynchronize(c->stream), "aes tables sync");
}
}  // namespace

int tfhe_mi355_bootstrap_key_upload_seeded(TfheMi355Context *ctx, const uint64_t *bodies, size_t len,
                                           uint64_t seed_lo, uint64_t seed_hi) {
    return guarded([&] {
        if (!ctx || !bodies) fail("null argument");
        std::lock_guard<std::mutex> g(ctx->mu);
        check(hipSetDevice(ctx->device), "hipSetDevice");
        const size_t rows = ctx->ggsw_count() * ctx->p.pbs_level * (ctx->k() + 1);
        if (len != rows * ctx->N()) fail("seeded bootstrapping key has %zu body words, expected %zu", len, rows * ctx->N());
        DeviceBuffer tab;
        upload_aes_tables(ctx, seed_lo, seed_hi, tab);
        DeviceBuffer d_bodies;
        d_bodies.reserve(len * sizeof(uint64_t));
        check(hipMemcpyAsync(d_bodies.ptr, bodies, len * sizeof(uint64_t), hipMemcpyHostToDevice, ctx->stream),
              "upload bodies");
        ctx->std_staging.reserve(ctx->std_bsk_len() * sizeof(uint64_t));
        check(launch_seeded_decompress(tab.ptr, (const uint64_t *)d_bodies.ptr, rows, ctx->k() * ctx->N(), ctx->N(),
                                       (uint64_t *)ctx->std_staging.ptr, ctx->stream),
              "seeded bsk decompression");
        ctx->fbsk.reserve(ctx->fourier_bsk_bytes());
        check(convert_bsk(ctx, (const uint64_t *)ctx->std_staging.ptr, ctx->std_bsk_len() / ctx->N(), ctx->stream),
              "bsk conversion");
        check(hipStreamSynchronize(ctx->stream), "seeded bsk sync");
        ctx->std_staging.release();
        d_bodies.release();
        tab.release();
        ctx->fbsk_ready = true;
    });
}

int tfhe_mi355_keyswitch_key_upload_seeded(TfheMi355Context *ctx, const uint64_t *bodies, size_t len,
                                           uint64_t seed_lo, uint64_t seed_hi) {
    return guarded([&] {
        if (!ctx || !bodies) fail("null argument");
        std::lock_guard<std::mutex> g(ctx->mu);
        check(hipSetDevice(ctx->device), "hipSetDevice");
        const size_t rows = ctx->big_dim() * ctx->p.ks_level;
        if (len != rows) fail("seeded keyswitching key has %zu body words, expected %zu", len, rows);
        DeviceBuffer tab;
        upload_aes_tables(ctx, seed_lo, seed_hi, tab);
        DeviceBuffer d_bodies;
        d_bodies.reserve(len * sizeof(uint64_t));
        check(hipMemcpyAsync(d_bodies.ptr, bodies, len * sizeof(uint64_t), hipMemcpyHostToDevice, ctx->stream),
              "upload bodies");
        ctx->ksk_ready = false;
        ctx->ksk.reserve(ctx->ksk_len() * sizeof(uint64_t));
        check(launch_seeded_decompress(tab.ptr, (const uint64_t *)d_bodies.ptr, rows, ctx->n(), 1,
                                       (uint64_t *)ctx->ksk.ptr, ctx->stream),
              "seeded ksk decompression");
        repack_ksk(ctx, ctx->stream);
        check(hipStreamSynchronize(ctx->stream), "seeded ksk sync");
        d_bodies.release();
        tab.release();
        ctx->ksk_ready = true;
    });
}

int tfhe_mi355_csprng_mask_words(TfheMi355Context *ctx, uint64_t seed_lo, uint64_t seed_hi, uint64_t *out,
                                 size_t words) {
    return guarded([&] {
        if (!ctx || (!out && words)) fail("null argument");
        std::lock_guard<std::mutex> g(ctx->mu);
        check(hipSetDevice(ctx->device), "hipSetDevice");
        if (words == 0) return;
        DeviceBuffer tab;
        upload_aes_tables(ctx, seed_lo, seed_hi, tab);
        ctx->io_out.reserve(words * sizeof(uint64_t));
        check(launch_seeded_decompress(tab.ptr, nullptr, 1, words, 0, (uint64_t *)ctx->io_out.ptr, ctx->stream),
              "csprng");
        check(hipMemcpyAsync(out, ctx->io_out.ptr, words * sizeof(uint64_t), hipMemcpyDeviceToHost, ctx->stream),
              "D2H words");
        check(hipStreamSynchronize(ctx->stream), "csprng sync");
        tab.release();
    });
}

int tfhe_mi355_bootstrap_key_convert_async(TfheMi355Context *ctx, const uint64_t *d_bsk, size_t len,
                                           void *stream) {
    return guarded([&] {
        if (!ctx || !d_bsk) fail("null argument");
        std::lock_guard<std::mutex> g(ctx->mu);
        check(hipSetDevice(ctx->device), "hipSetDevice");
        if (len != ctx->std_bsk_len()) fail("bootstrapping key has %zu words, expected %zu", len, ctx->std_bsk_len());
        ctx->fbsk.reserve(ctx->fourier_bsk_bytes());
        check(convert_bsk(ctx, d_bsk, len / ctx->N(), (hipStream_t)stream), "bsk conversion");
        ctx->fbsk_ready = true;
    });
}

int tfhe_mi355_bootstrap_key_fourier(TfheMi355Context *ctx, void **d_ptr, size_t *bytes) {
    return guarded([&] {
        if (!ctx || !d_ptr || !bytes) fail("null argument");
        *d_ptr = nullptr;
        *bytes = 0;
        std::lock_guard<std::mutex> g(ctx->mu);
        check(hipSetDevice(ctx->device), "hipSetDevice");
        ctx->fbsk.reserve(ctx->fourier_bsk_bytes());
        *d_ptr = ctx->fbsk.ptr;
        *bytes = ctx->fourier_bsk_bytes();
    });
}

int tfhe_mi355_bootstrap_key_fourier_set_ready(TfheMi355Context *ctx) {
    return guarded([&] {
        if (!ctx) fail("null ctx");
        if (!ctx->fbsk.ptr) fail("no Fourier key buffer");
        ctx->fbsk_ready = true;
    });
}

int tfhe_mi355_keyswitch_key_upload(TfheMi355Context *ctx, const uint64_t *ksk, size_t len) {
    return guarded([&] {
        if (!ctx || !ksk) fail("null argument");
        std::lock_guard<std::mutex> g(ctx->mu);
        check(hipSetDevice(ctx->device), "hipSetDevice");
        if (len != ctx->ksk_len()) fail("keyswitching key has %zu words, expected %zu", len, ctx->ksk_len());
        ctx->ksk.reserve(len * sizeof(uint64_t));
        check(hipMemcpy(ctx->ksk.ptr, ksk, len * sizeof(uint64_t), hipMemcpyHostToDevice), "upload ksk");
        repack_ksk(ctx, ctx->stream);
        check(hipStreamSynchronize(ctx->stream), "ksk repack sync");
        ctx->ksk_ready = true;
    });
}

int tfhe_mi355_keyswitch_key_upload_async(TfheMi355Context *ctx, const uint64_t *d_ksk, size_t len,
                                          void *stream) {
    return guarded([&] {
        if (!ctx || !d_ksk) fail("null argument");
        std::lock_guard<std::mutex> g(ctx->mu);
        check(hipSetDevice(ctx->device), "hipSetDevice");
        if (len != ctx->ksk_len()) fail("keyswitching key has %zu words, expected %zu", len, ctx->ksk_len());
        ctx->ksk.reserve(len * sizeof(uint64_t));
        check(hipMemcpyAsync(ctx->ksk.ptr, d_ksk, len * sizeof(uint64_t), hipMemcpyDeviceToDevice,
                             (hipStream_t)stream), "copy ksk");
        repack_ksk(ctx, (hipStream_t)stream);
        ctx->ksk_ready = true;
    });
}

int tfhe_mi355_keyswitch_key_device(TfheMi355Context *ctx, void **d_ptr, size_t *bytes) {
    return guarded([&] {
        if (!ctx || !d_ptr || !bytes) fail("null argument");
        *d_ptr = nullptr;
        *bytes = 0;
        std::lock_guard<std::mutex> g(ctx->mu);
        check(hipSetDevice(ctx->device), "hipSetDevice");
        ctx->ksk.reserve(ctx->ksk_len() * sizeof(uint64_t));
        *d_ptr = ctx->ksk.ptr;
        *bytes = ctx->ksk_len() * sizeof(uint64_t);
    });
}

int tfhe_mi355_keyswitch_key_set_ready(TfheMi355Context *ctx) {
    return guarded([&] {
        if (!ctx) fail("null ctx");
        if (!ctx->ksk.ptr) fail("no keyswitching key buffer");
        check(hipSetDevice(ctx->device), "hipSetDevice");
        repack_ksk(ctx, ctx->stream);
        check(hipStreamSynchronize(ctx->stream), "ksk repack sync");
        ctx->ksk_ready = true;
    });
}

int tfhe_mi355_programmable_bootstrap(TfheMi355Context *ctx, const uint64_t *lwe_in, uint64_t *lwe_out,
                                      const uint64_t *luts, size_t lut_count, const uint32_t *lut_indexes,
                                      size_t count) {
    return guarded([&] {
        if (!ctx || (!lwe_in && count) || (!lwe_out && count) || !luts) fail("null argument");
        std::lock_guard<std::mutex> g(ctx->mu);
        check(hipSetDevice(ctx->device), "hipSetDevice");
        require_fbsk(ctx);
        if (count == 0) return;
        validate_lut_indexes(lut_indexes, count, lut_count);
        const size_t in_b = count * (ctx->n() + 1) * 8, out_b = count * (ctx->big_dim() + 1) * 8;
        const size_t lut_b = lut_count * ctx->glwe_len() * 8;
        ctx->io_in.reserve(in_b);
        ctx->io_out.reserve(out_b);
        ctx->io_luts.reserve(lut_b);
        if (lut_indexes) ctx->io_idx.reserve(count * 4);
        hipStream_t s = ctx->stream;
        check(hipMemcpyAsync(ctx->io_in.ptr, lwe_in, in_b, hipMemcpyHostToDevice, s), "H2D in");
        check(hipMemcpyAsync(ctx->io_luts.ptr, luts, lut_b, hipMemcpyHostToDevice, s), "H2D luts");
        if (lut_indexes)
            check(hipMemcpyAsync(ctx->io_idx.ptr, lut_indexes, count * 4, hipMemcpyHostToDevice, s), "H2D idx");
        launch_pbs_dev(ctx, (const uint64_t *)ctx->io_in.ptr, (uint64_t *)ctx->io_out.ptr,
                       (const uint64_t *)ctx->io_luts.ptr, lut_count,
                       lut_indexes ? (const uint32_t *)ctx->io_idx.ptr : nullptr, count, s);
        check(hipMemcpyAsync(lwe_out, ctx->io_out.ptr, out_b, hipMemcpyDeviceToHost, s), "D2H out");
        check(hipStreamSynchronize(s), "pbs sync");
    });
}

int tfhe_mi355_programmable_bootstrap_async(TfheMi355Context *ctx, const uint64_t *d_in, uint64_t *d_out,
                                            const uint64_t *d_luts, size_t lut_count,
                                            const uint32_t *d_idx, size_t count, void *stream) {
    return guarded([&] {
        if (!ctx || (!d_in && count) || (!d_out && count) || !d_luts) fail("null argument");
        check(hipSetDevice(ctx->device), "hipSetDevice");
        launch_pbs_dev(ctx, d_in, d_out, d_luts, lut_count, d_idx, count, (hipStream_t)stream);
    });
}

int tfhe_mi355_blind_rotate(TfheMi355Context *ctx, const uint64_t *lwe_in, uint64_t *glwe_out, const uint64_t *luts,
                            size_t lut_count, const uint32_t *lut_indexes, size_t count) {
    return guarded([&] {
        if (!ctx || (!lwe_in && count) || (!glwe_out && count) || !luts) fail("null argument");
        std::lock_guard<std::mutex> g(ctx->mu);
        check(hipSetDevice(ctx->device), "hipSetDevice");
        require_fbsk(ctx);
        if (count == 0) return;
        validate_lut_indexes(lut_indexes, count, lut_count);
        const size_t in_b = count * (ctx->n() + 1) * 8, out_b = count * ctx->glwe_len() * 8;
        const size_t lut_b = lut_count * ctx->glwe_len() * 8;
        ctx->io_in.reserve(in_b);
        ctx->io_out.reserve(out_b);
        ctx->io_luts.reserve(lut_b);
        if (lut_indexes) ctx->io_idx.reserve(count * 4);
        hipStream_t s = ctx->stream;
        check(hipMemcpyAsync(ctx->io_in.ptr, lwe_in, in_b, hipMemcpyHostToDevice, s), "H2D in");
        check(hipMemcpyAsync(ctx->io_luts.ptr, luts, lut_b, hipMemcpyHostToDevice, s), "H2D luts");
        if (lut_indexes)
            check(hipMemcpyAsync(ctx->io_idx.ptr, lut_indexes, count * 4, hipMemcpyHostToDevice, s), "H2D idx");
        launch_pbs_dev(ctx, (const uint64_t *)ctx->io_in.ptr, (uint64_t *)ctx->io_out.ptr,
                       (const uint64_t *)ctx->io_luts.ptr, lut_count,
                       lut_indexes ? (const uint32_t *)ctx->io_idx.ptr : nullptr, count, s, true);
        check(hipMemcpyAsync(glwe_out, ctx->io_out.ptr, out_b, hipMemcpyDeviceToHost, s), "D2H out");
        check(hipStreamSynchronize(s), "blind rotate sync");
    });
}

int tfhe_mi355_blind_rotate_async(TfheMi355Context *ctx, const uint64_t *d_in, uint64_t *d_glwe_out,
                                  const uint64_t *d_luts, size_t lut_count, const uint32_t *d_lut_indexes,
                                  size_t count, void *stream) {
    return guarded([&] {
        if (!ctx || (!d_in && count) || (!d_glwe_out && count) || !d_luts) fail("null argument");
        check(hipSetDevice(ctx->device), "hipSetDevice");
        launch_pbs_dev(ctx, d_in, d_glwe_out, d_luts, lut_count, d_lut_indexes, count, (hipStream_t)stream, true);
    });
}

int tfhe_mi355_packing_keyswitch_key_upload(TfheMi355Context *ctx, const uint64_t *pksk, size_t len,
                                            uint32_t base_log, uint32_t level) {
    return guarded([&] {
        if (!ctx || !pksk) fail("null argument");
        if (level == 0 || base_log == 0 || base_log * level >= 64) fail("invalid packing ks decomposition");
        std::lock_guard<std::mutex> g(ctx->mu);
        check(hipSetDevice(ctx->device), "hipSetDevice");
        if (len != ctx->pksk_len(level))
            fail("packing keyswitching key has %zu words, expected %zu", len, ctx->pksk_len(level));
        ctx->pksk_ready = ctx->pksk_planes_ready = false;
        ctx->pksk.reserve(len * sizeof(uint64_t));
        check(hipMemcpy(ctx->pksk.ptr, pksk, len * sizeof(uint64_t), hipMemcpyHostToDevice), "upload pksk");
        ctx->pks_base_log = base_log;
        ctx->pks_level = level;
        const int in_dim = (int)ctx->big_dim(), out_dim = (int)ctx->glwe_len() - 1;
        const char *no_mfma = std::getenv("TFHE_MI355_KS_NO_MFMA");
        if (!(no_mfma && *no_mfma && *no_mfma != '0') && ks_mfma_supported(in_dim, (int)level, (int)base_log)) {
            ctx->pksk_planes.reserve(8 * ks_mfma_rows(in_dim, (int)level) * ks_mfma_cols(out_dim));
            check(launch_ksk_repack((const uint64_t *)ctx->pksk.ptr, (int8_t *)ctx->pksk_planes.ptr, in_dim,
                                    (int)level, out_dim, ctx->stream),
                  "pksk repack");
            ctx->pksk_planes_ready = true;
        }
        check(hipStreamSynchronize(ctx->stream), "pksk repack sync");
        ctx->pksk_ready = true;
    });
}

int tfhe_mi355_packing_keyswitch(TfheMi355Context *ctx, const uint64_t *lwe_in, uint64_t *glwe_out, size_t count) {
    return guarded([&] {
        if (!ctx || (!lwe_in && count) || (!glwe_out && count)) fail("null argument");
        std::lock_guard<std::mutex> g(ctx->mu);
        check(hipSetDevice(ctx->device), "hipSetDevice");
        if (!ctx->pksk_ready) fail("packing keyswitching key not uploaded");
        if (count == 0) return;
        const size_t in_b = count * (ctx->big_dim() + 1) * 8, out_b = count * ctx->glwe_len() * 8;
        ctx->io_in.reserve(in_b);
        ctx->io_out.reserve(out_b);
        hipStream_t s = ctx->stream;
        check(hipMemcpyAsync(ctx->io_in.ptr, lwe_in, in_b, hipMemcpyHostToDevice, s), "H2D in");
        launch_packing_ks_dev(ctx, (const uint64_t *)ctx->io_in.ptr, (uint64_t *)ctx->io_out.ptr, count, s);
        check(hipMemcpyAsync(glwe_out, ctx->io_out.ptr, out_b, hipMemcpyDeviceToHost, s), "D2H out");
        check(hipStreamSynchronize(s), "packing ks sync");
    });
}

int tfhe_mi355_packing_keyswitch_async(TfheMi355Context *ctx, const uint64_t *d_lwe_in, uint64_t *d_glwe_out,
                                       size_t count, void *stream) {
    return guarded([&] {
        if (!ctx || (!d_lwe_in && count) || (!d_glwe_out && count)) fail("null argument");
        check(hipSetDevice(ctx->device), "hipSetDevice");
        launch_packing_ks_dev(ctx, d_lwe_in, d_glwe_out, count, (hipStream_t)stream);
    });
}

int tfhe_mi355_glwe_poly_mul(TfheMi355Context *ctx, const uint64_t *glwe_in, size_t glwe_per_item,
                             const uint64_t *polys, size_t npoly, size_t count, int extract, uint64_t *out) {
    return guarded([&] {
        if (!ctx || (!glwe_in && count) || (!polys && npoly) || (!out && count && npoly)) fail("null argument");
        std::lock_guard<std::mutex> g(ctx->mu);
        check(hipSetDevice(ctx->device), "hipSetDevice");
        if (count == 0 || npoly == 0) return;
        const size_t out_words = extract ? ctx->big_dim() + 1 : ctx->glwe_len();
        const size_t in_b = count * glwe_per_item * ctx->glwe_len() * 8;
        const size_t poly_b = npoly * glwe_per_item * ctx->N() * 8, out_b = count * npoly * out_words * 8;
        ctx->io_in.reserve(in_b);
        ctx->io_luts.reserve(poly_b);
        ctx->io_out.reserve(out_b);
        hipStream_t s = ctx->stream;
        check(hipMemcpyAsync(ctx->io_in.ptr, glwe_in, in_b, hipMemcpyHostToDevice, s), "H2D glwe");
        check(hipMemcpyAsync(ctx->io_luts.ptr, polys, poly_b, hipMemcpyHostToDevice, s), "H2D polys");
        launch_glwe_poly_mul_dev(ctx, (const uint64_t *)ctx->io_in.ptr, glwe_per_item,
                                 (const uint64_t *)ctx->io_luts.ptr, npoly, count, extract != 0,
                                 (uint64_t *)ctx->io_out.ptr, s);
        check(hipMemcpyAsync(out, ctx->io_out.ptr, out_b, hipMemcpyDeviceToHost, s), "D2H out");
        check(hipStreamSynchronize(s), "glwe poly mul sync");
    });
}

int tfhe_mi355_glwe_poly_mul_async(TfheMi355Context *ctx, const uint64_t *d_glwe_in, size_t glwe_per_item,
                                   const uint64_t *d_polys, size_t npoly, size_t count, int extract,
                                   uint64_t *d_out, void *stream) {
    return guarded([&] {
        if (!ctx || (!d_glwe_in && count) || (!d_polys && npoly) || (!d_out && count && npoly))
            fail("null argument");
        check(hipSetDevice(ctx->device), "hipSetDevice");
        if (count == 0 || npoly == 0) return;
        launch_glwe_poly_mul_dev(ctx, d_glwe_in, glwe_per_item, d_polys, npoly, count, extract != 0, d_out,
                                 (hipStream_t)stream);
    });
}

int tfhe_mi355_keyswitch(TfheMi355Context *ctx, const uint64_t *lwe_in, uint64_t *lwe_out, size_t count) {
    return guarded([&] {
        if (!ctx || (!lwe_in && count) || (!lwe_out && count)) fail("null argument");
        std::lock_guard<std::mutex> g(ctx->mu);
        check(hipSetDevice(ctx->device), "hipSetDevice");
        require_ksk(ctx);
        if (count == 0) return;
        const size_t in_b = count * (ctx->big_dim() + 1) * 8, out_b = count * (ctx->n() + 1) * 8;
        ctx->io_in.reserve(in_b);
        ctx->io_out.reserve(out_b);
        hipStream_t s = ctx->stream;
        check(hipMemcpyAsync(ctx->io_in.ptr, lwe_in, in_b, hipMemcpyHostToDevice, s), "H2D in");
        launch_ks_dev(ctx, (const uint64_t *)ctx->io_in.ptr, (uint64_t *)ctx->io_out.ptr, count, s);
        check(hipMemcpyAsync(lwe_out, ctx->io_out.ptr, out_b, hipMemcpyDeviceToHost, s), "D2H out");
        check(hipStreamSynchronize(s), "ks sync");
    });
}

int tfhe_mi355_keyswitch_async(TfheMi355Context *ctx, const uint64_t *d_in, uint64_t *d_out, size_t count,
                               void *stream) {
    return guarded([&] {
        if (!ctx || (!d_in && count) || (!d_out && count)) fail("null argument");
        check(hipSetDevice(ctx->device), "hipSetDevice");
        launch_ks_dev(ctx, d_in, d_out, count, (hipStream_t)stream);
    });
}

int tfhe_mi355_keyswitch_programmable_bootstrap_scratch(TfheMi355Context *ctx, size_t count, size_t *bytes) {
    return guarded([&] {
        if (!ctx || !bytes) fail("null argument");
        *bytes = count * (ctx->n() + 1) * 8;
    });
}

int tfhe_mi355_keyswitch_programmable_bootstrap_async(TfheMi355Context *ctx, const uint64_t *d_in,
                                                      uint64_t *d_out, const uint64_t *d_luts, size_t lut_count,
                                                      const uint32_t *d_idx, size_t count, void *d_scratch,
                                                      void *stream) {
    return guarded([&] {
        if (!ctx || (!d_in && count) || (!d_out && count) || !d_luts || (!d_scratch && count))
            fail("null argument");
        check(hipSetDevice(ctx->device), "hipSetDevice");
        launch_ks_dev(ctx, d_in, (uint64_t *)d_scratch, count, (hipStream_t)stream);
        launch_pbs_dev(ctx, (const uint64_t *)d_scratch, d_out, d_luts, lut_count, d_idx, count,
                       (hipStream_t)stream);
    });
}

int tfhe_mi355_keyswitch_programmable_bootstrap(TfheMi355Context *ctx, const uint64_t *lwe_in,
                                                uint64_t *lwe_out, const uint64_t *luts, size_t lut_count,
                                                const uint32_t *lut_indexes, size_t count) {
    return guarded([&] {
        if (!ctx || (!lwe_in && count) || (!lwe_out && count) || !luts) fail("null argument");
        std::lock_guard<std::mutex> g(ctx->mu);
        check(hipSetDevice(ctx->device), "hipSetDevice");
        require_fbsk(ctx);
        require_ksk(ctx);
        if (count == 0) return;
        validate_lut_indexes(lut_indexes, count, lut_count);
        const size_t big_b = count * (ctx->big_dim() + 1) * 8, small_b = count * (ctx->n() + 1) * 8;
        const size_t lut_b = lut_count * ctx->glwe_len() * 8;
        ctx->io_in.reserve(big_b);
        ctx->io_out.reserve(big_b);
        ctx->io_tmp.reserve(small_b);
        ctx->io_luts.reserve(lut_b);
        if (lut_indexes) ctx->io_idx.reserve(count * 4);
        hipStream_t s = ctx->stream;
        check(hipMemcpyAsync(ctx->io_in.ptr, lwe_in, big_b, hipMemcpyHostToDevice, s), "H2D in");
        check(hipMemcpyAsync(ctx->io_luts.ptr, luts, lut_b, hipMemcpyHostToDevice, s), "H2D luts");
        if (lut_indexes)
            check(hipMemcpyAsync(ctx->io_idx.ptr, lut_indexes, count * 4, hipMemcpyHostToDevice, s), "H2D idx");
        launch_ks_dev(ctx, (const uint64_t *)ctx->io_in.ptr, (uint64_t *)ctx->io_tmp.ptr, count, s);
        launch_pbs_dev(ctx, (const uint64_t *)ctx->io_tmp.ptr, (uint64_t *)ctx->io_out.ptr,
                       (const uint64_t *)ctx->io_luts.ptr, lut_count,
                       lut_indexes ? (const uint32_t *)ctx->io_idx.ptr : nullptr, count, s);
        check(hipMemcpyAsync(lwe_out, ctx->io_out.ptr, big_b, hipMemcpyDeviceToHost, s), "D2H out");
        check(hipStreamSynchronize(s), "ks-pbs sync");
    });
}

int tfhe_mi355_programmable_bootstrap_keyswitch(TfheMi355Context *ctx, const uint64_t *lwe_in,
                                                uint64_t *lwe_out, const uint64_t *luts, size_t lut_count,
                                                const uint32_t *lut_indexes, size_t count) {
    return guarded([&] {
        if (!ctx || (!lwe_in && count) || (!lwe_out && count) || !luts) fail("null argument");
        std::lock_guard<std::mutex> g(ctx->mu);
        check(hipSetDevice(ctx->device), "hipSetDevice");
        require_fbsk(ctx);
        require_ksk(ctx);
        if (count == 0) return;
        validate_lut_indexes(lut_indexes, count, lut_count);
        const size_t big_b = count * (ctx->big_dim() + 1) * 8, small_b = count * (ctx->n() + 1) * 8;
        const size_t lut_b = lut_count * ctx->glwe_len() * 8;
        ctx->io_in.reserve(small_b);
        ctx->io_out.reserve(small_b);
        ctx->io_tmp.reserve(big_b);
        ctx->io_luts.reserve(lut_b);
        if (lut_indexes) ctx->io_idx.reserve(count * 4);
        hipStream_t s = ctx->stream;
        check(hipMemcpyAsync(ctx->io_in.ptr, lwe_in, small_b, hipMemcpyHostToDevice, s), "H2D in");
        check(hipMemcpyAsync(ctx->io_luts.ptr, luts, lut_b, hipMemcpyHostToDevice, s), "H2D luts");
        if (lut_indexes)
            check(hipMemcpyAsync(ctx->io_idx.ptr, lut_indexes, count * 4, hipMemcpyHostToDevice, s), "H2D idx");
        launch_pbs_dev(ctx, (const uint64_t *)ctx->io_in.ptr, (uint64_t *)ctx->io_tmp.ptr,
                       (const uint64_t *)ctx->io_luts.ptr, lut_count,
                       lut_indexes ? (const uint32_t *)ctx->io_idx.ptr : nullptr, count, s);
        launch_ks_dev(ctx, (const uint64_t *)ctx->io_tmp.ptr, (uint64_t *)ctx->io_out.ptr, count, s);
        check(hipMemcpyAsync(lwe_out, ctx->io_out.ptr, small_b, hipMemcpyDeviceToHost, s), "D2H out");
        check(hipStreamSynchronize(s), "pbs-ks sync");
    });
}

int tfhe_mi355_lwe_scalar_mul_add_async(TfheMi355Context *ctx, uint64_t *d_y, const uint64_t *d_x, uint64_t scalar,
                                        size_t rows, size_t words, size_t y_stride, size_t x_stride, void *stream) {
    return guarded([&] {
        if (!ctx || (!d_y && rows * words)) fail("null argument");
        if (words > y_stride || (d_x && words > x_stride)) fail("row stride smaller than the row");
        check(hipSetDevice(ctx->device), "hipSetDevice");
        check(launch_lwe_scalar_mul_add(d_y, d_x, scalar, rows, words, y_stride, x_stride, (hipStream_t)stream),
              "lwe scalar_mul_add");
    });
}

int tfhe_mi355_trivial_pbs_async(TfheMi355Context *ctx, uint64_t *d_body, size_t rows, size_t stride,
                                 const uint64_t *d_lut, void *stream) {
    return guarded([&] {
        if (!ctx || ((!d_body || !d_lut) && rows)) fail("null argument");
        const uint64_t msup = (uint64_t)ctx->p.message_modulus * ctx->p.carry_modulus;
        if (msup == 0 || ctx->N() % msup) fail("message space does not divide the polynomial size");
        check(hipSetDevice(ctx->device), "hipSetDevice");
        check(launch_trivial_pbs(d_body, rows, stride, d_lut + ctx->k() * ctx->N(), (1ULL << 63) / msup, msup,
                                 ctx->N() / msup, (hipStream_t)stream),
              "trivial pbs");
    });
}

int tfhe_mi355_debug_torus_from_fraction(int device, const double *fr, uint64_t *acc_inout, uint64_t *set_out,
                                         size_t n) {
    return guarded([&] {
        if ((!fr || !acc_inout || !set_out) && n) fail("null argument");
        if (n == 0) return;
        check(hipSetDevice(device), "hipSetDevice");
        DeviceBuffer d_fr, d_acc, d_set;
        struct Release {
            DeviceBuffer *b[3];
            ~Release() {
                for (DeviceBuffer *x : b) x->release();
            }
        } release{{&d_fr, &d_acc, &d_set}};
        d_fr.reserve(n * sizeof(double));
        d_acc.reserve(n * sizeof(uint64_t));
        d_set.reserve(n * sizeof(uint64_t));
        check(hipMemcpy(d_fr.ptr, fr, n * sizeof(double), hipMemcpyHostToDevice), "H2D fr");
        check(hipMemcpy(d_acc.ptr, acc_inout, n * sizeof(uint64_t), hipMemcpyHostToDevice), "H2D acc");
        check(launch_torus_from_fraction((const double *)d_fr.ptr, (uint64_t *)d_acc.ptr, (uint64_t *)d_set.ptr, n,
                                         nullptr),
              "torus conversion");
        check(hipMemcpy(acc_inout, d_acc.ptr, n * sizeof(uint64_t), hipMemcpyDeviceToHost), "D2H acc");
        check(hipMemcpy(set_out, d_set.ptr, n * sizeof(uint64_t), hipMemcpyDeviceToHost), "D2H set");
    });
}

int tfhe_mi355_fill_accumulator(const TfheMi355Parameters *params, const uint64_t *f_values, uint64_t *acc) {
    return guarded([&] {
        if (!params || !f_values || !acc) fail("null argument");
        const size_t N = params->polynomial_size, k = params->glwe_dimension;
        const size_t p = (size_t)params->message_modulus * params->carry_modulus;
        if (p == 0 || N % p) fail("polynomial_size must be a multiple of message_modulus*carry_modulus");
        const size_t box = N / p, half = box / 2;
        const uint64_t delta = (1ULL << 63) / p;
        std::vector<uint64_t> body(N);
        for (size_t i = 0; i < p; i++)
            for (size_t j = 0; j < box; j++) body[i * box + j] = f_values[i] * delta;
        for (size_t j = 0; j < half; j++) body[j] = 0 - body[j];
        std::memset(acc, 0, sizeof(uint64_t) * k * N);
        for (size_t j = 0; j < N; j++) acc[k * N + j] = body[(j + half) % N];
    });
}

}  // extern "C"
