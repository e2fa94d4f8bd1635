// serde.cpp -- ingestion of the reference's serialized shortint server keys.
//
// A tfhe-rs 0.5 server key reaches a server as the bincode 1.3.3 encoding of its serde derive
// (tfhe/Cargo.toml:36,57; the docs' `bincode::serialize(&server_key)`).  bincode's default options:
// fixed-width little-endian integers, usize as u64, u128 as 16 bytes (low word first), Vec and
// serialize_seq as a u64 length then the elements, enum variants as a u32 index, bool as one byte,
// newtype structs (LweSize(usize), ...) as their field, structs as their fields in order.
//
//   CompressedServerKey (shortint/server_key/compressed.rs:43-55)
//     key_switching_key: SeededLweKeyswitchKey<Vec<u64>>  (entities/seeded_lwe_keyswitch_key.rs:11-21)
//         data Vec<u64> [in_dim][level] bodies, decomp_base_log, decomp_level_count, output_lwe_size,
//         compression_seed: CompressionSeed{Seed(u128)} (commons/math/random/generator.rs:36-39),
//         ciphertext_modulus (commons/ciphertext_modulus.rs:41-64: {modulus: u128, scalar_bits: usize})
//     bootstrapping_key: ShortintCompressedBootstrappingKey (compressed.rs:10-17)
//         0 Classic(SeededLweBootstrapKey{ggsw_list})               (seeded_lwe_bootstrap_key.rs:16-24)
//         1 MultiBit{seeded_bsk: SeededLweMultiBitBootstrapKey{ggsw_list, grouping_factor},
//                    deterministic_execution: bool}          (seeded_lwe_multi_bit_bootstrap_key.rs:16-25)
//         ggsw_list = SeededGgswCiphertextList (entities/seeded_ggsw_ciphertext_list.rs:12-23):
//           data Vec<u64> [ggsw][level][k+1][N] bodies, glwe_size, polynomial_size, decomp_base_log,
//           decomp_level_count, compression_seed, ciphertext_modulus
//     message_modulus, carry_modulus, max_degree: usize; ciphertext_modulus; pbs_order: PBSOrder (u32)
//
//   ServerKey (shortint/server_key/mod.rs:283-297)
//     key_switching_key: LweKeyswitchKey<Vec<u64>> (entities/lwe_keyswitch_key.rs:77-86):
//         data Vec<u64> [in_dim][level][out_size], decomp_base_log, decomp_level_count, output_lwe_size,
//         ciphertext_modulus
//     bootstrapping_key: SerializableShortintBootstrappingKey (server_key/mod.rs:112-119)
//         0 Classic(FourierLweBootstrapKey{fourier, input_lwe_dimension, glwe_size, base_log, level})
//                                                              (fft64/crypto/bootstrap.rs:25-33)
//         1 MultiBit{fourier_bsk: FourierLweMultiBitBootstrapKey{.., grouping_factor},
//                    deterministic_execution: bool}          (entities/lwe_multi_bit_bootstrap_key.rs:316-325)
//         fourier = FourierPolynomialList (fft64/math/fft/mod.rs:588-632): a seq of 2 + P elements:
//           polynomial_size, P, then P Fourier polynomials, each written by concrete-fft 0.3.0's
//           Plan::serialize_fourier_buffer (absent crate, restated): a seq of M = N/2 c64 = (re, im)
//           f64 pairs in natural DFT order X[f] = sum_j z_j e^(-2 pi i j f / M) of the twisted
//           folded input (the plan-ordered buffer is reordered so keys move between machines).
//     message_modulus, carry_modulus, max_degree, max_noise_level: usize; ciphertext_modulus; pbs_order
//
// Seeded keys enter the GPU through the seeded uploads (masks regenerated from the AES-CTR stream
// on the device); the standard KSK through the plain upload; the Fourier BSK is mapped on the host
// from natural frequency order into the engine layout with the inverse FFT's 1/M
// folded in (an exact power-of-two scale) and copied to the device.  The reference holds no
// serialized keys, so the byte layout is pinned by the reference's type definitions above and
// the bincode spec; the concrete-fft buffer order is "parity unpinned" (DESIGN.md 4).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <initializer_list>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/tfhe_mi355.h"
#include "engine.h"
#include "errors.h"

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

template <class F>
int guarded(F &&f) {
    try {
        f();
        tfhe_mi355::last_error_text().clear();
        return TFHE_MI355_OK;
    } catch (const std::exception &ex) {
        tfhe_mi355::last_error_text() = ex.what();
        return TFHE_MI355_ERROR;
    }
}

// a call of the C ABI from inside this file: propagate its failure text
void abi(int rc) {
    if (rc != TFHE_MI355_OK) throw Failure(tfhe_mi355_last_error());
}

// bincode 1.3 default-options reader over a byte buffer (bounds-checked)
struct Reader {
    const uint8_t *p;
    size_t n, off = 0;
    void need(size_t b, const char *what) const {
        if (n - off < b) fail("serialized key truncated: %s at byte %zu needs %zu bytes, %zu left", what, off, b, n - off);
    }
    uint8_t u8(const char *what) {
        need(1, what);
        return p[off++];
    }
    uint32_t u32(const char *what) {
        need(4, what);
        uint32_t v;
        std::memcpy(&v, p + off, 4);
        off += 4;
        return v;
    }
    uint64_t u64(const char *what) {
        need(8, what);
        uint64_t v;
        std::memcpy(&v, p + off, 8);
        off += 8;
        return v;
    }
    void u128(const char *what, uint64_t &lo, uint64_t &hi) {
        lo = u64(what);
        hi = u64(what);
    }
    bool boolean(const char *what) {
        const uint8_t b = u8(what);
        if (b > 1) fail("invalid bool %u in %s at byte %zu", b, what, off - 1);
        return b;
    }
    // Vec<u64>: length, then the words (left in place; possibly unaligned)
    size_t vec_u64(const char *what, size_t &count) {
        count = u64(what);
        if (count > (n - off) / 8) fail("serialized key truncated: %s declares %zu words, %zu bytes left", what, count, n - off);
        const size_t at = off;
        off += count * 8;
        return at;
    }
};

void ciphertext_modulus(Reader &r, const char *what) {
    uint64_t lo, hi;
    r.u128(what, lo, hi);
    const uint64_t bits = r.u64(what);
    if (bits != 64) fail("%s: ciphertext modulus of a %llu-bit scalar, the engine is u64", what, (unsigned long long)bits);
    if (lo || hi) fail("%s: non-native ciphertext modulus (the engine computes modulo 2^64)", what);
}

struct SeededGgswList {
    size_t data = 0, words = 0;
    uint64_t glwe_size = 0, N = 0, base_log = 0, level = 0, seed_lo = 0, seed_hi = 0;
};
SeededGgswList seeded_ggsw_list(Reader &r) {
    SeededGgswList g;
    g.data = r.vec_u64("seeded GGSW list data", g.words);
    g.glwe_size = r.u64("glwe_size");
    g.N = r.u64("polynomial_size");
    g.base_log = r.u64("decomp_base_log");
    g.level = r.u64("decomp_level_count");
    r.u128("compression_seed", g.seed_lo, g.seed_hi);
    ciphertext_modulus(r, "seeded GGSW list");
    return g;
}

// Upper bounds on the header fields, checked before they enter any product (a crafted key with
// e.g. glwe_size = N = 2^32 would otherwise wrap a word count to 0 and divide by it).  Generous
// against every reference parameter set (N <= 2^15, k + 1 <= 6, levels <= 7, n <= 2^11).
constexpr uint64_t kMaxPolySize = 1ull << 17;
constexpr uint64_t kMaxGlweSize = 64;
constexpr uint64_t kMaxLevels = 64;
constexpr uint64_t kMaxLweSize = 1ull << 20;

void check_range(uint64_t v, uint64_t lo, uint64_t hi, const char *what) {
    if (v < lo || v > hi)
        fail("%s = %llu out of range [%llu, %llu]", what, (unsigned long long)v, (unsigned long long)lo,
             (unsigned long long)hi);
}

struct FourierList {
    uint64_t N = 0, polys = 0;
    size_t first = 0;  // byte offset of the first polynomial's length word
};
FourierList fourier_list(Reader &r) {
    FourierList f;
    const uint64_t seq = r.u64("Fourier polynomial list length");
    f.N = r.u64("Fourier polynomial_size");
    f.polys = r.u64("Fourier polynomial count");
    if (seq != 2 + f.polys) fail("Fourier polynomial list: sequence of %llu elements for %llu polynomials",
                                 (unsigned long long)seq, (unsigned long long)f.polys);
    // bounded before any size arithmetic (M * 16 below must not wrap)
    if (f.N < 2 || f.N > kMaxPolySize || (f.N & (f.N - 1)))
        fail("Fourier polynomial list: polynomial size %llu", (unsigned long long)f.N);
    f.first = r.off;
    const uint64_t M = f.N / 2;
    for (uint64_t q = 0; q < f.polys; q++) {
        const uint64_t m = r.u64("Fourier polynomial length");
        if (m != M) fail("Fourier polynomial %llu has %llu coefficients, expected %llu", (unsigned long long)q,
                         (unsigned long long)m, (unsigned long long)M);
        r.need(M * 16, "Fourier polynomial");
        r.off += M * 16;
    }
    return f;
}

struct Key {
    bool compressed = false;
    // keyswitching key
    size_t ksk_data = 0, ksk_words = 0;
    uint64_t ks_base_log = 0, ks_level = 0, ks_out_size = 0, ksk_seed_lo = 0, ksk_seed_hi = 0;
    // bootstrapping key
    uint32_t variant = 0;  // 0 classic, 1 multi-bit
    uint64_t grouping = 0;
    bool deterministic = false;
    SeededGgswList sbsk;                                        // compressed
    FourierList fbsk;                                           // standard
    uint64_t n = 0, glwe_size = 0, pbs_base_log = 0, pbs_level = 0;  // standard (fields)
    uint64_t message_modulus = 0, carry_modulus = 0, max_degree = 0, max_noise_level = 0;
    uint32_t pbs_order = 0;
    TfheMi355Parameters params{};
};

uint32_t u32_field(uint64_t v, const char *what) {
    if (v > 0xffffffffull) fail("%s = %llu out of range", what, (unsigned long long)v);
    return (uint32_t)v;
}

void finish(Key &k, Reader &r) {
    k.message_modulus = r.u64("message_modulus");
    k.carry_modulus = r.u64("carry_modulus");
    k.max_degree = r.u64("max_degree");
    if (!k.compressed) k.max_noise_level = r.u64("max_noise_level");
    ciphertext_modulus(r, "server key");
    k.pbs_order = r.u32("pbs_order");
    if (k.pbs_order > 1) fail("pbs_order variant %u", k.pbs_order);
    if (r.off != r.n) fail("%zu trailing bytes after the server key", r.n - r.off);

    // parameters implied by the key material
    TfheMi355Parameters &p = k.params;
    const uint64_t glwe_size = k.compressed ? k.sbsk.glwe_size : k.glwe_size;
    const uint64_t N = k.compressed ? k.sbsk.N : k.fbsk.N;
    const uint64_t L = k.compressed ? k.sbsk.level : k.pbs_level;
    // every field that enters a product below is range-checked first (no wrap-around)
    check_range(glwe_size, 2, kMaxGlweSize, "bootstrapping key glwe_size");
    check_range(N, 2, kMaxPolySize, "bootstrapping key polynomial_size");
    if (N & (N - 1)) fail("bootstrapping key polynomial_size %llu is not a power of two", (unsigned long long)N);
    check_range(L, 1, kMaxLevels, "bootstrapping key decomp_level_count");
    check_range(k.ks_level, 1, kMaxLevels, "keyswitching key decomp_level_count");
    check_range(k.ks_out_size, 2, kMaxLweSize, "keyswitching key output_lwe_size");
    if (!k.compressed) check_range(k.n, 1, kMaxLweSize, "input_lwe_dimension");
    const uint64_t k1 = glwe_size;
    uint64_t ggsw = 0;
    if (k.compressed) {
        const uint64_t per = L * k1 * N;  // bodies per GGSW
        if (k.sbsk.words % per) fail("seeded bootstrapping key: %zu words is not a whole number of GGSWs", k.sbsk.words);
        ggsw = k.sbsk.words / per;
    } else {
        const uint64_t per = L * k1 * k1;  // Fourier polynomials per GGSW
        if (k.fbsk.N != N || k.fbsk.polys % per) fail("Fourier bootstrapping key: %llu polynomials", (unsigned long long)k.fbsk.polys);
        ggsw = k.fbsk.polys / per;
    }
    uint64_t n = ggsw;
    if (k.variant == 1) {
        const uint64_t g = k.grouping;
        if (g < 1 || g > 6 || ggsw % (1ull << g)) fail("multi-bit key: %llu GGSWs at grouping factor %llu",
                                                      (unsigned long long)ggsw, (unsigned long long)g);
        n = ggsw / (1ull << g) * g;
    }
    if (!k.compressed && k.n != n) fail("Fourier bootstrapping key: input_lwe_dimension %llu but %llu GGSWs",
                                        (unsigned long long)k.n, (unsigned long long)ggsw);
    const uint64_t big = (k1 - 1) * N;
    if (k.ks_out_size != n + 1)
        fail("keyswitching key output size %llu does not match the bootstrapping key's n = %llu",
             (unsigned long long)k.ks_out_size, (unsigned long long)n);
    const uint64_t per_in = k.compressed ? k.ks_level : k.ks_level * k.ks_out_size;
    if (k.ksk_words != big * per_in)
        fail("keyswitching key has %zu words, expected %llu for an input dimension k N = %llu", k.ksk_words,
             (unsigned long long)(big * per_in), (unsigned long long)big);
    p.lwe_dimension = u32_field(n, "lwe_dimension");
    p.glwe_dimension = u32_field(k1 - 1, "glwe_dimension");
    p.polynomial_size = u32_field(N, "polynomial_size");
    p.pbs_base_log = u32_field(k.compressed ? k.sbsk.base_log : k.pbs_base_log, "pbs_base_log");
    p.pbs_level = u32_field(L, "pbs_level");
    p.ks_base_log = u32_field(k.ks_base_log, "ks_base_log");
    p.ks_level = u32_field(k.ks_level, "ks_level");
    p.message_modulus = u32_field(k.message_modulus, "message_modulus");
    p.carry_modulus = u32_field(k.carry_modulus, "carry_modulus");
    p.grouping_factor = k.variant == 1 ? u32_field(k.grouping, "grouping_factor") : 0;
}

Key parse_compressed(const uint8_t *bytes, size_t len) {
    Reader r{bytes, len};
    Key k;
    k.compressed = true;
    k.ksk_data = r.vec_u64("seeded keyswitching key data", k.ksk_words);
    k.ks_base_log = r.u64("ks decomp_base_log");
    k.ks_level = r.u64("ks decomp_level_count");
    k.ks_out_size = r.u64("ks output_lwe_size");
    r.u128("ks compression_seed", k.ksk_seed_lo, k.ksk_seed_hi);
    ciphertext_modulus(r, "seeded keyswitching key");
    k.variant = r.u32("ShortintCompressedBootstrappingKey variant");
    if (k.variant > 1) fail("ShortintCompressedBootstrappingKey variant %u", k.variant);
    k.sbsk = seeded_ggsw_list(r);
    if (k.variant == 1) {
        k.grouping = r.u64("grouping_factor");
        k.deterministic = r.boolean("deterministic_execution");
    }
    finish(k, r);
    return k;
}

Key parse_standard(const uint8_t *bytes, size_t len) {
    Reader r{bytes, len};
    Key k;
    k.ksk_data = r.vec_u64("keyswitching key data", k.ksk_words);
    k.ks_base_log = r.u64("ks decomp_base_log");
    k.ks_level = r.u64("ks decomp_level_count");
    k.ks_out_size = r.u64("ks output_lwe_size");
    ciphertext_modulus(r, "keyswitching key");
    k.variant = r.u32("ShortintBootstrappingKey variant");
    if (k.variant > 1) fail("ShortintBootstrappingKey variant %u", k.variant);
    k.fbsk = fourier_list(r);
    k.n = r.u64("input_lwe_dimension");
    k.glwe_size = r.u64("glwe_size");
    k.pbs_base_log = r.u64("decomposition_base_log");
    k.pbs_level = r.u64("decomposition_level_count");
    if (k.variant == 1) {
        k.grouping = r.u64("grouping_factor");
        k.deterministic = r.boolean("deterministic_execution");
    }
    finish(k, r);
    return k;
}

void fill_info(const Key &k, TfheMi355ServerKeyInfo *info) {
    std::memset(info, 0, sizeof *info);
    info->params = k.params;
    info->pbs_order = k.pbs_order;
    info->deterministic_execution = k.deterministic;
    info->max_degree = k.max_degree;
    info->max_noise_level = k.max_noise_level;
    info->ksk_seed_lo = k.ksk_seed_lo;
    info->ksk_seed_hi = k.ksk_seed_hi;
    info->bsk_seed_lo = k.sbsk.seed_lo;
    info->bsk_seed_hi = k.sbsk.seed_hi;
}

std::vector<uint64_t> words(const uint8_t *bytes, size_t at, size_t count) {
    std::vector<uint64_t> v(count);
    if (count) std::memcpy(v.data(), bytes + at, count * 8);  // bincode data is unaligned
    return v;
}

void require_same(const TfheMi355Parameters &key, const TfheMi355Parameters &ctx) {
#define SAME(f) \
    if (key.f != ctx.f) fail("server key " #f " = %u but the context was created with %u", key.f, ctx.f);
    SAME(lwe_dimension) SAME(glwe_dimension) SAME(polynomial_size) SAME(pbs_base_log) SAME(pbs_level)
    SAME(ks_base_log) SAME(ks_level) SAME(grouping_factor)
#undef SAME
}

}  // namespace

// engine Fourier layout: element e of a polynomial -> natural frequency index
int tfhe_mi355_fourier_engine_frequency(uint32_t N, uint32_t *freq) {
    return guarded([&] {
        if (!freq) fail("null argument");
        auto f1024 = [](uint32_t e) {  // WaveFft<1024>: element s*64 + lane (fft_device.h freq_lane/slot)
            const uint32_t lane = e & 63, s = e >> 6;
            return (lane & 15) + 64 * (lane >> 4) + 16 * (s >> 2) + 256 * (s & 3);
        };
        // DIF output position P = sum_i c_i M / (R_0 ... R_i) holds frequency sum_i c_i R_0 ... R_{i-1}
        // (the plan's digit reversal, oracle pos_freq)
        auto digit_reverse = [](uint32_t M, std::initializer_list<uint32_t> plan, uint32_t P) {
            uint32_t f = 0, stride = M, weight = 1;
            for (uint32_t R : plan) {
                stride /= R;
                f += (P / stride % R) * weight;
                weight *= R;
            }
            return f;
        };
        if (N == 2048) {
            for (uint32_t e = 0; e < 1024; e++) freq[e] = f1024(e);
        } else if (N == 1024) {
            // WaveFft<512>, plan [8, 8, 8]: element s*64 + lane holds P = 64 (lane & 7) + 8 (lane >> 3) + s
            for (uint32_t e = 0; e < 512; e++) {
                const uint32_t lane = e & 63, s = e >> 6;
                freq[e] = digit_reverse(512, {8, 8, 8}, 64 * (lane & 7) + 8 * (lane >> 3) + s);
            }
        } else if (N == 512) {
            // WaveFft<256>, plan [16, 16]: element q*64 + lane holds P = 16 (lane & 15) + (lane >> 4) + 4 q
            for (uint32_t e = 0; e < 256; e++) {
                const uint32_t lane = e & 63, q = e >> 6;
                freq[e] = digit_reverse(256, {16, 16}, 16 * (lane & 15) + (lane >> 4) + 4 * q);
            }
        } else if (N == 256) {
            // WaveFft<128>, plan [16, 8]: element e holds P = e (natural = Fourier layout)
            for (uint32_t e = 0; e < 128; e++) freq[e] = digit_reverse(128, {16, 8}, e);
        } else if (N == 4096 || N == 8192 || N == 16384 || N == 32768) {
            // element ((q 16 + s) 64 + lane): sub-block q (top DIF radix-R output digit, R = N/2048)
            // of the [R | 16, 16, 4] plan, then the 1024-point layout inside it
            const uint32_t R = N / 2048;
            for (uint32_t e = 0; e < N / 2; e++) freq[e] = (e >> 10) + R * f1024(e & 1023);
        } else {
            fail("Fourier key ingestion supports N = 256 ... 32768 (got %u)", N);
        }
    });
}

int tfhe_mi355_compressed_server_key_inspect(const uint8_t *bytes, size_t len, TfheMi355ServerKeyInfo *info) {
    return guarded([&] {
        if (!bytes || !info) fail("null argument");
        fill_info(parse_compressed(bytes, len), info);
    });
}

int tfhe_mi355_server_key_inspect(const uint8_t *bytes, size_t len, TfheMi355ServerKeyInfo *info) {
    return guarded([&] {
        if (!bytes || !info) fail("null argument");
        fill_info(parse_standard(bytes, len), info);
    });
}

int tfhe_mi355_compressed_server_key_upload(TfheMi355Context *ctx, const uint8_t *bytes, size_t len) {
    return guarded([&] {
        if (!ctx || !bytes) fail("null argument");
        const Key k = parse_compressed(bytes, len);
        const auto txn = tfhe_mi355::begin_key_transaction(ctx);  // both keys change as one
        TfheMi355Parameters cp;
        abi(tfhe_mi355_context_parameters(ctx, &cp));
        require_same(k.params, cp);
        {
            const std::vector<uint64_t> b = words(bytes, k.ksk_data, k.ksk_words);
            abi(tfhe_mi355_keyswitch_key_upload_seeded(ctx, b.data(), b.size(), k.ksk_seed_lo, k.ksk_seed_hi));
        }
        const std::vector<uint64_t> b = words(bytes, k.sbsk.data, k.sbsk.words);
        abi(tfhe_mi355_bootstrap_key_upload_seeded(ctx, b.data(), b.size(), k.sbsk.seed_lo, k.sbsk.seed_hi));
    });
}

int tfhe_mi355_server_key_upload(TfheMi355Context *ctx, const uint8_t *bytes, size_t len) {
    return guarded([&] {
        if (!ctx || !bytes) fail("null argument");
        const Key k = parse_standard(bytes, len);
        // no coalesced batch between the keyswitching key, the Fourier buffer and its ready flag
        const auto txn = tfhe_mi355::begin_key_transaction(ctx);
        TfheMi355Parameters cp;
        abi(tfhe_mi355_context_parameters(ctx, &cp));
        require_same(k.params, cp);
        const uint32_t N = k.params.polynomial_size, M = N / 2;
        std::vector<uint32_t> freq(M);
        abi(tfhe_mi355_fourier_engine_frequency(N, freq.data()));
        {
            const std::vector<uint64_t> b = words(bytes, k.ksk_data, k.ksk_words);
            abi(tfhe_mi355_keyswitch_key_upload(ctx, b.data(), b.size()));
        }
        void *d = nullptr;
        size_t dbytes = 0;
        abi(tfhe_mi355_bootstrap_key_fourier(ctx, &d, &dbytes));
        if (dbytes != (size_t)k.fbsk.polys * M * 16) fail("Fourier key size mismatch (%zu device bytes)", dbytes);
        // natural order -> engine layout, times 1/M (the resident key carries the inverse FFT's
        // normalisation), in slices of polynomials through a host buffer
        const double scale = 1.0 / (double)M;
        const size_t slice = std::max<size_t>(1, ((size_t)64 << 20) / ((size_t)M * 16));
        std::vector<double> host(std::min<size_t>(slice, k.fbsk.polys) * M * 2);
        for (size_t q0 = 0; q0 < k.fbsk.polys; q0 += slice) {
            const size_t cnt = std::min<size_t>(slice, k.fbsk.polys - q0);
            for (size_t q = 0; q < cnt; q++) {
                const uint8_t *src = bytes + k.fbsk.first + (q0 + q) * (8 + (size_t)M * 16) + 8;
                double *dst = host.data() + q * M * 2;
                for (uint32_t e = 0; e < M; e++) {
                    double c[2];
                    std::memcpy(c, src + (size_t)freq[e] * 16, 16);
                    dst[2 * e] = c[0] * scale;
                    dst[2 * e + 1] = c[1] * scale;
                }
            }
            if (hipMemcpy((char *)d + q0 * M * 16, host.data(), cnt * M * 16, hipMemcpyHostToDevice) != hipSuccess)
                fail("Fourier key copy to the device failed");
        }
        abi(tfhe_mi355_bootstrap_key_fourier_set_ready(ctx));
    });
}
