// client.cpp -- client-side helpers of the engine (key generation, LWE encryption/decryption).
// Not on the PBS hot path; they let a standalone user (and bench.py) build valid server keys
// without the Rust client.  They follow the reference's rules:
//   binary secret keys                  (LweSecretKey::generate_new_binary)
//   Gaussian noise, Marsaglia polar      (commons/math/random/gaussian.rs:15-52) + from_torus
//                                         (commons/math/torus/mod.rs:71-78)
//   GGSW rows of the BSK                 (algorithms/ggsw_encryption.rs:116-150, 300-331)
//   KSK levels stored L..1               (algorithms/lwe_keyswitch_key_generation.rs:60-135)
// The randomness source is a seeded xoshiro256**; keys are deterministic per (seed, index)
// whatever the thread count.  Seeded keys take their masks from the reference's AES-CTR mask
// stream of the compression seed (csprng.hip), so that the GPU can regenerate them.
#include <cmath>
#include <complex>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>
#include <atomic>
#include <algorithm>

namespace tfhe_mi355 {  // csprng.hip (host side): AES-128 tables / block function
size_t aes_tables_bytes();
void aes_tables_build(uint64_t seed_lo, uint64_t seed_hi, void *host_tables);
void aes128_encrypt_host(const void *host_tables, uint32_t s[4]);
}  // namespace tfhe_mi355

#include "../../include/tfhe_mi355.h"
#include "errors.h"

namespace {

struct Rng {
    uint64_t s[4];
    static uint64_t splitmix(uint64_t &x) {
        uint64_t z = (x += 0x9E3779B97F4A7C15ULL);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
        return z ^ (z >> 31);
    }
    Rng(uint64_t seed, uint64_t stream) {
        uint64_t x = seed ^ (stream * 0xD1B54A32D192ED03ULL) ^ 0xA5A5A5A5F00DF00DULL;
        for (auto &v : s) v = splitmix(x);
    }
    static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
    uint64_t next() {
        uint64_t r = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
        s[2] ^= s[0];
        s[3] ^= s[1];
        s[1] ^= s[2];
        s[0] ^= s[3];
        s[2] ^= t;
        s[3] = rotl(s[3], 45);
        return r;
    }
    uint64_t gaussian_torus(double std) {
        for (;;) {
            double u = (double)(int64_t)next() * 0x1p-63;
            double v = (double)(int64_t)next() * 0x1p-63;
            double s2 = u * u + v * v;
            if (s2 > 0.0 && s2 < 1.0) {
                double x = u * std * std::sqrt(-2.0 * std::log(s2) / s2);
                double fract = x - std::round(x);
                fract = std::round(fract * 18446744073709551616.0);
                if (fract >= 9223372036854775808.0) return 0x8000000000000000ULL;
                return (uint64_t)(int64_t)fract;
            }
        }
    }
};

template <class F>
int guard(F &&f) {
    try {
        f();
        tfhe_mi355::last_error_text().clear();
        return TFHE_MI355_OK;
    } catch (const std::exception &e) {
        tfhe_mi355::last_error_text() = e.what();
        return TFHE_MI355_ERROR;
    }
}

// Complex radix-2 FFT (host), used for exact negacyclic products at large N.
struct HostFft {
    int n;
    std::vector<std::complex<double>> w, psi;  // w[k] = exp(-2 pi i k / n); psi[j] = exp(i pi j / n)
    std::vector<int> rev;
    explicit HostFft(int n_) : n(n_), w(n_ / 2), psi(n_), rev(n_) {
        for (int k = 0; k < n / 2; k++) w[k] = std::polar(1.0, -2.0 * M_PI * k / n);
        for (int j = 0; j < n; j++) psi[j] = std::polar(1.0, M_PI * j / n);
        int lg = 0;
        while ((1 << lg) < n) lg++;
        for (int i = 0; i < n; i++) {
            int r = 0;
            for (int b = 0; b < lg; b++) r |= ((i >> b) & 1) << (lg - 1 - b);
            rev[i] = r;
        }
    }
    void run(std::complex<double> *x, bool inverse) const {
        for (int i = 0; i < n; i++)
            if (i < rev[i]) std::swap(x[i], x[rev[i]]);
        for (int len = 2; len <= n; len <<= 1) {
            const int half = len / 2, step = n / len;
            for (int i = 0; i < n; i += len)
                for (int k = 0; k < half; k++) {
                    std::complex<double> t = inverse ? std::conj(w[k * step]) : w[k * step];
                    std::complex<double> u = x[i + k], v = x[i + k + half] * t;
                    x[i + k] = u + v;
                    x[i + k + half] = u - v;
                }
        }
    }
};

const HostFft &host_fft(int n) {
    static std::mutex mu;
    static std::map<int, std::unique_ptr<HostFft>> cache;
    std::lock_guard<std::mutex> g(mu);
    auto &p = cache[n];
    if (!p) p.reset(new HostFft(n));
    return *p;
}

// body += a * s (negacyclic, s binary), exact mod 2^64: four 16-bit limbs of a, each convolved
// with s in f64 through a psi-weighted FFT (|limb conv| < 2^31, so rounding is exact; checked).
void negacyclic_binary_add_fft(uint64_t *body, const uint64_t *a, const uint64_t *s, int N) {
    const HostFft &F = host_fft(N);
    std::vector<std::complex<double>> S(N), A(N);
    for (int j = 0; j < N; j++) S[j] = (double)s[j] * F.psi[j];
    F.run(S.data(), false);
    for (int limb = 0; limb < 4; limb++) {
        for (int j = 0; j < N; j++) A[j] = (double)((a[j] >> (16 * limb)) & 0xffff) * F.psi[j];
        F.run(A.data(), false);
        for (int j = 0; j < N; j++) A[j] *= S[j];
        F.run(A.data(), true);
        for (int j = 0; j < N; j++) {
            const double v = (A[j] * std::conj(F.psi[j])).real() / N;
            const double r = std::nearbyint(v);
            if (std::fabs(v - r) > 0.25) throw std::runtime_error("inexact negacyclic product");
            body[j] += (uint64_t)(int64_t)r << (16 * limb);
        }
    }
}

void negacyclic_binary_add(uint64_t *body, const uint64_t *a, const uint64_t *s, int N) {
    if (N >= 4096) return negacyclic_binary_add_fft(body, a, s, N);
    for (int i = 0; i < N; i++) {
        if (!s[i]) continue;
        for (int j = 0; j < i; j++) body[j] -= a[j - i + N];
        for (int j = i; j < N; j++) body[j] += a[j - i];
    }
}

// AES-CTR mask words of a compression seed (csprng.hip; the reference's seeded-key mask stream:
// word w = little-endian bytes [1 + 8w, 9 + 8w) of the AES-CTR table)
struct SeededMask {
    std::vector<unsigned char> tables;
    SeededMask(uint64_t lo, uint64_t hi) : tables(tfhe_mi355::aes_tables_bytes()) {
        tfhe_mi355::aes_tables_build(lo, hi, tables.data());
    }
    void words(uint64_t first, size_t count, uint64_t *out) const {
        uint64_t cur = UINT64_MAX;
        unsigned char blk[16];
        unsigned char *dst = reinterpret_cast<unsigned char *>(out);
        for (size_t i = 0; i < 8 * count; i++) {
            const uint64_t g = 1 + 8 * first + i, a = g / 16;
            if (a != cur) {
                uint32_t st[4] = {(uint32_t)a, (uint32_t)(a >> 32), 0u, 0u};
                tfhe_mi355::aes128_encrypt_host(tables.data(), st);
                std::memcpy(blk, st, 16);
                cur = a;
            }
            dst[i] = blk[g % 16];
        }
    }
};

void glwe_encrypt_assign(Rng &r, uint64_t *glwe, const uint64_t *key, int k, int N, double std,
                         const SeededMask *mask = nullptr, uint64_t mask_first_word = 0) {
    uint64_t *body = glwe + (size_t)k * N;
    if (mask)
        mask->words(mask_first_word, (size_t)k * N, glwe);
    else
        for (size_t i = 0; i < (size_t)k * N; i++) glwe[i] = r.next();
    for (int j = 0; j < N; j++) body[j] += r.gaussian_torus(std);
    for (int p = 0; p < k; p++) negacyclic_binary_add(body, glwe + (size_t)p * N, key + (size_t)p * N, N);
}

void lwe_encrypt(Rng &r, const uint64_t *sk, int n, uint64_t pt, double std, uint64_t *ct,
                 const SeededMask *mask = nullptr, uint64_t mask_first_word = 0) {
    uint64_t b = pt + r.gaussian_torus(std);
    if (mask) mask->words(mask_first_word, (size_t)n, ct);
    for (int i = 0; i < n; i++) {
        if (!mask) ct[i] = r.next();
        b += ct[i] * sk[i];
    }
    ct[n] = b;
}

}  // namespace

extern "C" {

int tfhe_mi355_client_gen_binary_key(uint64_t seed, uint64_t stream, uint64_t *key, size_t len) {
    return guard([&] {
        if (!key) throw std::invalid_argument("null key");
        Rng r(seed, stream);
        for (size_t i = 0; i < len; i++) key[i] = r.next() >> 63;
    });
}

}  // extern "C"

namespace {
// GGSW list generation shared by the classic and multi-bit keys: GGSW i encrypts the constant
// plaintext msg(i) (ggsw_encryption.rs:116-150,300-331), with its own RNG stream.
// mask: optional seeded mask stream (GLWE row j of the list takes mask words [j kN, (j+1) kN))
template <class Msg>
void gen_ggsw_list(uint64_t seed, uint64_t stream_base, uint32_t items, const uint64_t *glwe_sk, uint32_t k,
                   uint32_t N, uint32_t base_log, uint32_t level, double std, uint64_t *out, uint32_t threads,
                   Msg msg, const SeededMask *mask = nullptr) {
    const size_t glwe_len = (size_t)(k + 1) * N, ggsw_len = (size_t)level * (k + 1) * glwe_len;
    std::atomic<uint32_t> next{0};
    auto work = [&] {
        for (;;) {
            uint32_t i = next++;
            if (i >= items) break;
            Rng r(seed, stream_base + i);
            const uint64_t m = msg(i);
            uint64_t *ggsw = out + (size_t)i * ggsw_len;
            for (uint32_t lvl = 1; lvl <= level; lvl++) {
                uint64_t factor = (0 - m) * (1ULL << (64 - base_log * lvl));
                for (uint32_t row = 0; row <= k; row++) {
                    uint64_t *g = ggsw + ((size_t)(lvl - 1) * (k + 1) + row) * glwe_len;
                    uint64_t *body = g + (size_t)k * N;
                    if (row < k) {
                        for (uint32_t j = 0; j < N; j++) body[j] = glwe_sk[(size_t)row * N + j] * factor;
                    } else {
                        std::memset(body, 0, sizeof(uint64_t) * N);
                        body[0] = 0 - factor;
                    }
                    const uint64_t row_index = ((uint64_t)i * level + (lvl - 1)) * (k + 1) + row;
                    glwe_encrypt_assign(r, g, glwe_sk, (int)k, (int)N, std, mask, row_index * k * N);
                }
            }
        }
    };
    uint32_t nt = threads ? threads : std::max(1u, std::thread::hardware_concurrency());
    std::vector<std::thread> th;
    for (uint32_t t = 1; t < nt; t++) th.emplace_back(work);
    work();
    for (auto &t : th) t.join();
}
}  // namespace

extern "C" {

int tfhe_mi355_client_gen_bootstrap_key(uint64_t seed, const uint64_t *lwe_sk, uint32_t n,
                                        const uint64_t *glwe_sk, uint32_t k, uint32_t N, uint32_t base_log,
                                        uint32_t level, double std, uint64_t *bsk, uint32_t threads) {
    return guard([&] {
        if (!lwe_sk || !glwe_sk || !bsk) throw std::invalid_argument("null argument");
        gen_ggsw_list(seed, 0x1000000ULL, n, glwe_sk, k, N, base_log, level, std, bsk, threads,
                      [&](uint32_t i) { return lwe_sk[i]; });
    });
}

// [n/g][2^g][L][k+1][k+1][N]; GGSW (j, sel) encrypts combine_key_bits(sel, s_{gj..gj+g-1})
// (lwe_multi_bit_bootstrap_key_generation.rs:87-173, 401-427)
int tfhe_mi355_client_gen_multi_bit_bootstrap_key(uint64_t seed, const uint64_t *lwe_sk, uint32_t n,
                                                  const uint64_t *glwe_sk, uint32_t k, uint32_t N,
                                                  uint32_t base_log, uint32_t level, uint32_t grouping_factor,
                                                  double std, uint64_t *bsk, uint32_t threads) {
    return guard([&] {
        if (!lwe_sk || !glwe_sk || !bsk) throw std::invalid_argument("null argument");
        const uint32_t g = grouping_factor;
        if (g == 0 || g > 6 || n % g) throw std::invalid_argument("invalid grouping factor");
        gen_ggsw_list(seed, 0x4000000ULL, (n / g) << g, glwe_sk, k, N, base_log, level, std, bsk, threads,
                      [&](uint32_t i) {
                          const uint32_t sel = i & ((1u << g) - 1);
                          const uint64_t *key = lwe_sk + (size_t)(i >> g) * g;
                          uint64_t p = 1;
                          for (uint32_t b = 0; b < g; b++) p *= key[b] ^ (uint64_t)(((sel >> (g - 1 - b)) & 1) ^ 1);
                          return p;
                      });
    });
}

int tfhe_mi355_client_gen_keyswitch_key(uint64_t seed, const uint64_t *in_sk, uint32_t in_dim,
                                        const uint64_t *out_sk, uint32_t out_dim, uint32_t base_log,
                                        uint32_t level, double std, uint64_t *ksk) {
    return guard([&] {
        if (!in_sk || !out_sk || !ksk) throw std::invalid_argument("null argument");
        Rng r(seed, 0x2000000ULL);
        for (uint32_t i = 0; i < in_dim; i++)
            for (uint32_t l = 0; l < level; l++) {
                uint32_t lvl = level - l;
                uint64_t msg = in_sk[i] << (64 - base_log * lvl);
                lwe_encrypt(r, out_sk, (int)out_dim, msg, std, ksk + ((size_t)i * level + l) * (out_dim + 1));
            }
    });
}

// LWE -> GLWE packing keyswitching key [in_dim][level][(k+1)N], levels stored L..1: GLWE
// encryptions of the constant polynomial in_sk[i] * 2^(64 - base_log*lvl)
// (lwe_packing_keyswitch_key_generation.rs:74-149); input coefficient i draws from its own stream.
int tfhe_mi355_client_gen_packing_keyswitch_key(uint64_t seed, const uint64_t *in_sk, uint32_t in_dim,
                                                const uint64_t *glwe_sk, uint32_t k, uint32_t N,
                                                uint32_t base_log, uint32_t level, double std, uint64_t *pksk,
                                                uint32_t threads) {
    return guard([&] {
        if (!in_sk || !glwe_sk || !pksk) throw std::invalid_argument("null argument");
        if (level == 0 || base_log == 0 || base_log * level >= 64) throw std::invalid_argument("invalid decomposition");
        const size_t glwe_len = (size_t)(k + 1) * N;
        std::atomic<uint32_t> next{0};
        auto work = [&] {
            for (;;) {
                const uint32_t i = next++;
                if (i >= in_dim) break;
                Rng r(seed, 0x5000000ULL + i);
                for (uint32_t l = 0; l < level; l++) {
                    const uint32_t lvl = level - l;
                    uint64_t *g = pksk + ((size_t)i * level + l) * glwe_len;
                    std::memset(g + (size_t)k * N, 0, sizeof(uint64_t) * N);
                    g[(size_t)k * N] = in_sk[i] << (64 - base_log * lvl);
                    glwe_encrypt_assign(r, g, glwe_sk, (int)k, (int)N, std);
                }
            }
        };
        uint32_t nt = threads ? threads : std::max(1u, std::thread::hardware_concurrency());
        std::vector<std::thread> th;
        for (uint32_t t = 1; t < nt; t++) th.emplace_back(work);
        work();
        for (auto &t : th) t.join();
    });
}

// Seeded keys (the reference's SeededLweBootstrapKey / SeededLweKeyswitchKey with a
// CompressionSeed, seeded_lwe_bootstrap_key_generation.rs, seeded_lwe_keyswitch_key_generation.rs):
// masks from the AES-CTR stream of (mask_seed_lo, mask_seed_hi), noise from the engine's own RNG;
// only the bodies are returned -- [n][L][k+1][N] and [in_dim][L].
int tfhe_mi355_client_gen_seeded_bootstrap_key(uint64_t noise_seed, uint64_t mask_seed_lo, uint64_t mask_seed_hi,
                                               const uint64_t *lwe_sk, uint32_t n, const uint64_t *glwe_sk,
                                               uint32_t k, uint32_t N, uint32_t base_log, uint32_t level, double std,
                                               uint64_t *bodies, uint32_t threads) {
    return guard([&] {
        if (!lwe_sk || !glwe_sk || !bodies) throw std::invalid_argument("null argument");
        const SeededMask mask(mask_seed_lo, mask_seed_hi);
        const size_t glwe = (size_t)(k + 1) * N, rows = (size_t)n * level * (k + 1);
        std::vector<uint64_t> full(glwe * rows);
        gen_ggsw_list(noise_seed, 0x6000000ULL, n, glwe_sk, k, N, base_log, level, std, full.data(), threads,
                      [&](uint32_t i) { return lwe_sk[i]; }, &mask);
        for (size_t row = 0; row < rows; row++)
            std::memcpy(bodies + row * N, full.data() + row * glwe + (size_t)k * N, sizeof(uint64_t) * N);
    });
}

int tfhe_mi355_client_gen_seeded_keyswitch_key(uint64_t noise_seed, uint64_t mask_seed_lo, uint64_t mask_seed_hi,
                                               const uint64_t *in_sk, uint32_t in_dim, const uint64_t *out_sk,
                                               uint32_t out_dim, uint32_t base_log, uint32_t level, double std,
                                               uint64_t *bodies) {
    return guard([&] {
        if (!in_sk || !out_sk || !bodies) throw std::invalid_argument("null argument");
        const SeededMask mask(mask_seed_lo, mask_seed_hi);
        Rng r(noise_seed, 0x7000000ULL);
        std::vector<uint64_t> ct((size_t)out_dim + 1);
        for (uint32_t i = 0; i < in_dim; i++)
            for (uint32_t l = 0; l < level; l++) {
                const uint32_t lvl = level - l;
                const uint64_t j = (uint64_t)i * level + l;
                lwe_encrypt(r, out_sk, (int)out_dim, in_sk[i] << (64 - base_log * lvl), std, ct.data(), &mask,
                            j * out_dim);
                bodies[j] = ct[out_dim];
            }
    });
}

int tfhe_mi355_client_csprng_mask_words(uint64_t seed_lo, uint64_t seed_hi, uint64_t first_word, size_t count,
                                        uint64_t *out) {
    return guard([&] {
        if (!out && count) throw std::invalid_argument("null argument");
        SeededMask(seed_lo, seed_hi).words(first_word, count, out);
    });
}

int tfhe_mi355_client_lwe_encrypt(uint64_t seed, const uint64_t *sk, uint32_t n, const uint64_t *pts,
                                  size_t count, double std, uint64_t *cts) {
    return guard([&] {
        if (!sk || (!pts && count) || (!cts && count)) throw std::invalid_argument("null argument");
        Rng r(seed, 0x3000000ULL);
        for (size_t c = 0; c < count; c++) lwe_encrypt(r, sk, (int)n, pts[c], std, cts + c * (n + 1));
    });
}

int tfhe_mi355_client_lwe_decrypt(const uint64_t *sk, uint32_t n, const uint64_t *cts, size_t count,
                                  uint64_t *pts) {
    return guard([&] {
        if (!sk || (!pts && count) || (!cts && count)) throw std::invalid_argument("null argument");
        for (size_t c = 0; c < count; c++) {
            const uint64_t *ct = cts + c * (n + 1);
            uint64_t b = ct[n];
            for (uint32_t i = 0; i < n; i++) b -= ct[i] * sk[i];
            pts[c] = b;
        }
    });
}

}  // extern "C"
