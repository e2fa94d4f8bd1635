// csprng.hip -- seeded-key decompression on the GPU.
//
// Replaces decompress_seeded_lwe_bootstrap_key / decompress_seeded_lwe_keyswitch_key and the
// multi-bit variant (core_crypto/algorithms/seeded_{lwe_bootstrap_key,lwe_keyswitch_key,
// lwe_multi_bit_bootstrap_key}_decompression.rs) with the concrete-csprng AES-CTR mask generator
// they drive (concrete-csprng/src/generators/aes_ctr/*.rs).  The reference's nested forks
// (BSK -> GGSW -> level -> GLWE row; KSK -> LWE) hand out contiguous byte ranges of ONE AES-CTR
// stream keyed with the compression seed, starting at table index (0, 1), and every native u64 mask
// word is the little-endian value of 8 consecutive bytes: mask word w of a key is stream bytes
// [1 + 8w, 9 + 8w) (oracle/csprng_oracle.c restates the derivation with file:line).  So the whole
// mask of a key is one counter-mode pass: thread a encrypts counter a and scatters its 16 bytes
// to the (up to three) mask words they belong to, directly into the standard key layout; the
// bodies are copied beside them.
//
// AES-128: T-table form (Te0 and the S-box in LDS, Te1..Te3 as byte rotations of Te0), round
// keys expanded once on the host.  Checked bit-exact against the oracle's FIPS-197 restatement.
#include "engine.h"

namespace tfhe_mi355 {

namespace {
__device__ __forceinline__ uint32_t rotl32(uint32_t x, int s) { return (x << s) | (x >> (32 - s)); }
}  // namespace

// columns packed little-endian: word c = s[4c] | s[4c+1] << 8 | s[4c+2] << 16 | s[4c+3] << 24
__device__ __forceinline__ void aes128_encrypt_block(const uint32_t *__restrict__ rk, const uint32_t *te,
                                                     const uint8_t *sb, uint32_t s[4]) {
#pragma unroll
    for (int c = 0; c < 4; c++) s[c] ^= rk[c];
#pragma unroll
    for (int round = 1; round < 10; round++) {
        uint32_t t[4];
#pragma unroll
        for (int c = 0; c < 4; c++) {
            t[c] = te[s[c] & 0xff] ^ rotl32(te[(s[(c + 1) & 3] >> 8) & 0xff], 8) ^
                   rotl32(te[(s[(c + 2) & 3] >> 16) & 0xff], 16) ^ rotl32(te[s[(c + 3) & 3] >> 24], 24) ^
                   rk[4 * round + c];
        }
#pragma unroll
        for (int c = 0; c < 4; c++) s[c] = t[c];
    }
    uint32_t t[4];
#pragma unroll
    for (int c = 0; c < 4; c++) {
        t[c] = ((uint32_t)sb[s[c] & 0xff] | ((uint32_t)sb[(s[(c + 1) & 3] >> 8) & 0xff] << 8) |
                ((uint32_t)sb[(s[(c + 2) & 3] >> 16) & 0xff] << 16) | ((uint32_t)sb[s[(c + 3) & 3] >> 24] << 24)) ^
               rk[40 + c];
    }
#pragma unroll
    for (int c = 0; c < 4; c++) s[c] = t[c];
}

struct AesTables {
    uint32_t rk[44];
    uint32_t te0[256];
    uint8_t sbox[256];
};

// Mask words [0, words) of the key, written into rows: word w -> out[(w / row_words) * stride +
// w % row_words].  Thread a encrypts counter a: its bytes 1..8 are word 2a, bytes 9..15 the low 7
// bytes of word 2a+1, byte 0 the top byte of word 2a-1.
__global__ void __launch_bounds__(256) csprng_mask_kernel(const AesTables *__restrict__ tab, size_t words,
                                                          size_t row_words, size_t stride, uint8_t *__restrict__ out) {
    __shared__ uint32_t te[256];
    __shared__ uint8_t sb[256];
    __shared__ uint32_t rk[44];
    te[threadIdx.x] = tab->te0[threadIdx.x];
    sb[threadIdx.x] = tab->sbox[threadIdx.x];
    if (threadIdx.x < 44) rk[threadIdx.x] = tab->rk[threadIdx.x];
    __syncthreads();
    const size_t blocks = (words + 1) / 2 + 1;  // counters touching words [0, words)
    for (size_t a = (size_t)blockIdx.x * 256 + threadIdx.x; a < blocks; a += (size_t)gridDim.x * 256) {
        uint32_t s[4] = {(uint32_t)a, (uint32_t)((uint64_t)a >> 32), 0u, 0u};  // u128 counter, LE
        aes128_encrypt_block(rk, te, sb, s);
        auto word_addr = [&](size_t w) { return out + ((w / row_words) * stride + w % row_words) * 8; };
        const size_t w0 = 2 * a;
        if (w0 < words) {  // bytes 1..8 -> word 2a
            const uint64_t lo = (uint64_t)s[0] | ((uint64_t)s[1] << 32), hi = (uint64_t)s[2] | ((uint64_t)s[3] << 32);
            *reinterpret_cast<uint64_t *>(word_addr(w0)) = (lo >> 8) | (hi << 56);
        }
        if (w0 + 1 < words) {  // bytes 9..15 -> bytes 0..6 of word 2a+1
            uint8_t *p = word_addr(w0 + 1);
            const uint64_t hi = (uint64_t)s[2] | ((uint64_t)s[3] << 32);
#pragma unroll
            for (int b = 0; b < 7; b++) p[b] = (uint8_t)(hi >> (8 * (b + 1)));
        }
        if (a >= 1 && w0 - 1 < words) word_addr(w0 - 1)[7] = (uint8_t)s[0];  // byte 0 -> top of word 2a-1
    }
}

// bodies[row][body_words] -> out[row * stride + row_words + j]
__global__ void __launch_bounds__(256) seeded_body_kernel(const uint64_t *__restrict__ bodies, size_t rows,
                                                          size_t body_words, size_t row_words, size_t stride,
                                                          uint64_t *__restrict__ out) {
    const size_t e = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= rows * body_words) return;
    const size_t r = e / body_words, j = e % body_words;
    out[r * stride + row_words + j] = bodies[e];
}

hipError_t launch_seeded_decompress(const void *d_tables, const uint64_t *d_bodies, size_t rows, size_t row_words,
                                    size_t body_words, uint64_t *d_out, hipStream_t s) {
    if (rows == 0) return hipSuccess;
    const size_t stride = row_words + body_words;
    const size_t words = rows * row_words;
    if (words) {
        const size_t blocks = (words + 1) / 2 + 1;
        const unsigned grid = (unsigned)std::min<size_t>((blocks + 255) / 256, 65536);
        hipLaunchKernelGGL(csprng_mask_kernel, dim3(grid), dim3(256), 0, s,
                           reinterpret_cast<const AesTables *>(d_tables), words, row_words, stride,
                           reinterpret_cast<uint8_t *>(d_out));
    }
    const size_t n = rows * body_words;
    if (n)
        hipLaunchKernelGGL(seeded_body_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, d_bodies, rows,
                           body_words, row_words, stride, d_out);
    return hipGetLastError();
}

// host copy of the block function (client-side seeded keygen uses the same tables)
void aes128_encrypt_host(const void *host_tables, uint32_t s[4]) {
    const AesTables &t = *reinterpret_cast<const AesTables *>(host_tables);
    auto rot = [](uint32_t x, int k) { return (x << k) | (x >> (32 - k)); };
    for (int c = 0; c < 4; c++) s[c] ^= t.rk[c];
    for (int round = 1; round < 10; round++) {
        uint32_t u[4];
        for (int c = 0; c < 4; c++)
            u[c] = t.te0[s[c] & 0xff] ^ rot(t.te0[(s[(c + 1) & 3] >> 8) & 0xff], 8) ^
                   rot(t.te0[(s[(c + 2) & 3] >> 16) & 0xff], 16) ^ rot(t.te0[s[(c + 3) & 3] >> 24], 24) ^
                   t.rk[4 * round + c];
        for (int c = 0; c < 4; c++) s[c] = u[c];
    }
    uint32_t u[4];
    for (int c = 0; c < 4; c++)
        u[c] = ((uint32_t)t.sbox[s[c] & 0xff] | ((uint32_t)t.sbox[(s[(c + 1) & 3] >> 8) & 0xff] << 8) |
                ((uint32_t)t.sbox[(s[(c + 2) & 3] >> 16) & 0xff] << 16) |
                ((uint32_t)t.sbox[s[(c + 3) & 3] >> 24] << 24)) ^
               t.rk[40 + c];
    for (int c = 0; c < 4; c++) s[c] = u[c];
}

// host side: FIPS-197 tables and key schedule in the kernel's packing
size_t aes_tables_bytes() { return sizeof(AesTables); }

void aes_tables_build(uint64_t seed_lo, uint64_t seed_hi, void *host_tables) {
    AesTables &t = *reinterpret_cast<AesTables *>(host_tables);
    auto gmul = [](uint8_t a, uint8_t b) {
        uint8_t p = 0;
        while (b) {
            if (b & 1) p ^= a;
            a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0));
            b >>= 1;
        }
        return p;
    };
    for (int x = 0; x < 256; x++) {
        uint8_t inv = 0;
        for (int y = 1; x && y < 256; y++)
            if (gmul((uint8_t)x, (uint8_t)y) == 1) {
                inv = (uint8_t)y;
                break;
            }
        uint8_t sv = inv, r = inv;
        for (int i = 0; i < 4; i++) {
            r = (uint8_t)((r << 1) | (r >> 7));
            sv ^= r;
        }
        t.sbox[x] = (uint8_t)(sv ^ 0x63);
    }
    for (int x = 0; x < 256; x++) {
        const uint8_t sv = t.sbox[x];
        t.te0[x] = (uint32_t)gmul(sv, 2) | ((uint32_t)sv << 8) | ((uint32_t)sv << 16) | ((uint32_t)gmul(sv, 3) << 24);
    }
    uint8_t rk[176];
    for (int i = 0; i < 8; i++) {  // key = seed (u128) little-endian bytes
        rk[i] = (uint8_t)(seed_lo >> (8 * i));
        rk[8 + i] = (uint8_t)(seed_hi >> (8 * i));
    }
    uint8_t rcon = 1;
    for (int i = 4; i < 44; i++) {
        uint8_t w[4] = {rk[4 * i - 4], rk[4 * i - 3], rk[4 * i - 2], rk[4 * i - 1]};
        if (i % 4 == 0) {
            const uint8_t u = w[0];
            w[0] = (uint8_t)(t.sbox[w[1]] ^ rcon);
            w[1] = t.sbox[w[2]];
            w[2] = t.sbox[w[3]];
            w[3] = t.sbox[u];
            rcon = gmul(rcon, 2);
        }
        for (int j = 0; j < 4; j++) rk[4 * i + j] = (uint8_t)(rk[4 * i - 16 + j] ^ w[j]);
    }
    for (int i = 0; i < 44; i++)
        t.rk[i] = (uint32_t)rk[4 * i] | ((uint32_t)rk[4 * i + 1] << 8) | ((uint32_t)rk[4 * i + 2] << 16) |
                  ((uint32_t)rk[4 * i + 3] << 24);
}

}  // namespace tfhe_mi355
