/* csprng_oracle.c -- TEST INFRASTRUCTURE ONLY: CPU restatement of the reference's seeded-key
 * mask generator, the checker of the engine's seeded-key decompression.
 *
 * The reference generates every public mask of a seeded key from concrete-csprng's AES-CTR
 * generator keyed with the CompressionSeed (concrete-csprng 0.4, in-tree at
 * /root/reference/concrete-csprng; the AES block itself comes from the `aes` 0.8 crate or AES-NI):
 *   - key bytes = seed (u128).to_ne_bytes()   (implem/soft/block_cipher.rs:12-17; x86: LE)
 *   - the byte at table index (a, b) is byte b of AES_key(a.to_ne_bytes())   (block_cipher.rs:19-33,
 *     aes_ctr/states.rs:24-37: batches of 8 consecutive counters, buffer pointer = byte index)
 *   - a fresh generator starts at TableIndex::SECOND = (0, 1)   (aes_ctr/generic.rs:36-44)
 *   - forks hand each child a contiguous byte range starting right after the parent's last
 *     byte (generic.rs:89-120), so nested forks of a whole key tile its byte stream in order
 *   - a native-modulus u64 mask word is u64::from_le_bytes of 8 consecutive bytes
 *     (commons/math/random/uniform.rs:15-24, generator.rs:250-265)
 * Fork sizes: mask_bytes_per_{glwe,ggsw_level,ggsw,lwe} (encryption/mask_random_generator.rs:347-393)
 * => mask word w of a key = bytes [1 + 8w, 9 + 8w) of the stream.
 * Decompression order: seeded_ggsw_ciphertext_list_decompression.rs:8-47 (GGSW -> levels -> GLWE
 * rows, mask then body), seeded_lwe_ciphertext_list_decompression.rs:13-70 (LWE list).
 *
 * AES-128 restated from FIPS-197 (S-box from the GF(2^8) inverse + affine map); pinned by the
 * FIPS-197 known-answer vectors in tests/test_csprng.py.
 */
#include <stdint.h>
#include <string.h>

static uint8_t SBOX[256], MUL2[256], MUL3[256];
static int sbox_ready;

static uint8_t gf_mul(uint8_t a, uint8_t b) {
    uint8_t p = 0;
    while (b) {
        if (b & 1) p ^= a;
        a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0));
        b >>= 1;
    }
    return p;
}

static void build_sbox(void) {
    for (int x = 0; x < 256; x++) {
        uint8_t inv = 0;
        if (x)
            for (int y = 1; y < 256; y++)
                if (gf_mul((uint8_t)x, (uint8_t)y) == 1) {
                    inv = (uint8_t)y;
                    break;
                }
        uint8_t s = inv;
        uint8_t r = s;
        for (int i = 0; i < 4; i++) {
            r = (uint8_t)((r << 1) | (r >> 7));
            s ^= r;
        }
        SBOX[x] = (uint8_t)(s ^ 0x63);
        MUL2[x] = gf_mul((uint8_t)x, 2);
        MUL3[x] = gf_mul((uint8_t)x, 3);
    }
    sbox_ready = 1;
}

/* FIPS-197 5.2 key expansion: 11 round keys of 16 bytes */
void orc_aes128_expand(const uint8_t key[16], uint8_t rk[176]) {
    if (!sbox_ready) build_sbox();
    memcpy(rk, key, 16);
    uint8_t rcon = 1;
    for (int i = 4; i < 44; i++) {
        uint8_t t[4];
        memcpy(t, rk + 4 * (i - 1), 4);
        if (i % 4 == 0) {
            uint8_t u = t[0];
            t[0] = (uint8_t)(SBOX[t[1]] ^ rcon);
            t[1] = SBOX[t[2]];
            t[2] = SBOX[t[3]];
            t[3] = SBOX[u];
            rcon = gf_mul(rcon, 2);
        }
        for (int j = 0; j < 4; j++) rk[4 * i + j] = (uint8_t)(rk[4 * (i - 4) + j] ^ t[j]);
    }
}

/* FIPS-197 5.1 cipher; state column-major (s[4c + r]) as the byte order of the block */
void orc_aes128_encrypt(const uint8_t rk[176], const uint8_t in[16], uint8_t out[16]) {
    if (!sbox_ready) build_sbox();
    uint8_t s[16];
    for (int i = 0; i < 16; i++) s[i] = (uint8_t)(in[i] ^ rk[i]);
    for (int round = 1; round <= 10; round++) {
        uint8_t t[16];
        /* SubBytes + ShiftRows: row r shifted left by r */
        for (int c = 0; c < 4; c++)
            for (int r = 0; r < 4; r++) t[4 * c + r] = SBOX[s[4 * ((c + r) & 3) + r]];
        if (round < 10) { /* MixColumns */
            for (int c = 0; c < 4; c++) {
                uint8_t a0 = t[4 * c], a1 = t[4 * c + 1], a2 = t[4 * c + 2], a3 = t[4 * c + 3];
                s[4 * c] = (uint8_t)(MUL2[a0] ^ MUL3[a1] ^ a2 ^ a3);
                s[4 * c + 1] = (uint8_t)(a0 ^ MUL2[a1] ^ MUL3[a2] ^ a3);
                s[4 * c + 2] = (uint8_t)(a0 ^ a1 ^ MUL2[a2] ^ MUL3[a3]);
                s[4 * c + 3] = (uint8_t)(MUL3[a0] ^ a1 ^ a2 ^ MUL2[a3]);
            }
        } else {
            memcpy(s, t, 16);
        }
        for (int i = 0; i < 16; i++) s[i] ^= rk[16 * round + i];
    }
    memcpy(out, s, 16);
}

static void seed_key(uint64_t seed_lo, uint64_t seed_hi, uint8_t rk[176]) {
    uint8_t key[16];
    for (int i = 0; i < 8; i++) {
        key[i] = (uint8_t)(seed_lo >> (8 * i));
        key[8 + i] = (uint8_t)(seed_hi >> (8 * i));
    }
    orc_aes128_expand(key, rk);
}

/* bytes [offset, offset + count) of the AES-CTR table of `seed` (offset 0 = table index FIRST) */
void orc_csprng_bytes(uint64_t seed_lo, uint64_t seed_hi, uint64_t offset, size_t count, uint8_t *out) {
    uint8_t rk[176], ctr[16], blk[16];
    seed_key(seed_lo, seed_hi, rk);
    uint64_t cur = UINT64_MAX;
    for (size_t i = 0; i < count; i++) {
        uint64_t g = offset + i, a = g / 16;
        if (a != cur) {
            memset(ctr, 0, 16);
            for (int j = 0; j < 8; j++) ctr[j] = (uint8_t)(a >> (8 * j)); /* u128 counter, LE */
            orc_aes128_encrypt(rk, ctr, blk);
            cur = a;
        }
        out[i] = blk[g % 16];
    }
}

/* the first `count` mask words of a key seeded with `seed`: word w = LE u64 of bytes 1 + 8w.. */
void orc_seeded_mask_words(uint64_t seed_lo, uint64_t seed_hi, uint64_t first_word, size_t count, uint64_t *out) {
    orc_csprng_bytes(seed_lo, seed_hi, 1 + 8 * first_word, 8 * count, (uint8_t *)out); /* host is LE */
}

/* decompress_seeded_lwe_bootstrap_key (classic; multi-bit: n_ggsw = (n/g) 2^g, same order):
 * bodies [n_ggsw][L][k+1][N] -> standard key [n_ggsw][L][k+1 rows][k+1 polys][N] */
void orc_decompress_seeded_bsk(uint64_t seed_lo, uint64_t seed_hi, const uint64_t *bodies, size_t n_ggsw, int L,
                               int k, int N, uint64_t *bsk) {
    const size_t glwe = (size_t)(k + 1) * N, mask = (size_t)k * N;
    const size_t rows = n_ggsw * (size_t)L * (k + 1);
    for (size_t row = 0; row < rows; row++) {
        uint64_t *g = bsk + row * glwe;
        orc_seeded_mask_words(seed_lo, seed_hi, row * mask, mask, g);
        memcpy(g + mask, bodies + row * N, sizeof(uint64_t) * N);
    }
}

/* decompress_seeded_lwe_keyswitch_key: bodies [in_dim][L] -> [in_dim][L][out_dim + 1] */
void orc_decompress_seeded_ksk(uint64_t seed_lo, uint64_t seed_hi, const uint64_t *bodies, size_t in_dim, int L,
                               int out_dim, uint64_t *ksk) {
    const size_t lwes = in_dim * (size_t)L;
    for (size_t j = 0; j < lwes; j++) {
        uint64_t *c = ksk + j * (size_t)(out_dim + 1);
        orc_seeded_mask_words(seed_lo, seed_hi, j * (size_t)out_dim, out_dim, c);
        c[out_dim] = bodies[j];
    }
}
