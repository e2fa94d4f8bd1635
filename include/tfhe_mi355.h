/*
 * tfhe_mi355.h -- C ABI of the MI355X programmable-bootstrap engine.
 *
 * This is the drop-in boundary for the reference's PBS hot path (tfhe-rs-odd = tfhe 0.5.0
 * fork, CPU-only Rust).  Each entry point names the reference interface it replaces.  The
 * Rust-side binding a maintainer would add (a `ShortintBootstrappingKey::Gpu` arm calling
 * these functions through `extern "C"`) is shown in INTEGRATION.md.
 *
 * Conventions (mirroring tfhe/src/c_api/utils.rs:3-73 and c_api/core_crypto/mod.rs:37-121):
 *   - every function returns int: 0 = success, 1 = failure; the failure text is returned by
 *     tfhe_mi355_last_error() (thread-local);
 *   - out-params of handle type are nulled first (c_api/shortint/server_key/pbs.rs:25-28);
 *   - buffers are plain uint64_t arrays in the reference's entity layouts:
 *       LWE ciphertext   = mask[0..n) || body                      (lwe_ciphertext.rs:598-599)
 *       GLWE ciphertext  = k mask polys || body poly, N coeffs each (glwe_ciphertext.rs:423-425)
 *       standard BSK     = [n][L][k+1 rows][k+1 polys][N]          (ggsw_ciphertext.rs:185-216)
 *       multi-bit BSK    = [n/g][2^g][L][k+1][k+1][N]              (lwe_multi_bit_bootstrap_key.rs)
 *       KSK              = [in_dim][L_ks][out_dim+1], levels stored L..1
 *                          (lwe_keyswitch_key.rs:102-108, lwe_keyswitch_key_generation.rs:109);
 *   - "_async" entry points take DEVICE pointers and a hipStream_t (as void*), enqueue the work
 *     and return immediately; the others take HOST pointers and return after the outputs are
 *     written (synchronous).  The host-pointer forms pipeline the batch in chunks through
 *     page-locked staging on two streams (copies of one chunk overlap the kernels of the next);
 *   - a context is bound to one GPU (tfhe_mi355_context_create) or to a list of GPUs
 *     (tfhe_mi355_context_create_devices: keys replicated, batches split over the devices, see
 *     there); host-pointer calls on one context are thread-safe, so
 *     rayon-style concurrent callers sharing a key are safe (SURVEY.md 8b "Threading"): calls of
 *     more than 64 ciphertexts are serialised by an internal mutex, smaller concurrent calls of
 *     the same entry point are coalesced into shared batches that a dispatcher thread of the
 *     context runs on its own stream, each caller blocking until its own rows are written
 *     (a batch closes when no call has arrived for TFHE_MI355_COALESCE_GAP_US = 50, after at most
 *     _WINDOW_US = 1000, at _BATCH = 1024 ciphertexts, or -- blocking callers only -- as soon as
 *     as many rows are queued as the previous batch of the entry point had; _SLOTS, _OVERFLOW: a
 *     second batch runs concurrently only when half a batch is queued; a call that finds the
 *     coalescer idle runs at once on the calling thread, TFHE_MI355_COALESCE_DIRECT=0 turns that
 *     off; the one-ciphertext-per-call pattern, shortint/server_key/mod.rs:783-857;
 *     TFHE_MI355_COALESCE_MAX_COUNT=0 turns coalescing off).  At N = 2048, k = 1, L = 1, batches
 *     of at most three (classic) / two (multi-bit g = 2, 3) passes of one ciphertext per CU (768 /
 *     512 rows on 256 CUs: the measured crossovers against the throughput kernels) run the
 *     one-ciphertext-per-CU latency kernels (same outputs; TFHE_MI355_LATENCY_MAX = rows
 *     overrides, 0 = never).  At N = 8192 / 4096, k = 1, L = 1 or 2 (classic), batches of at least
 *     3/8 / 5/8 of the CU count (96 / 160 rows on 256 CUs) run the on-chip CMUX (the whole blind
 *     rotation in one workgroup per ciphertext, two per CU at N = 4096, no scratch used), smaller
 *     ones the split CMUX (same outputs; TFHE_MI355_ONCHIP_MIN = rows overrides,
 *     TFHE_MI355_ONCHIP=0 = never); at N = 8192 / 4096 (L = 1 or 2) batches of at most CUs / 4 / CUs / 2
 *     rows run the quad CMUX instead (four / two CUs per ciphertext exchanging sub-blocks every CMUX
 *     through the scratch; same outputs; TFHE_MI355_QUAD_MAX = rows overrides, TFHE_MI355_QUAD=0 =
 *     never).  The quad
 *     CMUX's workgroups wait on each other, so its launches are serialised per device within the
 *     process; two PROCESSES running quad CMUX kernels on one GPU at once can starve each other's
 *     workgroups -- the waits are bounded, and a synchronous call whose quad launch timed out
 *     fails (rc 1, outputs invalid) instead of hanging (an _async call's failure is reported by
 *     the context's next synchronous call); set TFHE_MI355_QUAD=0 where processes share a GPU.
 *     The _async calls hold no per-context mutable state: every device scratch buffer they
 *     need comes from the caller (d_scratch, sized by the matching *_scratch query; a call
 *     given less than its query fails with an error, and only a query returning 0 allows
 *     d_scratch = NULL), so concurrent callers on different streams only need scratch buffers
 *     of their own, and the calls can be captured into a hipGraph (no allocation or
 *     synchronisation inside);
 *   - keys: a key upload (any *_key_upload*, *_set_ready) waits for the coalesced batches in
 *     flight and blocks new ones until it is done (a pending upload also keeps new batches from
 *     starting, so uploads are not starved under load); the serialized-key uploads hold the key
 *     lock from their first key write to the ready flag; a caller that fills the buffer of
 *     tfhe_mi355_bootstrap_key_fourier / _keyswitch_key_device itself owns that window (calls made
 *     before its _set_ready see whatever the buffer holds; on a multi-device context the hand-out
 *     marks that key not uploaded on every device, so batched calls fail until _set_ready, which
 *     replicates the buffer to the other devices); _async calls are not ordered with
 *     uploads: do not re-upload a key while _async work that reads it may still run;
 *   - _async lut index arrays are not checked on the host (they live on the device): an entry
 *     >= lut_count is clamped to lut_count - 1 by the kernels (no out-of-bounds read); the
 *     host-pointer forms reject such an entry with an error;
 *   - keys uploaded through the _async/device forms are complete when the upload call returns
 *     (it waits for its stream), so any later call on any stream sees the whole key.
 */
#ifndef TFHE_MI355_H
#define TFHE_MI355_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TFHE_MI355_OK 0
#define TFHE_MI355_ERROR 1

typedef struct TfheMi355Context TfheMi355Context;

/* Parameter set.  Mirrors shortint ClassicPBSParameters / MultiBitPBSParameters
 * (shortint/parameters/mod.rs:60-75, multi_bit.rs:173-190). grouping_factor = 0: classic PBS. */
typedef struct {
    uint32_t lwe_dimension;   /* n: small LWE dimension (PBS input)            */
    uint32_t glwe_dimension;  /* k                                             */
    uint32_t polynomial_size; /* N                                             */
    uint32_t pbs_base_log;
    uint32_t pbs_level;
    uint32_t ks_base_log;
    uint32_t ks_level;
    uint32_t message_modulus;
    uint32_t carry_modulus;
    uint32_t grouping_factor; /* 0 = classic; 2, 3 = multi-bit: N = 2048 (k = 1, L = 1),
                                 N = 512 (k = 3, L = 1), N = 8192 (k = 1, L = 2)  */
} TfheMi355Parameters;

/* Thread-local text of the last failure ("" if none). */
const char *tfhe_mi355_last_error(void);

/* Number of visible GPUs. */
int tfhe_mi355_device_count(int *out_count);

/* Per-kernel timing (profiling aid; the counterpart of the reference's `__profiling` feature,
 * tfhe/Cargo.toml:131, which un-inlines the FFT and external-product pieces for perf): with
 * `every` > 0 the device launchers of this context bracket every `every`-th launch of each kernel
 * family with HIP events on the launch stream (never while the stream is being captured);
 * `every` = 0 turns it off.  Enabling clears earlier totals.  Entries are read one by one:
 * index -> (kernel family name, total ms, timed launches); the call waits for the recorded
 * events and fails past the last entry. */
int tfhe_mi355_kernel_timing_enable(TfheMi355Context *ctx, int every);
int tfhe_mi355_kernel_timing_entry(TfheMi355Context *ctx, size_t index, char *name, size_t name_len,
                                   double *total_ms, uint64_t *launches);

/* Asynchronous form of the small host-pointer calls (the coalescer's queue):
 * tfhe_mi355_submit enqueues 1..1024 ciphertexts of one op (0: programmable_bootstrap,
 * 1: keyswitch_programmable_bootstrap, 2: programmable_bootstrap_keyswitch, 3: keyswitch; arguments
 * as those entry points, luts ignored for op 3) and returns at once with a request handle;
 * tfhe_mi355_wait blocks until the outputs are written and frees the handle (every submitted
 * request must be waited on exactly once, before the buffers are reused or the context is
 * destroyed; a request still queued when tfhe_mi355_context_destroy runs is not run: destroy
 * returns 1, and that request's wait returns 1 with a message).  One thread can keep many requests in flight: a rayon worker can submit every block
 * of its share of an integer layer, then wait for them (the reference calls
 * keyswitch_programmable_bootstrap_assign per block, shortint/server_key/mod.rs:783-857), so the
 * coalesced batch is no longer capped by the number of threads. */
typedef struct TfheMi355Request TfheMi355Request;
int tfhe_mi355_submit(TfheMi355Context *ctx, int op, const uint64_t *lwe_in, uint64_t *lwe_out,
                      const uint64_t *luts, size_t lut_count, const uint32_t *lut_indexes, size_t count,
                      TfheMi355Request **out_req);
int tfhe_mi355_wait(TfheMi355Request *req);

/* Request-coalescing counters of this context (all ops): batches run, ciphertexts in them, the
 * most batches in flight at once, and the summed wall time of the batches (staging, copies,
 * kernels, sync); `reset` != 0 clears them after reading.  Profiling aid, no reference
 * counterpart (the reference has no batching layer). */
int tfhe_mi355_coalesce_stats(TfheMi355Context *ctx, int reset, uint64_t *batches, uint64_t *rows,
                              uint64_t *max_in_flight, double *batch_seconds);

/* Page-locked (pinned) host memory for batch buffers.  The synchronous host-pointer entry points
 * detect pinned input/output buffers and DMA them directly, chunk by chunk, overlapped with the
 * kernels (no host staging copies); pageable buffers go through the engine's pinned staging.
 * A Rust binding allocates its LWE batch Vecs here to get the device rate over PCIe.
 * (No reference counterpart: the reference is CPU-only; the buffers replace Vec<u64> batches.) */
int tfhe_mi355_host_alloc(size_t bytes, void **out_ptr);
int tfhe_mi355_host_free(void *ptr);

/* Create / destroy an engine context on `device`.
 * Accepted decompositions: 2 <= pbs_base_log and pbs_base_log * pbs_level <= 30 for N <= 2048 and
 * multi-bit; <= 63 for classic N >= 4096, with pbs_base_log <= 15 when pbs_level > 1 (the split
 * CMUX packs signed digits into int16).  Every reference parameter set is inside these bounds.
 * Replaces Fft::new + the shortint engine's thread-local buffers
 * (fft64/math/fft/mod.rs:146-193, shortint/engine/mod.rs:23-70,163-235). */
int tfhe_mi355_context_create(const TfheMi355Parameters *params, int device,
                              TfheMi355Context **out_ctx);
/* One context over several GPUs of this process (SURVEY.md 8b ctx_create(params, device_mask);
 * the reference's one process with its rayon pool, shortint/engine/mod.rs:23-25, calling one KS+PBS
 * per block from par_iter, integer/server_key/radix_parallel/mul.rs:347-407).  `devices` lists
 * device ordinals (a device may repeat: its shards then run side by side on their own streams);
 * devices = NULL with device_count = 0 takes every visible device; one device is the same as
 * tfhe_mi355_context_create.  Behaviour of every entry point on such a context:
 *   - key uploads (host or device pointer, seeded, serialized, the _fourier/_device + _set_ready
 *     pairs) go to the first device and are replicated from its memory: RCCL ncclBroadcast among
 *     the distinct devices (one rank per device, over xGMI; librccl is opened at run time), then
 *     device-to-device copies to further shards of the same device (TFHE_MI355_REPLICATE=copy:
 *     peer copies instead of RCCL; the default "auto" also falls back to peer copies when librccl
 *     cannot be loaded or its communicator is refused); device-pointer key inputs live on the first
 *     device.  Peer access is enabled between the distinct devices at creation.  A failed upload
 *     or replication leaves that key part not uploaded on EVERY device;
 *   - the calling thread's current HIP device is left as it was by every entry point;
 *   - batched host-pointer calls (PBS, KS, KS->PBS, PBS->KS, blind rotation, packing KS,
 *     GLWE products) are split into contiguous row shares, one per device, run concurrently and
 *     joined before the call returns; outputs are bit-identical to a single-device context;
 *   - calls of at most TFHE_MI355_COALESCE_MAX_COUNT ciphertexts and tfhe_mi355_submit go to the
 *     devices' coalescers in turn (round robin);
 *   - device-pointer (_async) calls and the *_scratch queries address the FIRST device (a device
 *     pointer belongs to one GPU): use tfhe_mi355_context_device_context for the others;
 *   - kernel timing and coalescing statistics are summed over the devices. */
int tfhe_mi355_context_create_devices(const TfheMi355Parameters *params, const int *devices, size_t device_count,
                                      TfheMi355Context **out_ctx);
/* How the last key replication of a context ran: TFHE_MI355_REPLICATION_NONE (a single-device
 * context, or nothing replicated yet), _RCCL (ncclBroadcast), _PEER_COPY (hipMemcpyPeerAsync between
 * distinct devices), _DEVICE_COPY (one distinct device: device-to-device copies only).  `note`
 * (optional, borrowed until the next upload) says why auto mode did not use RCCL, else "". */
#define TFHE_MI355_REPLICATION_NONE 0
#define TFHE_MI355_REPLICATION_RCCL 1
#define TFHE_MI355_REPLICATION_PEER_COPY 2
#define TFHE_MI355_REPLICATION_DEVICE_COPY 3
int tfhe_mi355_context_replication(TfheMi355Context *ctx, int *mode, const char **note);
/* Number of devices (shards) of a context: 1 for a single-device context. */
int tfhe_mi355_context_devices(TfheMi355Context *ctx, size_t *count);
/* The single-device context of shard `index` and its device ordinal (borrowed: owned and destroyed
 * by `ctx`; destroying it directly fails).  For a single-device context, index 0 is ctx itself. */
int tfhe_mi355_context_device_context(TfheMi355Context *ctx, size_t index, TfheMi355Context **out_ctx,
                                      int *device);
/* Destroy stops the request coalescer first (a batch already running completes), then frees the
 * device state.  Requests still queued are failed, not run: their tfhe_mi355_wait returns 1, and
 * destroy itself returns 1 saying how many there were (the context is destroyed all the same). */
int tfhe_mi355_context_destroy(TfheMi355Context *ctx);

/* Upload a standard-domain (u64) bootstrapping key and convert it to the engine's Fourier
 * layout on the GPU.  Replaces convert_standard_lwe_bootstrap_key_to_fourier /
 * par_convert_standard_lwe_bootstrap_key_to_fourier (lwe_bootstrap_key_conversion.rs:21-151)
 * and, for grouping_factor > 0, par_convert_standard_lwe_multi_bit_bootstrap_key_to_fourier
 * (lwe_multi_bit_bootstrap_key_conversion.rs).  `len` is in u64 words. */
int tfhe_mi355_bootstrap_key_upload(TfheMi355Context *ctx, const uint64_t *standard_bsk, size_t len);

/* Device-pointer form of the above (standard BSK already in this context's GPU memory). */
int tfhe_mi355_bootstrap_key_convert_async(TfheMi355Context *ctx, const uint64_t *d_standard_bsk,
                                           size_t len, void *stream);

/* Fourier BSK held by the context: device pointer and byte size, for RCCL broadcast of the
 * converted key to the other GPUs of the node. */
int tfhe_mi355_bootstrap_key_fourier(TfheMi355Context *ctx, void **d_ptr, size_t *bytes);
/* Mark the Fourier BSK as valid after it was filled externally (e.g. by a broadcast into the
 * buffer returned above). */
int tfhe_mi355_bootstrap_key_fourier_set_ready(TfheMi355Context *ctx);

/* Upload a keyswitching key (big LWE key -> small LWE key).  `len` in u64 words. */
int tfhe_mi355_keyswitch_key_upload(TfheMi355Context *ctx, const uint64_t *ksk, size_t len);
/* Device-pointer form of the KSK upload (device-to-device copy on `stream`). */
int tfhe_mi355_keyswitch_key_upload_async(TfheMi355Context *ctx, const uint64_t *d_ksk, size_t len,
                                          void *stream);
int tfhe_mi355_keyswitch_key_device(TfheMi355Context *ctx, void **d_ptr, size_t *bytes);
int tfhe_mi355_keyswitch_key_set_ready(TfheMi355Context *ctx);

/* Batched programmable bootstrap: for c < count,
 *   lwe_out[c] = PBS(lwe_in[c], luts[lut_indexes ? lut_indexes[c] : 0]).
 * lwe_in: count x (n+1); lwe_out: count x (k*N+1); luts: lut_count x (k+1)*N (GLWE accumulators,
 * e.g. from shortint generate_lookup_table).
 * Replaces programmable_bootstrap_lwe_ciphertext[_mem_optimized]
 * (lwe_programmable_bootstrapping.rs:1017-1111) = FourierLweBootstrapKeyView::bootstrap
 * (fft64/crypto/bootstrap.rs:346-380) and, for grouping_factor > 0,
 * multi_bit_programmable_bootstrap_lwe_ciphertext (lwe_multi_bit_programmable_bootstrapping.rs:1035). */
int tfhe_mi355_programmable_bootstrap(TfheMi355Context *ctx, const uint64_t *lwe_in, uint64_t *lwe_out,
                                      const uint64_t *luts, size_t lut_count,
                                      const uint32_t *lut_indexes, size_t count);
int tfhe_mi355_programmable_bootstrap_async(TfheMi355Context *ctx, const uint64_t *d_lwe_in,
                                            uint64_t *d_lwe_out, const uint64_t *d_luts,
                                            size_t lut_count, const uint32_t *d_lut_indexes,
                                            size_t count, void *d_scratch, size_t scratch_bytes,
                                            void *stream);
/* Device scratch (bytes) of the async PBS for `count` ciphertexts (count >= 1):
 *   - classic N <= 2048: 256 bytes (the persistent grid's ciphertext ticket) at the shapes that
 *     run it -- N = 2048 k = 1 L = 1 (every 2_2-like shortint set), N = 1024 k = 1 L = 2,
 *     N = 1024 k = 2 L = 3, N = 256 k = 5 L = 1 -- and 0 at the other classic shapes;
 *   - multi-bit N = 2048 / 512: 0;
 *   - N >= 4096, classic and multi-bit (N = 8192): the accumulators + spectra of one pass of
 *     the split CMUX (also asked for where the on-chip CMUX will run: the call picks by count)
 *     min(count, chunk) ciphertexts (chunk = 128 at N = 32768, 1024 for multi-bit (N = 8192,
 *     400 MiB); otherwise ~200 MiB worth in multiples of 64, at most 1024: 1024 at N = 4096, 512
 *     at N = 8192 (3_3), 256 / 192 at N = 16384, L = 2 / 3; TFHE_MI355_LARGE_CHUNK overrides;
 *     e.g. 1.5 MiB per ciphertext at 4_4).  Less scratch runs smaller passes; the call fails below
 *     one ciphertext's worth.
 * tfhe_mi355_programmable_bootstrap_async fails when given less than this (N <= 2048) -- it never
 * falls back silently.  tfhe_mi355_blind_rotate_async takes no scratch and runs the one-pass grid. */
int tfhe_mi355_programmable_bootstrap_scratch(TfheMi355Context *ctx, size_t count, size_t *bytes);

/* Batched blind rotation WITHOUT sample extraction: glwe_out[c] = the rotated accumulator
 * ((k+1)*N words, GLWE layout) of lwe_in[c] with LUT luts[lut_indexes ? lut_indexes[c] : 0].
 * Replaces the fork's FourierLweBootstrapKeyView::bootstrap_without_sample_extract
 * (fft64/crypto/bootstrap.rs:383-412), the first step of its multi-value bootstrapping.
 * Classic and multi-bit contexts with N <= 2048. */
int tfhe_mi355_blind_rotate(TfheMi355Context *ctx, const uint64_t *lwe_in, uint64_t *glwe_out,
                            const uint64_t *luts, size_t lut_count, const uint32_t *lut_indexes, size_t count);
int tfhe_mi355_blind_rotate_async(TfheMi355Context *ctx, const uint64_t *d_lwe_in, uint64_t *d_glwe_out,
                                  const uint64_t *d_luts, size_t lut_count, const uint32_t *d_lut_indexes,
                                  size_t count, void *stream);

/* The parameter set a context was created with. */
int tfhe_mi355_context_parameters(TfheMi355Context *ctx, TfheMi355Parameters *out);

/* ---- serialized server keys (wire formats; csrc/serde.cpp) ----
 * A tfhe-rs server key arrives as the bincode 1.3.3 encoding of its serde derive
 * (`bincode::serialize(&key)`, tfhe/Cargo.toml:36,57): these entry points take those bytes.
 *   CompressedServerKey (shortint/server_key/compressed.rs:43-55): seeded LWE keyswitching key +
 *     ShortintCompressedBootstrappingKey (Classic / MultiBit seeded BSK) -> regenerated on the GPU
 *     (tfhe_mi355_{keyswitch,bootstrap}_key_upload_seeded).  Replaces
 *     CompressedServerKey::decompress (compressed.rs) + the Fourier conversion.
 *   ServerKey (shortint/server_key/mod.rs:283-297): standard LWE keyswitching key +
 *     Fourier bootstrapping key in concrete-fft's serialized form (FourierPolynomialList,
 *     fft64/math/fft/mod.rs:588-717: natural DFT order), mapped into the engine layout
 *     (every N = 256 ... 32768).  Replaces the ServerKey deserialisation feeding the CPU PBS.
 * Only native (2^64) ciphertext moduli.  *_inspect parses and validates without a GPU and
 * reports the parameter set the key implies (create the context from info.params); *_upload
 * requires a context with exactly that parameter set.  Truncated or inconsistent input fails
 * with a message naming the field and byte offset. */
typedef struct {
    TfheMi355Parameters params;        /* implied by the key material (std devs are not serialized) */
    uint32_t pbs_order;                /* PBSOrder: 0 KeyswitchBootstrap, 1 BootstrapKeyswitch */
    uint32_t deterministic_execution;  /* multi-bit keys */
    uint64_t max_degree;
    uint64_t max_noise_level;          /* ServerKey only (a CompressedServerKey has none: 0) */
    uint64_t ksk_seed_lo, ksk_seed_hi; /* CompressedServerKey: CompressionSeed of each key */
    uint64_t bsk_seed_lo, bsk_seed_hi;
} TfheMi355ServerKeyInfo;
int tfhe_mi355_compressed_server_key_inspect(const uint8_t *bytes, size_t len, TfheMi355ServerKeyInfo *info);
int tfhe_mi355_compressed_server_key_upload(TfheMi355Context *ctx, const uint8_t *bytes, size_t len);
int tfhe_mi355_server_key_inspect(const uint8_t *bytes, size_t len, TfheMi355ServerKeyInfo *info);
int tfhe_mi355_server_key_upload(TfheMi355Context *ctx, const uint8_t *bytes, size_t len);
/* engine Fourier layout: freq[e] = natural DFT index held by element e of a polynomial, M = N/2
 * entries, for every N = 256 ... 32768 -- host-only, no GPU needed */
int tfhe_mi355_fourier_engine_frequency(uint32_t N, uint32_t *freq);

/* Seeded (compressed) keys: the reference's SeededLweBootstrapKey / SeededLweKeyswitchKey
 * (shortint CompressedServerKey) hold only the bodies and a CompressionSeed (u128 = hi:lo); every
 * mask is regenerated on the GPU from the concrete-csprng AES-CTR stream of that seed.
 * Replace decompress_seeded_lwe_bootstrap_key (seeded_lwe_bootstrap_key_decompression.rs) +
 * the Fourier conversion, and decompress_seeded_lwe_keyswitch_key
 * (seeded_lwe_keyswitch_key_decompression.rs).  bodies: BSK [ggsw_count][L][k+1][N] (multi-bit:
 * ggsw_count = (n/g) 2^g, grouped as the standard key), KSK [k*N][ks_level]. */
int tfhe_mi355_bootstrap_key_upload_seeded(TfheMi355Context *ctx, const uint64_t *bodies, size_t len,
                                           uint64_t seed_lo, uint64_t seed_hi);
int tfhe_mi355_keyswitch_key_upload_seeded(TfheMi355Context *ctx, const uint64_t *bodies, size_t len,
                                           uint64_t seed_lo, uint64_t seed_hi);
/* the raw mask stream on the device: word w = little-endian bytes [1 + 8w, 9 + 8w) of the
 * AES-CTR table of the seed (concrete-csprng generators/aes_ctr, started at TableIndex::SECOND) */
int tfhe_mi355_csprng_mask_words(TfheMi355Context *ctx, uint64_t seed_lo, uint64_t seed_hi, uint64_t *out,
                                 size_t words);

/* LWE -> GLWE packing keyswitch of the fork's tree bootstrapping (gadget ServerKey
 * lwe_packing_keyswitch_key, gadget/engine/bootstrapping.rs:345-352, used at :713,:744).
 * Key layout [k*N][level][(k+1)*N] (levels stored L..1), input key = the big LWE key.
 * Replaces keyswitch_lwe_ciphertext_into_glwe_ciphertext (lwe_packing_keyswitch.rs:102-186):
 * lwe_in count x (k*N+1) -> glwe_out count x (k+1)*N. */
int tfhe_mi355_packing_keyswitch_key_upload(TfheMi355Context *ctx, const uint64_t *pksk, size_t len,
                                            uint32_t base_log, uint32_t level);
int tfhe_mi355_packing_keyswitch(TfheMi355Context *ctx, const uint64_t *lwe_in, uint64_t *glwe_out, size_t count);
int tfhe_mi355_packing_keyswitch_async(TfheMi355Context *ctx, const uint64_t *d_lwe_in, uint64_t *d_glwe_out,
                                       size_t count, void *d_scratch, size_t scratch_bytes, void *stream);
/* Device scratch (bytes) of the async packing keyswitch.  The packing key's decomposition (base,
 * level) belongs to the key, not to the parameter set: this query fails until the packing key is
 * uploaded, and its answer then depends only on that decomposition and `count`. */
int tfhe_mi355_packing_keyswitch_scratch(TfheMi355Context *ctx, size_t count, size_t *bytes);

/* GLWE x plaintext-polynomial products over (Z/2^64)[X]/(X^N+1):
 *   out[c][i] = sum_{j < glwe_per_item} glwe_in[c][j] * polys[i][j]   (each GLWE polynomial)
 * glwe_in [count][glwe_per_item][(k+1)N], polys [npoly][glwe_per_item][N],
 * out [count][npoly][(k+1)N], or [count][npoly][k*N+1] when extract != 0 (degree-0 sample
 * extraction of each product).  Replaces the fork's MVB products v0 * v_i + extraction
 * (gadget/engine/bootstrapping.rs:567-620, polynomial_karatsuba_wrapping_mul at
 * polynomial_algorithms.rs:683-742) and the window sums of pack_into_new_accumulator (:690-773). */
int tfhe_mi355_glwe_poly_mul(TfheMi355Context *ctx, const uint64_t *glwe_in, size_t glwe_per_item,
                             const uint64_t *polys, size_t npoly, size_t count, int extract, uint64_t *out);
int tfhe_mi355_glwe_poly_mul_async(TfheMi355Context *ctx, const uint64_t *d_glwe_in, size_t glwe_per_item,
                                   const uint64_t *d_polys, size_t npoly, size_t count, int extract,
                                   uint64_t *d_out, void *stream);

/* Batched LWE keyswitch (big key -> small key): lwe_in count x (k*N+1) -> lwe_out count x (n+1).
 * Replaces keyswitch_lwe_ciphertext (lwe_keyswitch.rs:96-170). */
int tfhe_mi355_keyswitch(TfheMi355Context *ctx, const uint64_t *lwe_in, uint64_t *lwe_out, size_t count);
int tfhe_mi355_keyswitch_async(TfheMi355Context *ctx, const uint64_t *d_lwe_in, uint64_t *d_lwe_out,
                               size_t count, void *d_scratch, size_t scratch_bytes, void *stream);
/* Device scratch (bytes) of the async keyswitch: the int8-MFMA path's digit matrix. */
int tfhe_mi355_keyswitch_scratch(TfheMi355Context *ctx, size_t count, size_t *bytes);

/* shortint KS -> PBS (PBSOrder::KeyswitchBootstrap): lwe_in/out count x (k*N+1).
 * Replaces ServerKey::keyswitch_programmable_bootstrap_assign (shortint/server_key/mod.rs:783-857). */
int tfhe_mi355_keyswitch_programmable_bootstrap(TfheMi355Context *ctx, const uint64_t *lwe_in,
                                                uint64_t *lwe_out, const uint64_t *luts, size_t lut_count,
                                                const uint32_t *lut_indexes, size_t count);
int tfhe_mi355_keyswitch_programmable_bootstrap_async(TfheMi355Context *ctx, const uint64_t *d_lwe_in,
                                                      uint64_t *d_lwe_out, const uint64_t *d_luts,
                                                      size_t lut_count, const uint32_t *d_lut_indexes,
                                                      size_t count, void *d_scratch, size_t scratch_bytes,
                                                      void *stream);
/* Device scratch (bytes) needed by the async KS->PBS for `count` ciphertexts: the small-LWE
 * intermediate plus the larger of the keyswitch and PBS scratch. */
int tfhe_mi355_keyswitch_programmable_bootstrap_scratch(TfheMi355Context *ctx, size_t count,
                                                        size_t *bytes);

/* shortint PBS -> KS (PBSOrder::BootstrapKeyswitch): lwe_in/out count x (n+1).
 * Replaces ServerKey::programmable_bootstrap_keyswitch_assign (shortint/server_key/mod.rs:859-932). */
int tfhe_mi355_programmable_bootstrap_keyswitch(TfheMi355Context *ctx, const uint64_t *lwe_in,
                                                uint64_t *lwe_out, const uint64_t *luts, size_t lut_count,
                                                const uint32_t *lut_indexes, size_t count);
int tfhe_mi355_programmable_bootstrap_keyswitch_async(TfheMi355Context *ctx, const uint64_t *d_lwe_in,
                                                      uint64_t *d_lwe_out, const uint64_t *d_luts,
                                                      size_t lut_count, const uint32_t *d_lut_indexes,
                                                      size_t count, void *d_scratch, size_t scratch_bytes,
                                                      void *stream);
/* Device scratch (bytes) of the async PBS->KS: the big-LWE intermediate plus the larger of the
 * PBS and keyswitch scratch. */
int tfhe_mi355_programmable_bootstrap_keyswitch_scratch(TfheMi355Context *ctx, size_t count, size_t *bytes);

/* Batched LWE linear algebra on device rows of u64 words (wrapping mod 2^64):
 *   y[r] = y[r] * scalar + (d_x ? x[r] : 0)   for r < rows, `words` words per row,
 * row strides in words.  Replaces shortint unchecked_add_assign / unchecked_scalar_mul_assign and
 * the bivariate packing left*factor + right (shortint/server_key/bivariate_pbs.rs:167-182) for
 * device-resident radix ciphertexts. */
int tfhe_mi355_lwe_scalar_mul_add_async(TfheMi355Context *ctx, uint64_t *d_y, const uint64_t *d_x, uint64_t scalar,
                                        size_t rows, size_t words, size_t y_stride, size_t x_stride, void *stream);
/* trivial_pbs_assign (shortint/server_key/mod.rs:763-781) on the bodies of `rows` trivial
 * ciphertexts (d_body points at the first body, rows `stride` words apart) with the GLWE
 * accumulator d_lut ((k+1)*N words, device). */
int tfhe_mi355_trivial_pbs_async(TfheMi355Context *ctx, uint64_t *d_body, size_t rows, size_t stride,
                                 const uint64_t *d_lut, void *stream);

/* Fill a shortint lookup table (GLWE accumulator, (k+1)*N words) from f(i), i < msg*carry.
 * Replaces shortint fill_accumulator (shortint/engine/mod.rs:72-128). */
int tfhe_mi355_fill_accumulator(const TfheMi355Parameters *params, const uint64_t *f_values,
                                uint64_t *accumulator);

/* Diagnostic (test hook, host buffers, synchronous): the PBS kernels' backward torus conversion
 * (x86.rs:823-874 + 961-1044 after the fract) applied to n given fractions fr in [-1/2, 1/2]:
 * acc_inout[i] += X_i and set_out[i] = X_i, X_i = rint_half_even(fr[i] * 2^64) mod 2^64. */
int tfhe_mi355_debug_torus_from_fraction(int device, const double *fr, uint64_t *acc_inout, uint64_t *set_out,
                                         size_t n);

/* ---- client-side helpers (not on the PBS path; seeded, deterministic per (seed, index)) ----
 * Binary secret keys, Gaussian noise (commons/math/random/gaussian.rs:15-52), GGSW/BSK
 * (ggsw_encryption.rs:116-150,300-331), KSK (lwe_keyswitch_key_generation.rs:60-135),
 * LWE encryption/decryption (lwe_encryption.rs).  The randomness is a seeded xoshiro256**,
 * not the reference's AES-CTR CSPRNG: use the Rust client for production keys. */
int tfhe_mi355_client_gen_binary_key(uint64_t seed, uint64_t stream, uint64_t *key, size_t len);
int tfhe_mi355_client_gen_bootstrap_key(uint64_t seed, const uint64_t *lwe_sk, uint32_t n,
                                        const uint64_t *glwe_sk, uint32_t k, uint32_t N,
                                        uint32_t base_log, uint32_t level, double std_dev,
                                        uint64_t *bsk, uint32_t threads);
/* multi-bit BSK [n/g][2^g][L][k+1][k+1][N] (lwe_multi_bit_bootstrap_key_generation.rs:87-173) */
int tfhe_mi355_client_gen_multi_bit_bootstrap_key(uint64_t seed, const uint64_t *lwe_sk, uint32_t n,
                                                  const uint64_t *glwe_sk, uint32_t k, uint32_t N,
                                                  uint32_t base_log, uint32_t level, uint32_t grouping_factor,
                                                  double std_dev, uint64_t *bsk, uint32_t threads);
int tfhe_mi355_client_gen_keyswitch_key(uint64_t seed, const uint64_t *in_sk, uint32_t in_dim,
                                        const uint64_t *out_sk, uint32_t out_dim, uint32_t base_log,
                                        uint32_t level, double std_dev, uint64_t *ksk);
/* packing KSK [in_dim][level][(k+1)N] (lwe_packing_keyswitch_key_generation.rs:74-149) */
int tfhe_mi355_client_gen_packing_keyswitch_key(uint64_t seed, const uint64_t *in_sk, uint32_t in_dim,
                                                const uint64_t *glwe_sk, uint32_t k, uint32_t N,
                                                uint32_t base_log, uint32_t level, double std_dev,
                                                uint64_t *pksk, uint32_t threads);
/* seeded keys (masks from the AES-CTR stream of mask_seed, noise from noise_seed); bodies only */
int tfhe_mi355_client_gen_seeded_bootstrap_key(uint64_t noise_seed, uint64_t mask_seed_lo, uint64_t mask_seed_hi,
                                               const uint64_t *lwe_sk, uint32_t n, const uint64_t *glwe_sk,
                                               uint32_t k, uint32_t N, uint32_t base_log, uint32_t level,
                                               double std_dev, uint64_t *bodies, uint32_t threads);
int tfhe_mi355_client_gen_seeded_keyswitch_key(uint64_t noise_seed, uint64_t mask_seed_lo, uint64_t mask_seed_hi,
                                               const uint64_t *in_sk, uint32_t in_dim, const uint64_t *out_sk,
                                               uint32_t out_dim, uint32_t base_log, uint32_t level, double std_dev,
                                               uint64_t *bodies);
int tfhe_mi355_client_csprng_mask_words(uint64_t seed_lo, uint64_t seed_hi, uint64_t first_word, size_t count,
                                        uint64_t *out);
int tfhe_mi355_client_lwe_encrypt(uint64_t seed, const uint64_t *sk, uint32_t n, const uint64_t *plaintexts,
                                  size_t count, double std_dev, uint64_t *cts);
int tfhe_mi355_client_lwe_decrypt(const uint64_t *sk, uint32_t n, const uint64_t *cts, size_t count,
                                  uint64_t *plaintexts);

#ifdef __cplusplus
}
#endif

#endif /* TFHE_MI355_H */
