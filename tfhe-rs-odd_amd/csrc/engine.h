// engine.h -- internal launchers of the MI355X PBS engine (host side, no torch types).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

struct TfheMi355Context;  // include/tfhe_mi355.h (opaque there), capi.cpp

namespace tfhe_mi355 {

// Key transaction (capi.cpp): holds the context's key locks (every shard's, for a multi-device
// context) exclusively until the returned holder is released.  Key uploads made from this thread in
// the meantime skip their own locking, so a multi-call upload (serde.cpp: keyswitching key, Fourier
// buffer, ready flag) is seen by coalesced batches only as a whole.
std::shared_ptr<void> begin_key_transaction(TfheMi355Context *ctx);

// Per-kernel durations measured on the launch stream (a profiling aid, off unless enabled through
// tfhe_mi355_kernel_timing_enable): the launchers bracket every `every`-th launch of a kernel
// family with HIP events; collect() waits for them and accumulates per-name totals.  bench.py
// reads the dominant kernel's average from here for its roofline.  Nothing is recorded while the
// stream is being captured into a graph.
struct KernelTimer {
    int every = 0;  // 0: off
    std::mutex mu;
    struct Rec {
        std::string name;
        hipEvent_t a, b;
    };
    std::vector<Rec> pending;
    std::vector<hipEvent_t> pool;
    std::map<std::string, std::pair<double, uint64_t>> totals;  // name -> (ms, launches)
    std::map<std::string, uint64_t> calls;                      // launches seen per name (sampling)

    // true when this launch of `name` is to be timed
    bool want(const char *name, hipStream_t s) {
        if (every <= 0) return false;
        hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing(s, &st) != hipSuccess || st != hipStreamCaptureStatusNone) return false;
        std::lock_guard<std::mutex> g(mu);
        return calls[name]++ % (uint64_t)every == 0;
    }
    hipEvent_t record(hipStream_t s) {
        hipEvent_t e = nullptr;
        {
            std::lock_guard<std::mutex> g(mu);
            if (!pool.empty()) {
                e = pool.back();
                pool.pop_back();
            }
        }
        if (!e && hipEventCreate(&e) != hipSuccess) return nullptr;
        (void)hipEventRecord(e, s);
        return e;
    }
    void done(const char *name, hipEvent_t a, hipStream_t s) {
        hipEvent_t b = record(s);
        if (!a || !b) return;
        std::lock_guard<std::mutex> g(mu);
        pending.push_back({name, a, b});
    }
    void collect() {
        std::vector<Rec> recs;
        {
            std::lock_guard<std::mutex> g(mu);
            recs.swap(pending);
        }
        for (auto &r : recs) {
            float ms = 0.f;
            if (hipEventSynchronize(r.b) == hipSuccess && hipEventElapsedTime(&ms, r.a, r.b) == hipSuccess) {
                std::lock_guard<std::mutex> g(mu);
                auto &t = totals[r.name];
                t.first += ms;
                t.second += 1;
            }
            std::lock_guard<std::mutex> g(mu);
            pool.push_back(r.a);
            pool.push_back(r.b);
        }
    }
    void reset() {
        collect();
        std::lock_guard<std::mutex> g(mu);
        totals.clear();
        calls.clear();
    }
    ~KernelTimer() {
        collect();
        for (hipEvent_t e : pool) (void)hipEventDestroy(e);
    }
};

// RAII bracket of one kernel launch (no-op without a timer or when this launch is not sampled)
struct TimedLaunch {
    KernelTimer *t;
    const char *name;
    hipStream_t s;
    hipEvent_t a = nullptr;
    TimedLaunch(KernelTimer *t_, const char *name_, hipStream_t s_) : t(t_), name(name_), s(s_) {
        if (t && t->want(name, s)) a = t->record(s);
        else t = nullptr;
    }
    ~TimedLaunch() {
        if (t) t->done(name, a, s);
    }
};

struct FftTables {
    // device tables, M entries each (M = N/2)
    double2 *W = nullptr;          // exp(-2 pi i t / M)
    double2 *twist = nullptr;      // exp(i pi j / N)            (fft/mod.rs:58-69)
    double2 *wtop = nullptr;       // N = 32768: top-stage twiddles wtop[c-1][a] = W[a c] (a < M/16, c < 16)
    int N = 0;
};

struct ClassicPbsLaunch {
    const uint64_t *lwe_in;      // [count][n+1]
    uint64_t *lwe_out;           // [count][k*N+1]
    const uint64_t *luts;        // [lut_count][(k+1)*N]
    const uint32_t *lut_indexes; // [count] or null; entries >= lut_count read LUT lut_count-1
    uint32_t lut_count;
    const double2 *fbsk;         // engine Fourier layout
    const double2 *W, *twist;
    int n;
    int base_log;
    int count;
    int glwe_out;                // 1: write the rotated accumulator [count][(k+1)N] (no sample extract)
    uint32_t *ticket = nullptr;  // zeroed device word: dynamic ciphertext queue of the persistent grid (null: one pass)
    int cpw_eff = 0;             // set by the launcher: ciphertexts per workgroup actually used (0: all slots)
};

// Returns false if (N, k, L) has no compiled specialisation.
bool classic_pbs_supported(int N, int k, int L);
// device scratch (zeroed by the caller before each launch) for the persistent grid's ticket
size_t classic_pbs_ticket_bytes(int N, int k, int L);
hipError_t launch_classic_pbs(int N, int k, int L, const ClassicPbsLaunch &a, hipStream_t s);
// latency form (pbs_latency.hip): one ciphertext per workgroup of 8 waves, same outputs; for small
// batches (the one-ciphertext-per-call pattern).  N = 2048, k = 1, L = 1 only; no ticket, no scratch.
bool latency_pbs_supported(int N, int k, int L);
hipError_t launch_latency_pbs(const ClassicPbsLaunch &a, hipStream_t s);

struct MultiBitPbsLaunch {
    const uint64_t *lwe_in;      // [count][n+1]
    uint64_t *lwe_out;           // [count][k*N+1]
    const uint64_t *luts;        // [lut_count][(k+1)*N]
    const uint32_t *lut_indexes; // [count] or null; entries >= lut_count read LUT lut_count-1
    uint32_t lut_count;
    const double2 *fbsk;         // [n/g][2^g][L][k+1][k+1] polys, engine Fourier layout
    const double2 *W, *twist;
    int n;
    int base_log;
    int count;
    int glwe_out;                // 1: write the rotated accumulator [count][(k+1)N] (no sample extract)
};
bool multibit_pbs_supported(int N, int k, int L, int g);
hipError_t launch_multibit_pbs(int N, int k, int L, int g, const MultiBitPbsLaunch &a, hipStream_t s);
// latency form (pbs_latency.hip): one ciphertext per workgroup of 8 waves, keybundle built into LDS
// beside the forward transform; same outputs.  N = 2048, k = 1, L = 1, g = 2 / 3; no scratch.
bool latency_multibit_supported(int N, int k, int L, int g);
hipError_t launch_latency_multibit_pbs(int g, const MultiBitPbsLaunch &a, hipStream_t s);

// N = 32768 classic PBS: accumulator and spectra in device scratch, three launches per CMUX
struct LargePbsLaunch {
    const uint64_t *lwe_in;      // [count][n+1]
    uint64_t *lwe_out;           // [count][k*N+1]
    const uint64_t *luts;        // [lut_count][(k+1)*N]
    const uint32_t *lut_indexes; // [count] or null; entries >= lut_count read LUT lut_count-1
    uint32_t lut_count;
    const double2 *fbsk;         // engine Fourier layout
    const double2 *W, *twist;
    const double2 *wtop;         // FftTables::wtop
    int n;
    int base_log;
    int count;
    void *scratch;               // >= large_pbs_scratch_per_ct() bytes per ciphertext of a chunk
    size_t scratch_bytes;
    uint64_t *acc;               // set by the launcher
    double2 *spectra;            // set by the launcher
    int levels;                  // set by the launcher (= pbs_level)
    int chunk_count;             // set by the launcher: ciphertexts in the current chunk
    KernelTimer *timer = nullptr;  // optional per-kernel timing
    int grouping = 0;              // > 0: multi-bit PBS (fbsk = [n/g][2^g][L][k+1][k+1] polys)
    int onchip_min_count = 0;      // N = 8192, L = 2 classic: the on-chip CMUX from this many ciphertexts on
    // N = 32768 grouped CMUX on two CU-masked streams: lane_c runs the
    // FP64 group kernels of one chunk while lane_m runs the streaming kernels (top_inv, digits) of
    // another; null: everything on the launch stream
    hipStream_t lane_c = nullptr, lane_m = nullptr;
    // N = 8192, L = 2 classic: the quad CMUX (R workgroups per ciphertext) for batches
    // of at most quad_max_count ciphertexts, quad_pass ciphertexts per launch (CUs / R: one workgroup
    // per CU, all resident at once); 0 = never
    int quad_pass = 0, quad_max_count = 0;
    uint32_t *quad_fail = nullptr;  // device word set by a quad workgroup whose partners never arrived
};
bool large_pbs_supported(int N, int k, int L);
bool large_multibit_supported(int N, int k, int L, int g);
size_t large_pbs_scratch_per_ct(int N, int k, int L);
hipError_t launch_large_pbs(int N, int k, int L, const LargePbsLaunch &a, hipStream_t s);
hipError_t launch_large_bsk_to_fourier(const uint64_t *std_polys, double2 *fourier, size_t npoly,
                                       const FftTables &t, hipStream_t s);

// standard BSK polys (npoly x N u64) -> Fourier (npoly x M double2, engine layout)
hipError_t launch_bsk_to_fourier(int N, const uint64_t *std_polys, double2 *fourier, size_t npoly,
                                 const FftTables &t, hipStream_t s);

struct KeyswitchLaunch {
    const uint64_t *lwe_in;  // [count][in_dim+1]
    uint64_t *lwe_out;       // [count][out_dim+1]
    const uint64_t *ksk;     // [in_dim][level][out_dim+1]
    int in_dim, out_dim, base_log, level;
    int count;
    // output column receiving the input body: out_dim for an LWE keyswitch, k*N for the LWE ->
    // GLWE packing keyswitch (lwe_packing_keyswitch.rs:159-161, the GLWE body's constant term)
    int body_col = -1;
    __host__ __device__ int body() const { return body_col < 0 ? out_dim : body_col; }
};
hipError_t launch_keyswitch(const KeyswitchLaunch &a, hipStream_t s);
// int8-MFMA keyswitch: KSK repacked once into 8 byte planes (ks_mfma_cols x ks_mfma_rows each)
bool ks_mfma_supported(int in_dim, int level, int base_log);
size_t ks_mfma_rows(int in_dim, int level);
size_t ks_mfma_cols(int out_dim);
size_t ks_mfma_scratch_bytes(int in_dim, int level, int count);
hipError_t launch_ksk_repack(const uint64_t *ksk, int8_t *kt, int in_dim, int level, int out_dim, hipStream_t s);
hipError_t launch_keyswitch_mfma(const KeyswitchLaunch &a, const int8_t *kt, void *scratch, hipStream_t s);

// batched LWE linear algebra / trivial PBS (lwe_ops.hip)
hipError_t launch_torus_from_fraction(const double *fr, uint64_t *acc, uint64_t *set, size_t n, hipStream_t s);
hipError_t launch_lwe_scalar_mul_add(uint64_t *y, const uint64_t *x, uint64_t scalar, size_t rows, size_t words,
                                     size_t y_stride, size_t x_stride, hipStream_t s);
hipError_t launch_trivial_pbs(uint64_t *body, size_t rows, size_t stride, const uint64_t *lut_body, uint64_t delta,
                              uint64_t modulus_sup, uint64_t box, hipStream_t s);

// GLWE x plaintext-polynomial products (glwe_ops.hip):
//   out[c][i] = sum_{j<J} glwe_in[c][j] * polys[i][j]   in (Z/2^64)[X]/(X^N+1), per GLWE polynomial,
// optionally sample-extracted at degree 0.  Serves the fork's MVB products v0 * v_i
// (gadget/engine/bootstrapping.rs:567-620) and the window sums of the tree-bootstrapping packing
// (:690-773).  Cost scales with the polys' nonzero count.
struct GlwePolyMulLaunch {
    const uint64_t *glwe_in;  // [count][J][(k+1)N]
    const uint64_t *polys;    // [npoly][J][N]
    uint64_t *out;            // [count][npoly][(k+1)N], or [count][npoly][kN+1] when extract
    int k, N, J, npoly;
    size_t count;
    bool extract;
};
hipError_t launch_glwe_poly_mul(const GlwePolyMulLaunch &a, hipStream_t s);

// seeded-key decompression (csprng.hip): AES-CTR mask stream of the compression seed written as
// `row_words` mask words per row, followed by `body_words` copied from d_bodies, for `rows` rows
size_t aes_tables_bytes();
void aes_tables_build(uint64_t seed_lo, uint64_t seed_hi, void *host_tables);
void aes128_encrypt_host(const void *host_tables, uint32_t s[4]);
hipError_t launch_seeded_decompress(const void *d_tables, const uint64_t *d_bodies, size_t rows, size_t row_words,
                                    size_t body_words, uint64_t *d_out, hipStream_t s);

}  // namespace tfhe_mi355
