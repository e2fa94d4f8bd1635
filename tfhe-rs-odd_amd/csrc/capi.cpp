// capi.cpp -- C ABI implementation (include/tfhe_mi355.h).  Host-side runtime of the engine:
// context = device + parameter set + key material + FFT tables, guarded by a mutex so that
// concurrent callers (the reference's rayon workers, shortint/engine/mod.rs:23-25) can share one
// key.  Error convention: 0/1 return + thread-local message (tfhe/src/c_api/utils.rs:3-73).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>  // types only: librccl is opened at run time, when keys are replicated

#include <algorithm>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdlib>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <atomic>
#include <shared_mutex>
#include <stdexcept>
#include <string>
#include <thread>
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

// The calling thread's current HIP device is the caller's (a Rust or C caller may use HIP itself):
// every entry point that selects another device puts the caller's back before it returns, success
// or failure.  A thread without a device (no GPU, or HIP not initialised) keeps none.
struct CallerDevice {
    int d = -1;
    CallerDevice() {
        if (hipGetDevice(&d) != hipSuccess) d = -1;
    }
    ~CallerDevice() {
        int now = -1;
        if (d >= 0 && (hipGetDevice(&now) != hipSuccess || now != d)) (void)hipSetDevice(d);
    }
    CallerDevice(const CallerDevice &) = delete;
    CallerDevice &operator=(const CallerDevice &) = delete;
};

template <class F>
int guarded(F &&f) {
    CallerDevice keep;
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
    DeviceBuffer() = default;
    DeviceBuffer(const DeviceBuffer &) = delete;
    DeviceBuffer &operator=(const DeviceBuffer &) = delete;
    ~DeviceBuffer() { release(); }
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

// page-locked host staging of the host-pointer entry points (hipHostMalloc), one per pipeline lane
struct PinnedBuffer {
    void *ptr = nullptr;
    size_t bytes = 0;
    PinnedBuffer() = default;
    PinnedBuffer(const PinnedBuffer &) = delete;
    PinnedBuffer &operator=(const PinnedBuffer &) = delete;
    ~PinnedBuffer() { release(); }
    void reserve(size_t b) {
        if (b <= bytes) return;
        release();
        check(hipHostMalloc(&ptr, b, hipHostMallocDefault), "hipHostMalloc");
        bytes = b;
    }
    void release() {
        if (ptr) (void)hipHostFree(ptr);
        ptr = nullptr;
        bytes = 0;
    }
};

// an environment switch is on when set to a non-empty value other than "0"
bool env_flag(const char *name) {
    const char *e = std::getenv(name);
    return e && *e && std::strcmp(e, "0") != 0;
}

size_t align256(size_t b) { return (b + 255) / 256 * 256; }

bool is_pow2(uint32_t x) { return x && !(x & (x - 1)); }
}  // namespace

// one small host-pointer call waiting to be coalesced into a batch (see "request coalescing")
enum CoalescedOp { CO_PBS = 0, CO_KS_PBS, CO_PBS_KS, CO_KS, CO_OPS };
struct CoalescedReq {
    const uint64_t *in;
    uint64_t *out;
    const uint64_t *luts;
    size_t lut_count;
    const uint32_t *idx;
    size_t count;
    bool sync = false;  // a blocking caller (coalesced_call), not a submitted request
    // blocking callers copy their own rows out of the slot's pinned staging once woken (in parallel
    // instead of one after the other on the dispatcher), then release the slot (pending)
    const uint64_t *src = nullptr;
    size_t src_bytes = 0;
    std::atomic<int> *pending = nullptr;
    // completion: set by the dispatcher, waited on by the caller alone (no shared mutex, so a
    // finished batch wakes its callers without a thundering herd on the queue lock)
    std::mutex m;
    std::condition_variable cv;
    bool done = false;
    std::string err;
};

struct RcclComms;  // communicator over a multi-device context's distinct devices (key replication)

// Worker threads of a multi-device context, one per shard after the first, started with the context
// and joined by its destroy: a batched host-pointer call hands each of them its shard's row share
// (split_rows) instead of starting threads per call.  Each worker runs its queue in
// order; concurrent calls queue behind each other per shard, as they would on the shard's lock.
struct ShardWorker {
    std::mutex m;
    std::condition_variable cv;
    std::deque<std::function<void()>> q;
    bool stop = false;
    std::thread t;
    void post(std::function<void()> f) {
        {
            std::lock_guard<std::mutex> g(m);
            q.push_back(std::move(f));
        }
        cv.notify_one();
    }
    void loop() {
        for (;;) {
            std::function<void()> f;
            {
                std::unique_lock<std::mutex> g(m);
                cv.wait(g, [&] { return stop || !q.empty(); });
                if (q.empty()) return;  // stop with nothing queued
                f = std::move(q.front());
                q.pop_front();
            }
            f();
        }
    }
    ~ShardWorker() {
        {
            std::lock_guard<std::mutex> g(m);
            stop = true;
        }
        cv.notify_one();
        if (t.joinable()) t.join();
    }
};

struct TfheMi355Context {
    TfheMi355Parameters p{};
    int device = 0;
    int cus = 256;  // compute units of the device (the latency kernels run one ciphertext per CU)
    std::mutex mu;
    // Key material vs the coalescer's batches: every key upload holds it exclusively, every
    // dispatcher batch shared, so a re-upload waits for the batches in flight and no batch starts
    // on a half-written key (the large host-pointer calls are ordered with uploads by `mu`).
    // Uploads go through KeyWrite, batches through KeyRead.
    std::shared_mutex keys_mu;
    // key writers waiting or running: a batch does not take keys_mu while one is pending, so an
    // upload is never starved by back-to-back batches (libstdc++'s shared_mutex lets new readers
    // in ahead of a waiting writer)
    std::atomic<int> key_writers{0};
    // Multi-device context (tfhe_mi355_context_create_devices): one single-device context per
    // listed device (a device may repeat), owned by this one; empty for a single-device context.
    // Every entry point of a multi-device context dispatches to them (see "multi-device").
    std::vector<TfheMi355Context *> shards;
    std::atomic<size_t> next_shard{0};  // round robin of coalesced calls and submits
    std::vector<std::unique_ptr<ShardWorker>> workers;  // shards 1.. (split_rows)
    int replication = 0;  // how the last key replication ran (tfhe_mi355_context_replication)
    RcclComms *rccl = nullptr;
    std::string replicate_note;  // why the last replication did not use RCCL in auto mode (empty: it did, or no need)
    TfheMi355Context *owner = nullptr;  // a shard: its multi-device context (destroyed with it)
    bool multi() const { return !shards.empty(); }
    hipStream_t stream = nullptr;
    FftTables tables;
    DeviceBuffer fbsk, ksk, std_staging;
    DeviceBuffer io_luts, io_tmp;
    DeviceBuffer ksk_planes;   // int8 byte planes of the KSK for the MFMA keyswitch
    // Host-pointer entry points: kernels run in chunk order on `stream`; each of two lanes has a
    // copy stream, page-locked staging and device in/out buffers, so that chunk i's copies (and
    // the host-side copies into and out of the staging) overlap chunk i+-1's kernels.  Only the
    // synchronous entry points use these, under `mu`; the _async entry points take all their
    // scratch from the caller (no shared mutable state, capturable into a hipGraph).
    struct Lane {
        hipStream_t stream = nullptr;
        hipEvent_t h2d = nullptr, kern = nullptr, done = nullptr;
        PinnedBuffer h_in, h_out, h_idx;
        DeviceBuffer d_in, d_out, d_idx;
        bool pending = false;
        bool direct_out = false;  // this chunk's D2H went straight into the caller's pinned buffer
        size_t first = 0, count = 0;
    } lanes[2];
    bool ksk_planes_ready = false;
    bool fbsk_ready = false, ksk_ready = false;
    // LWE -> GLWE packing keyswitching key of the gadget layer (big LWE key -> GLWE key)
    DeviceBuffer pksk, pksk_planes;
    uint32_t pks_base_log = 0, pks_level = 0;
    bool pksk_ready = false, pksk_planes_ready = false;
    KernelTimer timer;  // per-kernel durations (tfhe_mi355_kernel_timing_*), off by default
    // CU-masked lanes of the N = 32768 grouped CMUX (large_lanes), created at first use
    std::mutex lanes_mu;
    bool lanes_made = false;
    long lanes_mcus = 0, lanes_chunk = 0;  // TFHE_MI355_LANES_MCUS / _CHUNK at creation
    DeviceBuffer quad_fail;  // one u32 the quad CMUX sets when a flag wait timed out (check_quad_fail)
    bool lanes_block = false;              // TFHE_MI355_LANES_MASK=block
    hipStream_t lane_c = nullptr, lane_m = nullptr;
    // Request coalescing of small host-pointer calls (the reference calls the PBS one ciphertext
    // at a time from rayon workers: shortint/server_key/mod.rs:783-857, radix_parallel/mul.rs:
    // 347-407).  Concurrent calls are queued per op; dispatcher threads (one per batch slot,
    // started with the first coalesced call) each gather a queue into a batch (after a short
    // window or when the batch is full) and run it on their slot's stream, staging and scratch;
    // every caller gets its rows back bit-identical to a call of its own.
    struct Coalescer {
        std::mutex m;
        std::condition_variable cv;  // dispatchers: work queued / stop
        std::vector<CoalescedReq *> queue[CO_OPS];
        size_t queued[CO_OPS] = {};
        size_t queued_sync[CO_OPS] = {};  // of queued[]: rows from blocking callers
        size_t last_sync_rows[CO_OPS] = {};  // rows of the op's previous batch if all were blocking calls
        std::chrono::steady_clock::time_point last_arrival[CO_OPS];
        bool stop = false;
        std::vector<std::thread> workers;
        struct Slot {
            hipStream_t stream = nullptr;
            PinnedBuffer h_in, h_out;            // h_in / d_in: [LUT sets | input rows | LUT indexes]
            DeviceBuffer d_in, d_out, d_scratch;
            std::atomic<int> copies{0};          // callers of the last batch still copying out of h_out
        } slots[9];  // 0-7: dispatchers; 8: direct calls (coalesced_call)
        bool direct_busy = false;  // slot 8 in use, under m
        // statistics (tfhe_mi355_coalesce_stats), under m
        uint64_t batches = 0, rows = 0, in_flight = 0, max_in_flight = 0;
        double batch_seconds = 0;
    } co;
    KernelTimer *timer_or_null() { return timer.every > 0 ? &timer : nullptr; }

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

// ---- key transactions ------------------------------------------------------------------------
// A key write holds the context's mutex and keys_mu exclusively.  It is re-entrant per thread: a
// transaction (tfhe_mi355::begin_key_transaction, e.g. the serialized-key upload, which uploads the
// KSK, fills the Fourier buffer and marks it ready through three ABI calls) keeps both locks for its
// whole duration, and the nested calls on the same context from the same thread skip the locking.
thread_local std::vector<const TfheMi355Context *> tl_key_writes;

struct KeyWrite {
    TfheMi355Context *c = nullptr;
    std::unique_lock<std::mutex> g;
    std::unique_lock<std::shared_mutex> k;
    explicit KeyWrite(TfheMi355Context *c_) {
        if (std::find(tl_key_writes.begin(), tl_key_writes.end(), c_) != tl_key_writes.end()) return;
        c = c_;
        c->key_writers.fetch_add(1, std::memory_order_acq_rel);
        g = std::unique_lock<std::mutex>(c->mu);
        k = std::unique_lock<std::shared_mutex>(c->keys_mu);
        tl_key_writes.push_back(c);
    }
    KeyWrite(const KeyWrite &) = delete;
    KeyWrite &operator=(const KeyWrite &) = delete;
    ~KeyWrite() {
        if (!c) return;
        tl_key_writes.erase(std::find(tl_key_writes.begin(), tl_key_writes.end(), c));
        k.unlock();
        g.unlock();
        c->key_writers.fetch_sub(1, std::memory_order_acq_rel);
    }
};

// a coalesced batch reads the keys: it waits while an upload is pending (writer preference), then
// holds keys_mu shared for the batch
struct KeyRead {
    std::shared_lock<std::shared_mutex> k;
    explicit KeyRead(TfheMi355Context *c) {
        if (std::find(tl_key_writes.begin(), tl_key_writes.end(), c) != tl_key_writes.end()) return;
        while (c->key_writers.load(std::memory_order_acquire) > 0)
            std::this_thread::sleep_for(std::chrono::microseconds(20));
        k = std::shared_lock<std::shared_mutex>(c->keys_mu);
    }
};

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
    if (N >= 4096) {
        // the split CMUX's top radix-R stage (R = M / 1024) reads W[a c] for a < 1024: laid out
        // [c-1][a] so that a wave's 64 consecutive butterflies read 1 KiB contiguously instead of
        // 64 scattered lines
        const int A = 1024, R = M / A;
        std::vector<double2> top((size_t)(R - 1) * A);
        for (int c = 1; c < R; c++)
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

// ---- scratch sizes -----------------------------------------------------------------------------
// Every launcher takes its device scratch explicitly: the _async entry points pass the caller's
// d_scratch (sized by the *_scratch queries), the host-pointer entry points a lane's own buffer.

// the split CMUX of N >= 4096 (classic, or multi-bit at the N = 8192 sets): accumulators in scratch
bool is_large(const TfheMi355Context *c) {
    if (c->p.grouping_factor)
        return large_multibit_supported((int)c->N(), (int)c->k(), (int)c->p.pbs_level, (int)c->p.grouping_factor);
    return large_pbs_supported((int)c->N(), (int)c->k(), (int)c->p.pbs_level);
}

// N >= 4096: ciphertexts per pass of the split CMUX.  The chunk's accumulators + spectra should
// stay resident in the 256 MiB Infinity Cache: 128 at N = 32768 (1.5 MiB per ciphertext at 4_4,
// best of 64..1024 measured), otherwise ~200 MiB of scratch in multiples of 64 (64..1024) --
// round 4 sweeps (profiles/r04_chunk_sweep.log): 3_3 384 / 512 / 768 -> 5.94k / 6.17k / 5.55k,
// 2_5 192 / 256 -> 2268 / 2307, 1_4 832 / 1024 -> 13.5k / 14.3k KS+PBS/s (160 MiB gave 384 / 192 / 832);
// multi-bit mb3_3g3 (512 here) 384 / 512 / 768 / 1024 -> 9.11k / 9.30k / 8.59k / 8.19k (r04_mbchunk_*.log).
// Round 5, after the paired multi-bit kernel (large_mb_pair2_kernel) and the fused top_inv/top_fwd
// made the chunk's spectra traffic the smaller share: 512 / 768 / 1024 / 1280 / 2048 ->
// mb3_3g3 12.04k / 12.24k / 12.18k / 11.52k / 11.54k, mb3_3g2 10.21k / 10.44k / 10.63k / 9.65k /
// 9.65k (profiles/r05_mbchunk_*.json), so multi-bit takes 1024 (400 MiB of scratch).
// N = 32768 on two CU-masked lanes (pbs_large.hip launch_grouped_lanes): TFHE_MI355_LANES_MCUS =
// CUs per XCD of the streaming lane (0 = one stream, the default until measured), the group lane takes
// the rest; TFHE_MI355_LANES_MASK = "interleave" (CU mask bit i on XCD i mod 8, the driver's
// symmetric mapping) or "block"; TFHE_MI355_LANES_CHUNK = ciphertexts per lane chunk (default: one
// group-kernel round of the group lane's CUs twice over, i.e. its CUs / 2 since a ciphertext has 4
// group workgroups)
// (read per context at its creation, so that a process can hold contexts of both kinds)
long env_long(const char *name, long dflt) {
    const char *e = std::getenv(name);
    return e && *e ? std::max(0L, std::atol(e)) : dflt;
}
bool large_lanes_on(const TfheMi355Context *c) {
    return c->N() >= 32768 && c->p.pbs_level == 2 && !c->p.grouping_factor && c->lanes_mcus > 0 &&
           c->lanes_mcus * 8 < c->cus;
}
size_t lanes_chunk(const TfheMi355Context *c) {
    if (c->lanes_chunk > 0) return (size_t)c->lanes_chunk;
    return std::max<size_t>(8, ((size_t)c->cus - (size_t)c->lanes_mcus * 8) / 2 / 8 * 8);
}
void make_lanes(TfheMi355Context *c) {
    std::lock_guard<std::mutex> g(c->lanes_mu);
    if (c->lanes_made) return;
    const int cus = c->cus, m = (int)c->lanes_mcus * 8;
    const bool block = c->lanes_block;
    std::vector<uint32_t> mc((cus + 31) / 32, 0), mm((cus + 31) / 32, 0);
    for (int i = 0; i < cus; i++) {
        // interleave: the last m bits (bit i -> XCD i mod 8: m / 8 CUs of every XCD); block: the last
        // m / 8 CUs of each 32-CU run of bits
        const bool mem = block ? (i % (cus / 8)) >= (cus / 8) - m / 8 : i >= cus - m;
        (mem ? mm : mc)[i / 32] |= 1u << (i % 32);
    }
    check(hipSetDevice(c->device), "hipSetDevice");
    check(hipExtStreamCreateWithCUMask(&c->lane_c, (uint32_t)mc.size(), mc.data()), "hipExtStreamCreateWithCUMask");
    check(hipExtStreamCreateWithCUMask(&c->lane_m, (uint32_t)mm.size(), mm.data()), "hipExtStreamCreateWithCUMask");
    c->lanes_made = true;
}

size_t large_chunk(const TfheMi355Context *c) {
    static const size_t forced = [] {
        const char *e = std::getenv("TFHE_MI355_LARGE_CHUNK");
        const long x = e ? std::atol(e) : 0;
        return x > 0 ? (size_t)x : (size_t)0;
    }();
    if (forced) return forced;
    if (large_lanes_on(c)) return 2 * lanes_chunk(c);  // one chunk per lane
    if (c->N() >= 32768) return 128;
    if (c->p.grouping_factor) return 1024;
    const size_t per = large_pbs_scratch_per_ct((int)c->N(), (int)c->k(), (int)c->p.pbs_level);
    return std::min<size_t>(1024, std::max<size_t>(64, ((size_t)200 << 20) / per / 64 * 64));
}

size_t pbs_scratch_bytes(const TfheMi355Context *c, size_t count) {
    if (count == 0 || (c->p.grouping_factor && !is_large(c))) return 0;
    if (!is_large(c)) return classic_pbs_ticket_bytes((int)c->N(), (int)c->k(), (int)c->p.pbs_level);
    const size_t per_ct = large_pbs_scratch_per_ct((int)c->N(), (int)c->k(), (int)c->p.pbs_level);
    return per_ct * std::min(count, large_chunk(c));
}

// The on-chip CMUX (the whole blind rotation in one workgroup: one ciphertext per CU at N = 8192,
// two per CU at N = 4096) against the split CMUX (a ciphertext's sub-blocks over several CUs, in several
// launches per CMUX): at 3_3 the split path takes 16.3 / 18.8 / 23.2 / 25.4 ms for 1 / 64 / 96 / 128
// ciphertexts, the on-chip one 22.9-25.1 ms for any count up to one per CU
// (profiles/r05_sweep33_onchip{0,1}.json); at 1_4 (N = 4096) split 11.0 / 13.3 / 14.0 / 19.3 ms for
// 1 / 96 / 128 / 192, on-chip 18.6-18.9 ms up to two per CU (r05_sweep14_onchip{0,1}.json).  So the
// on-chip kernel from 3/8 (N = 8192) / 5/8 (N = 4096) of the CU count on: 96 / 160 on MI355X.
// TFHE_MI355_ONCHIP_MIN overrides.
size_t onchip_min(const TfheMi355Context *c) {
    static const long env = [] {
        const char *e = std::getenv("TFHE_MI355_ONCHIP_MIN");
        return e && *e ? std::strtol(e, nullptr, 10) : -1L;
    }();
    if (env >= 0) return (size_t)env;
    return c->N() == 4096 ? (size_t)c->cus * 5 / 8 : (size_t)c->cus * 3 / 8;
}

// The quad CMUX (N = 8192, L = 1 or 2 classic, four CUs per ciphertext, pbs_large.hip; N = 4096: two CUs,
// the "duo") for batches of at most this many ciphertexts: one pass of CUs / R by default (R = N / 2048
// sub-blocks); TFHE_MI355_QUAD_MAX overrides (0 = never)
size_t quad_sub_blocks(const TfheMi355Context *c) { return c->N() / 2048; }
size_t quad_max(const TfheMi355Context *c) {
    if ((c->N() != 8192 && c->N() != 4096) || (c->p.pbs_level != 2 && c->p.pbs_level != 1) || c->p.grouping_factor ||
        c->k() != 1)
        return 0;
    static const long env = [] {
        const char *e = std::getenv("TFHE_MI355_QUAD_MAX");
        return e && *e ? std::strtol(e, nullptr, 10) : -1L;
    }();
    return env >= 0 ? (size_t)env : (size_t)c->cus / quad_sub_blocks(c);
}

// Batches of at most this many ciphertexts run the latency kernels (one ciphertext per CU) at the
// shapes they support.  Chosen by predicted time: the latency kernel takes one pass per CU-full of
// ciphertexts, the throughput kernel a time that steps with its ciphertexts per CU (<= 1024 rows:
// small batches spread over the CUs), so latency wins while passes x T_latency < T_throughput.
// Measured at 2_2 (profiles/r05_lat_sweep_{lat,thr}.json, 1..1024 rows): latency 2.54-2.60 ms per
// pass; throughput 5.6 / 6.0 / 8.6 / 8.8 ms at 1 / 2 / 3 / 4 ciphertexts per CU -> the latency
// kernel up to 3 passes (768 rows on 256 CUs: 7.7-8.0 vs 8.6 ms), the throughput kernel from the
// 4th (10.3 vs 8.8 ms).  Multi-bit (profiles/r05_lat_sweep_mb{3,2}_{lat,thr}.json): latency kernel
// 1.8-2.1 ms per pass (g = 3; 2.0 at g = 2), the slot-split throughput kernel 4.7-5.2 ms (g = 3;
// 5.0 at g = 2) for any batch up to 1024 rows -> two passes (512 rows: 4.25 vs 4.72 ms), not three
// (6.0 vs 4.7 ms).  TFHE_MI355_LATENCY_MAX overrides the row count for every shape (0 = never).
constexpr size_t kLatPassesClassic = 3, kLatPassesMb = 2;
size_t latency_max(const TfheMi355Context *c) {
    static const long forced = [] {
        const char *e = std::getenv("TFHE_MI355_LATENCY_MAX");
        return e && *e ? std::max(0L, std::atol(e)) : -1L;
    }();
    if (forced >= 0) return (size_t)forced;
    return (c->p.grouping_factor ? kLatPassesMb : kLatPassesClassic) * (size_t)c->cus;
}

bool ks_use_mfma(const TfheMi355Context *c) {
    static const bool disabled = env_flag("TFHE_MI355_KS_NO_MFMA");
    return !disabled && ks_mfma_supported((int)c->big_dim(), (int)c->p.ks_level, (int)c->p.ks_base_log);
}

size_t ks_scratch_bytes(const TfheMi355Context *c, size_t count) {
    if (!c->ksk_planes_ready && !ks_use_mfma(c)) return 0;
    return count ? ks_mfma_scratch_bytes((int)c->big_dim(), (int)c->p.ks_level, (int)count) : 0;
}

// The packing key's decomposition (base, level) is part of the key, not of the parameter set, so
// this size is defined from the key's upload on (the scratch query fails before it); it follows
// from the decomposition and the MFMA eligibility alone, not from the repack having run.
bool pks_use_mfma(const TfheMi355Context *c) {
    static const bool disabled = env_flag("TFHE_MI355_KS_NO_MFMA");
    return !disabled && c->pks_level &&
           ks_mfma_supported((int)c->big_dim(), (int)c->pks_level, (int)c->pks_base_log);
}
size_t pks_scratch_bytes(const TfheMi355Context *c, size_t count) {
    if (!pks_use_mfma(c) || count == 0) return 0;
    return ks_mfma_scratch_bytes((int)c->big_dim(), (int)c->pks_level, (int)count);
}

// KS -> PBS: the small-LWE intermediate, then (reused in stream order) the KS digits or the PBS
// chunk scratch
size_t ks_pbs_scratch_bytes(const TfheMi355Context *c, size_t count) {
    return align256(count * (c->n() + 1) * 8) + std::max(ks_scratch_bytes(c, count), pbs_scratch_bytes(c, count));
}
// PBS -> KS: the big-LWE intermediate, then the PBS or KS scratch
size_t pbs_ks_scratch_bytes(const TfheMi355Context *c, size_t count) {
    return align256(count * (c->big_dim() + 1) * 8) + std::max(ks_scratch_bytes(c, count), pbs_scratch_bytes(c, count));
}

void require_scratch(size_t have, size_t need) {
    if (have < need) fail("device scratch too small: %zu bytes given, %zu needed (see the *_scratch queries)", have, need);
}

// ---- launchers ---------------------------------------------------------------------------------

void launch_pbs_dev(TfheMi355Context *c, const uint64_t *d_in, uint64_t *d_out, const uint64_t *d_luts,
                    size_t lut_count, const uint32_t *d_idx, size_t count, void *scratch, size_t scratch_bytes,
                    hipStream_t s, bool glwe_out = false) {
    require_fbsk(c);
    if (lut_count == 0) fail("lut_count must be >= 1");
    if (lut_count > 0xffffffffu) fail("lut_count too large");
    if (count > 0x7fffffff) fail("batch too large");
    if (count == 0) return;
    if (c->p.grouping_factor && !is_large(c)) {
        MultiBitPbsLaunch a;
        a.lwe_in = d_in;
        a.lwe_out = d_out;
        a.luts = d_luts;
        a.lut_indexes = d_idx;
        a.lut_count = (uint32_t)lut_count;
        a.fbsk = reinterpret_cast<const double2 *>(c->fbsk.ptr);
        a.W = c->tables.W;
        a.twist = c->tables.twist;
        a.n = (int)c->n();
        a.base_log = (int)c->p.pbs_base_log;
        a.count = (int)count;
        a.glwe_out = glwe_out;
        if (count <= latency_max(c) && latency_multibit_supported((int)c->N(), (int)c->k(), (int)c->p.pbs_level,
                                                                 (int)c->p.grouping_factor)) {
            TimedLaunch tl(c->timer_or_null(), "pbs_mb_latency_kernel", s);
            check(launch_latency_multibit_pbs((int)c->p.grouping_factor, a, s), "launch multi-bit latency pbs");
            return;
        }
        TimedLaunch tl(c->timer_or_null(), "pbs_multibit", s);
        check(launch_multibit_pbs((int)c->N(), (int)c->k(), (int)c->p.pbs_level, (int)c->p.grouping_factor, a, s),
              "launch multi-bit pbs");
        return;
    }
    if (is_large(c)) {
        if (glwe_out) fail("blind rotation without sample extraction is not available at N = %zu", c->N());
        const size_t per_ct = large_pbs_scratch_per_ct((int)c->N(), (int)c->k(), (int)c->p.pbs_level);
        if (!scratch || scratch_bytes < per_ct)
            fail("N = %zu PBS needs >= %zu bytes of device scratch per chunk ciphertext (%zu given)", c->N(), per_ct,
                 scratch_bytes);
        LargePbsLaunch a{};
        a.lwe_in = d_in;
        a.lwe_out = d_out;
        a.luts = d_luts;
        a.lut_indexes = d_idx;
        a.lut_count = (uint32_t)lut_count;
        a.fbsk = reinterpret_cast<const double2 *>(c->fbsk.ptr);
        a.W = c->tables.W;
        a.twist = c->tables.twist;
        a.wtop = c->tables.wtop;
        a.n = (int)c->n();
        a.base_log = (int)c->p.pbs_base_log;
        a.count = (int)count;
        a.scratch = scratch;
        a.scratch_bytes = std::min(scratch_bytes, per_ct * large_chunk(c));
        a.timer = c->timer_or_null();
        a.grouping = (int)c->p.grouping_factor;
        a.onchip_min_count = (int)onchip_min(c);
        a.quad_pass = (int)(c->cus / quad_sub_blocks(c));
        a.quad_max_count = (int)quad_max(c);
        if (a.quad_max_count > 0 && count <= (size_t)a.quad_max_count) {
            if (!c->quad_fail.ptr) {  // created zeroed at the first quad launch of the context
                std::lock_guard<std::mutex> g(c->lanes_mu);
                if (!c->quad_fail.ptr) {
                    c->quad_fail.reserve(4);
                    check(hipMemset(c->quad_fail.ptr, 0, 4), "quad fail word");
                }
            }
            a.quad_fail = static_cast<uint32_t *>(c->quad_fail.ptr);
        }
        if (large_lanes_on(c) && count > lanes_chunk(c)) {  // two chunks in flight at once
            make_lanes(c);
            a.lane_c = c->lane_c;
            a.lane_m = c->lane_m;
        }
        check(launch_large_pbs((int)c->N(), (int)c->k(), (int)c->p.pbs_level, a, s), "launch large pbs");
        return;
    }
    ClassicPbsLaunch a;
    a.lwe_in = d_in;
    a.lwe_out = d_out;
    a.luts = d_luts;
    a.lut_indexes = d_idx;
    a.lut_count = (uint32_t)lut_count;
    a.fbsk = reinterpret_cast<const double2 *>(c->fbsk.ptr);
    a.W = c->tables.W;
    a.twist = c->tables.twist;
    a.n = (int)c->n();
    a.base_log = (int)c->p.pbs_base_log;
    a.count = (int)count;
    a.glwe_out = glwe_out;
    // small batches: the latency kernel (one ciphertext per CU, all 8 waves on it; same outputs)
    if (count <= latency_max(c) && latency_pbs_supported((int)c->N(), (int)c->k(), (int)c->p.pbs_level)) {
#if LAT_STAMPS
        a.ticket = reinterpret_cast<uint32_t *>(scratch);  // diagnostic builds: the stamp buffer
#endif
        TimedLaunch tl(c->timer_or_null(), "pbs_latency_kernel", s);
        check(launch_latency_pbs(a, s), "launch latency pbs");
        return;
    }
    // persistent grid: a zeroed ticket word from the caller's scratch (none given: one pass)
    if (classic_pbs_ticket_bytes((int)c->N(), (int)c->k(), (int)c->p.pbs_level) && scratch && scratch_bytes >= 4) {
        a.ticket = reinterpret_cast<uint32_t *>(scratch);
        check(hipMemsetAsync(a.ticket, 0, sizeof(uint32_t), s), "zero pbs ticket");
    }
    TimedLaunch tl(c->timer_or_null(), "pbs_classic_kernel", s);
    check(launch_classic_pbs((int)c->N(), (int)c->k(), (int)c->p.pbs_level, a, s), "launch pbs");
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

void launch_ks_dev(TfheMi355Context *c, const uint64_t *d_in, uint64_t *d_out, size_t count, void *scratch,
                   size_t scratch_bytes, hipStream_t s) {
    require_ksk(c);
    if (count == 0) return;
    if (count > 0x7fffffffu) fail("count too large");
    KeyswitchLaunch a;
    a.lwe_in = d_in;
    a.lwe_out = d_out;
    a.ksk = reinterpret_cast<const uint64_t *>(c->ksk.ptr);
    a.in_dim = (int)c->big_dim();
    a.out_dim = (int)c->n();
    a.base_log = (int)c->p.ks_base_log;
    a.level = (int)c->p.ks_level;
    a.count = (int)count;
    TimedLaunch tl(c->timer_or_null(), "keyswitch", s);
    if (c->ksk_planes_ready) {
        require_scratch(scratch ? scratch_bytes : 0, ks_scratch_bytes(c, count));
        check(launch_keyswitch_mfma(a, (const int8_t *)c->ksk_planes.ptr, scratch, s), "launch mfma keyswitch");
        return;
    }
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

void launch_packing_ks_dev(TfheMi355Context *c, const uint64_t *d_in, uint64_t *d_out, size_t count, void *scratch,
                           size_t scratch_bytes, hipStream_t s) {
    if (!c->pksk_ready) fail("packing keyswitching key not uploaded");
    if (count == 0) return;
    if (count > 0x7fffffffu) fail("count too large");
    KeyswitchLaunch a = packing_ks_args(c, d_in, d_out, count);
    if (c->pksk_planes_ready) {
        require_scratch(scratch ? scratch_bytes : 0, pks_scratch_bytes(c, count));
        check(launch_keyswitch_mfma(a, (const int8_t *)c->pksk_planes.ptr, scratch, s),
              "launch mfma packing keyswitch");
    } else {
        check(launch_keyswitch(a, s), "launch packing keyswitch");
    }
}

// shortint KS -> PBS on device: scratch = [small LWE intermediate | KS digits or PBS chunk scratch]
void launch_ks_pbs_dev(TfheMi355Context *c, const uint64_t *d_in, uint64_t *d_out, const uint64_t *d_luts,
                       size_t lut_count, const uint32_t *d_idx, size_t count, void *scratch, size_t scratch_bytes,
                       hipStream_t s) {
    require_fbsk(c);
    require_ksk(c);
    if (count == 0) return;
    require_scratch(scratch ? scratch_bytes : 0, ks_pbs_scratch_bytes(c, count));
    const size_t head = align256(count * (c->n() + 1) * 8);
    uint64_t *small = reinterpret_cast<uint64_t *>(scratch);
    void *rest = reinterpret_cast<char *>(scratch) + head;
    launch_ks_dev(c, d_in, small, count, rest, scratch_bytes - head, s);
    launch_pbs_dev(c, small, d_out, d_luts, lut_count, d_idx, count, rest, scratch_bytes - head, s);
}

// shortint PBS -> KS on device: scratch = [big LWE intermediate | PBS or KS scratch]
void launch_pbs_ks_dev(TfheMi355Context *c, const uint64_t *d_in, uint64_t *d_out, const uint64_t *d_luts,
                       size_t lut_count, const uint32_t *d_idx, size_t count, void *scratch, size_t scratch_bytes,
                       hipStream_t s) {
    require_fbsk(c);
    require_ksk(c);
    if (count == 0) return;
    require_scratch(scratch ? scratch_bytes : 0, pbs_ks_scratch_bytes(c, count));
    const size_t head = align256(count * (c->big_dim() + 1) * 8);
    uint64_t *big = reinterpret_cast<uint64_t *>(scratch);
    void *rest = reinterpret_cast<char *>(scratch) + head;
    launch_pbs_dev(c, d_in, big, d_luts, lut_count, d_idx, count, rest, scratch_bytes - head, s);
    launch_ks_dev(c, big, d_out, count, rest, scratch_bytes - head, s);
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

// ---- host-pointer pipeline ------------------------------------------------------------------------
// The synchronous entry points (host buffers in and out, the form the Rust binding calls) run the
// batch in chunks: per chunk, the host input slice is copied into a lane's page-locked buffer and
// DMA'd up on the lane's copy stream, the kernels run on ctx->stream (chunks in order, so the GPU
// stays busy), and the output is DMA'd back on the copy stream and copied into the caller's
// buffer while the next chunk's kernels run.  The LUTs go up once per call.  Callers are
// serialised by ctx->mu.

using ChunkLaunch = void (*)(TfheMi355Context *c, const uint64_t *d_in, uint64_t *d_out, const uint64_t *d_luts,
                             size_t lut_count, const uint32_t *d_idx, size_t count, void *scratch,
                             size_t scratch_bytes, hipStream_t s);
using ScratchSize = size_t (*)(const TfheMi355Context *c, size_t count);

size_t host_chunk(const TfheMi355Context *c, size_t count) {
    static const size_t forced = [] {
        const char *e = std::getenv("TFHE_MI355_HOST_CHUNK");
        const long x = e ? std::atol(e) : 0;
        return x > 0 ? (size_t)x : (size_t)0;
    }();
    if (forced) return forced;
    if (is_large(c)) return large_chunk(c);
    // >= 4 chunks so that copies hide behind kernels (also with pinned caller buffers: 2 chunks
    // measured 93.5k vs 112.9k PBS/s at 4096); >= one full wave of PBS slots (256 CUs x 4
    // ciphertexts) and <= 4 waves per launch
    const size_t slots = 1024;
    const size_t quarter = (count + 3) / 4;
    return std::min<size_t>(4 * slots, std::max(slots, (quarter + slots - 1) / slots * slots));
}

// true when [p, p + bytes) is page-locked host memory (tfhe_mi355_host_alloc, hipHostMalloc or
// hipHostRegister): the pipeline then DMAs straight from / into the caller's buffer
bool is_pinned(const void *p, size_t bytes) {
    if (!p || !bytes) return false;
    for (const void *q : {p, (const void *)((const char *)p + bytes - 1)}) {
        hipPointerAttribute_t at{};
        if (hipPointerGetAttributes(&at, q) != hipSuccess) {
            (void)hipGetLastError();  // pageable memory: clear the non-sticky error
            return false;
        }
        if (at.type != hipMemoryTypeHost) return false;
    }
    return true;
}

void lane_finish(TfheMi355Context::Lane &L, void *out, size_t out_words) {
    if (!L.pending) return;
    L.pending = false;
    check(hipEventSynchronize(L.done), "chunk sync");
    if (!L.direct_out)
        std::memcpy(static_cast<uint64_t *>(out) + L.first * out_words, L.h_out.ptr, L.count * out_words * 8);
}

// after a synchronous call's device work: a quad CMUX launch of this context whose flag wait timed
// out (its partner workgroups never became resident -- e.g. another process's quad grid held the
// CUs) left invalid outputs; fail the call loudly instead of returning them
void check_quad_fail(TfheMi355Context *c) {
    if (!c->quad_fail.ptr) return;
    uint32_t v = 0;
    check(hipMemcpy(&v, c->quad_fail.ptr, 4, hipMemcpyDeviceToHost), "quad fail word");
    if (v) {
        (void)hipMemset(c->quad_fail.ptr, 0, 4);
        fail("quad CMUX: a workgroup waited in vain for its partners (is another process running quad CMUX "
             "kernels on this GPU?); the outputs are invalid -- TFHE_MI355_QUAD=0 disables the quad CMUX");
    }
}

void run_host_pipeline(TfheMi355Context *c, const uint64_t *in, size_t in_words, uint64_t *out, size_t out_words,
                       const uint64_t *luts, size_t lut_words, size_t lut_count, const uint32_t *idx, size_t count,
                       ChunkLaunch launch, ScratchSize scratch_size) {
    if (count == 0) return;
    hipStream_t cs = c->stream;
    const uint64_t *d_luts = nullptr;
    if (luts) {  // on the kernel stream: ordered before every chunk's kernels
        c->io_luts.reserve(lut_count * lut_words * 8);
        check(hipMemcpyAsync(c->io_luts.ptr, luts, lut_count * lut_words * 8, hipMemcpyHostToDevice, cs),
              "H2D luts");
        d_luts = (const uint64_t *)c->io_luts.ptr;
    }
    // page-locked caller buffers are DMA'd directly (no staging copies on the host)
    const bool pin_in = is_pinned(in, count * in_words * 8), pin_out = is_pinned(out, count * out_words * 8);
    const size_t chunk = std::min(count, host_chunk(c, count));
    // kernels of consecutive chunks are ordered on cs: one scratch serves them all
    const size_t need_scratch = scratch_size ? scratch_size(c, chunk) : 0;
    if (need_scratch) c->io_tmp.reserve(need_scratch);
    try {
        size_t next = 0;
        for (int q = 0; next < count; q ^= 1) {
            TfheMi355Context::Lane &L = c->lanes[q];
            lane_finish(L, out, out_words);  // this lane's previous chunk: all its device work is done
            const size_t cnt = std::min(chunk, count - next);
            if (!pin_in) L.h_in.reserve(chunk * in_words * 8);
            if (!pin_out) L.h_out.reserve(chunk * out_words * 8);
            L.d_in.reserve(chunk * in_words * 8);
            L.d_out.reserve(chunk * out_words * 8);
            const uint64_t *src = in + next * in_words;
            if (!pin_in) {
                std::memcpy(L.h_in.ptr, src, cnt * in_words * 8);
                src = (const uint64_t *)L.h_in.ptr;
            }
            check(hipMemcpyAsync(L.d_in.ptr, src, cnt * in_words * 8, hipMemcpyHostToDevice, L.stream), "H2D in");
            const uint32_t *d_idx = nullptr;
            if (idx) {
                L.h_idx.reserve(chunk * 4);
                L.d_idx.reserve(chunk * 4);
                std::memcpy(L.h_idx.ptr, idx + next, cnt * 4);
                check(hipMemcpyAsync(L.d_idx.ptr, L.h_idx.ptr, cnt * 4, hipMemcpyHostToDevice, L.stream), "H2D idx");
                d_idx = (const uint32_t *)L.d_idx.ptr;
            }
            check(hipEventRecord(L.h2d, L.stream), "h2d event");
            check(hipStreamWaitEvent(cs, L.h2d, 0), "wait h2d");
            launch(c, (const uint64_t *)L.d_in.ptr, (uint64_t *)L.d_out.ptr, d_luts, lut_count, d_idx, cnt,
                   need_scratch ? c->io_tmp.ptr : nullptr, need_scratch ? c->io_tmp.bytes : 0, cs);
            check(hipEventRecord(L.kern, cs), "kernel event");
            check(hipStreamWaitEvent(L.stream, L.kern, 0), "wait kernels");
            L.direct_out = pin_out;
            check(hipMemcpyAsync(pin_out ? (void *)(out + next * out_words) : L.h_out.ptr, L.d_out.ptr,
                                 cnt * out_words * 8, hipMemcpyDeviceToHost, L.stream),
                  "D2H out");
            check(hipEventRecord(L.done, L.stream), "chunk event");
            L.pending = true;
            L.first = next;
            L.count = cnt;
            next += cnt;
        }
        // retire in chunk order: the lane holding the older chunk first
        TfheMi355Context::Lane &a = c->lanes[0], &b = c->lanes[1];
        if (a.pending && b.pending && b.first < a.first) {
            lane_finish(b, out, out_words);
            lane_finish(a, out, out_words);
        } else {
            lane_finish(a, out, out_words);
            lane_finish(b, out, out_words);
        }
        check_quad_fail(c);
    } catch (...) {
        (void)hipStreamSynchronize(cs);
        for (auto &L : c->lanes) {
            (void)hipStreamSynchronize(L.stream);
            L.pending = false;
        }
        throw;
    }
}

// adapters of the launchers to ChunkLaunch
void chunk_pbs(TfheMi355Context *c, const uint64_t *i, uint64_t *o, const uint64_t *l, size_t lc, const uint32_t *x,
               size_t n, void *sc, size_t sb, hipStream_t s) {
    launch_pbs_dev(c, i, o, l, lc, x, n, sc, sb, s);
}
void chunk_blind_rotate(TfheMi355Context *c, const uint64_t *i, uint64_t *o, const uint64_t *l, size_t lc,
                        const uint32_t *x, size_t n, void *sc, size_t sb, hipStream_t s) {
    launch_pbs_dev(c, i, o, l, lc, x, n, sc, sb, s, true);
}
void chunk_ks(TfheMi355Context *c, const uint64_t *i, uint64_t *o, const uint64_t *, size_t, const uint32_t *,
              size_t n, void *sc, size_t sb, hipStream_t s) {
    launch_ks_dev(c, i, o, n, sc, sb, s);
}
void chunk_pks(TfheMi355Context *c, const uint64_t *i, uint64_t *o, const uint64_t *, size_t, const uint32_t *,
               size_t n, void *sc, size_t sb, hipStream_t s) {
    launch_packing_ks_dev(c, i, o, n, sc, sb, s);
}

// ---- request coalescing ---------------------------------------------------------------------------
// Calls of at most coalesce_max_count() ciphertexts (default 64; TFHE_MI355_COALESCE_MAX_COUNT,
// 0 = off) are coalesced: up to coalesce_batch() ciphertexts (default 1024, one ciphertext per PBS
// slot of the chip at 2_2) gathered until no call has arrived for coalesce_gap() (default 50 us),
// for at most coalesce_window() (default 1000 us) from the first queued call.  Both are small next
// to a PBS (milliseconds), and a full batch leaves at once.
size_t env_size(const char *name, size_t dflt) {
    const char *e = std::getenv(name);
    if (!e || !*e) return dflt;
    const long x = std::atol(e);
    return x >= 0 ? (size_t)x : dflt;
}
size_t coalesce_batch() {
    static const size_t v = std::max<size_t>(env_size("TFHE_MI355_COALESCE_BATCH", 1024), 1);
    return v;
}
// never above the batch size: a dispatcher always takes its queue's first request whole, and the
// slot staging is sized for one batch
size_t coalesce_max_count() {
    static const size_t v = std::min(env_size("TFHE_MI355_COALESCE_MAX_COUNT", 64), coalesce_batch());
    return v;
}
// batch slots (dispatcher threads, up to 8): batches in flight at once, each on its own stream.
// A PBS batch takes about one CMUX chain (6-9 ms at 2_2) whatever its size up to a chip-full, so
// by Little's law T callers get at most T / (chain + window) calls/s; a second slot that starts
// whenever work is queued only splits the callers into half batches that the device does not
// overlap (measured at 64 / 256 synchronous callers: 1 slot 10.4k / 37.5k calls/s, 2 slots
// 10.3k / 30.4k, 3 slots 7.6k / 26.7k).  So a slot other than the first starts only when
// coalesce_overflow() rows are queued (coalesce_dispatcher): synchronous callers see one slot,
// while submit/wait callers with thousands of requests in flight overlap host staging with the
// device (64 threads x 64 in flight: 92k calls/s with 1 slot, 108-113k with 2).  Default 2.
size_t coalesce_slots() {
    static const size_t v = std::min<size_t>(std::max<size_t>(env_size("TFHE_MI355_COALESCE_SLOTS", 2), 1), 8);
    return v;
}
// queued ciphertexts of one op that start a batch on a second slot while another runs (default
// half a batch: 16 threads x 64 submitted requests 62.6k calls/s at a full batch, 67.5k at half;
// 256 synchronous callers never queue that many, so they keep one slot)
size_t coalesce_overflow() {
    static const size_t v = std::max<size_t>(env_size("TFHE_MI355_COALESCE_OVERFLOW", coalesce_batch() / 2), 1);
    return v;
}
std::chrono::microseconds coalesce_window() {
    static const size_t v = env_size("TFHE_MI355_COALESCE_WINDOW_US", 1000);
    return std::chrono::microseconds(v);
}
// the batch also closes once no request of its op has arrived for this long: callers woken one by
// one after a batch (or a thread submitting a burst) re-queue within microseconds of each other
std::chrono::microseconds coalesce_gap() {
    static const size_t v = env_size("TFHE_MI355_COALESCE_GAP_US", 50);
    return std::chrono::microseconds(v);
}

struct CoalescedOpDesc {
    size_t in_words, out_words;
    bool lut;
    ChunkLaunch launch;
    ScratchSize scratch;
};
CoalescedOpDesc coalesced_op(const TfheMi355Context *c, CoalescedOp op) {
    const size_t small = c->n() + 1, big = c->big_dim() + 1;
    switch (op) {
        case CO_PBS: return {small, big, true, chunk_pbs, pbs_scratch_bytes};
        case CO_KS_PBS: return {big, big, true, launch_ks_pbs_dev, ks_pbs_scratch_bytes};
        case CO_PBS_KS: return {small, small, true, launch_pbs_ks_dev, pbs_ks_scratch_bytes};
        default: return {big, small, false, chunk_ks, ks_scratch_bytes};
    }
}

// one batch on one slot: concatenated inputs, LUT sets deduplicated by pointer with per-row LUT
// indexes shifted to the set's offset, one launch of the _async path on the slot's stream
void run_coalesced_batch(TfheMi355Context *c, TfheMi355Context::Coalescer::Slot &sl, CoalescedOp op,
                         const std::vector<CoalescedReq *> &batch) {
    check(hipSetDevice(c->device), "hipSetDevice");
    const CoalescedOpDesc d = coalesced_op(c, op);
    if (!sl.stream) check(hipStreamCreateWithFlags(&sl.stream, hipStreamNonBlocking), "hipStreamCreate(slot)");
    // the previous batch's blocking callers copy their rows out of h_out themselves (a few us each)
    while (sl.copies.load(std::memory_order_acquire) != 0) std::this_thread::yield();
    size_t total = 0;
    for (auto *r : batch) total += r->count;
    // sized for a full batch once (no hipFree between batches: it would wait for the device); a
    // batch is at most `cap` rows (coalesce_max_count() <= cap, submit counts <= cap), the max()
    // keeps the copies below in bounds whatever the settings
    const size_t cap = std::max(coalesce_batch(), total), glwe = c->glwe_len();
    sl.h_out.reserve(cap * d.out_words * 8);
    sl.d_out.reserve(cap * d.out_words * 8);
    const size_t scratch = d.scratch(c, cap);
    if (scratch) sl.d_scratch.reserve(scratch);
    size_t rows = 0, sets = 0;
    std::vector<std::pair<const uint64_t *, size_t>> seen;  // LUT pointer -> first set index
    std::vector<size_t> seen_count;                           // its lut_count
    std::vector<size_t> base(batch.size(), 0);
    if (d.lut) {  // distinct LUT sets (by pointer) and their offsets
        for (size_t b = 0; b < batch.size(); b++) {
            const CoalescedReq *r = batch[b];
            base[b] = (size_t)-1;
            for (size_t q = 0; q < seen.size(); q++)  // same buffer, same number of tables
                if (seen[q].first == r->luts && seen_count[q] == r->lut_count) base[b] = seen[q].second;
            if (base[b] == (size_t)-1) {
                base[b] = sets;
                seen.push_back({r->luts, sets});
                seen_count.push_back(r->lut_count);
                sets += r->lut_count;
            }
        }
    }
    // ONE host->device copy per batch: [LUT sets | input rows | per-row LUT indexes (> 1 set)] packed
    // in the slot's pinned staging and its device twin (each copy is a DMA with its own ~10 us of
    // setup: a one-ciphertext call paid three of them).  Capacity: a full batch of rows plus the
    // sets seen so far, grown (rarely) on demand.
    const size_t lut_bytes = d.lut ? sets * glwe * 8 : 0;
    const size_t in_off = align256(lut_bytes), in_bytes = total * d.in_words * 8;
    const bool with_idx = d.lut && sets > 1;
    const size_t idx_off = align256(in_off + in_bytes), span = idx_off + (with_idx ? total * 4 : 0);
    const size_t room = align256(lut_bytes) + align256(cap * d.in_words * 8) + cap * 4;
    sl.h_in.reserve(std::max(span, room));
    sl.d_in.reserve(std::max(span, room));
    char *hs = static_cast<char *>(sl.h_in.ptr);
    for (size_t q = 0; q < seen.size(); q++)
        std::memcpy(hs + seen[q].second * glwe * 8, seen[q].first, seen_count[q] * glwe * 8);
    uint32_t *hidx = reinterpret_cast<uint32_t *>(hs + idx_off);
    for (size_t b = 0; b < batch.size(); b++) {
        const CoalescedReq *r = batch[b];
        std::memcpy(hs + in_off + rows * d.in_words * 8, r->in, r->count * d.in_words * 8);
        if (with_idx)
            for (size_t i = 0; i < r->count; i++) hidx[rows + i] = (uint32_t)(base[b] + (r->idx ? r->idx[i] : 0));
        rows += r->count;
    }
    const hipStream_t s = sl.stream;
    check(hipMemcpyAsync(sl.d_in.ptr, sl.h_in.ptr, span, hipMemcpyHostToDevice, s), "H2D batch");
    char *ds = static_cast<char *>(sl.d_in.ptr);
    d.launch(c, (const uint64_t *)(ds + in_off), (uint64_t *)sl.d_out.ptr, (const uint64_t *)ds,
             d.lut ? sets : 0, with_idx ? (const uint32_t *)(ds + idx_off) : nullptr, total,
             scratch ? sl.d_scratch.ptr : nullptr, scratch ? sl.d_scratch.bytes : 0, s);
    check(hipMemcpyAsync(sl.h_out.ptr, sl.d_out.ptr, total * d.out_words * 8, hipMemcpyDeviceToHost, s), "D2H batch");
    check(hipStreamSynchronize(s), "batch sync");
    check_quad_fail(c);
    rows = 0;
    int deferred = 0;
    for (auto *r : batch) {
        const uint64_t *src = static_cast<uint64_t *>(sl.h_out.ptr) + rows * d.out_words;
        if (r->sync) {  // copied by its caller after the wake-up (coalesce_wait)
            r->src = src;
            r->src_bytes = r->count * d.out_words * 8;
            r->pending = &sl.copies;
            deferred++;
        } else {
            std::memcpy(r->out, src, r->count * d.out_words * 8);
        }
        rows += r->count;
    }
    sl.copies.store(deferred, std::memory_order_release);  // before any caller is woken
}

// dispatcher of batch slot q: waits for queued work, lets the window fill the batch, takes the
// longest-waiting op's queue (up to a full batch) and runs it; callers are woken one by one
void coalesce_dispatcher(TfheMi355Context *c, size_t q) {
    auto &co = c->co;
    auto &sl = co.slots[q];
    const size_t cap = coalesce_batch();
    size_t rr = 0;  // round robin over the ops
    for (;;) {
        std::vector<CoalescedReq *> batch;
        CoalescedOp op = CO_PBS;
        size_t cts = 0;
        {
            std::unique_lock<std::mutex> lk(co.m);
            auto pending = [&] {
                for (int o = 0; o < CO_OPS; o++)
                    if (!co.queue[o].empty()) return true;
                return false;
            };
            auto full = [&] {
                for (int o = 0; o < CO_OPS; o++)
                    if (co.queued[o] >= coalesce_overflow()) return true;
                return false;
            };
            // a batch starts when no other slot is busy, or when a full batch is waiting (overflow:
            // callers with many requests in flight, e.g. through tfhe_mi355_submit)
            co.cv.wait(lk, [&] { return co.stop || (pending() && (co.in_flight == 0 || full())); });
            if (co.stop && !pending()) return;
            co.max_in_flight = std::max(co.max_in_flight, ++co.in_flight);  // claimed before the window
            for (int k = 0; k < CO_OPS; k++) {
                const int o = (int)((rr + k) % CO_OPS);
                if (!co.queue[o].empty()) {
                    op = (CoalescedOp)o;
                    break;
                }
            }
            rr = (size_t)op + 1;
            // the window also closes as soon as the blocking callers of the op's previous batch can
            // all be back (as many blocking rows queued as it had; each such caller has one call
            // outstanding).  Submitted requests keep the gap rule: a burst from one thread says
            // nothing about how many more are coming.
            const auto close = std::chrono::steady_clock::now() + coalesce_window();
            while (!co.stop && co.queued[op] < cap &&
                   !(co.last_sync_rows[op] && co.queued_sync[op] >= co.last_sync_rows[op])) {
                const auto t = std::min(close, co.last_arrival[op] + coalesce_gap());
                if (std::chrono::steady_clock::now() >= t) break;
                co.cv.wait_until(lk, t);
            }
            auto &qu = co.queue[op];
            size_t take = 0;
            size_t sync_rows = 0;
            while (take < qu.size() && (batch.empty() || cts + qu[take]->count <= cap)) {
                cts += qu[take]->count;
                if (qu[take]->sync) sync_rows += qu[take]->count;
                batch.push_back(qu[take++]);
            }
            qu.erase(qu.begin(), qu.begin() + take);
            co.queued[op] -= cts;
            co.queued_sync[op] -= sync_rows;
            if (batch.empty()) {  // another slot took the queue during the window
                co.in_flight--;
                continue;
            }
            co.last_sync_rows[op] = sync_rows == cts ? cts : 0;  // only a batch that ran says how many callers
            if (full()) co.cv.notify_one();  // another full batch: an idle slot can run it now
        }
        std::string err;
        const auto t0 = std::chrono::steady_clock::now();
        try {
            KeyRead keys(c);  // no key upload mid-batch
            run_coalesced_batch(c, sl, op, batch);
        } catch (const std::exception &ex) {
            err = ex.what();
        }
        const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        for (auto *x : batch) {  // notified under its lock: the caller may free x as soon as it wakes
            std::lock_guard<std::mutex> g(x->m);
            x->err = err;
            x->done = true;
            x->cv.notify_one();
        }
        {  // the slot counts as busy until its callers are all woken, so the next batch's window
           // (on whichever slot) starts after they have had the chance to queue again
            std::lock_guard<std::mutex> g(co.m);
            co.in_flight--;
            co.batches++;
            co.rows += cts;
            co.batch_seconds += dt;
        }
        co.cv.notify_one();  // a slot waiting for this one to finish
    }
}

// a request joins its op's queue (the dispatchers start with the first one)
void coalesce_enqueue(TfheMi355Context *c, CoalescedOp op, CoalescedReq &r) {
    auto &co = c->co;
    {
        std::lock_guard<std::mutex> g(co.m);
        if (co.workers.empty())
            for (size_t q = 0; q < coalesce_slots(); q++) co.workers.emplace_back(coalesce_dispatcher, c, q);
        co.queue[op].push_back(&r);
        co.queued[op] += r.count;
        if (r.sync) co.queued_sync[op] += r.count;
        co.last_arrival[op] = std::chrono::steady_clock::now();
    }
    co.cv.notify_one();
}

void coalesce_wait(CoalescedReq &r) {
    {
        std::unique_lock<std::mutex> lk(r.m);
        r.cv.wait(lk, [&] { return r.done; });
    }
    if (r.pending) {  // this caller's rows are in the slot's staging: copy them, release the slot
        std::memcpy(r.out, r.src, r.src_bytes);
        r.pending->fetch_sub(1, std::memory_order_release);
    }
    if (!r.err.empty()) fail("%s", r.err.c_str());
}

// A synchronous call that finds the coalescer idle (nothing queued, no batch in flight) runs at once
// on the calling thread as a batch of its own, on slot 8 (TFHE_MI355_COALESCE_DIRECT=0: never):
// it skips the batching window and two thread hand-offs (~0.1 ms of a ~2.6 ms call).  It is not
// counted in in_flight, so calls arriving meanwhile are batched by the dispatchers on their own
// slots and run beside it (the latency kernel puts each ciphertext on its own CU).
bool coalesce_direct() {
    static const bool v = env_size("TFHE_MI355_COALESCE_DIRECT", 1) != 0;
    return v;
}

// the calling thread's request joins its op's queue and waits for its own completion
void coalesced_call(TfheMi355Context *c, CoalescedOp op, CoalescedReq &r) {
    auto &co = c->co;
    bool direct = false;
    if (coalesce_direct()) {
        std::lock_guard<std::mutex> g(co.m);
        // ... and only while this entry point's traffic is one blocking caller at a time (its last
        // dispatcher batch had at most one blocking row): with several callers a direct call would
        // split their batch in two
        bool idle = !co.stop && !co.direct_busy && co.in_flight == 0 && co.last_sync_rows[op] <= 1;
        for (int o = 0; o < CO_OPS && idle; o++) idle = co.queue[o].empty();
        if (idle) co.direct_busy = direct = true;
    }
    if (!direct) {
        r.sync = true;
        coalesce_enqueue(c, op, r);
        coalesce_wait(r);
        return;
    }
    std::string err;
    const auto t0 = std::chrono::steady_clock::now();
    try {
        KeyRead keys(c);  // no key upload mid-batch
        const std::vector<CoalescedReq *> one{&r};
        run_coalesced_batch(c, co.slots[8], op, one);
    } catch (const std::exception &ex) {
        err = ex.what();
    }
    {
        std::lock_guard<std::mutex> g(co.m);
        co.direct_busy = false;
        co.batches++;
        co.rows += r.count;
        co.batch_seconds += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    }
    if (!err.empty()) fail("%s", err.c_str());
}

bool coalescible(size_t count) { return count > 0 && count <= coalesce_max_count(); }

// an ABI call made from inside another one: its failure text becomes ours
void abi(int rc) {
    if (rc != TFHE_MI355_OK) fail("%s", tfhe_mi355_last_error());
}

// ---- multi-device contexts ----------------------------------------------------------------------
// SURVEY.md 8b `ctx_create(params, device_mask)` / 8e: ONE process drives several GPUs through one
// context, the way the reference's one process drives its rayon pool (a thread-local ShortintEngine
// per worker, shortint/engine/mod.rs:23-25, and one KS+PBS per block from par_iter,
// integer/server_key/radix_parallel/mul.rs:347-407, through the ShortintBootstrappingKey arms,
// shortint/server_key/mod.rs:104-111,783-857).  A multi-device context owns one single-device context
// ("shard") per listed device; a device may be listed more than once (shards on one GPU then run
// side by side on their own streams).
//   keys: uploaded once, to the first shard, and replicated from its device memory: an RCCL
//     broadcast over xGMI among the distinct devices (librccl opened at run time; ncclCommInitAll
//     over the device list, one rank per distinct device), then device-to-device copies to further
//     shards on the same device.  TFHE_MI355_REPLICATE=copy uses peer copies instead of RCCL,
//     =rccl forces the broadcast even with one distinct device (a one-rank communicator copying
//     into the second shard of that device; a test hook);
//   batched host-pointer calls: split into contiguous shares, one per shard, each run by the shard's
//     own entry point on a thread of its own (its own stream, staging, lock) and joined before the
//     call returns;
//   small calls (the coalesced ones) and submitted requests: round-robin to the shards' coalescers;
//   device-pointer (_async) calls and their scratch queries: the first device's shard (a device
//     pointer belongs to one device; tfhe_mi355_context_device_context hands out each shard).
}  // namespace

struct RcclComms {
    void *lib = nullptr;
    decltype(&ncclCommInitAll) init_all = nullptr;
    decltype(&ncclBroadcast) broadcast = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    std::vector<int> devices;  // rank -> device
    std::vector<ncclComm_t> comms;
    ~RcclComms() {
        for (size_t r = 0; r < comms.size(); r++)
            if (comms[r] && comm_destroy) {
                (void)hipSetDevice(devices[r]);
                (void)comm_destroy(comms[r]);
            }
        if (lib) dlclose(lib);
    }
};

namespace {

void check_nccl(const RcclComms &rc, ncclResult_t r, const char *what) {
    if (r != ncclSuccess) fail("%s: %s", what, rc.error_string ? rc.error_string(r) : "RCCL error");
}

// the communicator over `devices` (rank 0 = the source's device), created once per context
RcclComms &rccl_for(TfheMi355Context *m, const std::vector<int> &devices) {
    if (m->rccl && m->rccl->devices == devices) return *m->rccl;
    delete m->rccl;
    m->rccl = nullptr;
    auto rc = std::make_unique<RcclComms>();
    rc->lib = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!rc->lib) rc->lib = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
    if (!rc->lib) fail("RCCL is not available for key replication (%s); TFHE_MI355_REPLICATE=copy uses peer copies",
                       dlerror());
    auto sym = [&](const char *name) {
        void *f = dlsym(rc->lib, name);
        if (!f) fail("librccl lacks %s", name);
        return f;
    };
    rc->init_all = reinterpret_cast<decltype(rc->init_all)>(sym("ncclCommInitAll"));
    rc->broadcast = reinterpret_cast<decltype(rc->broadcast)>(sym("ncclBroadcast"));
    rc->group_start = reinterpret_cast<decltype(rc->group_start)>(sym("ncclGroupStart"));
    rc->group_end = reinterpret_cast<decltype(rc->group_end)>(sym("ncclGroupEnd"));
    rc->comm_destroy = reinterpret_cast<decltype(rc->comm_destroy)>(sym("ncclCommDestroy"));
    rc->error_string = reinterpret_cast<decltype(rc->error_string)>(sym("ncclGetErrorString"));
    rc->devices = devices;
    rc->comms.assign(devices.size(), nullptr);
    check_nccl(*rc, rc->init_all(rc->comms.data(), (int)devices.size(), devices.data()), "ncclCommInitAll");
    m->rccl = rc.release();
    return *m->rccl;
}

// TFHE_MI355_REPLICATE: "auto" (default), "rccl", "copy" ("fail": a replication failure, test hook)
std::string replicate_mode() {
    const char *e = std::getenv("TFHE_MI355_REPLICATE");
    return e && *e ? std::string(e) : std::string("auto");
}

enum class KeyPart { Fourier, Ksk };

// shard 0's key part -> every other shard (see above); the ready flags are the caller's business
void replicate(TfheMi355Context *m, KeyPart part) {
    auto &S = m->shards;
    TfheMi355Context *src = S[0];
    const size_t bytes = part == KeyPart::Fourier ? src->fourier_bsk_bytes() : src->ksk_len() * sizeof(uint64_t);
    auto buffer = [&](TfheMi355Context *s) -> DeviceBuffer & { return part == KeyPart::Fourier ? s->fbsk : s->ksk; };
    if (!buffer(src).ptr || buffer(src).bytes < bytes) fail("no key on the first device to replicate");
    // distinct devices in order of first appearance (rank 0: the source's) and the shards on each
    std::vector<int> devs;
    std::vector<std::vector<size_t>> on;
    for (size_t i = 0; i < S.size(); i++) {
        const auto it = std::find(devs.begin(), devs.end(), S[i]->device);
        if (it == devs.end()) {
            devs.push_back(S[i]->device);
            on.push_back({i});
        } else {
            on[it - devs.begin()].push_back(i);
        }
    }
    for (size_t i = 1; i < S.size(); i++) {
        check(hipSetDevice(S[i]->device), "hipSetDevice");
        buffer(S[i]).reserve(bytes);
    }
    // the shard of each device that receives the broadcast: the first one on it (on the source's
    // device: a second shard there, else the source itself, in place)
    std::vector<size_t> holder(devs.size());
    for (size_t r = 0; r < devs.size(); r++) holder[r] = r == 0 && on[0].size() > 1 ? on[0][1] : on[r][0];
    const std::string mode = replicate_mode();
    m->replicate_note.clear();
    if (mode == "fail") fail("key replication failed (TFHE_MI355_REPLICATE=fail test hook)");
    bool use_rccl = mode == "rccl" || (mode != "copy" && devs.size() > 1);
    RcclComms *rcp = nullptr;
    if (use_rccl) {
        try {
            rcp = &rccl_for(m, devs);
        } catch (const Failure &e) {
            if (mode == "rccl") throw;
            // auto: librccl missing or its communicator refused -> the peer-copy path
            m->replicate_note = std::string("RCCL unavailable, peer copies: ") + e.what();
            use_rccl = false;
        }
    }
    auto sync_all = [&] {
        for (auto *s : S) {
            check(hipSetDevice(s->device), "hipSetDevice");
            check(hipStreamSynchronize(s->stream), "key replication sync");
        }
    };
    check(hipSetDevice(src->device), "hipSetDevice");
    check(hipStreamSynchronize(src->stream), "key source sync");
    m->replication = use_rccl ? TFHE_MI355_REPLICATION_RCCL
                     : devs.size() > 1 ? TFHE_MI355_REPLICATION_PEER_COPY : TFHE_MI355_REPLICATION_DEVICE_COPY;
    if (use_rccl) {
        RcclComms &rc = *rcp;
        check_nccl(rc, rc.group_start(), "ncclGroupStart");
        for (size_t r = 0; r < devs.size(); r++) {
            check(hipSetDevice(devs[r]), "hipSetDevice");
            TfheMi355Context *h = S[holder[r]];
            const ncclResult_t e =
                rc.broadcast(buffer(src).ptr, buffer(h).ptr, bytes, ncclUint8, 0, rc.comms[r], h->stream);
            if (e != ncclSuccess) {
                (void)rc.group_end();
                check_nccl(rc, e, "ncclBroadcast");
            }
        }
        check_nccl(rc, rc.group_end(), "ncclGroupEnd");
    } else {
        for (size_t r = 0; r < devs.size(); r++) {
            if (holder[r] == 0) continue;
            TfheMi355Context *h = S[holder[r]];
            check(hipSetDevice(h->device), "hipSetDevice");
            check(h->device == src->device
                      ? hipMemcpyAsync(buffer(h).ptr, buffer(src).ptr, bytes, hipMemcpyDeviceToDevice, h->stream)
                      : hipMemcpyPeerAsync(buffer(h).ptr, h->device, buffer(src).ptr, src->device, bytes, h->stream),
                  "key peer copy");
        }
    }
    sync_all();
    for (size_t r = 0; r < devs.size(); r++)  // the other shards of each device: from its holder
        for (size_t i : on[r]) {
            if (i == 0 || i == holder[r]) continue;
            check(hipSetDevice(S[i]->device), "hipSetDevice");
            check(hipMemcpyAsync(buffer(S[i]).ptr, buffer(S[holder[r]]).ptr, bytes, hipMemcpyDeviceToDevice,
                                 S[i]->stream),
                  "key device copy");
        }
    if (part == KeyPart::Ksk)  // each shard repacks its own byte planes for the MFMA keyswitch
        for (size_t i = 1; i < S.size(); i++) {
            check(hipSetDevice(S[i]->device), "hipSetDevice");
            repack_ksk(S[i], S[i]->stream);
        }
    sync_all();
    check(hipSetDevice(src->device), "hipSetDevice");
}

// the context itself, or the first shard of a multi-device one (device-pointer calls)
TfheMi355Context *primary(TfheMi355Context *c) { return c && c->multi() ? c->shards[0] : c; }

// the shard that takes the next small call / submitted request
TfheMi355Context *pick_shard(TfheMi355Context *m) {
    return m->shards[m->next_shard.fetch_add(1, std::memory_order_relaxed) % m->shards.size()];
}

// key writes of a multi-device context: its own lock (uploads in turn), then every shard's (no
// coalesced batch on any device while the key changes)
std::vector<std::unique_ptr<KeyWrite>> key_write_all(TfheMi355Context *c) {
    std::vector<std::unique_ptr<KeyWrite>> w;
    w.emplace_back(new KeyWrite(c));
    for (auto *s : c->shards) w.emplace_back(new KeyWrite(s));
    return w;
}

void set_ready_all(TfheMi355Context *m, KeyPart part, bool ready) {
    for (auto *s : m->shards) {
        if (part == KeyPart::Fourier) s->fbsk_ready = ready;
        else s->ksk_ready = ready;
    }
}

// a batched host-pointer call of a multi-device context: shard i runs rows [count i / S, count (i+1)
// / S) through `f(shard, first, count)` (an entry point of the shard, 0 = ok), shard 0 on the calling
// thread and the others on threads of their own; joined, then the first failure is reported
// The whole call holds the multi-device context's key lock shared, so a concurrent key upload
// (key_write_all: this context exclusively first) lands before or after it, never between two
// shards' shares.
template <class F>
void split_rows(TfheMi355Context *m, size_t count, F &&f) {
    const size_t S = m->shards.size();
    KeyRead keys(m);
    std::vector<std::string> errs(S);
    auto run = [&](size_t i) {
        const size_t a = count * i / S, b = count * (i + 1) / S;
        if (a == b) return;
        try {
            if (f(m->shards[i], a, b - a) != TFHE_MI355_OK) errs[i] = tfhe_mi355_last_error();
        } catch (const std::exception &e) {
            errs[i] = e.what();
        }
    };
    std::mutex dm;
    std::condition_variable dcv;
    size_t left = 0;
    for (size_t i = 1; i < S; i++) {
        if (count * i / S == count * (i + 1) / S) continue;
        left++;
        m->workers[i - 1]->post([&, i] {
            run(i);
            std::lock_guard<std::mutex> g(dm);
            if (--left == 0) dcv.notify_one();
        });
    }
    run(0);
    {
        std::unique_lock<std::mutex> g(dm);
        dcv.wait(g, [&] { return left == 0; });
    }
    for (size_t i = 0; i < S; i++)
        if (!errs[i].empty()) fail("device %d (shard %zu): %s", m->shards[i]->device, i, errs[i].c_str());
}

// peer access between every two distinct devices of a multi-device context, so that the peer-copy
// replication (TFHE_MI355_REPLICATE=copy, or auto without RCCL) is a direct xGMI copy rather than
// a staged one; a pair the platform cannot map keeps the staged path (not an error)
void enable_peer_access(const std::vector<int> &devs) {
    std::vector<int> d = devs;
    std::sort(d.begin(), d.end());
    d.erase(std::unique(d.begin(), d.end()), d.end());
    for (int a : d)
        for (int b : d) {
            if (a == b) continue;
            int can = 0;
            if (hipDeviceCanAccessPeer(&can, a, b) != hipSuccess || !can) continue;
            if (hipSetDevice(a) != hipSuccess) continue;
            (void)hipDeviceEnablePeerAccess(b, 0);  // hipErrorPeerAccessAlreadyEnabled is fine too
            (void)hipGetLastError();                 // ... and leaves its code behind
        }
}

// parameter checks shared by the single- and multi-device constructors
void validate_parameters(const TfheMi355Parameters &p) {
    if (!is_pow2(p.polynomial_size)) fail("polynomial_size must be a power of two");
    if (p.grouping_factor != 0) {
        if (!multibit_pbs_supported((int)p.polynomial_size, (int)p.glwe_dimension, (int)p.pbs_level,
                                    (int)p.grouping_factor) &&
            !large_multibit_supported((int)p.polynomial_size, (int)p.glwe_dimension, (int)p.pbs_level,
                                      (int)p.grouping_factor))
            fail("no multi-bit kernel for N=%u k=%u pbs_level=%u grouping_factor=%u", p.polynomial_size,
                 p.glwe_dimension, p.pbs_level, p.grouping_factor);
        if (p.lwe_dimension % p.grouping_factor)
            fail("lwe_dimension %u is not a multiple of grouping_factor %u", p.lwe_dimension, p.grouping_factor);
    } else if (!classic_pbs_supported((int)p.polynomial_size, (int)p.glwe_dimension, (int)p.pbs_level) &&
               !large_pbs_supported((int)p.polynomial_size, (int)p.glwe_dimension, (int)p.pbs_level)) {
        fail("no kernel for N=%u k=%u pbs_level=%u", p.polynomial_size, p.glwe_dimension, p.pbs_level);
    }
    // the N <= 2048 kernels (and the grouped N = 32768 CMUX) decompose in 32-bit registers;
    // the split CMUX of N >= 4096 in 64-bit ones (the shortint sets reach 11 x 3 = 33 bits)
    const bool split = !p.grouping_factor && p.polynomial_size >= 4096;
    const uint32_t max_bits = split ? 63 : 30;
    if (p.pbs_base_log < 2 || p.pbs_base_log * p.pbs_level > max_bits)
        fail("pbs decomposition base_log*level must be in [2, %u] (got %u x %u)", max_bits, p.pbs_base_log,
             p.pbs_level);
    // the split CMUX keeps the lower levels' digits as int16 between passes: a signed digit lies
    // in [-2^(beta-1), 2^(beta-1)], so beta <= 15 (beta = 16 would wrap +2^15 to -2^15); this
    // also keeps the grouped N = 32768, L = 2 path's 32-bit decomposition at beta * L <= 30
    if (split && p.pbs_level > 1 && p.pbs_base_log > 15)
        fail("pbs base_log %u > 15 with %u levels at N = %u (digits are packed as int16)", p.pbs_base_log,
             p.pbs_level, p.polynomial_size);
    if (p.ks_level && (p.ks_base_log == 0 || p.ks_base_log * p.ks_level >= 64)) fail("invalid ks decomposition");
    if (p.lwe_dimension == 0) fail("lwe_dimension must be > 0");
}

TfheMi355Context *create_single(const TfheMi355Parameters &p, int device) {
    check(hipSetDevice(device), "hipSetDevice");
    auto *c = new TfheMi355Context();
    c->p = p;
    c->device = device;
    c->lanes_mcus = env_long("TFHE_MI355_LANES_MCUS", 0);
    c->lanes_chunk = env_long("TFHE_MI355_LANES_CHUNK", 0);
    {
        const char *e = std::getenv("TFHE_MI355_LANES_MASK");
        c->lanes_block = e && std::strcmp(e, "block") == 0;
    }
    try {
        check(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking), "hipStreamCreate");
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0)
            c->cus = cus;
        for (auto &L : c->lanes) {
            check(hipStreamCreateWithFlags(&L.stream, hipStreamNonBlocking), "hipStreamCreate(lane)");
            for (hipEvent_t *e : {&L.h2d, &L.kern, &L.done})
                check(hipEventCreateWithFlags(e, hipEventDisableTiming), "hipEventCreate(lane)");
        }
        build_tables(c);
    } catch (...) {
        tfhe_mi355_context_destroy(c);
        throw;
    }
    return c;
}
}  // namespace

// key transaction of serde.cpp's serialized-key uploads (engine.h)
std::shared_ptr<void> tfhe_mi355::begin_key_transaction(TfheMi355Context *ctx) {
    return std::make_shared<std::vector<std::unique_ptr<KeyWrite>>>(key_write_all(ctx));
}

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

int tfhe_mi355_kernel_timing_enable(TfheMi355Context *ctx, int every) {
    return guarded([&] {
        if (!ctx) fail("null argument");
        if (every < 0) fail("sampling interval must be >= 0");
        if (ctx->multi()) {
            for (auto *s : ctx->shards) abi(tfhe_mi355_kernel_timing_enable(s, every));
            return;
        }
        check(hipSetDevice(ctx->device), "hipSetDevice");
        ctx->timer.reset();
        ctx->timer.every = every;
    });
}

int tfhe_mi355_kernel_timing_entry(TfheMi355Context *ctx, size_t index, char *name, size_t name_len,
                                   double *total_ms, uint64_t *launches) {
    return guarded([&] {
        if (!ctx || !name || !name_len || !total_ms || !launches) fail("null argument");
        name[0] = 0;
        *total_ms = 0;
        *launches = 0;
        if (ctx->multi()) {  // summed over the devices, by kernel family
            std::map<std::string, std::pair<double, uint64_t>> all;
            char nm[256];
            for (auto *s : ctx->shards) {
                double ms = 0;
                uint64_t cnt = 0;
                for (size_t i = 0; tfhe_mi355_kernel_timing_entry(s, i, nm, sizeof nm, &ms, &cnt) == TFHE_MI355_OK; i++) {
                    all[nm].first += ms;
                    all[nm].second += cnt;
                }
            }
            if (index >= all.size()) fail("kernel timing index %zu out of range (%zu entries)", index, all.size());
            auto it = all.begin();
            std::advance(it, index);
            std::snprintf(name, name_len, "%s", it->first.c_str());
            *total_ms = it->second.first;
            *launches = it->second.second;
            return;
        }
        check(hipSetDevice(ctx->device), "hipSetDevice");
        ctx->timer.collect();
        std::lock_guard<std::mutex> g(ctx->timer.mu);
        if (index >= ctx->timer.totals.size()) fail("kernel timing index %zu out of range (%zu entries)", index,
                                                    ctx->timer.totals.size());
        auto it = ctx->timer.totals.begin();
        std::advance(it, index);
        std::snprintf(name, name_len, "%s", it->first.c_str());
        *total_ms = it->second.first;
        *launches = it->second.second;
    });
}

struct TfheMi355Request {
    CoalescedReq req;
};

int tfhe_mi355_submit(TfheMi355Context *ctx, int op, const uint64_t *lwe_in, uint64_t *lwe_out, const uint64_t *luts,
                      size_t lut_count, const uint32_t *lut_indexes, size_t count, TfheMi355Request **out_req) {
    return guarded([&] {
        if (!out_req) fail("null argument");
        *out_req = nullptr;
        if (!ctx || !lwe_in || !lwe_out) fail("null argument");
        if (op < 0 || op >= CO_OPS) fail("unknown op %d (0 PBS, 1 KS->PBS, 2 PBS->KS, 3 KS)", op);
        if (ctx->multi()) {  // round robin over the devices' coalescers
            abi(tfhe_mi355_submit(pick_shard(ctx), op, lwe_in, lwe_out, luts, lut_count, lut_indexes, count, out_req));
            return;
        }
        if (count == 0 || count > coalesce_batch())
            fail("submit takes 1..%zu ciphertexts (larger batches: the batched entry points)", coalesce_batch());
        check(hipSetDevice(ctx->device), "hipSetDevice");
        const bool lut = op != CO_KS;
        if (lut) {
            require_fbsk(ctx);
            if (!luts || lut_count == 0) fail("lut_count must be >= 1");
            validate_lut_indexes(lut_indexes, count, lut_count);
        }
        if (op != CO_PBS) require_ksk(ctx);
        auto *h = new TfheMi355Request{{lwe_in, lwe_out, lut ? luts : nullptr, lut ? lut_count : 0,
                                        lut ? lut_indexes : nullptr, count}};
        coalesce_enqueue(ctx, (CoalescedOp)op, h->req);
        *out_req = h;
    });
}

int tfhe_mi355_wait(TfheMi355Request *req) {
    return guarded([&] {
        if (!req) fail("null request");
        std::unique_ptr<TfheMi355Request> own(req);
        coalesce_wait(own->req);
    });
}

int tfhe_mi355_coalesce_stats(TfheMi355Context *ctx, int reset, uint64_t *batches, uint64_t *rows,
                              uint64_t *max_in_flight, double *batch_seconds) {
    return guarded([&] {
        if (!ctx || !batches || !rows || !max_in_flight || !batch_seconds) fail("null argument");
        if (ctx->multi()) {  // summed over the devices (max_in_flight: the sum of the devices' maxima)
            *batches = *rows = *max_in_flight = 0;
            *batch_seconds = 0;
            for (auto *s : ctx->shards) {
                uint64_t b = 0, r = 0, m = 0;
                double t = 0;
                abi(tfhe_mi355_coalesce_stats(s, reset, &b, &r, &m, &t));
                *batches += b;
                *rows += r;
                *max_in_flight += m;
                *batch_seconds += t;
            }
            return;
        }
        auto &co = ctx->co;
        std::lock_guard<std::mutex> g(co.m);
        *batches = co.batches;
        *rows = co.rows;
        *max_in_flight = co.max_in_flight;
        *batch_seconds = co.batch_seconds;
        if (reset) {
            co.batches = co.rows = 0;
            co.max_in_flight = co.in_flight;
            co.batch_seconds = 0;
        }
    });
}

int tfhe_mi355_host_alloc(size_t bytes, void **out_ptr) {
    return guarded([&] {
        if (!out_ptr) fail("null out_ptr");
        *out_ptr = nullptr;
        if (!bytes) fail("zero-byte host allocation");
        void *p = nullptr;
        check(hipHostMalloc(&p, bytes, hipHostMallocPortable), "hipHostMalloc");
        *out_ptr = p;
    });
}

int tfhe_mi355_host_free(void *ptr) {
    return guarded([&] {
        if (ptr) check(hipHostFree(ptr), "hipHostFree");
    });
}

int tfhe_mi355_context_create(const TfheMi355Parameters *params, int device, TfheMi355Context **out_ctx) {
    return guarded([&] {
        if (!out_ctx) fail("null out_ctx");
        *out_ctx = nullptr;
        if (!params) fail("null params");
        validate_parameters(*params);
        *out_ctx = create_single(*params, device);
    });
}

int tfhe_mi355_context_create_devices(const TfheMi355Parameters *params, const int *devices, size_t device_count,
                                      TfheMi355Context **out_ctx) {
    return guarded([&] {
        if (!out_ctx) fail("null out_ctx");
        *out_ctx = nullptr;
        if (!params || (!devices && device_count)) fail("null argument");
        validate_parameters(*params);
        int visible = 0;
        check(hipGetDeviceCount(&visible), "hipGetDeviceCount");
        std::vector<int> devs(devices, devices + device_count);
        if (devs.empty())  // no list: every visible device
            for (int d = 0; d < visible; d++) devs.push_back(d);
        if (devs.empty()) fail("no GPU visible");
        if (devs.size() > 64) fail("at most 64 devices per context (%zu listed)", devs.size());
        for (int d : devs)
            if (d < 0 || d >= visible) fail("device %d is not visible (%d devices)", d, visible);
        if (devs.size() == 1) {
            *out_ctx = create_single(*params, devs[0]);
            return;
        }
        auto *m = new TfheMi355Context();
        m->p = *params;
        m->device = devs[0];
        try {
            for (int d : devs) {
                m->shards.push_back(create_single(*params, d));
                m->shards.back()->owner = m;
            }
            for (size_t i = 1; i < devs.size(); i++) {
                m->workers.emplace_back(new ShardWorker());
                ShardWorker *w = m->workers.back().get();
                w->t = std::thread([w] { w->loop(); });
            }
            enable_peer_access(devs);
        } catch (...) {
            tfhe_mi355_context_destroy(m);
            throw;
        }
        *out_ctx = m;
    });
}

int tfhe_mi355_context_devices(TfheMi355Context *ctx, size_t *count) {
    return guarded([&] {
        if (!ctx || !count) fail("null argument");
        *count = ctx->multi() ? ctx->shards.size() : 1;
    });
}

int tfhe_mi355_context_replication(TfheMi355Context *ctx, int *mode, const char **note) {
    return guarded([&] {
        if (!ctx || !mode) fail("null argument");
        *mode = ctx->multi() ? ctx->replication : TFHE_MI355_REPLICATION_NONE;
        if (note) *note = ctx->replicate_note.c_str();
    });
}

int tfhe_mi355_context_device_context(TfheMi355Context *ctx, size_t index, TfheMi355Context **out_ctx,
                                      int *device) {
    return guarded([&] {
        if (!out_ctx) fail("null out_ctx");
        *out_ctx = nullptr;
        if (!ctx) fail("null ctx");
        const size_t n = ctx->multi() ? ctx->shards.size() : 1;
        if (index >= n) fail("device index %zu out of range (%zu devices)", index, n);
        TfheMi355Context *s = ctx->multi() ? ctx->shards[index] : ctx;
        if (device) *device = s->device;
        *out_ctx = s;
    });
}

int tfhe_mi355_context_destroy(TfheMi355Context *ctx) {
    return guarded([&] {
        if (!ctx) return;
        if (ctx->owner) fail("this context belongs to a multi-device context: destroy that one");
        if (ctx->multi()) {  // every shard (each reports its own queued requests), then the communicator
            ctx->workers.clear();  // joins the shard workers (a split call still running finishes first)
            std::string errs;
            for (auto *s : ctx->shards) {
                s->owner = nullptr;
                if (tfhe_mi355_context_destroy(s) != TFHE_MI355_OK)
                    errs += std::string(errs.empty() ? "" : "; ") + tfhe_mi355_last_error();
            }
            delete ctx->rccl;
            delete ctx;
            if (!errs.empty()) fail("%s", errs.c_str());
            return;
        }
        (void)hipSetDevice(ctx->device);
        // 1. The coalescer first: take every still-queued request out of the queues and stop the
        //    dispatchers (a batch already running completes; its callers get their rows), join
        //    them, then fail the taken requests with rc = 1 -- they never launch a kernel on the
        //    tables and streams freed below (c_api/utils.rs:3-11 error convention).
        std::vector<CoalescedReq *> orphans;
        {
            std::lock_guard<std::mutex> g(ctx->co.m);
            ctx->co.stop = true;
            for (int o = 0; o < CO_OPS; o++) {
                orphans.insert(orphans.end(), ctx->co.queue[o].begin(), ctx->co.queue[o].end());
                ctx->co.queue[o].clear();
                ctx->co.queued[o] = 0;
                ctx->co.queued_sync[o] = 0;
            }
        }
        ctx->co.cv.notify_all();
        for (auto &t : ctx->co.workers) t.join();
        ctx->co.workers.clear();
        // a direct call (coalesced_call on an idle coalescer) still running on another thread
        // finishes on slot 8 before the slots' streams and the tables go (none starts after stop)
        for (;;) {
            {
                std::lock_guard<std::mutex> g(ctx->co.m);
                if (!ctx->co.direct_busy) break;
            }
            std::this_thread::sleep_for(std::chrono::microseconds(100));
        }
        for (auto *x : orphans) {
            std::lock_guard<std::mutex> g(x->m);
            x->err = "the context was destroyed before this request ran (wait on every request first)";
            x->done = true;
            x->cv.notify_one();
        }
        for (auto &sl : ctx->co.slots)  // woken callers still copying their rows out of the staging
            while (sl.copies.load(std::memory_order_acquire) != 0) std::this_thread::yield();
        for (auto &sl : ctx->co.slots)
            if (sl.stream) {
                (void)hipStreamSynchronize(sl.stream);
                (void)hipStreamDestroy(sl.stream);
                sl.stream = nullptr;
            }
        // 2. then the device work of the synchronous paths, the tables and the streams
        if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
        for (auto &L : ctx->lanes)
            if (L.stream) (void)hipStreamSynchronize(L.stream);
        if (ctx->tables.W) (void)hipFree(ctx->tables.W);
        if (ctx->tables.twist) (void)hipFree(ctx->tables.twist);
        if (ctx->tables.wtop) (void)hipFree(ctx->tables.wtop);
        for (auto &L : ctx->lanes) {
            for (hipEvent_t e : {L.h2d, L.kern, L.done})
                if (e) (void)hipEventDestroy(e);
            if (L.stream) (void)hipStreamDestroy(L.stream);
        }
        if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
        for (hipStream_t l : {ctx->lane_c, ctx->lane_m})
            if (l) {
                (void)hipStreamSynchronize(l);
                (void)hipStreamDestroy(l);
            }
        delete ctx;  // device and pinned buffers free themselves
        if (!orphans.empty())
            fail("context destroyed with %zu request(s) still queued: they were not run and their wait returns 1",
                 orphans.size());
    });
}

}  // extern "C"

namespace {
// a key upload of a multi-device context: `first` (the same entry point) on the first device's
// shard, then the key part replicated to the other shards (RCCL broadcast / device copies)
template <class F>
void multi_key_upload(TfheMi355Context *m, KeyPart part, F &&first) {
    auto w = key_write_all(m);
    set_ready_all(m, part, false);
    try {
        abi(first(m->shards[0]));
        replicate(m, part);
    } catch (...) {  // the first shard may hold the new key already: no shard serves a half-replicated one
        set_ready_all(m, part, false);
        throw;
    }
    set_ready_all(m, part, true);
}
}  // namespace

extern "C" {

int tfhe_mi355_bootstrap_key_upload(TfheMi355Context *ctx, const uint64_t *bsk, size_t len) {
    return guarded([&] {
        if (!ctx || !bsk) fail("null argument");
        if (ctx->multi())
            return multi_key_upload(ctx, KeyPart::Fourier, [&](TfheMi355Context *s) {
                return tfhe_mi355_bootstrap_key_upload(s, bsk, len);
            });
        KeyWrite kw(ctx);  // no coalesced batch in flight, none starts until done
        check(hipSetDevice(ctx->device), "hipSetDevice");
        if (len != ctx->std_bsk_len()) fail("bootstrapping key has %zu words, expected %zu", len, ctx->std_bsk_len());
        ctx->fbsk_ready = false;
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
        if (ctx->multi())
            return multi_key_upload(ctx, KeyPart::Fourier, [&](TfheMi355Context *s) {
                return tfhe_mi355_bootstrap_key_upload_seeded(s, bodies, len, seed_lo, seed_hi);
            });
        KeyWrite kw(ctx);  // no coalesced batch in flight, none starts until done
        check(hipSetDevice(ctx->device), "hipSetDevice");
        const size_t rows = ctx->ggsw_count() * ctx->p.pbs_level * (ctx->k() + 1);
        if (len != rows * ctx->N()) fail("seeded bootstrapping key has %zu body words, expected %zu", len, rows * ctx->N());
        ctx->fbsk_ready = false;
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
        if (ctx->multi())
            return multi_key_upload(ctx, KeyPart::Ksk, [&](TfheMi355Context *s) {
                return tfhe_mi355_keyswitch_key_upload_seeded(s, bodies, len, seed_lo, seed_hi);
            });
        KeyWrite kw(ctx);  // no coalesced batch in flight, none starts until done
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
        ctx = primary(ctx);  // device pointers: the first device's shard
        if (!ctx || (!out && words)) fail("null argument");
        std::lock_guard<std::mutex> g(ctx->mu);
        check(hipSetDevice(ctx->device), "hipSetDevice");
        if (words == 0) return;
        DeviceBuffer tab;
        upload_aes_tables(ctx, seed_lo, seed_hi, tab);
        DeviceBuffer d_words;
        d_words.reserve(words * sizeof(uint64_t));
        check(launch_seeded_decompress(tab.ptr, nullptr, 1, words, 0, (uint64_t *)d_words.ptr, ctx->stream),
              "csprng");
        check(hipMemcpyAsync(out, d_words.ptr, words * sizeof(uint64_t), hipMemcpyDeviceToHost, ctx->stream),
              "D2H words");
        check(hipStreamSynchronize(ctx->stream), "csprng sync");
        tab.release();
    });
}

int tfhe_mi355_bootstrap_key_convert_async(TfheMi355Context *ctx, const uint64_t *d_bsk, size_t len,
                                           void *stream) {
    return guarded([&] {
        if (!ctx || !d_bsk) fail("null argument");
        if (ctx->multi())  // d_bsk on the first device
            return multi_key_upload(ctx, KeyPart::Fourier, [&](TfheMi355Context *s) {
                return tfhe_mi355_bootstrap_key_convert_async(s, d_bsk, len, stream);
            });
        KeyWrite kw(ctx);  // no coalesced batch in flight, none starts until done
        check(hipSetDevice(ctx->device), "hipSetDevice");
        if (len != ctx->std_bsk_len()) fail("bootstrapping key has %zu words, expected %zu", len, ctx->std_bsk_len());
        ctx->fbsk_ready = false;
        ctx->fbsk.reserve(ctx->fourier_bsk_bytes());
        check(convert_bsk(ctx, d_bsk, len / ctx->N(), (hipStream_t)stream), "bsk conversion");
        // the key counts as ready only once the conversion has run: every later call (on any
        // stream, including ctx->stream, which is not ordered after the caller's) sees it whole
        check(hipStreamSynchronize((hipStream_t)stream), "bsk conversion sync");
        ctx->fbsk_ready = true;
    });
}

int tfhe_mi355_context_parameters(TfheMi355Context *ctx, TfheMi355Parameters *out) {
    return guarded([&] {
        if (!ctx || !out) fail("null argument");
        *out = ctx->p;
    });
}

int tfhe_mi355_bootstrap_key_fourier(TfheMi355Context *ctx, void **d_ptr, size_t *bytes) {
    return guarded([&] {
        if (!ctx || !d_ptr || !bytes) fail("null argument");
        *d_ptr = nullptr;
        *bytes = 0;
        if (ctx->multi()) {  // the first device's buffer; _set_ready replicates it to the others
            auto w = key_write_all(ctx);
            abi(tfhe_mi355_bootstrap_key_fourier(ctx->shards[0], d_ptr, bytes));
            // the caller now rewrites shard 0's copy: no device serves this key part until _set_ready
            // (batches fail cleanly instead of mixing a half-written key with the old replicas)
            set_ready_all(ctx, KeyPart::Fourier, false);
            return;
        }
        KeyWrite kw(ctx);  // no coalesced batch in flight, none starts until done
        check(hipSetDevice(ctx->device), "hipSetDevice");
        ctx->fbsk.reserve(ctx->fourier_bsk_bytes());
        *d_ptr = ctx->fbsk.ptr;
        *bytes = ctx->fourier_bsk_bytes();
    });
}

int tfhe_mi355_bootstrap_key_fourier_set_ready(TfheMi355Context *ctx) {
    return guarded([&] {
        if (!ctx) fail("null ctx");
        if (ctx->multi())
            return multi_key_upload(ctx, KeyPart::Fourier, [&](TfheMi355Context *s) {
                return tfhe_mi355_bootstrap_key_fourier_set_ready(s);
            });
        KeyWrite kw(ctx);  // no coalesced batch in flight, none starts until done
        if (!ctx->fbsk.ptr) fail("no Fourier key buffer");
        ctx->fbsk_ready = true;
    });
}

int tfhe_mi355_keyswitch_key_upload(TfheMi355Context *ctx, const uint64_t *ksk, size_t len) {
    return guarded([&] {
        if (!ctx || !ksk) fail("null argument");
        if (ctx->multi())
            return multi_key_upload(ctx, KeyPart::Ksk, [&](TfheMi355Context *s) {
                return tfhe_mi355_keyswitch_key_upload(s, ksk, len);
            });
        KeyWrite kw(ctx);  // no coalesced batch in flight, none starts until done
        check(hipSetDevice(ctx->device), "hipSetDevice");
        if (len != ctx->ksk_len()) fail("keyswitching key has %zu words, expected %zu", len, ctx->ksk_len());
        ctx->ksk_ready = false;
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
        if (ctx->multi())  // d_ksk on the first device
            return multi_key_upload(ctx, KeyPart::Ksk, [&](TfheMi355Context *s) {
                return tfhe_mi355_keyswitch_key_upload_async(s, d_ksk, len, stream);
            });
        KeyWrite kw(ctx);  // no coalesced batch in flight, none starts until done
        check(hipSetDevice(ctx->device), "hipSetDevice");
        if (len != ctx->ksk_len()) fail("keyswitching key has %zu words, expected %zu", len, ctx->ksk_len());
        ctx->ksk.reserve(len * sizeof(uint64_t));
        ctx->ksk_ready = false;
        check(hipMemcpyAsync(ctx->ksk.ptr, d_ksk, len * sizeof(uint64_t), hipMemcpyDeviceToDevice,
                             (hipStream_t)stream), "copy ksk");
        repack_ksk(ctx, (hipStream_t)stream);
        check(hipStreamSynchronize((hipStream_t)stream), "ksk upload sync");  // see bootstrap_key_convert_async
        ctx->ksk_ready = true;
    });
}

int tfhe_mi355_keyswitch_key_device(TfheMi355Context *ctx, void **d_ptr, size_t *bytes) {
    return guarded([&] {
        if (!ctx || !d_ptr || !bytes) fail("null argument");
        *d_ptr = nullptr;
        *bytes = 0;
        if (ctx->multi()) {  // the first device's buffer; _set_ready replicates it to the others
            auto w = key_write_all(ctx);
            abi(tfhe_mi355_keyswitch_key_device(ctx->shards[0], d_ptr, bytes));
            // the caller now rewrites shard 0's copy: no device serves this key part until _set_ready
            // (batches fail cleanly instead of mixing a half-written key with the old replicas)
            set_ready_all(ctx, KeyPart::Ksk, false);
            return;
        }
        KeyWrite kw(ctx);  // no coalesced batch in flight, none starts until done
        check(hipSetDevice(ctx->device), "hipSetDevice");
        ctx->ksk.reserve(ctx->ksk_len() * sizeof(uint64_t));
        *d_ptr = ctx->ksk.ptr;
        *bytes = ctx->ksk_len() * sizeof(uint64_t);
    });
}

int tfhe_mi355_keyswitch_key_set_ready(TfheMi355Context *ctx) {
    return guarded([&] {
        if (!ctx) fail("null ctx");
        if (ctx->multi())
            return multi_key_upload(ctx, KeyPart::Ksk, [&](TfheMi355Context *s) {
                return tfhe_mi355_keyswitch_key_set_ready(s);
            });
        KeyWrite kw(ctx);  // no coalesced batch in flight, none starts until done
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
        if (ctx->multi()) {
            const size_t wi = ctx->n() + 1, wo = ctx->big_dim() + 1;
            if (coalescible(count))
                return abi(tfhe_mi355_programmable_bootstrap(pick_shard(ctx), lwe_in, lwe_out, luts, lut_count,
                                                             lut_indexes, count));
            return split_rows(ctx, count, [&](TfheMi355Context *s, size_t a, size_t n) {
                return tfhe_mi355_programmable_bootstrap(s, lwe_in + a * wi, lwe_out + a * wo, luts, lut_count,
                                                         lut_indexes ? lut_indexes + a : nullptr, n);
            });
        }
        check(hipSetDevice(ctx->device), "hipSetDevice");
        require_fbsk(ctx);
        if (lut_count == 0) fail("lut_count must be >= 1");
        validate_lut_indexes(lut_indexes, count, lut_count);
        if (coalescible(count)) {
            CoalescedReq r{lwe_in, lwe_out, luts, lut_count, lut_indexes, count};
            return coalesced_call(ctx, CO_PBS, r);
        }
        std::lock_guard<std::mutex> g(ctx->mu);
        run_host_pipeline(ctx, lwe_in, ctx->n() + 1, lwe_out, ctx->big_dim() + 1, luts, ctx->glwe_len(), lut_count,
                          lut_indexes, count, chunk_pbs, pbs_scratch_bytes);
    });
}

int tfhe_mi355_programmable_bootstrap_scratch(TfheMi355Context *ctx, size_t count, size_t *bytes) {
    return guarded([&] {
        ctx = primary(ctx);  // device pointers: the first device's shard
        if (!ctx || !bytes) fail("null argument");
        *bytes = pbs_scratch_bytes(ctx, count);
    });
}

int tfhe_mi355_programmable_bootstrap_async(TfheMi355Context *ctx, const uint64_t *d_in, uint64_t *d_out,
                                            const uint64_t *d_luts, size_t lut_count, const uint32_t *d_idx,
                                            size_t count, void *d_scratch, size_t scratch_bytes, void *stream) {
    return guarded([&] {
        ctx = primary(ctx);  // device pointers: the first device's shard
        if (!ctx || (!d_in && count) || (!d_out && count) || !d_luts) fail("null argument");
        check(hipSetDevice(ctx->device), "hipSetDevice");
        // the scratch query is the contract: the persistent grid's ticket word at the classic
        // shapes that use one (a NULL scratch there would silently run the slower one-pass grid);
        // at N >= 4096 at least one ciphertext's worth (smaller passes below the query's size)
        if (count && !is_large(ctx)) require_scratch(d_scratch ? scratch_bytes : 0, pbs_scratch_bytes(ctx, count));
        launch_pbs_dev(ctx, d_in, d_out, d_luts, lut_count, d_idx, count, d_scratch, scratch_bytes,
                       (hipStream_t)stream);
    });
}

int tfhe_mi355_blind_rotate(TfheMi355Context *ctx, const uint64_t *lwe_in, uint64_t *glwe_out, const uint64_t *luts,
                            size_t lut_count, const uint32_t *lut_indexes, size_t count) {
    return guarded([&] {
        if (!ctx || (!lwe_in && count) || (!glwe_out && count) || !luts) fail("null argument");
        if (ctx->multi())
            return split_rows(ctx, count, [&](TfheMi355Context *s, size_t a, size_t n) {
                return tfhe_mi355_blind_rotate(s, lwe_in + a * (ctx->n() + 1), glwe_out + a * ctx->glwe_len(), luts,
                                               lut_count, lut_indexes ? lut_indexes + a : nullptr, n);
            });
        std::lock_guard<std::mutex> g(ctx->mu);
        check(hipSetDevice(ctx->device), "hipSetDevice");
        require_fbsk(ctx);
        if (lut_count == 0) fail("lut_count must be >= 1");
        if (is_large(ctx)) fail("blind rotation without sample extraction is not available at N = %zu", ctx->N());
        validate_lut_indexes(lut_indexes, count, lut_count);
        run_host_pipeline(ctx, lwe_in, ctx->n() + 1, glwe_out, ctx->glwe_len(), luts, ctx->glwe_len(), lut_count,
                          lut_indexes, count, chunk_blind_rotate, pbs_scratch_bytes);
    });
}

int tfhe_mi355_blind_rotate_async(TfheMi355Context *ctx, const uint64_t *d_in, uint64_t *d_glwe_out,
                                  const uint64_t *d_luts, size_t lut_count, const uint32_t *d_lut_indexes,
                                  size_t count, void *stream) {
    return guarded([&] {
        ctx = primary(ctx);  // device pointers: the first device's shard
        if (!ctx || (!d_in && count) || (!d_glwe_out && count) || !d_luts) fail("null argument");
        check(hipSetDevice(ctx->device), "hipSetDevice");
        launch_pbs_dev(ctx, d_in, d_glwe_out, d_luts, lut_count, d_lut_indexes, count, nullptr, 0,
                       (hipStream_t)stream, true);
    });
}

int tfhe_mi355_packing_keyswitch_key_upload(TfheMi355Context *ctx, const uint64_t *pksk, size_t len,
                                            uint32_t base_log, uint32_t level) {
    return guarded([&] {
        if (!ctx || !pksk) fail("null argument");
        if (level == 0 || base_log == 0 || base_log * level >= 64) fail("invalid packing ks decomposition");
        if (ctx->multi()) {  // a gadget-layer key: uploaded to every device from the host
            auto w = key_write_all(ctx);
            for (auto *s : ctx->shards) abi(tfhe_mi355_packing_keyswitch_key_upload(s, pksk, len, base_log, level));
            return;
        }
        KeyWrite kw(ctx);
        check(hipSetDevice(ctx->device), "hipSetDevice");
        if (len != ctx->pksk_len(level))
            fail("packing keyswitching key has %zu words, expected %zu", len, ctx->pksk_len(level));
        ctx->pksk_ready = ctx->pksk_planes_ready = false;
        ctx->pksk.reserve(len * sizeof(uint64_t));
        check(hipMemcpy(ctx->pksk.ptr, pksk, len * sizeof(uint64_t), hipMemcpyHostToDevice), "upload pksk");
        ctx->pks_base_log = base_log;
        ctx->pks_level = level;
        const int in_dim = (int)ctx->big_dim(), out_dim = (int)ctx->glwe_len() - 1;
        if (pks_use_mfma(ctx)) {
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
        if (ctx->multi())
            return split_rows(ctx, count, [&](TfheMi355Context *s, size_t a, size_t n) {
                return tfhe_mi355_packing_keyswitch(s, lwe_in + a * (ctx->big_dim() + 1), glwe_out + a * ctx->glwe_len(), n);
            });
        std::lock_guard<std::mutex> g(ctx->mu);
        check(hipSetDevice(ctx->device), "hipSetDevice");
        if (!ctx->pksk_ready) fail("packing keyswitching key not uploaded");
        run_host_pipeline(ctx, lwe_in, ctx->big_dim() + 1, glwe_out, ctx->glwe_len(), nullptr, 0, 0, nullptr, count,
                          chunk_pks, pks_scratch_bytes);
    });
}

int tfhe_mi355_packing_keyswitch_scratch(TfheMi355Context *ctx, size_t count, size_t *bytes) {
    return guarded([&] {
        ctx = primary(ctx);  // device pointers: the first device's shard
        if (!ctx || !bytes) fail("null argument");
        std::lock_guard<std::mutex> g(ctx->mu);
        if (!ctx->pksk_ready) fail("packing keyswitching key not uploaded: its decomposition sizes the scratch");
        *bytes = pks_scratch_bytes(ctx, count);
    });
}

int tfhe_mi355_packing_keyswitch_async(TfheMi355Context *ctx, const uint64_t *d_lwe_in, uint64_t *d_glwe_out,
                                       size_t count, void *d_scratch, size_t scratch_bytes, void *stream) {
    return guarded([&] {
        ctx = primary(ctx);  // device pointers: the first device's shard
        if (!ctx || (!d_lwe_in && count) || (!d_glwe_out && count)) fail("null argument");
        check(hipSetDevice(ctx->device), "hipSetDevice");
        launch_packing_ks_dev(ctx, d_lwe_in, d_glwe_out, count, d_scratch, scratch_bytes, (hipStream_t)stream);
    });
}

int tfhe_mi355_glwe_poly_mul(TfheMi355Context *ctx, const uint64_t *glwe_in, size_t glwe_per_item,
                             const uint64_t *polys, size_t npoly, size_t count, int extract, uint64_t *out) {
    return guarded([&] {
        if (!ctx || (!glwe_in && count) || (!polys && npoly) || (!out && count && npoly)) fail("null argument");
        if (ctx->multi()) {
            const size_t wo = npoly * (extract ? ctx->big_dim() + 1 : ctx->glwe_len());
            return split_rows(ctx, count, [&](TfheMi355Context *s, size_t a, size_t n) {
                return tfhe_mi355_glwe_poly_mul(s, glwe_in + a * glwe_per_item * ctx->glwe_len(), glwe_per_item, polys,
                                                npoly, n, extract, out + a * wo);
            });
        }
        std::lock_guard<std::mutex> g(ctx->mu);
        check(hipSetDevice(ctx->device), "hipSetDevice");
        if (count == 0 || npoly == 0) return;
        const size_t out_words = extract ? ctx->big_dim() + 1 : ctx->glwe_len();
        const size_t in_b = count * glwe_per_item * ctx->glwe_len() * 8;
        const size_t poly_b = npoly * glwe_per_item * ctx->N() * 8, out_b = count * npoly * out_words * 8;
        DeviceBuffer d_in, d_polys, d_out;
        d_in.reserve(in_b);
        d_polys.reserve(poly_b);
        d_out.reserve(out_b);
        hipStream_t s = ctx->stream;
        check(hipMemcpyAsync(d_in.ptr, glwe_in, in_b, hipMemcpyHostToDevice, s), "H2D glwe");
        check(hipMemcpyAsync(d_polys.ptr, polys, poly_b, hipMemcpyHostToDevice, s), "H2D polys");
        launch_glwe_poly_mul_dev(ctx, (const uint64_t *)d_in.ptr, glwe_per_item, (const uint64_t *)d_polys.ptr, npoly,
                                 count, extract != 0, (uint64_t *)d_out.ptr, s);
        check(hipMemcpyAsync(out, d_out.ptr, out_b, hipMemcpyDeviceToHost, s), "D2H out");
        check(hipStreamSynchronize(s), "glwe poly mul sync");
    });
}

int tfhe_mi355_glwe_poly_mul_async(TfheMi355Context *ctx, const uint64_t *d_glwe_in, size_t glwe_per_item,
                                   const uint64_t *d_polys, size_t npoly, size_t count, int extract,
                                   uint64_t *d_out, void *stream) {
    return guarded([&] {
        ctx = primary(ctx);  // device pointers: the first device's shard
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
        if (ctx->multi()) {
            const size_t wi = ctx->big_dim() + 1, wo = ctx->n() + 1;
            if (coalescible(count)) return abi(tfhe_mi355_keyswitch(pick_shard(ctx), lwe_in, lwe_out, count));
            return split_rows(ctx, count, [&](TfheMi355Context *s, size_t a, size_t n) {
                return tfhe_mi355_keyswitch(s, lwe_in + a * wi, lwe_out + a * wo, n);
            });
        }
        check(hipSetDevice(ctx->device), "hipSetDevice");
        require_ksk(ctx);
        if (coalescible(count)) {
            CoalescedReq r{lwe_in, lwe_out, nullptr, 0, nullptr, count};
            return coalesced_call(ctx, CO_KS, r);
        }
        std::lock_guard<std::mutex> g(ctx->mu);
        run_host_pipeline(ctx, lwe_in, ctx->big_dim() + 1, lwe_out, ctx->n() + 1, nullptr, 0, 0, nullptr, count,
                          chunk_ks, ks_scratch_bytes);
    });
}

int tfhe_mi355_keyswitch_scratch(TfheMi355Context *ctx, size_t count, size_t *bytes) {
    return guarded([&] {
        ctx = primary(ctx);  // device pointers: the first device's shard
        if (!ctx || !bytes) fail("null argument");
        std::lock_guard<std::mutex> g(ctx->mu);
        *bytes = ks_scratch_bytes(ctx, count);
    });
}

int tfhe_mi355_keyswitch_async(TfheMi355Context *ctx, const uint64_t *d_in, uint64_t *d_out, size_t count,
                               void *d_scratch, size_t scratch_bytes, void *stream) {
    return guarded([&] {
        ctx = primary(ctx);  // device pointers: the first device's shard
        if (!ctx || (!d_in && count) || (!d_out && count)) fail("null argument");
        check(hipSetDevice(ctx->device), "hipSetDevice");
        launch_ks_dev(ctx, d_in, d_out, count, d_scratch, scratch_bytes, (hipStream_t)stream);
    });
}

int tfhe_mi355_keyswitch_programmable_bootstrap_scratch(TfheMi355Context *ctx, size_t count, size_t *bytes) {
    return guarded([&] {
        ctx = primary(ctx);  // device pointers: the first device's shard
        if (!ctx || !bytes) fail("null argument");
        std::lock_guard<std::mutex> g(ctx->mu);
        *bytes = ks_pbs_scratch_bytes(ctx, count);
    });
}

int tfhe_mi355_keyswitch_programmable_bootstrap_async(TfheMi355Context *ctx, const uint64_t *d_in,
                                                      uint64_t *d_out, const uint64_t *d_luts, size_t lut_count,
                                                      const uint32_t *d_idx, size_t count, void *d_scratch,
                                                      size_t scratch_bytes, void *stream) {
    return guarded([&] {
        ctx = primary(ctx);  // device pointers: the first device's shard
        if (!ctx || (!d_in && count) || (!d_out && count) || !d_luts || (!d_scratch && count))
            fail("null argument");
        check(hipSetDevice(ctx->device), "hipSetDevice");
        launch_ks_pbs_dev(ctx, d_in, d_out, d_luts, lut_count, d_idx, count, d_scratch, scratch_bytes,
                          (hipStream_t)stream);
    });
}

int tfhe_mi355_keyswitch_programmable_bootstrap(TfheMi355Context *ctx, const uint64_t *lwe_in,
                                                uint64_t *lwe_out, const uint64_t *luts, size_t lut_count,
                                                const uint32_t *lut_indexes, size_t count) {
    return guarded([&] {
        if (!ctx || (!lwe_in && count) || (!lwe_out && count) || !luts) fail("null argument");
        if (ctx->multi()) {
            const size_t wi = ctx->big_dim() + 1, wo = ctx->big_dim() + 1;
            if (coalescible(count))
                return abi(tfhe_mi355_keyswitch_programmable_bootstrap(pick_shard(ctx), lwe_in, lwe_out, luts, lut_count, lut_indexes, count));
            return split_rows(ctx, count, [&](TfheMi355Context *s, size_t a, size_t n) {
                return tfhe_mi355_keyswitch_programmable_bootstrap(s, lwe_in + a * wi, lwe_out + a * wo, luts, lut_count,
                            lut_indexes ? lut_indexes + a : nullptr, n);
            });
        }
        check(hipSetDevice(ctx->device), "hipSetDevice");
        require_fbsk(ctx);
        require_ksk(ctx);
        if (lut_count == 0) fail("lut_count must be >= 1");
        validate_lut_indexes(lut_indexes, count, lut_count);
        if (coalescible(count)) {
            CoalescedReq r{lwe_in, lwe_out, luts, lut_count, lut_indexes, count};
            return coalesced_call(ctx, CO_KS_PBS, r);
        }
        std::lock_guard<std::mutex> g(ctx->mu);
        run_host_pipeline(ctx, lwe_in, ctx->big_dim() + 1, lwe_out, ctx->big_dim() + 1, luts, ctx->glwe_len(),
                          lut_count, lut_indexes, count, launch_ks_pbs_dev, ks_pbs_scratch_bytes);
    });
}

int tfhe_mi355_programmable_bootstrap_keyswitch_scratch(TfheMi355Context *ctx, size_t count, size_t *bytes) {
    return guarded([&] {
        ctx = primary(ctx);  // device pointers: the first device's shard
        if (!ctx || !bytes) fail("null argument");
        std::lock_guard<std::mutex> g(ctx->mu);
        *bytes = pbs_ks_scratch_bytes(ctx, count);
    });
}

int tfhe_mi355_programmable_bootstrap_keyswitch_async(TfheMi355Context *ctx, const uint64_t *d_in,
                                                      uint64_t *d_out, const uint64_t *d_luts, size_t lut_count,
                                                      const uint32_t *d_idx, size_t count, void *d_scratch,
                                                      size_t scratch_bytes, void *stream) {
    return guarded([&] {
        ctx = primary(ctx);  // device pointers: the first device's shard
        if (!ctx || (!d_in && count) || (!d_out && count) || !d_luts || (!d_scratch && count))
            fail("null argument");
        check(hipSetDevice(ctx->device), "hipSetDevice");
        launch_pbs_ks_dev(ctx, d_in, d_out, d_luts, lut_count, d_idx, count, d_scratch, scratch_bytes,
                          (hipStream_t)stream);
    });
}

int tfhe_mi355_programmable_bootstrap_keyswitch(TfheMi355Context *ctx, const uint64_t *lwe_in,
                                                uint64_t *lwe_out, const uint64_t *luts, size_t lut_count,
                                                const uint32_t *lut_indexes, size_t count) {
    return guarded([&] {
        if (!ctx || (!lwe_in && count) || (!lwe_out && count) || !luts) fail("null argument");
        if (ctx->multi()) {
            const size_t wi = ctx->n() + 1, wo = ctx->n() + 1;
            if (coalescible(count))
                return abi(tfhe_mi355_programmable_bootstrap_keyswitch(pick_shard(ctx), lwe_in, lwe_out, luts, lut_count, lut_indexes, count));
            return split_rows(ctx, count, [&](TfheMi355Context *s, size_t a, size_t n) {
                return tfhe_mi355_programmable_bootstrap_keyswitch(s, lwe_in + a * wi, lwe_out + a * wo, luts, lut_count,
                            lut_indexes ? lut_indexes + a : nullptr, n);
            });
        }
        check(hipSetDevice(ctx->device), "hipSetDevice");
        require_fbsk(ctx);
        require_ksk(ctx);
        if (lut_count == 0) fail("lut_count must be >= 1");
        validate_lut_indexes(lut_indexes, count, lut_count);
        if (coalescible(count)) {
            CoalescedReq r{lwe_in, lwe_out, luts, lut_count, lut_indexes, count};
            return coalesced_call(ctx, CO_PBS_KS, r);
        }
        std::lock_guard<std::mutex> g(ctx->mu);
        run_host_pipeline(ctx, lwe_in, ctx->n() + 1, lwe_out, ctx->n() + 1, luts, ctx->glwe_len(), lut_count,
                          lut_indexes, count, launch_pbs_ks_dev, pbs_ks_scratch_bytes);
    });
}

int tfhe_mi355_lwe_scalar_mul_add_async(TfheMi355Context *ctx, uint64_t *d_y, const uint64_t *d_x, uint64_t scalar,
                                        size_t rows, size_t words, size_t y_stride, size_t x_stride, void *stream) {
    return guarded([&] {
        ctx = primary(ctx);  // device pointers: the first device's shard
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
        ctx = primary(ctx);  // device pointers: the first device's shard
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
