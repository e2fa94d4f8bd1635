// loadgen.cpp -- native closed-loop callers of the synchronous host-pointer C ABI (measurement
// tool for bench.py, built as lib/libtfhe_mi355_loadgen.so; not part of the engine library).
//
// The reference bootstraps one ciphertext per call from rayon worker threads
// (shortint/server_key/mod.rs:783-857, integer/server_key/radix_parallel/mul.rs:347-407).  A Rust
// caller of the drop-in does the same through tfhe_mi355_keyswitch_programmable_bootstrap with
// count = 1 from native threads; Python threads cannot stand in for that (each call holds the GIL
// for its argument marshalling), so this tool drives the ABI from std::threads: T threads, each
// issuing its next count = 1 call as soon as the previous one returns, for a fixed time.  Every
// output row is compared with the expected row (the same ciphertext through one batched call).
// tfhe_mi355_loadgen_submit_run drives the asynchronous submit / wait pair the same way.
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/tfhe_mi355.h"

extern "C" {

// op: 0 = tfhe_mi355_programmable_bootstrap, 1 = tfhe_mi355_keyswitch_programmable_bootstrap.
// in: [n_in][in_words], expected: [n_in][out_words] (or null), lut: one accumulator.
// Results: calls completed, wall seconds, mean call latency (seconds), rows differing from
// `expected`, failed calls.
int tfhe_mi355_loadgen_run(TfheMi355Context *ctx, int op, const uint64_t *in, size_t in_words, size_t n_in,
                           const uint64_t *expected, size_t out_words, const uint64_t *lut, int threads,
                           double seconds, uint64_t *calls, double *wall, double *mean_latency,
                           uint64_t *mismatches, uint64_t *failures) {
    if (!ctx || !in || !lut || !calls || !wall || !mean_latency || !mismatches || !failures || threads <= 0 ||
        n_in == 0)
        return 1;
    std::atomic<uint64_t> n_calls{0}, n_bad{0}, n_fail{0};
    std::atomic<uint64_t> lat_ns{0};
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    const auto stop = t0 + std::chrono::duration_cast<clk::duration>(std::chrono::duration<double>(seconds));
    auto worker = [&](int t) {
        std::vector<uint64_t> out(out_words);
        size_t i = (size_t)t % n_in;
        while (clk::now() < stop) {
            const auto c0 = clk::now();
            const uint64_t *x = in + i * in_words;
            const int rc = op == 0 ? tfhe_mi355_programmable_bootstrap(ctx, x, out.data(), lut, 1, nullptr, 1)
                                   : tfhe_mi355_keyswitch_programmable_bootstrap(ctx, x, out.data(), lut, 1, nullptr, 1);
            const auto c1 = clk::now();
            if (rc != 0) {
                n_fail++;
                continue;
            }
            lat_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(c1 - c0).count();
            n_calls++;
            if (expected && std::memcmp(out.data(), expected + i * out_words, out_words * 8) != 0) n_bad++;
            i = (i + (size_t)threads) % n_in;
        }
    };
    std::vector<std::thread> ts;
    for (int t = 0; t < threads; t++) ts.emplace_back(worker, t);
    for (auto &th : ts) th.join();
    *wall = std::chrono::duration<double>(clk::now() - t0).count();
    *calls = n_calls.load();
    *mean_latency = *calls ? (double)lat_ns.load() * 1e-9 / (double)*calls : 0.0;
    *mismatches = n_bad.load();
    *failures = n_fail.load();
    return 0;
}

// Same callers through tfhe_mi355_submit / tfhe_mi355_wait: each thread keeps `window` count = 1
// requests in flight (submits them, then waits for all), so the coalesced batches are no longer
// capped by the number of threads.  op as tfhe_mi355_submit (0 PBS, 1 KS -> PBS); latency is
// submit-to-wait-return per request.
int tfhe_mi355_loadgen_submit_run(TfheMi355Context *ctx, int op, const uint64_t *in, size_t in_words, size_t n_in,
                                  const uint64_t *expected, size_t out_words, const uint64_t *lut, int threads,
                                  int window, double seconds, uint64_t *calls, double *wall, double *mean_latency,
                                  uint64_t *mismatches, uint64_t *failures) {
    if (!ctx || !in || !lut || !calls || !wall || !mean_latency || !mismatches || !failures || threads <= 0 ||
        window <= 0 || n_in == 0)
        return 1;
    std::atomic<uint64_t> n_calls{0}, n_bad{0}, n_fail{0};
    std::atomic<uint64_t> lat_ns{0};
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    const auto stop = t0 + std::chrono::duration_cast<clk::duration>(std::chrono::duration<double>(seconds));
    auto worker = [&](int t) {
        std::vector<uint64_t> out((size_t)window * out_words);
        std::vector<TfheMi355Request *> req((size_t)window, nullptr);
        std::vector<size_t> row((size_t)window);
        size_t i = (size_t)t % n_in;
        while (clk::now() < stop) {
            const auto c0 = clk::now();
            for (int w = 0; w < window; w++) {
                row[w] = i;
                if (tfhe_mi355_submit(ctx, op, in + i * in_words, out.data() + (size_t)w * out_words, lut, 1, nullptr, 1,
                                      &req[w]) != 0) {
                    n_fail++;
                    req[w] = nullptr;
                }
                i = (i + (size_t)threads) % n_in;
            }
            for (int w = 0; w < window; w++) {
                if (!req[w]) continue;
                if (tfhe_mi355_wait(req[w]) != 0) {
                    n_fail++;
                    continue;
                }
                const auto c1 = clk::now();
                lat_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(c1 - c0).count();
                n_calls++;
                if (expected &&
                    std::memcmp(out.data() + (size_t)w * out_words, expected + row[w] * out_words, out_words * 8) != 0)
                    n_bad++;
            }
        }
    };
    std::vector<std::thread> ts;
    for (int t = 0; t < threads; t++) ts.emplace_back(worker, t);
    for (auto &th : ts) th.join();
    *wall = std::chrono::duration<double>(clk::now() - t0).count();
    *calls = n_calls.load();
    *mean_latency = *calls ? (double)lat_ns.load() * 1e-9 / (double)*calls : 0.0;
    *mismatches = n_bad.load();
    *failures = n_fail.load();
    return 0;
}
}
