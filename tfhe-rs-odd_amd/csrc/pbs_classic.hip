// pbs_classic.hip -- batched classic programmable bootstrap on gfx950.
//
// Replaces (reference tfhe-rs-odd, CPU Rust):
//   FourierLweBootstrapKeyView::blind_rotate_assign   fft64/crypto/bootstrap.rs:243-344
//   FourierLweBootstrapKeyView::bootstrap             fft64/crypto/bootstrap.rs:346-380
//   add_external_product_assign / update_with_fmadd   fft64/crypto/ggsw.rs:477-697
//   polynomial_wrapping_monic_monomial_{div,mul_and_subtract}
//                                                     algorithms/polynomial_algorithms.rs:219-490
//   fast_pbs_modulus_switch                           fft_impl/common.rs:26-43
//   extract_lwe_sample_from_glwe_ciphertext (deg 0)   algorithms/glwe_sample_extraction.rs:91-147
//   par_convert_polynomials_list_to_fourier           fft64/math/fft/mod.rs:719-764
// The fork's PATTERN msgpack dump (bootstrap.rs:340-342) is deliberately not reproduced.
//
// Design: a workgroup bootstraps CPW ciphertexts (4 at 2_2, else 1), one wavefront
// per GLWE polynomial ((k+1) waves per ciphertext).  Each wave keeps its accumulator polynomial in
// registers (u64), rotates it through its LDS buffer, decomposes and forward-FFTs it (row r = its
// polynomial); the (k+1) row spectra of a ciphertext are published to LDS and wave c computes
// output column c = sum_r F_r * GGSW[r][c] (GGSW streamed from L2/MALL, 16 B per lane, coalesced;
// MAC operands read back from LDS at N = 2048 and 1024), inverse-FFTs it and adds it back.  FFT
// twiddles and the twist live in LDS.  At 2_2: 2 waves per SIMD (<= 256 VGPRs, 244 used), LDS
// 31 KiB of tables + 8 x 16 KiB exchange buffers + sync flags = 159 KiB -> 4 ciphertexts per CU.
// The grid is persistent with a global ciphertext ticket queue at 2_2 (PbsConfig::PERSIST).
// Synchronisation: wave-private LDS reuse is ordered with wave-local fences; the spectrum exchange
// among the (k+1) waves of ONE ciphertext uses LDS flag words (GroupSync, pbs_common.h), so the
// ciphertexts of a workgroup drift apart instead of running in lockstep behind s_barrier.
//
// Control flow is uniform within a ciphertext's waves: a CMUX whose mask element is 0 (skipped by
// the reference, bootstrap.rs:285) is executed as a rotation by 0, which adds exactly 0 to the
// accumulator (ct1 = 0 -> digits 0 -> spectra +-0 -> increments 0), so the output bits are
// unchanged.
#include "engine.h"
#include "pbs_common.h"

#ifndef CLASSIC_DIGIT2
#define CLASSIC_DIGIT2 1  // L = 2 shapes: Digit2 (pbs_common.h) instead of the per-level digit loop (0: A/B)
#endif

namespace tfhe_mi355 {

#ifndef PBS_CPW
#define PBS_CPW 0  // ciphertexts per workgroup; 0: per-shape default
#endif
#ifndef PBS_TSKIP_ROT
#define PBS_TSKIP_ROT 0  // timing-only builds (wrong outputs): no rotation gather (what the rotation costs)
#endif
#ifndef PBS_GGSW_LDS
#define PBS_GGSW_LDS 0  // measured 2% slower than streaming from L2 (CPW=2 couples 4 waves); kept as an option
#endif
template <int N, int K, int L>
struct PbsConfig {
    static constexpr int M = N / 2;
    static constexpr size_t GGSW_ELEMS = (size_t)L * (K + 1) * (K + 1) * M;  // double2 per GGSW
    // 2_2 shape (N = 2048, k = 1, L = 1): 4 ciphertexts per workgroup at 2 waves/SIMD.  The MAC
    // reads every row spectrum back from LDS (the own row's 64 VGPRs are free by then: 226
    // VGPRs, no spills) and the twist/M table is dropped, so 31 KiB of tables + 8 x 16 KiB
    // exchange buffers fill the CU's LDS (159 KiB): 8 waves per CU instead of 4, 77.5k -> 96.9k PBS/s.
    static constexpr bool PACK4 = N == 2048 && K == 1 && L == 1;
    // MAC operands (every row spectrum, the wave's own included) read back from LDS instead of
    // kept in registers: frees the own row's VGPRs.  Per shape (measured, gadget sets): on at
    // N = 2048 (PACK4) and N = 1024 (TFHE_LIB 93.7k -> 109.3k, ASCON_40 34.3k -> 37.4k,
    // MANTICORE +2%), off at N = 512 (SIMON_40 -3%, AES_40 -5%: no spills to remove there)
    static constexpr bool MAC_LDS = PBS_MAC_FROM_LDS >= 0 ? (bool)PBS_MAC_FROM_LDS : (PACK4 || N == 1024);
    // GGSW_i staged in LDS by async global->LDS loads and shared by the workgroup's ciphertexts;
    // fits next to the tables and 2 x (k+1) exchange buffers when it is <= 64 KiB
    // (only without the twist/M table: both do not fit next to four exchange buffers)
    static constexpr bool STAGE = PBS_GGSW_LDS && !PACK4 && GGSW_ELEMS * 16 <= 65536;
    static constexpr int CPW = PBS_CPW > 0 ? PBS_CPW : STAGE ? 2 : PACK4 ? 4 : 1;
    static constexpr bool GSYNC = PBS_GROUP_SYNC && !STAGE;  // the staged GGSW is shared by the workgroup
    static constexpr size_t flags_off() { return PbsLds<M>::bytes((K + 1) * CPW) + (STAGE ? GGSW_ELEMS * 16 : 0); }
    static constexpr size_t lds_bytes() { return flags_off() + (GSYNC ? 4 * (K + 1) * CPW + 4 * CPW : 0); }
    static_assert(lds_bytes() <= 160 * 1024, "LDS per workgroup exceeds a CU");
    // register budget per wave: 2 waves/SIMD for the packed 2_2 shape and N = 1024 (<= 256),
    // 3 at N = 512 (<= 168), 1 for the other N = 2048 shapes (~430 VGPR+AGPR at L = 2)
    static constexpr int WPE = PBS_WAVES_PER_EU > 0 ? PBS_WAVES_PER_EU
                                                    : (PACK4 ? 2 : N >= 2048 ? 1 : N == 1024 ? 2 : 3);
    // Persistent grid with a dynamic ciphertext queue (needs GSYNC: slots never wait on each other).
    // With one ciphertext per slot and launch, a workgroup holds its CU until its slowest slot is
    // done; its ciphertexts drift apart (per-ciphertext sync), so on average only 1.6 of the 2
    // waves per SIMD are resident (PMC).  Here a slot that finishes takes the next ciphertext from
    // a global ticket (one atomic per ciphertext), and the grid is one resident wave of workgroups.
    // Measured A/B (4096 PBS, `profiles/r02_ab_persistent_ticket.json`, PMC: 1.6 -> 1.88 resident
    // waves/SIMD at 2_2): 2_2 115.0k -> 125.3k PBS/s, 2_2 KS+PBS 111.4k -> 121.2k, MANTICORE
    // 98.0k -> 108.7k, SHA3_40 99.3k -> 114.8k, ASCON_40 37.3k -> 40.6k; slower for TFHE_LIB
    // (1024, 2, 1) 108.9k -> 104.5k and SIMON_40 (512, 3, 2) 97.5k -> 91.9k, even for AES_40:
    // on for the shapes where it measured faster (PBS_PERSIST = 0/1 forces it off/on).
    static constexpr bool PERSIST_DEFAULT =
        (N == 2048 && K == 1 && L == 1) || (N == 1024 && K == 1 && L == 2) || (N == 256 && K == 5 && L == 1) ||
        (N == 1024 && K == 2 && L == 3);
    static constexpr bool PERSIST = GSYNC && (PBS_PERSIST >= 0 ? (bool)PBS_PERSIST : PERSIST_DEFAULT);
    static constexpr size_t ticket_off() { return flags_off() + (GSYNC ? 4 * (K + 1) * CPW : 0); }
};

template <int N, int K, int L>
__global__ void __launch_bounds__((64 * (K + 1) * PbsConfig<N, K, L>::CPW), (PbsConfig<N, K, L>::WPE))
    pbs_classic_kernel(ClassicPbsLaunch a) {
    constexpr int M = N / 2;
    constexpr int V = M / 64;
    constexpr int LOG2N = ilog2(N);
    using Cfg = PbsConfig<N, K, L>;
    constexpr int CPW = Cfg::CPW;
    constexpr bool STAGE = Cfg::STAGE;
    using Fft = WaveFft<M>;
    using Lay = PbsLds<M>;
    constexpr int XL = Lay::XL;
    static_assert(sizeof(cx) * XL >= sizeof(uint64_t) * N, "exchange buffer holds one polynomial");

    extern __shared__ __attribute__((aligned(16))) char smem[];
    double2 *lds = reinterpret_cast<double2 *>(smem);
    const double2 *s_twist = lds + Lay::twist_off;

    // wave-uniform ids in SGPRs: per-ciphertext pointers and the mask element loads stay scalar
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane0 = threadIdx.x & 63;
    // wave -> (ciphertext slot, polynomial).  PBS_SLOT_MAJOR: wave w = r CPW + slot, so with the
    // workgroup's waves placed round-robin on the CU's 4 SIMDs each SIMD hosts the (k+1) waves of
    // ONE ciphertext (CPW = 4, k = 1) instead of rows of two different ciphertexts
    const int wave = PBS_SLOT_MAJOR ? wid / CPW : wid % (K + 1);  // polynomial of the ciphertext this wave owns
    const int slot = PBS_SLOT_MAJOR ? wid % CPW : wid / (K + 1);  // ciphertext slot in the workgroup
    const int n = a.n;
    const int beta = a.base_log;
    const uint32_t dmask = (1u << beta) - 1;
    const DigitL1 digit_l1(beta);                      // L = 1 digits
    const Digit2 digit2(L == 2 ? beta : 2);             // L = 2: both levels of a pair at once (2 beta <= 30)
    BlockSync sync;       // cross-wave: spectrum exchange
#if PBS_WAVE_LOCAL
    WaveLocalSync wsync;  // wave-private buffer reuse
#else
    BlockSync wsync;
#endif

    // twiddles and twist -> LDS (once per workgroup)
    for (int e = threadIdx.x; e < M; e += blockDim.x) lds[Lay::twist_off + e] = a.twist[e];
    uint32_t *gflags = reinterpret_cast<uint32_t *>(smem + Cfg::flags_off());
    if (Cfg::GSYNC && threadIdx.x < (K + 1) * CPW) gflags[threadIdx.x] = 0;
    Fft::Lds::template fill<M>(lds + Lay::s1_off, lds + Lay::s2_off, a.W, threadIdx.x, blockDim.x);
    const typename Fft::Lds tw{lds + Lay::s1_off, lds + Lay::s2_off};
    sync();  // tables visible to every wave (the CMUX loop itself only syncs wave-locally)

    cx *xct = reinterpret_cast<cx *>(lds + Lay::xbuf_off) + (size_t)slot * (K + 1) * XL;  // this ct's buffers
    // spectrum exchange among this ciphertext's waves
    std::conditional_t<Cfg::GSYNC, GroupSync<K + 1>, BlockSync> xsync;
    if constexpr (Cfg::GSYNC)
        xsync = {lds_addr(gflags + slot * (K + 1)), lds_addr(gflags + slot * (K + 1) + wave)};
    cx *xb = xct + wave * XL;
    uint64_t *xb64 = reinterpret_cast<uint64_t *>(xb);

    // Ciphertext loop.  PERSIST (per-ciphertext sync: a slot's (k+1) waves never wait on the
    // other slots): the grid is at most one resident wave of workgroups (sized by the host) and
    // each slot walks the batch with stride gridDim.x * CPW.  Otherwise the grid covers the batch
    // (one trip); idle slots compute on a valid ciphertext and store nothing.
    // The launch arguments are read inside the per-ciphertext routine through a kernarg-segment
    // pointer laundered per call: in the persistent loop the compiler would otherwise keep every
    // argument in SGPRs across the CMUX loop (SGPR spills into VGPR lanes, +24 VGPRs, 3 spilled).
    using KArg = const __attribute__((address_space(4))) ClassicPbsLaunch;
    auto run_ct = [&](const int ct_raw) {
    KArg *ka = (KArg *)__builtin_amdgcn_kernarg_segment_ptr();
    if constexpr (Cfg::PERSIST) asm volatile("" : "+s"(ka));
    const ClassicPbsLaunch &A = *(const ClassicPbsLaunch *)ka;
    int lane = lane0;  // per-ciphertext opaque copy: lane-derived addresses are not hoisted across ciphertexts
    if constexpr (Cfg::PERSIST) asm volatile("" : "+v"(lane));
    const bool active = ct_raw < A.count;  // idle slots compute on a valid ct, store nothing
    const int ct = active ? ct_raw : A.count - 1;
    const uint64_t *in = A.lwe_in + (size_t)ct * (n + 1);
    // the input row is read-only for the whole launch: constant address space -> s_load
    const __attribute__((address_space(4))) uint64_t *in_s = (const __attribute__((address_space(4))) uint64_t *)(
        ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)((uintptr_t)in >> 32)) << 32) |
        (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)in));
    const uint32_t li = A.lut_indexes ? min(A.lut_indexes[ct], A.lut_count - 1u) : 0u;
    const uint64_t *lut = A.luts + (size_t)li * (K + 1) * N + (size_t)wave * N;

    // this wave's accumulator polynomial, in registers: c0[h] = position lane + 64 h
    // (h < V: j < M; h >= V: j = M + lane + 64 (h - V)).  ct0 = LUT / X^{b~}
    // (bootstrap.rs:255-275, polynomial_wrapping_monic_monomial_div)
    uint64_t c0[2 * V];
    {
        const uint32_t bt = pbs_modulus_switch<LOG2N>(in[n]);
        const int full = bt / N, rem = bt % N;
#pragma unroll
        for (int h = 0; h < 2 * V; h++) {
            const int src = lane + 64 * h + rem;
            const bool wrap = src >= N;
            uint64_t v = lut[wrap ? src - N : src];
            c0[h] = (wrap != (bool)(full & 1)) ? 0 - v : v;
        }
    }

    constexpr size_t ggsw_stride = (size_t)L * (K + 1) * (K + 1) * M;
    const double2 *gcol = A.fbsk + (size_t)wave * M + lane;  // column c = wave, this lane
    // staged GGSW: LDS image identical to the global one (lane-linear 1 KiB chunks)
    double2 *s_ggsw = lds + Lay::xbuf_off + (size_t)CPW * (K + 1) * XL;
    // The LDS-DMA is issued from inline asm: issued through the builtin, hipcc makes every later
    // LDS read wait vmcnt(0) (it cannot prove the DMA target disjoint), which drains the prefetch
    // at the first FFT twiddle read.  Hidden from it, the copy is retired explicitly before the
    // barrier that precedes its reader (stage_ggsw_wait); the loop issues no other vector loads.
    const uint32_t s_ggsw_addr = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) char *)(s_ggsw));
    auto stage_ggsw = [&](int i) {
        const double2 *src = A.fbsk + (size_t)i * ggsw_stride + lane0;
        for (int q = wid; q < (int)(ggsw_stride / 64); q += CPW * (K + 1)) {
            const uint32_t dst = __builtin_amdgcn_readfirstlane(s_ggsw_addr + (uint32_t)q * 1024u);
            uint32_t keep;
            asm volatile(
                "s_mov_b32 %0, m0\n\t"
                "s_mov_b32 m0, %2\n\t"
                "s_nop 0\n\t"
                "global_load_lds_dwordx4 %1, off\n\t"
                "s_mov_b32 m0, %0"
                : "=&s"(keep)
                : "v"(src + q * 64), "s"(dst)
                : "memory");
        }
    };
    auto stage_ggsw_wait = [&]() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); };
    if constexpr (STAGE) stage_ggsw(0);  // drained by the first spectrum-publish barrier
    // L = 1: this wave's GGSW column for the next CMUX is loaded into registers right after the
    // current MAC, so its L2/MALL latency hides behind the inverse FFT, the rotation and the
    // forward FFT (the vmcnt wait lands at the MAC; no other vector loads in the loop).
    constexpr bool PREF = PBS_GGSW_PREFETCH && L == 1 && !STAGE;
    double2 gpre[PREF ? V * (K + 1) : 1];
    auto prefetch = [&](int ii) {
        const double2 *g = gcol + (size_t)ii * ggsw_stride;
#pragma unroll
        for (int s = 0; s < V; s++)
#pragma unroll
            for (int r = 0; r <= K; r++) gpre[s * (K + 1) + r] = g[(size_t)r * (K + 1) * M + s * 64];
    };
    if constexpr (PREF) {
        prefetch(0);
        __builtin_amdgcn_sched_barrier(0);
    }

    const double k32 = torus_k32();
    for (int i = 0; i < n; i++) {
        // Every LDS/GGSW address below is a function of the lane only (loop invariant); hoisted
        // out of the CMUX loop they pin ~100 VGPRs and spill.  An opaque per-iteration copy of the
        // lane id makes them cheap per-iteration recomputations instead.
        int lane = lane0;
        asm volatile("" : "+v"(lane));
        // mask element through the scalar unit: an s_load waits on lgkmcnt, never on the vmcnt
        // that the GGSW LDS-DMA occupies
        const uint32_t at = pbs_modulus_switch<LOG2N>(in_s[i]);
        const bool full_odd = (at / N) & 1;
        const int rem = at % N;
        const double2 *ggsw = STAGE ? s_ggsw + (size_t)wave * M + lane : gcol + (size_t)i * ggsw_stride;

        // ct1 = X^{a~} ct0 - ct0 (polynomial_algorithms.rs:425-490) through the LDS buffer
        // (wave-private: the other waves' last reads of it ended at the post-MAC barrier)
        if (!PBS_TSKIP_ROT) {
            wsync();
#pragma unroll
            for (int h = 0; h < 2 * V; h++) xb64[lane + 64 * h] = c0[h];
            wsync();
        }
        // (X^d p)[j] = -p[N-d+j] for j < d, p[j-d] otherwise (sign flipped again when the
        // rotation passes a full N); only the top 32 bits of ct1 feed the decomposition.
        // Source index jj = lane - rem + 64 h wraps (jj < 0) exactly for h < hcut, so the gather
        // address is a select between two lane bases with 8*64*h in the ds_read offset field (no
        // per-coefficient index arithmetic); xpos may sit up to 8(N-1) bytes below xb64, which is
        // still inside LDS since the twist table (8N bytes) precedes every exchange buffer.
        const int rbase = lane - rem;  // in (-N, 64)
        const int hcut = (63 - rbase) >> 6;
        const uint64_t *xpos = xb64 + rbase;
        const uint64_t *xneg = xpos + N;
        auto ct1_hi = [&](int h) -> uint32_t {
            if (PBS_TSKIP_ROT) return (uint32_t)(c0[h] >> 32) ^ at;  // timing only: no rotation
            const bool wrap = h < hcut;
            const bool neg = wrap != full_odd;
            const uint64_t x = (wrap ? xneg : xpos)[64 * h];
            const uint64_t r = neg ? 0 - x : x;
            return (uint32_t)((r - c0[h]) >> 32);
        };
        uint32_t st[L > 1 ? 2 * V : 1];
        if constexpr (L == 2 && CLASSIC_DIGIT2) {
            // st[b] = level-L int16 pair of positions (b, V + b), st[V + b] = level L-1 (Digit2)
#pragma unroll
            for (int b = 0; b < V; b++) digit2.pair(ct1_hi(b), ct1_hi(V + b), st[b], st[V + b]);
        } else if constexpr (L > 1) {
#pragma unroll
            for (int h = 0; h < 2 * V; h++) st[h] = decomp_state32_hi<L>(ct1_hi(h), beta);
        }

        cx acc[L > 1 ? V : 1];
        // L > 1: a runtime level loop (one copy of the FFT/MAC code); unrolled, the compiler
        // overlaps consecutive levels and the register demand grows by ~(K+1)*V*4 per level
#pragma unroll 1
        for (int lvl = L; lvl >= 1; lvl--) {
            cx v[V];
#pragma unroll
            for (int b = 0; b < V; b++) {
                int32_t d0, d1;
                if constexpr (L == 1) {
                    d0 = digit_l1(ct1_hi(b));
                    d1 = digit_l1(ct1_hi(V + b));
                } else if constexpr (L == 2 && CLASSIC_DIGIT2) {
                    const uint32_t w = lvl == L ? st[b] : st[V + b];
                    d0 = (int32_t)(int16_t)(w & 0xffffu);
                    d1 = (int32_t)(int16_t)(w >> 16);
                } else {
                    d0 = decomp_digit32(st[b], beta, dmask);
                    d1 = decomp_digit32(st[V + b], beta, dmask);
                }
                const cx z = {(double)d0, (double)d1};
                const double2 w = s_twist[lane + 64 * b];
                v[b] = cmulw(z, w.x, w.y);  // convert_forward_integer (x86.rs:505-596)
            }
            Fft::forward(v, xb, tw, lane, wsync);
            // publish this row's spectrum to the ciphertext's other waves
            wsync();
#pragma unroll
            for (int s = 0; s < V; s++)
                reinterpret_cast<double2 *>(xb)[s * 64 + lane] = make_double2(v[s].re, v[s].im);
            if constexpr (STAGE) stage_ggsw_wait();  // this wave's part of GGSW_i has landed
            xsync();
            // output column c = wave: sum_r F_r * G[lvl][r][c]   (ggsw.rs:524-567, update_with_fmadd)
            const double2 *lm = ggsw + (size_t)(lvl - 1) * (K + 1) * (K + 1) * M;
#pragma unroll
            for (int s = 0; s < V; s++) {
                if (s % PBS_MAC_SB == 0) __builtin_amdgcn_sched_barrier(0);  // bound loads in flight
                cx o = (L > 1 && lvl != L) ? acc[L > 1 ? s : 0] : cx{0.0, 0.0};
#pragma unroll
                for (int r = 0; r <= K; r++) {
                    const double2 gg = PREF ? gpre[PREF ? s * (K + 1) + r : 0] : lm[(size_t)r * (K + 1) * M + s * 64];
                    double2 ff;
                    if (Cfg::MAC_LDS) {  // every row from LDS: no wave-dependent branch
                        ff = reinterpret_cast<const double2 *>(xct + r * XL)[s * 64 + lane];
                    } else if (r == wave) {
                        ff = make_double2(v[s].re, v[s].im);
                    } else {
                        ff = reinterpret_cast<const double2 *>(xct + r * XL)[s * 64 + lane];
                    }
                    if (lvl == L && r == 0) {
                        o.re = fma(gg.x, ff.x, -(gg.y * ff.y));
                        o.im = fma(gg.x, ff.y, gg.y * ff.x);
                    } else {
                        o.re = fma(gg.x, ff.x, fma(-gg.y, ff.y, o.re));
                        o.im = fma(gg.x, ff.y, fma(gg.y, ff.x, o.im));
                    }
                }
                if constexpr (L > 1) acc[s] = o;
                else v[s] = o;
            }
            xsync();  // every wave is done reading the published spectra (and the staged GGSW)
            if constexpr (PREF) {
                __builtin_amdgcn_sched_barrier(0);
                if (i + 1 < n) prefetch(i + 1);
                __builtin_amdgcn_sched_barrier(0);
            }
            if constexpr (STAGE) {
                // prefetch GGSW_{i+1} into LDS: overlaps the inverse FFT, the rotation and the
                // forward FFT; the next publish barrier (its vmcnt(0)) retires it
                if (lvl == 1 && i + 1 < n) stage_ggsw(i + 1);
            }
            if constexpr (L == 1) {
                Fft::inverse(v, xb, tw, lane, wsync);
#pragma unroll
                for (int b = 0; b < V; b++) {
                    if (b % PBS_BWD_SB == 0) __builtin_amdgcn_sched_barrier(0);
                    const double2 w = s_twist[lane + 64 * b];  // the resident key carries the 1/M
                    backward_add(v[b], cx{w.x, w.y}, c0[b], c0[V + b], k32);
                }
            }
        }
        if constexpr (L > 1) {
            Fft::inverse(acc, xb, tw, lane, wsync);
#pragma unroll
            for (int b = 0; b < V; b++) {
                const double2 w = s_twist[lane + 64 * b];
                backward_add(acc[b], cx{w.x, w.y}, c0[b], c0[V + b], k32);
            }
        }
    }

    if (A.glwe_out) {  // bootstrap_without_sample_extract (fork, bootstrap.rs:383-412)
        if (active) {
            uint64_t *g = A.lwe_out + ((size_t)ct * (K + 1) + wave) * N;
#pragma unroll
            for (int h = 0; h < 2 * V; h++) g[lane0 + 64 * h] = c0[h];
        }
        return;
    }
    // sample extract at degree 0 (glwe_sample_extraction.rs:91-147)
    wsync();
#pragma unroll
    for (int h = 0; h < 2 * V; h++) xb64[lane0 + 64 * h] = c0[h];
    wsync();
    if (active) {
        uint64_t *out = A.lwe_out + (size_t)ct * (K * N + 1);
        if (wave < K) {
            for (int j = lane0; j < N; j += 64) out[wave * N + j] = j == 0 ? xb64[0] : 0 - xb64[N - j];
        } else if (lane0 == 0) {
            out[K * N] = c0[0];
        }
    }
    wsync();  // the extract's reads of xb64 precede the next ciphertext's rotation writes
    };
    if constexpr (Cfg::PERSIST) {
        // first ciphertext: the slot's static index; then tickets (none without a ticket word: one
        // pass).  Row 0 of the slot takes the ticket (one lane, a vector atomic) and hands it to
        // its partner waves through LDS; the GroupSyncs that every wave of the slot executes once
        // per ciphertext order the handover.
        uint32_t *tslot = reinterpret_cast<uint32_t *>(smem + Cfg::ticket_off()) + slot;
        // a small batch is spread over the CUs (cpw_eff < CPW slots per workgroup, no tickets): a
        // ciphertext alone on its CU runs its CMUX chain ~1.5x faster than four sharing it
        const int cpw = a.cpw_eff > 0 ? a.cpw_eff : CPW;
        int ct_raw = slot < cpw ? (int)blockIdx.x * cpw + slot : a.count;
        while (ct_raw < a.count) {
            run_ct(ct_raw);
            if (!a.ticket) break;
            if (wave == 0) {
                uint32_t t = 0;
                if (lane0 == 0) t = atomicAdd(a.ticket, 1u);
                t = __builtin_amdgcn_readfirstlane(t);
                if (lane0 == 0) *tslot = t;
            }
            xsync();
            ct_raw = (int)gridDim.x * CPW + (int)__builtin_amdgcn_readfirstlane(*(volatile uint32_t *)tslot);
            xsync();  // every wave has read the ticket before row 0 may overwrite it
        }
    } else {
        run_ct(blockIdx.x * CPW + slot);
    }
}

template <int N, int K, int L>
static hipError_t launch_pbs_t(const ClassicPbsLaunch &a, hipStream_t s) {
    constexpr int CPW = PbsConfig<N, K, L>::CPW;
    const size_t lds = PbsConfig<N, K, L>::lds_bytes();
    if (a.count == 0) return hipSuccess;
    const int threads = 64 * (K + 1) * CPW;
    int blocks = (a.count + CPW - 1) / CPW;
    if (PbsConfig<N, K, L>::PERSIST && a.ticket) {
        const int res = resident_blocks((const void *)pbs_classic_kernel<N, K, L>, threads, lds);
        if (CPW > 1 && a.count <= res * (CPW - 1)) {
            // fewer ciphertexts than a packed resident grid: spread them, ceil(count / res) per
            // workgroup (latency of the coalesced small batches: 9.0 -> 5.8 ms at 2_2 alone on a CU)
            ClassicPbsLaunch b = a;
            b.cpw_eff = (a.count + res - 1) / res;
            b.ticket = nullptr;
            blocks = (a.count + b.cpw_eff - 1) / b.cpw_eff;
            hipLaunchKernelGGL((pbs_classic_kernel<N, K, L>), dim3(blocks), dim3(threads), lds, s, b);
            return hipGetLastError();
        }
        blocks = std::min(blocks, res);
    }
    hipLaunchKernelGGL((pbs_classic_kernel<N, K, L>), dim3(blocks), dim3(threads), lds, s, a);
    return hipGetLastError();
}

// Instantiated shapes: the shortint sets (k = 1, N = 2048 / 1024) and the fork's gadget sets
// (gadget/parameters/mod.rs:84-235: k = 2, 3 at N = 512 / 1024, levels 1-4; SHA3_40: k = 5, N = 256).
#define PBS_CLASSIC_SHAPES(X) \
    X(2048, 1, 1) X(2048, 1, 2) \
    X(1024, 1, 1) X(1024, 1, 2) X(1024, 1, 3) X(1024, 1, 4) \
    X(1024, 2, 1) X(1024, 2, 2) X(1024, 2, 3) X(1024, 2, 4) \
    X(1024, 3, 1) X(1024, 3, 2) X(1024, 3, 3) \
    X(512, 1, 1) X(512, 1, 2) X(512, 1, 3) X(512, 1, 4) \
    X(512, 2, 1) X(512, 2, 2) X(512, 2, 3) X(512, 2, 4) \
    X(512, 3, 1) X(512, 3, 2) X(512, 3, 3) X(512, 3, 4) \
    X(256, 5, 1)

// bytes of zeroed device scratch the launch wants for its ciphertext ticket (0: no persistent grid)
size_t classic_pbs_ticket_bytes(int N, int k, int L) {
#define PBS_TICKET(n_, k_, l_) if (N == n_ && k == k_ && L == l_) return PbsConfig<n_, k_, l_>::PERSIST ? 256 : 0;
    PBS_CLASSIC_SHAPES(PBS_TICKET)
#undef PBS_TICKET
    return 0;
}

bool classic_pbs_supported(int N, int k, int L) {
#define PBS_SUPPORTED(n_, k_, l_) if (N == n_ && k == k_ && L == l_) return true;
    PBS_CLASSIC_SHAPES(PBS_SUPPORTED)
#undef PBS_SUPPORTED
    return false;
}

hipError_t launch_classic_pbs(int N, int k, int L, const ClassicPbsLaunch &a, hipStream_t s) {
#define PBS_LAUNCH(n_, k_, l_) if (N == n_ && k == k_ && L == l_) return launch_pbs_t<n_, k_, l_>(a, s);
    PBS_CLASSIC_SHAPES(PBS_LAUNCH)
#undef PBS_LAUNCH
    return hipErrorInvalidValue;
}

// ---------------------------------------------------------------------------------------
// standard -> Fourier BSK (forward_as_torus, fft/mod.rs:197-218 + 378-385): one wave per
// polynomial; output in the engine layout [poly][slot*64 + lane].
// ---------------------------------------------------------------------------------------
template <int N>
__global__ void __launch_bounds__(64) bsk_to_fourier_kernel(const uint64_t *__restrict__ polys,
                                                            double2 *__restrict__ out, size_t npoly,
                                                            const double2 *__restrict__ W,
                                                            const double2 *__restrict__ twist) {
    constexpr int M = N / 2;
    constexpr int V = M / 64;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    cx *xb = reinterpret_cast<cx *>(smem);
    const int lane = threadIdx.x;
    const size_t p = blockIdx.x;
    if (p >= npoly) return;  // whole (single-wave) block exits together
    const uint64_t *x = polys + p * N;
    cx v[V];
#pragma unroll
    for (int b = 0; b < V; b++) {
        const int j = lane + 64 * b;
        double xr = (double)(int64_t)x[j] * fourier_key_scale(M);
        double xi = (double)(int64_t)x[j + M] * fourier_key_scale(M);
        cx w = gld(twist + j);
        v[b].re = xr * w.re - xi * w.im;
        v[b].im = xr * w.im + xi * w.re;
    }
    WaveFft<M>::forward(v, xb, GlobalTwiddles<M>{W}, lane, BlockSync{});
    double2 *o = out + p * M + lane;
#pragma unroll
    for (int s = 0; s < V; s++) o[s * 64] = make_double2(v[s].re, v[s].im);
}

hipError_t launch_bsk_to_fourier(int N, const uint64_t *std_polys, double2 *fourier, size_t npoly,
                                 const FftTables &t, hipStream_t s) {
    if (npoly == 0) return hipSuccess;
    if (N == 2048) {
        hipLaunchKernelGGL(bsk_to_fourier_kernel<2048>, dim3(npoly), dim3(64),
                           sizeof(cx) * WaveFft<1024>::XL, s, std_polys, fourier, npoly, t.W, t.twist);
    } else if (N == 1024) {
        hipLaunchKernelGGL(bsk_to_fourier_kernel<1024>, dim3(npoly), dim3(64),
                           sizeof(cx) * WaveFft<512>::XL, s, std_polys, fourier, npoly, t.W, t.twist);
    } else if (N == 512) {
        hipLaunchKernelGGL(bsk_to_fourier_kernel<512>, dim3(npoly), dim3(64),
                           sizeof(cx) * WaveFft<256>::XL, s, std_polys, fourier, npoly, t.W, t.twist);
    } else if (N == 256) {
        hipLaunchKernelGGL(bsk_to_fourier_kernel<256>, dim3(npoly), dim3(64),
                           sizeof(cx) * WaveFft<128>::XL, s, std_polys, fourier, npoly, t.W, t.twist);
    } else {
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace tfhe_mi355
