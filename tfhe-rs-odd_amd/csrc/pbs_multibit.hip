// pbs_multibit.hip -- batched multi-bit programmable bootstrap on gfx950.
//
// Replaces (reference tfhe-rs-odd, CPU Rust):
//   multi_bit_programmable_bootstrap_lwe_ciphertext    lwe_multi_bit_programmable_bootstrapping.rs:1035-1128
//   multi_bit_deterministic_blind_rotate_assign        same file :548-828 (group order 0..n/g-1)
//   prepare_multi_bit_ggsw_mem_optimized (keybundle)   same file :18-84
//   update_with_fmadd_factor                           fft64/crypto/ggsw.rs:699-754
//   incomplete_monomial_forward_as_integer             fft64/math/fft/mod.rs:407-445
//   add_external_product_assign                        fft64/crypto/ggsw.rs:477-598
//
// Design (DESIGN.md "Kernels"): the classic kernel's shape -- one workgroup per ciphertext, one
// wavefront per GLWE polynomial, accumulator in registers -- with the CMUX replaced by the
// multi-bit step  acc <- ExtProd(KB_j, acc),  KB_j = sum_sel X^{deg_sel} GGSW_{j,sel}.
// The keybundle is never materialised: wave c builds KB_j[lvl][r][c] for its column frequency
// by frequency in registers while it streams the 2^g GGSW columns, and immediately contracts it
// with the published row spectra.  The monomial spectra are 2N-th roots of unity read from the
// twist table in LDS (exact sign/swap, no rounding; oracle mono_spectrum), so the keybundle
// costs 2^g - 1 complex FMAs per GGSW element and one LDS read per (monomial, frequency).
// No rotation is needed (ct1 = acc), and the backward transform overwrites the accumulator
// (the reference's zeroed ping-pong destination, :782-800).
#include "engine.h"
#include "pbs_common.h"

namespace tfhe_mi355 {

// Ciphertexts per workgroup and register budget.  As the classic 2_2 kernel: 4 ciphertexts per
// workgroup at 2 waves/SIMD (31 KiB of tables + 8 x 16 KiB exchange buffers = 159 KiB of LDS),
// the MAC reading every row spectrum from LDS and a one-slot issue window for the GGSW loads so
// the wave fits 256 registers.
#ifndef PBS_MB_CPW
#define PBS_MB_CPW 4
#endif
#ifndef PBS_MB_WINDOW
#define PBS_MB_WINDOW 4  // MAC slots whose GGSW loads may be in flight (4: 234 VGPRs at g = 3; 8 spills)
#endif
#ifndef PBS_MB_MAC_LDS
#define PBS_MB_MAC_LDS 1
#endif
#ifndef PBS_MB_BUFLD
#define PBS_MB_BUFLD 1  // GGSW loads through a buffer resource: scalar offsets, no 64-bit VALU address adds
#endif
// TwistLds (the twist table in LDS, shared with the multi-bit latency kernel): pbs_common.h

constexpr int mb_wpe() { return PBS_WAVES_PER_EU > 0 ? PBS_WAVES_PER_EU : (PBS_MB_CPW >= 4 ? 2 : 1); }

template <int N, int K, int L, int G>
__global__ void __launch_bounds__(64 * (K + 1) * PBS_MB_CPW, mb_wpe())
    pbs_multibit_kernel(MultiBitPbsLaunch a) {
    constexpr int CPW = PBS_MB_CPW;
    constexpr int M = N / 2;
    constexpr int V = M / 64;
    constexpr int LOG2N = ilog2(N);
    constexpr int NSEL = 1 << G;
    using Fft = WaveFft<M>;
    using Lay = PbsLds<M>;
    constexpr int XL = Lay::XL;
    static_assert(sizeof(cx) * XL >= sizeof(uint64_t) * N, "exchange buffer holds one polynomial");

    extern __shared__ __attribute__((aligned(16))) char smem[];
    double2 *lds = reinterpret_cast<double2 *>(smem);
    using Tw = TwistLds<M>;

    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wave = wid % (K + 1);  // polynomial / column
    const int slot = wid / (K + 1);  // ciphertext slot in the workgroup
    const int lane0 = threadIdx.x & 63;
    int lane = lane0;
    const int ct_raw = blockIdx.x * CPW + slot;
    const bool active = ct_raw < a.count;  // idle slots compute on a valid ct, store nothing
    const int ct = active ? ct_raw : a.count - 1;
    const int n = a.n;
    const int beta = a.base_log;
    const uint32_t dmask = (1u << beta) - 1;
    const DigitL1 digit_l1(beta);
    BlockSync sync;
    WaveLocalSync wsync;

    Tw::fill(reinterpret_cast<double *>(lds + Lay::twist_off), a.twist, threadIdx.x, blockDim.x);
    // spectrum exchange among this ciphertext's waves (GroupSync, pbs_common.h): flags after the buffers
    uint32_t *gflags = reinterpret_cast<uint32_t *>(smem + Lay::bytes((K + 1) * CPW));
    if (PBS_GROUP_SYNC && threadIdx.x < (K + 1) * CPW) gflags[threadIdx.x] = 0;
    std::conditional_t<(bool)PBS_GROUP_SYNC, GroupSync<K + 1>, BlockSync> xsync;
    if constexpr ((bool)PBS_GROUP_SYNC) xsync = {lds_addr(gflags + slot * (K + 1)), lds_addr(gflags + wid)};
    Fft::Lds::template fill<M>(lds + Lay::s1_off, lds + Lay::s2_off, a.W, threadIdx.x, blockDim.x);
    const typename Fft::Lds tw{lds + Lay::s1_off, lds + Lay::s2_off};
    sync();

    cx *xct = reinterpret_cast<cx *>(lds + Lay::xbuf_off) + (size_t)slot * (K + 1) * XL;  // this ct's buffers
    cx *xb = xct + wave * XL;
    uint64_t *xb64 = reinterpret_cast<uint64_t *>(xb);
    const uint64_t *in = a.lwe_in + (size_t)ct * (n + 1);
    const uint32_t li = a.lut_indexes ? min(a.lut_indexes[ct], a.lut_count - 1u) : 0u;
    const uint64_t *lut = a.luts + (size_t)li * (K + 1) * N + (size_t)wave * N;

    // acc = LUT / X^{b~}  (:635-650), position lane + 64 h
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

    constexpr size_t ggsw_len = (size_t)L * (K + 1) * (K + 1) * M;
    constexpr size_t lvl_len = (size_t)(K + 1) * (K + 1) * M;
    const double2 *gcol = a.fbsk + (size_t)wave * M + lane;  // column c = wave, this lane
    // the same column as a buffer resource: per-lane byte offset (VGPR, loop invariant; laundered
    // through the issue window) + scalar offsets for group / selector / level / row / slot
    const __amdgpu_buffer_rsrc_t gres = make_rsrc(a.fbsk + (size_t)wave * M);
    const int groups = n / G;

    const double k32 = torus_k32();
    for (int j = 0; j < groups; j++) {
        int lane = lane0;
        asm volatile("" : "+v"(lane));
        // monomial degrees of the 2^g - 1 non-constant GGSWs (wave-uniform, :700-716)
        uint32_t d4[NSEL];
        {
            uint64_t av[G];
#pragma unroll
            for (int i = 0; i < G; i++) av[i] = in[j * G + i];
#pragma unroll
            for (int sel = 1; sel < NSEL; sel++) {
                uint64_t deg = 0;
#pragma unroll
                for (int i = 0; i < G; i++)
                    if ((sel >> (G - 1 - i)) & 1) deg += av[i];
                d4[sel] = pbs_modulus_switch<LOG2N>(deg);
            }
        }
        // per-lane part of t = d (1 - 4 f) mod 2N with f = freq_lane + freq_slot
        const uint32_t fl = Fft::freq_lane(lane);
        // the twist table is the first LDS object and the kernel has no static LDS, so its byte
        // address is 0 and the monomial read addresses need no base
        static_assert(Lay::twist_off == 0, "twist table at LDS offset 0");
        const uint32_t lb = Tw::lane_base(lane);
        uint32_t tb[NSEL];
#pragma unroll
        for (int sel = 1; sel < NSEL; sel++) {
            tb[sel] = d4[sel] - 4u * d4[sel] * fl;  // t mod 2^32 at freq_slot 0
            d4[sel] *= 4u;
        }
        const double2 *grp = gcol + (size_t)j * NSEL * ggsw_len;
        const uint32_t gsoff = (uint32_t)((size_t)j * NSEL * ggsw_len * 16);  // < 2^31 (MB-BSK bytes)

        uint32_t st[L > 1 ? 2 * V : 1];
        if constexpr (L > 1) {
#pragma unroll
            for (int h = 0; h < 2 * V; h++) st[h] = decomp_state32_hi<L>((uint32_t)(c0[h] >> 32), beta);
        }

        cx acc[L > 1 ? V : 1];
#pragma unroll
        for (int lvl = L; lvl >= 1; lvl--) {
            cx v[V];
#pragma unroll
            for (int b = 0; b < V; b++) {
                int32_t d0, d1;
                if constexpr (L == 1) {
                    d0 = digit_l1((uint32_t)(c0[b] >> 32));
                    d1 = digit_l1((uint32_t)(c0[V + b] >> 32));
                } else {
                    d0 = decomp_digit32(st[b], beta, dmask);
                    d1 = decomp_digit32(st[V + b], beta, dmask);
                }
                const cx z = {(double)d0, (double)d1};
                const cx w = Tw::linear(lb, b);
                v[b] = cmulw(z, w.re, w.im);
            }
            Fft::forward(v, xb, tw, lane, wsync);
            wsync();
#pragma unroll
            for (int s = 0; s < V; s++)
                reinterpret_cast<double2 *>(xb)[s * 64 + lane] = make_double2(v[s].re, v[s].im);
            xsync();
            const double2 *lm = grp + (size_t)(lvl - 1) * lvl_len;
            const uint32_t lsoff = gsoff + (uint32_t)((lvl - 1) * lvl_len * 16);
            uint32_t loff = 16u * (uint32_t)lane;
#pragma unroll
            for (int s = 0; s < V; s++) {
                // Issue window: slot s's GGSW loads and monomial reads take their addresses from
                // an opaque copy that depends on the result of slot s-2, so at most two slots of
                // operands are in flight (hoisted all at once they need ~1 KiB/lane and spill).
                if (s >= PBS_MB_WINDOW) {
                    const double dep = (L > 1) ? acc[L > 1 ? s - PBS_MB_WINDOW : 0].re : v[s - PBS_MB_WINDOW].re;
                    if (PBS_MB_BUFLD) asm volatile("" : "+v"(loff) : "v"(dep));
                    else asm volatile("" : "+v"(lm) : "v"(dep));
#pragma unroll
                    for (int sel = 1; sel < NSEL; sel++) asm volatile("" : "+v"(tb[sel]) : "v"(dep));
                }
                // monomial spectra at this frequency: i^q twist[r], t = q M + r
                cx mono[NSEL];
#pragma unroll
                for (int sel = 1; sel < NSEL; sel++) mono[sel] = Tw::mono(tb[sel] - d4[sel] * Fft::freq_slot(s));
                cx o = (L > 1 && lvl != L) ? acc[L > 1 ? s : 0] : cx{0.0, 0.0};
#pragma unroll
                for (int r = 0; r <= K; r++) {
                    // KB[lvl][r][c] at this frequency (keybundle, oracle mb_keybundle order)
                    const double2 *gp = lm + (size_t)r * (K + 1) * M + s * 64;
                    const uint32_t rsoff = lsoff + (uint32_t)((r * (K + 1) * M + s * 64) * 16);
                    double2 kb = PBS_MB_BUFLD ? buffer_ld_d2(gres, loff, rsoff) : gp[0];
#pragma unroll
                    for (int sel = 1; sel < NSEL; sel++) {
                        const double2 gg = PBS_MB_BUFLD ? buffer_ld_d2(gres, loff, rsoff + (uint32_t)(sel * ggsw_len * 16))
                                                        : gp[(size_t)sel * ggsw_len];
                        kb.x = fma(gg.x, mono[sel].re, fma(-gg.y, mono[sel].im, kb.x));
                        kb.y = fma(gg.x, mono[sel].im, fma(gg.y, mono[sel].re, kb.y));
                    }
                    double2 ff;
                    if (PBS_MB_MAC_LDS) {  // every row from LDS: no wave-dependent branch
                        ff = reinterpret_cast<const double2 *>(xct + r * XL)[s * 64 + lane];
                    } else if (r == wave) {
                        ff = make_double2(v[s].re, v[s].im);
                    } else {
                        ff = reinterpret_cast<const double2 *>(xct + r * XL)[s * 64 + lane];
                    }
                    if (lvl == L && r == 0) {
                        o.re = fma(kb.x, ff.x, -(kb.y * ff.y));
                        o.im = fma(kb.x, ff.y, kb.y * ff.x);
                    } else {
                        o.re = fma(kb.x, ff.x, fma(-kb.y, ff.y, o.re));
                        o.im = fma(kb.x, ff.y, fma(kb.y, ff.x, o.im));
                    }
                }
                if constexpr (L > 1) acc[s] = o;
                else v[s] = o;
            }
            xsync();  // every wave is done reading the published spectra before xb is reused
            if constexpr (L == 1) {
                Fft::inverse(v, xb, tw, lane, wsync);
#pragma unroll
                for (int b = 0; b < V; b++)  // the resident key carries the 1/M
                    backward_convert(v[b], Tw::linear(lb, b), c0[b], c0[V + b], k32);
            }
        }
        if constexpr (L > 1) {
            Fft::inverse(acc, xb, tw, lane, wsync);
#pragma unroll
            for (int b = 0; b < V; b++) backward_convert(acc[b], Tw::linear(lb, b), c0[b], c0[V + b], k32);
        }
    }

    if (a.glwe_out) {  // bootstrap_without_sample_extract (fork, bootstrap.rs:383-412)
        if (!active) return;
        uint64_t *g = a.lwe_out + ((size_t)ct * (K + 1) + wave) * N;
#pragma unroll
        for (int h = 0; h < 2 * V; h++) g[lane + 64 * h] = c0[h];
        return;
    }
    // sample extract at degree 0 (glwe_sample_extraction.rs:91-147)
    wsync();
#pragma unroll
    for (int h = 0; h < 2 * V; h++) xb64[lane + 64 * h] = c0[h];
    wsync();
    if (!active) return;
    uint64_t *out = a.lwe_out + (size_t)ct * (K * N + 1);
    if (wave < K) {
        for (int j = lane; j < N; j += 64) out[wave * N + j] = j == 0 ? xb64[0] : 0 - xb64[N - j];
    } else if (lane == 0) {
        out[K * N] = c0[0];
    }
}

#ifndef PBS_MB_SHARED
#define PBS_MB_SHARED 1  // slot-split MAC phase: each GGSW element is loaded once per workgroup
#endif

// Slot-split variant (PBS_MB_SHARED, L = 1).  The kernel above streams every GGSW column once per
// ciphertext: 2^g (k+1)^2 M 16 B = 512 KiB per group and ciphertext at g = 3 (155 MB per PBS) from
// L2/MALL -- ~20 TB/s of L2->CU traffic at 128k PBS/s, and its waves wait on it (PMC: s_waitcnt
// 0.48 of wave cycles, VALU 0.26).  Here the CPW ciphertexts of a workgroup share each load:
//   phase 1  wave (ct, r): digits of its accumulator row, twist, forward FFT, publish F_ct[r]
//   phase 2  wave w owns spectrum slots s = w SPW .. w SPW + SPW-1 for EVERY ciphertext and
//            column: it loads G[sel][r][c][s] once and builds KB_ct and the MAC for each of the
//            CPW ciphertexts (their monomials differ), writing out_ct[c][s] over F_ct[c][s] (no
//            other wave touches slot s)
//   phase 3  wave (ct, c): inverse FFT of out_ct[c], backward conversion into its accumulator
// Two workgroup barriers per group.  Per (ciphertext, column, frequency) the arithmetic and its
// order are those of the kernel above (keybundle in selector order, MAC over rows in order), so
// the outputs are bit-identical; a ciphertext's GGSW traffic drops by CPW (4x).
template <int N, int K, int L, int G>
__global__ void __launch_bounds__(64 * (K + 1) * PBS_MB_CPW, mb_wpe())
    pbs_multibit_shared_kernel(MultiBitPbsLaunch a) {
    static_assert(L == 1, "slot-split kernel: one decomposition level (every multi-bit set)");
    constexpr int CPW = PBS_MB_CPW;
    constexpr int W = (K + 1) * CPW;  // waves per workgroup
    constexpr int M = N / 2;
    constexpr int V = M / 64;
    static_assert(V % W == 0, "spectrum slots split evenly over the waves");
    constexpr int SPW = V / W;        // slots per wave in phase 2
    constexpr int LOG2N = ilog2(N);
    constexpr int NSEL = 1 << G;
    static_assert((K + 1) * (K + 1) * NSEL <= 32, "a slot's GGSW operands must fit the register budget");
    using Fft = WaveFft<M>;
    using Lay = PbsLds<M>;
    constexpr int XL = Lay::XL;
    static_assert(sizeof(cx) * XL >= sizeof(uint64_t) * N, "exchange buffer holds one polynomial");
    static_assert(Lay::twist_off == 0, "twist table at LDS offset 0");

    extern __shared__ __attribute__((aligned(16))) char smem[];
    double2 *lds = reinterpret_cast<double2 *>(smem);
    using Tw = TwistLds<M>;

    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wave = wid % (K + 1);  // row in phase 1, column in phase 3
    const int slot = wid / (K + 1);  // this wave's ciphertext in phases 1 and 3
    const int lane0 = threadIdx.x & 63;
    const int n = a.n;
    const int beta = a.base_log;
    const DigitL1 digit_l1(beta);
    WaveLocalSync wsync;

    Tw::fill(reinterpret_cast<double *>(lds + Lay::twist_off), a.twist, threadIdx.x, blockDim.x);
    Fft::Lds::template fill<M>(lds + Lay::s1_off, lds + Lay::s2_off, a.W, threadIdx.x, blockDim.x);
    const typename Fft::Lds tw{lds + Lay::s1_off, lds + Lay::s2_off};
    __syncthreads();

    cx *xbuf = reinterpret_cast<cx *>(lds + Lay::xbuf_off);  // buffer (ct, p) at (ct (K+1) + p) XL
    cx *xb = xbuf + (size_t)wid * XL;
    uint64_t *xb64 = reinterpret_cast<uint64_t *>(xb);
    // every ciphertext of the workgroup (idle slots compute on a valid one and store nothing)
    const int ct_raw = blockIdx.x * CPW + slot;
    const bool active = ct_raw < a.count;
    const int ct = active ? ct_raw : a.count - 1;
    const uint64_t *in = a.lwe_in + (size_t)ct * (n + 1);
    const uint32_t li = a.lut_indexes ? min(a.lut_indexes[ct], a.lut_count - 1u) : 0u;
    const uint64_t *lut = a.luts + (size_t)li * (K + 1) * N + (size_t)wave * N;

    uint64_t c0[2 * V];  // this wave's accumulator polynomial (row = wave), position lane + 64 h
    {
        const uint32_t bt = pbs_modulus_switch<LOG2N>(in[n]);
        const int full = bt / N, rem = bt % N;
#pragma unroll
        for (int h = 0; h < 2 * V; h++) {
            const int src = lane0 + 64 * h + rem;
            const bool wrap = src >= N;
            uint64_t v = lut[wrap ? src - N : src];
            c0[h] = (wrap != (bool)(full & 1)) ? 0 - v : v;
        }
    }

    constexpr size_t ggsw_len = (size_t)(K + 1) * (K + 1) * M;  // L = 1
    const __amdgpu_buffer_rsrc_t gres = make_rsrc(a.fbsk);
    const int groups = n / G;
    const double k32 = torus_k32();
    const int s0 = wid * SPW;  // phase-2 slots of this wave (wave-uniform)

    for (int j = 0; j < groups; j++) {
        int lane = lane0;
        asm volatile("" : "+v"(lane));
        const uint32_t lb = Tw::lane_base(lane);
        // ---- phase 1: forward FFT of row `wave` of ciphertext `slot`, published to xb ----
        {
            cx v[V];
#pragma unroll
            for (int b = 0; b < V; b++) {
                const int32_t d0 = digit_l1((uint32_t)(c0[b] >> 32));
                const int32_t d1 = digit_l1((uint32_t)(c0[V + b] >> 32));
                const cx w = Tw::linear(lb, b);
                v[b] = cmulw(cx{(double)d0, (double)d1}, w.re, w.im);
            }
            Fft::forward(v, xb, tw, lane, wsync);
            wsync();
#pragma unroll
            for (int s = 0; s < V; s++) reinterpret_cast<double2 *>(xb)[s * 64 + lane] = make_double2(v[s].re, v[s].im);
        }
        // ---- phase 2: keybundle + MAC of slots s0 .. s0+SPW-1 for every ciphertext ----
        // Every GGSW operand of a slot ((k+1)^2 2^g double2: 64 / 128 VGPRs at g = 2 / 3) is held
        // at once, so each ciphertext's monomials are built once per slot for both columns.  The
        // first slot's operands and the mask elements are loaded BEFORE the barrier that publishes
        // the row spectra (they do not depend on it), so their latency hides behind the wait.
        const uint32_t loff = 16u * (uint32_t)lane;
        double2 g[K + 1][K + 1][NSEL];
        auto load_slot = [&](int s) {
#pragma unroll
            for (int col = 0; col <= K; col++)
#pragma unroll
                for (int r = 0; r <= K; r++)
#pragma unroll
                    for (int sel = 0; sel < NSEL; sel++)
                        g[col][r][sel] = buffer_ld_d2(gres, loff,
                                                      (uint32_t)((((size_t)j * NSEL + sel) * ggsw_len + (size_t)r * (K + 1) * M +
                                                                  (size_t)col * M + (size_t)s * 64) * 16));
        };
        load_slot(s0);
        // monomial degrees d of the 2^g - 1 non-constant GGSWs of each ciphertext (:700-716),
        // wave-uniform: scalar loads through the constant address space -> SGPRs
        int32_t dd[CPW][NSEL];
#pragma unroll
        for (int c = 0; c < CPW; c++) {
            const int ctc = min((int)blockIdx.x * CPW + c, a.count - 1);
            const __attribute__((address_space(4))) uint64_t *inc =
                (const __attribute__((address_space(4))) uint64_t *)(a.lwe_in + (size_t)ctc * (n + 1) + (size_t)j * G);
            uint64_t av[G];
#pragma unroll
            for (int i = 0; i < G; i++) av[i] = inc[i];
#pragma unroll
            for (int sel = 1; sel < NSEL; sel++) {
                uint64_t deg = 0;
#pragma unroll
                for (int i = 0; i < G; i++)
                    if ((sel >> (G - 1 - i)) & 1) deg += av[i];
                dd[c][sel] = (int32_t)pbs_modulus_switch<LOG2N>(deg);  // <= 2N
            }
        }
        __syncthreads();
        {
            const int32_t fl = (int32_t)Fft::freq_lane(lane);
#pragma unroll
            for (int i = 0; i < SPW; i++) {
                const int s = s0 + i;
                if (i) {
                    __builtin_amdgcn_sched_barrier(0);
                    load_slot(s);
                }
                // t = d (1 - 4 f) mod 2N, f = freq_lane + freq_slot(s) < M: |1 - 4 f| < 2^12 and
                // d <= 2^12, so a 24-bit signed multiply is exact
                const int32_t w = 1 - 4 * (fl + 16 * (s >> 2) + 256 * (s & 3));
#pragma unroll
                for (int c = 0; c < CPW; c++) {
                    if (c) __builtin_amdgcn_sched_barrier(0);  // one ciphertext's monomials live at a time
                    // monomial spectra of ciphertext c at frequency f: i^q twist[r], t = q M + r
                    cx mono[NSEL];
#pragma unroll
                    for (int sel = 1; sel < NSEL; sel++) mono[sel] = Tw::mono((uint32_t)__mul24(dd[c][sel], w));
                    double2 ff[K + 1];
#pragma unroll
                    for (int r = 0; r <= K; r++)
                        ff[r] = reinterpret_cast<const double2 *>(xbuf + (size_t)(c * (K + 1) + r) * XL)[s * 64 + lane];
#pragma unroll
                    for (int col = 0; col <= K; col++) {
                        cx o;
#pragma unroll
                        for (int r = 0; r <= K; r++) {
                            // KB[r][col] at this frequency (keybundle, oracle mb_keybundle order)
                            double2 kb = g[col][r][0];
#pragma unroll
                            for (int sel = 1; sel < NSEL; sel++) {
                                const double2 gg = g[col][r][sel];
                                kb.x = fma(gg.x, mono[sel].re, fma(-gg.y, mono[sel].im, kb.x));
                                kb.y = fma(gg.x, mono[sel].im, fma(gg.y, mono[sel].re, kb.y));
                            }
                            // MAC over rows (update_with_fmadd order)
                            if (r == 0) {
                                o.re = fma(kb.x, ff[r].x, -(kb.y * ff[r].y));
                                o.im = fma(kb.x, ff[r].y, kb.y * ff[r].x);
                            } else {
                                o.re = fma(kb.x, ff[r].x, fma(-kb.y, ff[r].y, o.re));
                                o.im = fma(kb.x, ff[r].y, fma(kb.y, ff[r].x, o.im));
                            }
                        }
                        // out_c[col][s] over F_c[col][s]: ciphertext c's F of slot s is in registers
                        // and slot s is this wave's alone
                        reinterpret_cast<double2 *>(xbuf + (size_t)(c * (K + 1) + col) * XL)[s * 64 + lane] =
                            make_double2(o.re, o.im);
                    }
                }
            }
        }
        __syncthreads();
        // ---- phase 3: inverse FFT of column `wave` of ciphertext `slot`, into the accumulator ----
        {
            cx v[V];
#pragma unroll
            for (int s = 0; s < V; s++) {
                const double2 t = reinterpret_cast<const double2 *>(xb)[s * 64 + lane];
                v[s] = cx{t.x, t.y};
            }
            wsync();
            Fft::inverse(v, xb, tw, lane, wsync);
#pragma unroll
            for (int b = 0; b < V; b++)  // the resident key carries the 1/M
                backward_convert(v[b], Tw::linear(lb, b), c0[b], c0[V + b], k32);
        }
    }

    if (a.glwe_out) {  // bootstrap_without_sample_extract (fork, bootstrap.rs:383-412)
        if (!active) return;
        uint64_t *g = a.lwe_out + ((size_t)ct * (K + 1) + wave) * N;
#pragma unroll
        for (int h = 0; h < 2 * V; h++) g[lane0 + 64 * h] = c0[h];
        return;
    }
    // sample extract at degree 0 (glwe_sample_extraction.rs:91-147)
    wsync();
#pragma unroll
    for (int h = 0; h < 2 * V; h++) xb64[lane0 + 64 * h] = c0[h];
    wsync();
    if (!active) return;
    uint64_t *out = a.lwe_out + (size_t)ct * (K * N + 1);
    if (wave < K) {
        for (int jj = lane0; jj < N; jj += 64) out[wave * N + jj] = jj == 0 ? xb64[0] : 0 - xb64[N - jj];
    } else if (lane0 == 0) {
        out[K * N] = c0[0];
    }
}

template <int N, int K, int L, int G>
static hipError_t launch_mb_t(const MultiBitPbsLaunch &a, hipStream_t s) {
    constexpr int M = N / 2;
    constexpr size_t lds = PbsLds<M>::bytes((K + 1) * PBS_MB_CPW) + (PBS_GROUP_SYNC ? 4 * (K + 1) * PBS_MB_CPW : 0);
    static_assert(lds <= 160 * 1024, "LDS per workgroup exceeds a CU");
    if (a.count == 0) return hipSuccess;
    if (a.n % G) return hipErrorInvalidValue;
    const int blocks = (a.count + PBS_MB_CPW - 1) / PBS_MB_CPW;
    if constexpr (PBS_MB_SHARED && L == 1 && (K + 1) * (K + 1) * (1 << G) <= 32)
        hipLaunchKernelGGL((pbs_multibit_shared_kernel<N, K, L, G>), dim3(blocks), dim3(64 * (K + 1) * PBS_MB_CPW), lds, s, a);
    else
        hipLaunchKernelGGL((pbs_multibit_kernel<N, K, L, G>), dim3(blocks), dim3(64 * (K + 1) * PBS_MB_CPW), lds, s, a);
    return hipGetLastError();
}

// The reference's multi-bit parameter sets at N <= 2048 (shortint/parameters/multi_bit.rs): the
// 2_2 sets (N = 2048, k = 1; the slot-split kernel) and the 1_1 sets (N = 512, k = 3, :96,154; the
// per-ciphertext kernel: their (k+1)^2 2^g GGSW operands per slot exceed the slot-split register
// budget).  All use one decomposition level; the 3_3 sets (N = 8192) run the split CMUX.
bool multibit_pbs_supported(int N, int k, int L, int g) {
    return ((N == 2048 && k == 1) || (N == 512 && k == 3)) && L == 1 && (g == 2 || g == 3);
}

hipError_t launch_multibit_pbs(int N, int k, int L, int g, const MultiBitPbsLaunch &a, hipStream_t s) {
    if (N == 2048 && k == 1 && L == 1 && g == 3) return launch_mb_t<2048, 1, 1, 3>(a, s);
    if (N == 2048 && k == 1 && L == 1 && g == 2) return launch_mb_t<2048, 1, 1, 2>(a, s);
    if (N == 512 && k == 3 && L == 1 && g == 3) return launch_mb_t<512, 3, 1, 3>(a, s);
    if (N == 512 && k == 3 && L == 1 && g == 2) return launch_mb_t<512, 3, 1, 2>(a, s);
    return hipErrorInvalidValue;
}

}  // namespace tfhe_mi355
