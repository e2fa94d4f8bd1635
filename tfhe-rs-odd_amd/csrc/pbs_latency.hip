// pbs_latency.hip -- latency form of the classic PBS at N = 2048, k = 1, L = 1 (the 2_2 shape):
// ONE ciphertext per workgroup of 8 wavefronts, each GLWE polynomial's 1024-point FFT spread over
// four of them.
//
// Replaces the same reference functions as pbs_classic.hip (FourierLweBootstrapKeyView::
// bootstrap, fft64/crypto/bootstrap.rs:243-380; add_external_product_assign, ggsw.rs:477-697;
// fast_pbs_modulus_switch, fft_impl/common.rs:26-43; extract_lwe_sample_from_glwe_ciphertext,
// glwe_sample_extraction.rs:91-147) for the calling pattern of the reference itself: a handful
// of ciphertexts per call (keyswitch_programmable_bootstrap_assign bootstraps ONE ciphertext,
// shortint/server_key/mod.rs:783-857, from each rayon worker, radix_parallel/mul.rs:347-407).
// The throughput kernel puts a ciphertext on 2 waves (one per GLWE row) and needs four of them
// per CU to fill its SIMDs; alone on a CU its 742 dependent CMUXes take ~5.9 ms.  Here the 8 waves
// of a CU all work on one ciphertext, so a batch of up to 256 ciphertexts (one per CU) finishes
// in the time of one CMUX chain at 4x the per-CMUX parallelism.
//
// Same FFT DAG as WaveFft<1024> and the oracle ([16, 16, 4] DIF forward / mirrored DIT inverse,
// same twiddle products and fma forms, same MAC order), so outputs are bit-identical to the
// throughput kernel and to oracle/pbs_oracle.c.  Work split of one row's transform (waves
// w = 0..3 of that row; lane = 16 lrow + col):
//   stage 1 (R16, stride 64): butterfly a = 16 w + col, split over the four 16-lane rows as in
//     WaveFft<256> (in-row radix 4, row twiddles, v_permlane transpose, radix 4): lane holds
//     z[a + 64 (lrow + 4 j)], j < 4, and leaves output C = lrow + 4 q -> LDS X[a + 64 C];
//   stage 2 (R16 on blocks of 64, stride 4): block cc = 4 w + (col >> 2), a1 = col & 3, same
//     row split -> LDS Y[64 cc + a1 + 4 C2];
//   stage 3 (R4 on blocks of 4) is computed by the MAC lane that owns the block, for both rows
//     (the MAC needs both rows' spectra anyway): block t = 16 cc' + C2', cc' = 4 w + (col & 3),
//     C2' = lrow + 4 (col >> 2), positions 4 t + e, e < 4;
//   the inverse mirrors it; the stage-3 inverse output goes back to stage-2 lanes through this
//     wave's own quarter of X (wave-private, no barrier).
// That mapping (LAT_MAP = 0) has four workgroup barriers per CMUX: accumulator -> rotation gather,
// stage 1 -> 2, stage 2 -> MAC, inverse stage 2 -> 1.  LAT_MAP = 1 (default) gives wave w the
// stage-1 butterflies a = w + 4 col instead, so stage 2's butterfly a2 = w of EVERY block cc =
// col reads only this wave's stage-1 outputs (positions = w mod 4): stages 1 <-> 2 are wave-private
// both ways and the cross-wave hand-offs are stage 2 <-> 3, which the MAC's row join needs anyway.
// Three barriers: accumulator -> rotation (A), stage 2 -> MAC (C), inverse stage 3 -> 2 (E); the
// accumulator pairs move to their own buffer Z so one wave's rotation gather may overlap another's
// stage-2 stores.  Same operations on the same values, so the outputs are unchanged.
#include "engine.h"
#include "pbs_common.h"

namespace tfhe_mi355 {

namespace {

constexpr int LAT_N = 2048, LAT_M = 1024;
#ifndef LAT_MAP
#define LAT_MAP 1  // lane mapping of the transform stages (see the header: 1 = three barriers per CMUX)
#endif
// LDS layout in double2 units: per GLWE row an exchange buffer X (stages 1/2) and a buffer Y
// (stage-2 outputs; LAT_MAP = 0: also the accumulator pairs of the rotation).  LAT_MAP = 1 keeps
// the pairs in their own buffer Z: the rotation gather of one wave can then overlap another wave's
// stage-2 stores, with no barrier between them.  The twiddles and the twist a lane needs are 12
// constants per lane, kept in registers (read once from the global tables).
struct LatLds {
    static constexpr int X = 0;
    static constexpr int Y = X + 2 * LAT_M;
    static constexpr int Z = LAT_MAP ? Y + 2 * LAT_M : Y;
    static constexpr int end = Z + 2 * LAT_M;
    static constexpr size_t bytes = sizeof(double2) * end;
};
static_assert(LatLds::bytes <= 160 * 1024, "latency PBS LDS exceeds a CU");

__device__ __forceinline__ cx ld2(const double2 *p) {
    const double2 t = *p;
    return {t.x, t.y};
}
__device__ __forceinline__ void st2(double2 *p, cx v) { *p = make_double2(v.re, v.im); }
// X / Y slot of FFT position P: an XOR swizzle of the 16-byte slot's bank bits (0-3), found by
// exhaustive search to make all three access patterns of a wave free of bank conflicts for both
// ds_read_b128 lane groups and ds_write_b128's (the plain layout puts up to 4 lanes of a group on
// one bank).  LAT_MAP = 0 (stage 1 a1 + 64 C, a1 = 16 w + col; stage 2 64 cc + a2 + 4 C2; the
// MAC's blocks 4 t + e): bits 0-3 ^= bits 4, 7, 6, 6 (linear swizzles of bits 4-7).  LAT_MAP = 1
// (a1 = w + 4 col, cc = col, a2 = w; same blocks): no XOR of bits 4-9 into bits 0-3 works (the
// stage-1 stores of 8 contiguous lanes differ in bit 3), so bits 0-2 ^= bits 3, 4, 6, 7, 8 ->
// 1, 0, 2, 1, 0 and bit 3 ^= bit 6 (scripts/probes/lat_swizzle_search.c: 712,704 such maps
// qualify among the 2^27 with bit 3 as an input).  LAT_SWZ=0: plain.
#ifndef LAT_SWZ
#define LAT_SWZ 1
#endif
__device__ __forceinline__ int lswz(int P) {
    if (!LAT_SWZ) return P;
    if (LAT_MAP)
        return P ^ (((P >> 2) & 2) ^ ((P >> 4) & 1) ^ ((P >> 4) & 4) ^ ((P >> 6) & 2) ^ ((P >> 8) & 1) ^ ((P >> 3) & 8));
    return P ^ (((P >> 4) & 1) | ((P >> 6) & 2) | ((P >> 4) & 4) | ((P >> 3) & 8));
}
// Lane mapping of the transform stages (lane = 16 lrow + col, w = the wave's quarter of its row):
// stage-1 butterfly a1, stage-2 block cc and butterfly a2
__device__ __forceinline__ int lat_a1(int w, int col) { return LAT_MAP ? w + 4 * col : 16 * w + col; }
__device__ __forceinline__ int lat_cc(int w, int col) { return LAT_MAP ? col : 4 * w + (col >> 2); }
__device__ __forceinline__ int lat_a2(int w, int col) { return LAT_MAP ? w : col & 3; }
// Slot of accumulator pair j (acc[j], acc[j + M]) in its buffer.  LAT_MAP = 1: a lane's pairs are
// j = w + 4 col + 64 (lrow + 4 q), so the stores of 8 contiguous lanes and the rotation gather
// (pairs j - rem: in a 16-lane read group bits 2-5 take all 16 values, bits 0-1 are fixed) would
// share banks; bits 0-1 ^= (bit 3 ^ bit 5, bit 4) makes both conflict-free for every rem.
__device__ __forceinline__ int aswz(int j) { return LAT_MAP ? j ^ ((((j >> 3) ^ (j >> 5)) & 1) | ((j >> 3) & 2)) : j; }
// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations (lgkmcnt), not
// for its global loads, so the GGSW prefetch stays in flight across it (__syncthreads' fence
// would wait for vmcnt(0) too and expose the prefetch's latency at the first barrier).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

}  // namespace

#ifndef LAT_BF
#define LAT_BF 2  // row twiddles: 2 select-free fused products (RowTwF), 1 per-lane constants + selects, 0 row branches
#endif

// Row-split 16-point DFTs of dft16_fwd_rows / dft16_inv_rows (fft_device.h) with the internal
// twiddles omega16^(A k) (A = the lane's row, k = 1, 2, 3) computed without lane-divergent
// branches: every exponent E = A k is either a cmulw with a constant (E = 0: (1, 0), E = 4:
// (0, -1), value-identical to skipping / swapping; E = 1, 3, 9: the tw16 constants) or one of the
// two sqrt(1/2) forms (E = 2, 6); each lane computes both candidate forms and selects its own.
// Operation for operation the same as tw16_fwd<E> / tw16_inv<E> for the selected E.
struct RowTw {
    double cr[3], ci[3];  // cmulw constants of k = 1, 2, 3 (forward; the inverse conjugates)
    bool sp[3], e6[3];    // sqrt(1/2) form (E = 2 or 6) and which one
    __device__ explicit RowTw(int A) {
#pragma unroll
        for (int k = 0; k < 3; k++) {
            const int E = A * (k + 1);
            sp[k] = E == 2 || E == 6;
            e6[k] = E == 6;
            cr[k] = E == 0 ? 1.0 : E == 1 ? TM_C16_1 : E == 3 ? TM_S16_1 : E == 4 ? 0.0 : E == 9 ? -TM_C16_1 : 0.0;
            ci[k] = E == 0 ? 0.0 : E == 1 ? -TM_S16_1 : E == 3 ? -TM_C16_1 : E == 4 ? -1.0 : E == 9 ? TM_S16_1 : 0.0;
        }
    }
    template <bool INV>
    __device__ __forceinline__ cx apply(int k, cx x) const {
        const cx c = cmulw(x, cr[k], INV ? -ci[k] : ci[k]);
        // forward E = 2: ((r + i) h, (i - r) h), E = 6: ((i - r) h, -((r + i) h));
        // inverse E = 2: ((r - i) h, (r + i) h), E = 6: (-((r + i) h), (r - i) h)
        const double sh = (x.re + x.im) * TM_SQH;
        const double dh = (INV ? x.re - x.im : x.im - x.re) * TM_SQH;
        cx sq;
        if (INV) sq = e6[k] ? cx{-sh, dh} : cx{dh, sh};
        else sq = e6[k] ? cx{dh, -sh} : cx{sh, dh};
        return sp[k] ? sq : c;
    }
};
// Select-free form (LAT_BF = 2): every E as the same three fused products,
//   U = fma(im, be, re),  U2 = fma(im, be2, re),  out = (fma(U, c1, im s1), fma(U2, c2, im s2))
// with per-lane constants.  cmulw lanes (E = 0, 1, 3, 4, 9): be = be2 = 0, so U = U2 = re exactly,
// and (c1, s1, c2, s2) = (wr, -wi, wi, wr): cmulw's (fma(re, wr, -(im wi)), fma(re, wi, im wr)).
// sqrt(1/2) lanes: U, U2 = re + im or re - im with one rounding (the oracle's x.re + x.im etc.; its
// x.im - x.re is the negation of re - im, folded into the sign of c), s1 = s2 = 0, c1, c2 = +-h, so
// each output is the oracle's single rounding of (sum) * h.  Only the sign of a zero can differ from
// the branchy form (a +-0 addend), which no later rounding observes.
struct RowTwF {
    double be[3], be2[3], c1[3], s1[3], c2[3], s2[3];
    __device__ RowTwF(int A, bool inv) {
        // every member by a conditional expression (no if/else over members: those leave the
        // object in private memory instead of registers)
        const double h = TM_SQH;
#pragma unroll
        for (int k = 0; k < 3; k++) {
            const int E = A * (k + 1);
            const bool sq = E == 2 || E == 6, six = E == 6;
            const double wr = E == 0 ? 1.0 : E == 1 ? TM_C16_1 : E == 3 ? TM_S16_1 : E == 4 ? 0.0 : -TM_C16_1;
            const double wf = E == 0 ? 0.0 : E == 1 ? -TM_S16_1 : E == 3 ? -TM_C16_1 : E == 4 ? -1.0 : TM_S16_1;
            const double wi = inv ? -wf : wf;
            // fwd E=2: ((r+i)h, -((r-i)h))   fwd E=6: (-((r-i)h), -((r+i)h))
            // inv E=2: ((r-i)h, (r+i)h)      inv E=6: (-((r+i)h), (r-i)h)
            be[k] = !sq ? 0.0 : (inv ? six : !six) ? 1.0 : -1.0;
            be2[k] = !sq ? 0.0 : (inv ? !six : six) ? 1.0 : -1.0;
            c1[k] = !sq ? wr : six ? -h : h;
            s1[k] = sq ? 0.0 : -wi;
            c2[k] = !sq ? wi : inv ? h : -h;
            s2[k] = sq ? 0.0 : wr;
        }
    }
    __device__ __forceinline__ cx apply(int k, cx x) const {
        const double u = fma(x.im, be[k], x.re);
        const double u2 = fma(x.im, be2[k], x.re);
        return {fma(u, c1[k], x.im * s1[k]), fma(u2, c2[k], x.im * s2[k])};
    }
};
__device__ __forceinline__ void dft16_fwd_rows_sf(cx *v, const RowTwF &t) {
    r4_fwd(v[0], v[1], v[2], v[3]);
    v[1] = t.apply(0, v[1]);
    v[2] = t.apply(1, v[2]);
    v[3] = t.apply(2, v[3]);
    transpose_rows4(v[0], v[1], v[2], v[3]);
    r4_fwd(v[0], v[1], v[2], v[3]);
}
__device__ __forceinline__ void dft16_inv_rows_sf(cx *v, const RowTwF &t) {
    r4_inv(v[0], v[1], v[2], v[3]);
    transpose_rows4(v[0], v[1], v[2], v[3]);
    v[1] = t.apply(0, v[1]);
    v[2] = t.apply(1, v[2]);
    v[3] = t.apply(2, v[3]);
    r4_inv(v[0], v[1], v[2], v[3]);
}
__device__ __forceinline__ void dft16_fwd_rows_bf(cx *v, const RowTw &t) {
    r4_fwd(v[0], v[1], v[2], v[3]);
    v[1] = t.apply<false>(0, v[1]);
    v[2] = t.apply<false>(1, v[2]);
    v[3] = t.apply<false>(2, v[3]);
    transpose_rows4(v[0], v[1], v[2], v[3]);
    r4_fwd(v[0], v[1], v[2], v[3]);
}
__device__ __forceinline__ void dft16_inv_rows_bf(cx *v, const RowTw &t) {
    r4_inv(v[0], v[1], v[2], v[3]);
    transpose_rows4(v[0], v[1], v[2], v[3]);
    v[1] = t.apply<true>(0, v[1]);
    v[2] = t.apply<true>(1, v[2]);
    v[3] = t.apply<true>(2, v[3]);
    r4_inv(v[0], v[1], v[2], v[3]);
}

#ifndef LAT_PRIO
#define LAT_PRIO 0  // s_setprio for the second-dispatched half of the waves (the arbitration losers)
#endif
#ifndef LAT_PREF2
#define LAT_PREF2 0  // GGSW of CMUX i + 1 loaded during CMUX i (two register sets) instead of at its top
#endif

#ifndef LAT_HOIST
#define LAT_HOIST 1  // 1: the per-lane LDS / GGSW addresses are loop invariants (kept in VGPRs); 0: recomputed per CMUX
#endif

#ifndef LAT_EARLYACC
#define LAT_EARLYACC 1  // 1: each accumulator pair goes to LDS right after its backward conversion (0: at the CMUX top)
#endif

#ifndef LAT_TSKIP
#define LAT_TSKIP 0  // timing-only builds (wrong outputs): 1 = skip the inverse's wave-private exchange
#endif

#ifndef LAT_STAMPS
#define LAT_STAMPS 0  // diagnostic builds: s_memtime per CMUX phase of block 0 into the ticket buffer
#endif

// RPW = GLWE rows per wave: 1 -> 8 waves (wave (row, w), 2 per SIMD); 2 -> 4 waves, each doing
// quarter w of both rows (twice the independent work per lane, one wave per SIMD; the stage-2 ->
// MAC hand-off is then wave-private, so one workgroup barrier fewer per CMUX).
template <int RPW>
__global__ void __launch_bounds__(512 / RPW, 2 / RPW) pbs_latency_kernel(ClassicPbsLaunch a) {
    constexpr int N = LAT_N, M = LAT_M, K = 1, LOG2N = 11;
    static_assert(RPW == 1 || RPW == 2, "one or both GLWE rows per wave");
    static_assert(!LAT_MAP || RPW == 1, "the three-barrier lane mapping is written for one row per wave");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    double2 *lds = reinterpret_cast<double2 *>(smem);
    const int tid = threadIdx.x;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int row0 = (wid >> 2) * RPW;  // first GLWE row this wave transforms (rows row0 .. row0 + RPW - 1)
    const int w = wid & 3;              // quarter of the rows' transforms
    const int lane0 = tid & 63;

    // per-lane constants: stage-1 twiddles W[a1 C] (a1 = 16 w + col, C = lrow + 4 q; C = 0 gives
    // W[0] = (1, -0): value-identical to the oracle's skipped multiply), stage-2 twiddles
    // W[16 a2 C2] (a2 = col & 3), the twist of the lane's positions j_q = a1 + 64 (lrow + 4 q)
    cx tw1[4], tw2[4], tws[4];
    const RowTw rtw(lane0 >> 4);
    const RowTwF rtf(lane0 >> 4, false), rti(lane0 >> 4, true);  // LAT_BF = 2
    {
        const int lrow = lane0 >> 4, col = lane0 & 15, a1 = lat_a1(w, col), a2 = lat_a2(w, col);
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int C = lrow + 4 * q;
            tw1[q] = ld2(a.W + a1 * C);
            tw2[q] = ld2(a.W + 16 * a2 * C);
            tws[q] = ld2(a.twist + a1 + 64 * C);
        }
    }

    const int ct = blockIdx.x;
    const int n = a.n;
    const uint64_t *in = a.lwe_in + (size_t)ct * (n + 1);
    const __attribute__((address_space(4))) uint64_t *in_s = (const __attribute__((address_space(4))) uint64_t *)(
        ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)((uintptr_t)in >> 32)) << 32) |
        (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)in));
    const uint32_t li = a.lut_indexes ? min(a.lut_indexes[ct], a.lut_count - 1u) : 0u;
    const DigitL1 digit_l1(a.base_log);

    // this lane's accumulator coefficients of row row0 + r: j_q = a1 + 64 (lrow + 4 q) (a1 = 16 w +
    // col) and j_q + M (the stage-1 input positions and the backward conversion's output positions)
    uint64_t lo[RPW][4], hi[RPW][4];
    {
        const uint32_t bt = pbs_modulus_switch<LOG2N>(in[n]);
        const int full = bt / N, rem = bt % N;
#pragma unroll
        for (int r = 0; r < RPW; r++) {
            const uint64_t *lut = a.luts + (size_t)li * (K + 1) * N + (size_t)(row0 + r) * N;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int j = lat_a1(w, lane0 & 15) + 64 * (lane0 >> 4) + 256 * q;
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    const int src = j + h * M + rem;
                    const bool wrap = src >= N;
                    const uint64_t v = lut[wrap ? src - N : src];
                    const uint64_t c = (wrap != (bool)(full & 1)) ? 0 - v : v;
                    (h ? hi : lo)[r][q] = c;
                }
            }
        }
    }
    // per row: X = exchange buffer of stages 1 / 2, Y = stage-2 outputs; the accumulator pairs
    // (acc[p], acc[p + M]) live in Y between CMUXes (its stage-2 outputs are dead then)
    auto Xr = [&](int r) { return lds + LatLds::X + (row0 + r) * M; };
    auto Yr = [&](int r) { return lds + LatLds::Y + (row0 + r) * M; };
    auto Ar = [&](int r) { return reinterpret_cast<uint64_t *>(lds + LatLds::Z + (row0 + r) * M); };
    constexpr size_t ggsw_stride = (size_t)(K + 1) * (K + 1) * M;
    const double k32 = torus_k32();

    // diagnostic stamps (LAT_STAMPS builds only; written to a buffer nothing else reads): wave 0 and
    // (RPW = 1) wave 4 of workgroup 0, CMUX 200 .. 207, 12 stamps each
    uint64_t *stamp_buf = LAT_STAMPS ? reinterpret_cast<uint64_t *>(a.ticket) : nullptr;
    auto stamp = [&](int i, int k) {
        if constexpr (LAT_STAMPS) {
            if (blockIdx.x == 0 && (wid & 3) == 0 && lane0 == 0 && i >= 200 && i < 208) {
                int vo = lane0;  // a VGPR offset (0 here): the stamp goes out through a vector store
                asm volatile("" : "+v"(vo));
                stamp_buf[((wid >> 2) * 8 + (i - 200)) * 12 + k + vo] = __builtin_amdgcn_s_memtime();
            }
        }
    };
    // GGSW operands of the MAC lane's block (see the MAC below) for each output column of this
    // wave; engine layout: element s*64 + L <-> position 64 (L & 15) + 16 (L >> 4) + s, so position
    // 64 ccm + 4 (lrow + 4 xm) + e is element (4 lrow + e) 64 + 16 xm + ccm
    auto load_ggsw = [&](double2 (&gp)[RPW][K + 1][4], int ii, int lrow, int col) {
        const int ccm = 4 * w + (col & 3), xm = col >> 2;
        const double2 *g = a.fbsk + (size_t)ii * ggsw_stride + 256 * lrow + 16 * xm + ccm;
#pragma unroll
        for (int c = 0; c < RPW; c++)
#pragma unroll
            for (int rr = 0; rr <= K; rr++)
#pragma unroll
                for (int e = 0; e < 4; e++) gp[c][rr][e] = g[(size_t)(rr * (K + 1) + row0 + c) * M + 64 * e];
    };
    double2 gnext[RPW][K + 1][4];
    if (LAT_PREF2) load_ggsw(gnext, 0, lane0 >> 4, lane0 & 15);
    if (LAT_PRIO && wid >= (int)(blockDim.x >> 7)) __builtin_amdgcn_s_setprio(1);
    for (int i = 0; i < n; i++) {
        int lane = lane0;  // LAT_HOIST = 0: opaque per-iteration copy, lane-derived addresses not hoisted
        if (!LAT_HOIST) asm volatile("" : "+v"(lane));
        stamp(i, 0);
        const int lrow = lane >> 4, col = lane & 15;
        const int ccm = 4 * w + (col & 3), xm = col >> 2;
        // this CMUX's GGSW operands: loaded at its top, so that their L2/MALL latency hides behind
        // the rotation and the forward FFT (LAT_PREF2: during the previous CMUX)
        double2 gpre[RPW][K + 1][4];
        if (LAT_PREF2) {
#pragma unroll
            for (int c = 0; c < RPW; c++)
#pragma unroll
                for (int rr = 0; rr <= K; rr++)
#pragma unroll
                    for (int e = 0; e < 4; e++) gpre[c][rr][e] = gnext[c][rr][e];
            if (i + 1 < n) load_ggsw(gnext, i + 1, lrow, col);
        } else {
            load_ggsw(gpre, i, lrow, col);
        }
        __builtin_amdgcn_sched_barrier(0);
        const uint32_t at = pbs_modulus_switch<LOG2N>(in_s[i]);
        const bool full_odd = (at / N) & 1;
        const int rem = at % N;

        // ---- accumulator -> LDS pairs, rotation gather, ct1 = X^at acc - acc, digits, twist ----
        // (LAT_EARLYACC: the pairs were stored by the previous CMUX's backward conversion, or before
        // the loop; the pair buffer is free then -- LAT_MAP = 0: Y, whose last reads were the MAC's,
        // before barrier D; LAT_MAP = 1: Z, whose last reads were the rotation's, before barrier C)
        if (!LAT_EARLYACC || i == 0) {
#pragma unroll
            for (int r = 0; r < RPW; r++)
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const int j = aswz(lat_a1(w, col) + 64 * lrow + 256 * q);
                    Ar(r)[2 * j] = lo[r][q];
                    Ar(r)[2 * j + 1] = hi[r][q];
                }
        }
        lds_barrier();  // (A) every wave's pairs written
        stamp(i, 1);
        cx v[RPW][4];
#pragma unroll
        for (int r = 0; r < RPW; r++)
#pragma unroll
            for (int q = 0; q < 4; q++) {
                // (X^rem p) at j and j + M from ONE pair: u = j - rem, s = u mod M; u >= 0: (lo, hi);
                // -M <= u < 0: (-hi, lo) (X^M acts as i on the fold); u < -M: (-lo, -hi).
                // j = j0 + 256 q: the pair swizzle reads bits 3-5 and changes bits 0-1 only, so
                // aswz(s) = (aswz(s0) + 256 q) mod M with s0 the q = 0 slot (one add per q)
                const int u0 = lat_a1(w, col) + 64 * lrow - rem;
                const int u = u0 + 256 * q;
                const int s = (aswz(u0 & (M - 1)) + 256 * q) & (M - 1);
                const uint64_t plo = Ar(r)[2 * s], phi = Ar(r)[2 * s + 1];
                const bool swap = u < 0 && u >= -M;
                const bool n0 = (u < 0) != full_odd, n1 = (u < -M) != full_odd;
                const uint64_t x0 = swap ? phi : plo, x1 = swap ? plo : phi;
                const uint64_t r0 = n0 ? 0 - x0 : x0, r1 = n1 ? 0 - x1 : x1;
                const int32_t d0 = digit_l1((uint32_t)((r0 - lo[r][q]) >> 32));
                const int32_t d1 = digit_l1((uint32_t)((r1 - hi[r][q]) >> 32));
                v[r][q] = cmulw(cx{(double)d0, (double)d1}, tws[q].re, tws[q].im);  // convert_forward_integer (x86.rs:505-596)
            }

        stamp(i, 2);
        // ---- forward stage 1: butterfly a1 = 16 w + col, column lrow ----
#pragma unroll
        for (int r = 0; r < RPW; r++) {
            if constexpr (LAT_BF == 2) dft16_fwd_rows_sf(v[r], rtf);
            else if (LAT_BF) dft16_fwd_rows_bf(v[r], rtw);
            else dft16_fwd_rows(v[r], lrow);
            const int a1 = lat_a1(w, col);
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int C = lrow + 4 * q;
                st2(Xr(r) + lswz(a1 + 64 * C), cmulw(v[r][q], tw1[q].re, tw1[q].im));
            }
        }
        stamp(i, 3);
        // (B) LAT_MAP = 0: stage 2 reads other waves' stage-1 outputs; LAT_MAP = 1: only this wave's
        if constexpr (LAT_MAP) WaveLocalSync{}();
        else lds_barrier();
        stamp(i, 4);
        // ---- forward stage 2: block cc, butterfly a2 (LAT_MAP = 0: cc = 4 w + (col >> 2),
        //      a2 = col & 3; LAT_MAP = 1: cc = col, a2 = w) ----
        {
            const int cc = lat_cc(w, col), a2 = lat_a2(w, col);
#pragma unroll
            for (int r = 0; r < RPW; r++) {
#pragma unroll
                for (int q = 0; q < 4; q++) v[r][q] = ld2(Xr(r) + lswz(64 * cc + a2 + 4 * (lrow + 4 * q)));
                if constexpr (LAT_BF == 2) dft16_fwd_rows_sf(v[r], rtf);
                else if (LAT_BF) dft16_fwd_rows_bf(v[r], rtw);
                else dft16_fwd_rows(v[r], lrow);
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const int C2 = lrow + 4 * q;
                    st2(Yr(r) + lswz(64 * cc + a2 + 4 * C2), cmulw(v[r][q], tw2[q].re, tw2[q].im));
                }
            }
        }
        stamp(i, 5);
        // (C) both rows' stage-2 outputs of this wave's blocks: written by the other row's wave
        // (RPW = 1), or by this wave itself (RPW = 2: wave-private)
        if constexpr (RPW == 1) lds_barrier();
        else WaveLocalSync{}();
        stamp(i, 6);
        // ---- stage 3 of both rows + MAC of this wave's output columns on block t ----
        const int tb = 64 * ccm + 4 * (lrow + 4 * xm);  // first position of block t
        cx o[RPW][4];
        {
            cx f[K + 1][4];
#pragma unroll
            for (int rr = 0; rr <= K; rr++) {
                const double2 *y = lds + LatLds::Y + rr * M;
                f[rr][0] = ld2(y + lswz(tb));
                f[rr][1] = ld2(y + lswz(tb + 1));
                f[rr][2] = ld2(y + lswz(tb + 2));
                f[rr][3] = ld2(y + lswz(tb + 3));
                r4_fwd(f[rr][0], f[rr][1], f[rr][2], f[rr][3]);
            }
#pragma unroll
            for (int c = 0; c < RPW; c++)
#pragma unroll
                for (int rr = 0; rr <= K; rr++)
#pragma unroll
                    for (int e = 0; e < 4; e++) {
                        const double2 gg = gpre[c][rr][e];
                        const double2 ff = make_double2(f[rr][e].re, f[rr][e].im);
                        if (rr == 0) {  // update_with_fmadd (ggsw.rs:524-567), the throughput kernel's form
                            o[c][e].re = fma(gg.x, ff.x, -(gg.y * ff.y));
                            o[c][e].im = fma(gg.x, ff.y, gg.y * ff.x);
                        } else {
                            o[c][e].re = fma(gg.x, ff.x, fma(-gg.y, ff.y, o[c][e].re));
                            o[c][e].im = fma(gg.x, ff.y, fma(gg.y, ff.x, o[c][e].im));
                        }
                    }
        }
        // ---- inverse stage 3 (R4 on the block), back to the stage-2 lanes through this wave's
        //      own quarter of X (positions 256 w .. 256 w + 255: written and read by this wave only)
        stamp(i, 7);
#pragma unroll
        for (int c = 0; c < RPW; c++) {
            r4_inv(o[c][0], o[c][1], o[c][2], o[c][3]);
#pragma unroll
            for (int e = 0; e < 4; e++)
                if (!(LAT_TSKIP & 1)) st2(Xr(c) + lswz(tb + e), o[c][e]);
        }
        // LAT_MAP = 0: the blocks are this wave's own stage-2 blocks (wave-private); LAT_MAP = 1:
        // stage 2 reads one residue class mod 4 of every block, written by all four waves (E)
        if constexpr (LAT_MAP) lds_barrier();
        else if (!(LAT_TSKIP & 1)) WaveLocalSync{}();
        {
            const int cc = lat_cc(w, col), a2 = lat_a2(w, col);
#pragma unroll
            for (int r = 0; r < RPW; r++) {
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const int C2 = lrow + 4 * q;
                    // LAT_TSKIP & 1 (timing only, wrong outputs): no wave-private exchange
                    const cx x = (LAT_TSKIP & 1) ? o[r][q] : ld2(Xr(r) + lswz(64 * cc + a2 + 4 * C2));
                    v[r][q] = cmulw(x, tw2[q].re, -tw2[q].im);
                }
                if constexpr (LAT_BF == 2) dft16_inv_rows_sf(v[r], rti);
                else if (LAT_BF) dft16_inv_rows_bf(v[r], rtw);
                else dft16_inv_rows(v[r], lrow);
            }
            WaveLocalSync{}();
#pragma unroll
            for (int r = 0; r < RPW; r++)
#pragma unroll
                for (int q = 0; q < 4; q++) st2(Xr(r) + lswz(64 * cc + a2 + 4 * (lrow + 4 * q)), v[r][q]);
        }
        stamp(i, 8);
        // (D) LAT_MAP = 0: stage 1 reads other waves' stage-2 outputs; LAT_MAP = 1: only this wave's
        if constexpr (LAT_MAP) WaveLocalSync{}();
        else lds_barrier();
        stamp(i, 9);
        // ---- inverse stage 1 + backward conversion into the accumulator ----
        {
            const int a1 = lat_a1(w, col);
#pragma unroll
            for (int r = 0; r < RPW; r++) {
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const int C = lrow + 4 * q;
                    v[r][q] = cmulw(ld2(Xr(r) + lswz(a1 + 64 * C)), tw1[q].re, -tw1[q].im);
                }
                if constexpr (LAT_BF == 2) dft16_inv_rows_sf(v[r], rti);
                else if (LAT_BF) dft16_inv_rows_bf(v[r], rtw);
                else dft16_inv_rows(v[r], lrow);
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    backward_add(v[r][q], tws[q], lo[r][q], hi[r][q], k32);  // the resident key carries the 1/M
                    if constexpr (LAT_EARLYACC) {  // the next rotation's pair, stored as soon as it is final
                        const int j = aswz(lat_a1(w, col) + 64 * lrow + 256 * q);
                        Ar(r)[2 * j] = lo[r][q];
                        Ar(r)[2 * j + 1] = hi[r][q];
                    }
                }
            }
        }
        stamp(i, 10);
    }

    // ---- output ----
    const int lrow = lane0 >> 4, col = lane0 & 15;
    if (a.glwe_out) {  // bootstrap_without_sample_extract (fork, bootstrap.rs:383-412)
#pragma unroll
        for (int r = 0; r < RPW; r++) {
            uint64_t *g = a.lwe_out + ((size_t)ct * (K + 1) + row0 + r) * N;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int j = lat_a1(w, col) + 64 * lrow + 256 * q;
                g[j] = lo[r][q];
                g[j + M] = hi[r][q];
            }
        }
        return;
    }
    // sample extract at degree 0 (glwe_sample_extraction.rs:91-147): mask j = -acc0[N - j] (j > 0),
    // body = acc_k[0]
#pragma unroll
    for (int r = 0; r < RPW; r++)
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int j = aswz(lat_a1(w, col) + 64 * lrow + 256 * q);
            Ar(r)[2 * j] = lo[r][q];
            Ar(r)[2 * j + 1] = hi[r][q];
        }
    __syncthreads();
    uint64_t *out = a.lwe_out + (size_t)ct * (K * N + 1);
    const uint64_t *A0 = reinterpret_cast<const uint64_t *>(lds + LatLds::Z);  // row 0 (K = 1)
    for (int j = tid; j < N; j += (int)blockDim.x) {
        uint64_t x;
        if (j == 0) {
            x = A0[0];
        } else {
            const int src = N - j;  // acc0[src]: pair (src mod M), lo below M, hi above
            x = 0 - A0[2 * aswz(src & (M - 1)) + (src >= M)];
        }
        out[j] = x;
    }
    if (tid == 0) out[K * N] = reinterpret_cast<const uint64_t *>(lds + LatLds::Z + K * M)[0];
}

// ---------------------------------------------------------------------------------------------
// Multi-bit latency form (N = 2048, k = 1, L = 1, grouping g = 2, 3: the PARAM_MULTI_BIT_MESSAGE_2_
// CARRY_2 sets, shortint/parameters/multi_bit.rs:173-190), the reference's one-ciphertext call
// (shortint/server_key/mod.rs:829-851 -> multi_bit_programmable_bootstrap_lwe_ciphertext,
// lwe_multi_bit_programmable_bootstrapping.rs:1035-1128, deterministic group order :548-828).
// One ciphertext per workgroup of 8 waves with the transform split of the kernel above (LAT_MAP =
// 1 lane mapping), the CMUX replaced by  acc <- ExtProd(KB_j, acc),  KB_j = sum_sel X^{d_sel}
// GGSW_{j,sel}  (prepare_multi_bit_ggsw_mem_optimized :18-84, update_with_fmadd_factor ggsw.rs:
// 699-754).  The keybundle does not depend on the accumulator, so it is built into LDS by all 512
// lanes -- each lane two frequencies of all four (row, column) polynomials, its GGSW operands read
// coalesced (1 KiB per wave instruction) in the engine layout -- while the forward transform of the
// same group runs; the MAC lanes read it back by position after the stage-2 barrier.  No rotation
// (ct1 = acc), so a group has two workgroup barriers: stage 2 -> MAC (C, which also publishes the
// keybundle) and inverse stage 3 -> 2 (E); the backward conversion overwrites the accumulator (the
// reference's zeroed ping-pong destination).  Keybundle in selector order with the fma forms of
// pbs_multibit.hip and the oracle's mb_keybundle, MAC over rows in order: outputs bit-identical to
// the throughput kernels and to oracle/pbs_oracle.c.
// ---------------------------------------------------------------------------------------------
namespace {
// LDS (double2 units): twist planes (TwistLds<1024>: re [M] doubles | im [M] doubles, at byte 0
// for its address-free monomial reads) | X [2 rows][M] | Y [2 rows][M] | keybundle [row][col][M]
// (the accumulator pairs for the sample extraction reuse it at the end)
struct MbLatLds {
    static constexpr int TW = 0;
    static constexpr int X = LAT_M;
    static constexpr int Y = X + 2 * LAT_M;
    static constexpr int KB = Y + 2 * LAT_M;
    static constexpr int end = KB + 4 * LAT_M;
    static constexpr size_t bytes = sizeof(double2) * end;
};
static_assert(MbLatLds::bytes <= 160 * 1024, "multi-bit latency PBS LDS exceeds a CU");
// keybundle slot of engine element E (written by consecutive lanes, read by the MAC blocks:
// bit 2 ^= bit 4 spreads a MAC read group's 8 lanes over 8 distinct 16-byte slots mod 8)
__device__ __forceinline__ int kswz(int E) { return E ^ ((E >> 2) & 4); }
}  // namespace

#ifndef MBL_WINDOW
#define MBL_WINDOW 2  // keybundle elements whose GGSW loads may be in flight at once (register bound)
#endif

template <int G>
__global__ void __launch_bounds__(512, 2) pbs_mb_latency_kernel(MultiBitPbsLaunch a) {
    constexpr int N = LAT_N, M = LAT_M, K = 1, LOG2N = 11, NSEL = 1 << G;
    static_assert(LAT_MAP == 1, "written for the three-barrier lane mapping");
    using Tw = TwistLds<M>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    double2 *lds = reinterpret_cast<double2 *>(smem);
    const int tid = threadIdx.x;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int row0 = wid >> 2;  // this wave's GLWE row (transforms) and output column (MAC)
    const int w = wid & 3;      // quarter of the row's transform
    const int lane0 = tid & 63;

    Tw::fill(reinterpret_cast<double *>(lds + MbLatLds::TW), a.twist, tid, blockDim.x);
    cx tw1[4], tw2[4], tws[4];
    const RowTwF rtf(lane0 >> 4, false), rti(lane0 >> 4, true);
    {
        const int lrow = lane0 >> 4, col = lane0 & 15, a1 = lat_a1(w, col), a2 = lat_a2(w, col);
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int C = lrow + 4 * q;
            tw1[q] = ld2(a.W + a1 * C);
            tw2[q] = ld2(a.W + 16 * a2 * C);
            tws[q] = ld2(a.twist + a1 + 64 * C);
        }
    }

    const int ct = blockIdx.x;
    const int n = a.n, groups = n / G;
    const uint64_t *in = a.lwe_in + (size_t)ct * (n + 1);
    const __attribute__((address_space(4))) uint64_t *in_s = (const __attribute__((address_space(4))) uint64_t *)(
        ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)((uintptr_t)in >> 32)) << 32) |
        (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)in));
    const uint32_t li = a.lut_indexes ? min(a.lut_indexes[ct], a.lut_count - 1u) : 0u;
    const DigitL1 digit_l1(a.base_log);

    // acc = LUT / X^{b~} (:372-389): this lane's pairs j_q = a1 + 64 (lrow + 4 q), j_q + M of row row0
    uint64_t lo[4], hi[4];
    {
        const uint32_t bt = pbs_modulus_switch<LOG2N>(in[n]);
        const int full = bt / N, rem = bt % N;
        const uint64_t *lut = a.luts + (size_t)li * (K + 1) * N + (size_t)row0 * N;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int j = lat_a1(w, lane0 & 15) + 64 * (lane0 >> 4) + 256 * q;
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const int src = j + h * M + rem;
                const bool wrap = src >= N;
                const uint64_t v = lut[wrap ? src - N : src];
                const uint64_t c = (wrap != (bool)(full & 1)) ? 0 - v : v;
                (h ? hi : lo)[q] = c;
            }
        }
    }
    auto Xr = [&](int r) { return lds + MbLatLds::X + r * M; };
    auto Yr = [&](int r) { return lds + MbLatLds::Y + r * M; };
    double2 *kbl = lds + MbLatLds::KB;
    constexpr size_t ggsw_len = (size_t)(K + 1) * (K + 1) * M;
    const __amdgpu_buffer_rsrc_t gres = make_rsrc(a.fbsk);
    // keybundle elements of this lane: E = tid and tid + 512, frequency fl + freq_slot(wid) (+ 32)
    // (element s 64 + lane of WaveFft<1024>'s engine layout, s = wid and wid + 8)
    const int32_t kf0 = (int32_t)(WaveFft<M>::freq_lane(lane0) + WaveFft<M>::freq_slot(wid));
    const double k32 = torus_k32();
    __syncthreads();  // twist planes

    for (int j = 0; j < groups; j++) {
        int lane = lane0;
        asm volatile("" : "+v"(lane));
        const int lrow = lane >> 4, col = lane & 15;
        const int ccm = 4 * w + (col & 3), xm = col >> 2;

        // ---- keybundle of group j into LDS (every lane; independent of the accumulator) ----
        {
            int32_t dd[NSEL];  // monomial degrees of the 2^g - 1 non-constant GGSWs (:700-716), SGPRs
            {
                uint64_t av[G];
#pragma unroll
                for (int i = 0; i < G; i++) av[i] = in_s[j * G + i];
#pragma unroll
                for (int sel = 1; sel < NSEL; sel++) {
                    uint64_t deg = 0;
#pragma unroll
                    for (int i = 0; i < G; i++)
                        if ((sel >> (G - 1 - i)) & 1) deg += av[i];
                    dd[sel] = (int32_t)pbs_modulus_switch<LOG2N>(deg);  // <= 2N
                }
            }
            uint32_t loff = 16u * (uint32_t)tid;
            const uint32_t goff = (uint32_t)((size_t)j * NSEL * ggsw_len * 16);  // < 2^31 (MB-BSK bytes)
            double dep = 0.0;
            double depq[MBL_WINDOW];
#pragma unroll
            for (int q = 0; q < MBL_WINDOW; q++) depq[q] = 0.0;
#pragma unroll
            for (int h = 0; h < 2; h++) {
                // t = d (1 - 4 f) mod 2N as a 24-bit signed product (|1 - 4 f| < 2^12, d <= 2^12)
                const int32_t wf = 1 - 4 * (kf0 + 32 * h);
                cx mono[NSEL];
#pragma unroll
                for (int sel = 1; sel < NSEL; sel++) mono[sel] = Tw::mono((uint32_t)__mul24(dd[sel], wf));
#pragma unroll
                for (int p = 0; p < 4; p++) {  // polynomial (row rr = p >> 1, column c = p & 1)
                    const int e = 4 * h + p;
                    // issue window: this element's loads wait (as far as the compiler knows) for the
                    // element MBL_WINDOW back, so at most that many elements' operands are live
                    if (e >= MBL_WINDOW) {
                        dep = depq[e % MBL_WINDOW];
                        asm volatile("" : "+v"(loff) : "v"(dep));
                    }
                    const uint32_t eoff = goff + (uint32_t)(((size_t)p * M + (size_t)h * 512) * 16);
                    double2 kb = buffer_ld_d2(gres, loff, eoff);
#pragma unroll
                    for (int sel = 1; sel < NSEL; sel++) {
                        const double2 gg = buffer_ld_d2(gres, loff, eoff + (uint32_t)(sel * ggsw_len * 16));
                        kb.x = fma(gg.x, mono[sel].re, fma(-gg.y, mono[sel].im, kb.x));
                        kb.y = fma(gg.x, mono[sel].im, fma(gg.y, mono[sel].re, kb.y));
                    }
                    depq[e % MBL_WINDOW] = kb.x;
                    kbl[p * M + kswz(tid + 512 * h)] = kb;
                }
            }
        }

        // ---- digits of the accumulator (ct1 = acc), twist, forward stage 1 (wave-private) ----
        cx v[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int32_t d0 = digit_l1((uint32_t)(lo[q] >> 32));
            const int32_t d1 = digit_l1((uint32_t)(hi[q] >> 32));
            v[q] = cmulw(cx{(double)d0, (double)d1}, tws[q].re, tws[q].im);  // convert_forward_integer
        }
        dft16_fwd_rows_sf(v, rtf);
        {
            const int a1 = lat_a1(w, col);
#pragma unroll
            for (int q = 0; q < 4; q++) st2(Xr(row0) + lswz(a1 + 64 * (lrow + 4 * q)), cmulw(v[q], tw1[q].re, tw1[q].im));
        }
        WaveLocalSync{}();
        // ---- forward stage 2 (block cc = col, butterfly a2 = w) ----
        const int cc = lat_cc(w, col), a2 = lat_a2(w, col);
#pragma unroll
        for (int q = 0; q < 4; q++) v[q] = ld2(Xr(row0) + lswz(64 * cc + a2 + 4 * (lrow + 4 * q)));
        dft16_fwd_rows_sf(v, rtf);
#pragma unroll
        for (int q = 0; q < 4; q++) st2(Yr(row0) + lswz(64 * cc + a2 + 4 * (lrow + 4 * q)), cmulw(v[q], tw2[q].re, tw2[q].im));
        lds_barrier();  // (C) both rows' stage-2 outputs and the whole keybundle

        // ---- stage 3 of both rows + MAC of column row0 on block t with the keybundle ----
        const int tb = 64 * ccm + 4 * (lrow + 4 * xm);  // first position of block t
        cx o[4];
        {
            cx f[K + 1][4];
#pragma unroll
            for (int rr = 0; rr <= K; rr++) {
                const double2 *y = lds + MbLatLds::Y + rr * M;
#pragma unroll
                for (int e = 0; e < 4; e++) f[rr][e] = ld2(y + lswz(tb + e));
                r4_fwd(f[rr][0], f[rr][1], f[rr][2], f[rr][3]);
            }
#pragma unroll
            for (int rr = 0; rr <= K; rr++)
#pragma unroll
                for (int e = 0; e < 4; e++) {
                    // position tb + e is engine element (4 lrow + e) 64 + 16 xm + ccm
                    const double2 kb = kbl[(rr * (K + 1) + row0) * M + kswz((4 * lrow + e) * 64 + 16 * xm + ccm)];
                    const double2 ff = make_double2(f[rr][e].re, f[rr][e].im);
                    if (rr == 0) {  // MAC over rows (update_with_fmadd order)
                        o[e].re = fma(kb.x, ff.x, -(kb.y * ff.y));
                        o[e].im = fma(kb.x, ff.y, kb.y * ff.x);
                    } else {
                        o[e].re = fma(kb.x, ff.x, fma(-kb.y, ff.y, o[e].re));
                        o[e].im = fma(kb.x, ff.y, fma(kb.y, ff.x, o[e].im));
                    }
                }
        }
        r4_inv(o[0], o[1], o[2], o[3]);
#pragma unroll
        for (int e = 0; e < 4; e++) st2(Xr(row0) + lswz(tb + e), o[e]);
        lds_barrier();  // (E) inverse stage 2 reads one residue class of every block (all four waves)
#pragma unroll
        for (int q = 0; q < 4; q++)
            v[q] = cmulw(ld2(Xr(row0) + lswz(64 * cc + a2 + 4 * (lrow + 4 * q))), tw2[q].re, -tw2[q].im);
        dft16_inv_rows_sf(v, rti);
        WaveLocalSync{}();
#pragma unroll
        for (int q = 0; q < 4; q++) st2(Xr(row0) + lswz(64 * cc + a2 + 4 * (lrow + 4 * q)), v[q]);
        WaveLocalSync{}();
        // ---- inverse stage 1 + backward conversion (overwrites the accumulator) ----
        {
            const int a1 = lat_a1(w, col);
#pragma unroll
            for (int q = 0; q < 4; q++) v[q] = cmulw(ld2(Xr(row0) + lswz(a1 + 64 * (lrow + 4 * q))), tw1[q].re, -tw1[q].im);
            dft16_inv_rows_sf(v, rti);
#pragma unroll
            for (int q = 0; q < 4; q++) backward_convert(v[q], tws[q], lo[q], hi[q], k32);  // the key carries 1/M
        }
    }

    // ---- output ----
    const int lrow = lane0 >> 4, col = lane0 & 15;
    if (a.glwe_out) {  // bootstrap_without_sample_extract (fork, bootstrap.rs:383-412)
        uint64_t *g = a.lwe_out + ((size_t)ct * (K + 1) + row0) * N;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int jj = lat_a1(w, col) + 64 * lrow + 256 * q;
            g[jj] = lo[q];
            g[jj + M] = hi[q];
        }
        return;
    }
    __syncthreads();  // every wave's last keybundle reads are done: its area takes the pairs
    uint64_t *A = reinterpret_cast<uint64_t *>(lds + MbLatLds::KB);
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int jj = aswz(lat_a1(w, col) + 64 * lrow + 256 * q);
        A[2 * (row0 * M + jj)] = lo[q];
        A[2 * (row0 * M + jj) + 1] = hi[q];
    }
    __syncthreads();
    // sample extract at degree 0 (glwe_sample_extraction.rs:91-147)
    uint64_t *out = a.lwe_out + (size_t)ct * (K * N + 1);
    for (int jj = tid; jj < N; jj += (int)blockDim.x) {
        uint64_t x;
        if (jj == 0) {
            x = A[0];
        } else {
            const int src = N - jj;
            x = 0 - A[2 * aswz(src & (M - 1)) + (src >= M)];
        }
        out[jj] = x;
    }
    if (tid == 0) out[K * N] = A[2 * M * K];
}

bool latency_multibit_supported(int N, int k, int L, int g) { return N == 2048 && k == 1 && L == 1 && (g == 2 || g == 3); }

hipError_t launch_latency_multibit_pbs(int g, const MultiBitPbsLaunch &a, hipStream_t s) {
    if (a.count <= 0) return hipSuccess;
    if (a.n % g) return hipErrorInvalidValue;
    if (g == 3)
        hipLaunchKernelGGL(pbs_mb_latency_kernel<3>, dim3(a.count), dim3(512), MbLatLds::bytes, s, a);
    else if (g == 2)
        hipLaunchKernelGGL(pbs_mb_latency_kernel<2>, dim3(a.count), dim3(512), MbLatLds::bytes, s, a);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

bool latency_pbs_supported(int N, int k, int L) { return N == 2048 && k == 1 && L == 1; }

#ifndef LAT_RPW
#define LAT_RPW 1  // GLWE rows per wave (1: 8 waves per ciphertext, 2: 4 waves; 2 needs LAT_MAP=0)
#endif

hipError_t launch_latency_pbs(const ClassicPbsLaunch &a, hipStream_t s) {
    if (a.count <= 0) return hipSuccess;
    hipLaunchKernelGGL(pbs_latency_kernel<LAT_RPW>, dim3(a.count), dim3(512 / LAT_RPW), LatLds::bytes, s, a);
    return hipGetLastError();
}

}  // namespace tfhe_mi355
