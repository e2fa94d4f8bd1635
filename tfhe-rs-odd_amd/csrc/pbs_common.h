// pbs_common.h -- device helpers shared by the classic and multi-bit PBS kernels.
#pragma once
#include "fft_device.h"

#ifndef PBS_WAVE_LOCAL
#define PBS_WAVE_LOCAL 1
#endif
#ifndef PBS_BWD_SB
#define PBS_BWD_SB 2  // backward-conversion slots per scheduling region (bounds live f64 temporaries)
#endif
#ifndef PBS_MAC_SB
#define PBS_MAC_SB 4  // MAC slots per scheduling region
#endif
#ifndef PBS_GGSW_PREFETCH
#define PBS_GGSW_PREFETCH 0  // L = 1: GGSW_{i+1} column into registers during CMUX i's inverse FFT (measured 8% slower: AGPR shuffles)
#endif
#ifndef PBS_MAC_FROM_LDS
#define PBS_MAC_FROM_LDS -1  // classic kernel: -1 per-shape default (PbsConfig::MAC_LDS), 0/1 force
#endif
#ifndef PBS_WAVES_PER_EU
#define PBS_WAVES_PER_EU 0  // 0: per-shape default (PbsConfig::WPE); the multi-bit kernel uses 1
#endif

#ifndef PBS_SYNC_SLEEP
#define PBS_SYNC_SLEEP 1  // s_sleep argument between polls of a partner's flag (64 clocks per unit)
#endif
#define PBS_STR2(x) #x
#define PBS_STR(x) PBS_STR2(x)
#define PBS_SYNC_SLEEP_STR PBS_STR(PBS_SYNC_SLEEP)
#ifndef PBS_GROUP_SYNC
#define PBS_GROUP_SYNC 1  // CMUX-loop syncs between the (k+1) waves of ONE ciphertext (LDS flags), not s_barrier
#endif

#ifndef PBS_SLOT_MAJOR
#define PBS_SLOT_MAJOR 0  // classic kernel: 1 = wave w serves (row w / CPW, ciphertext w % CPW) -- one ciphertext per SIMD
#endif
#ifndef PBS_PERSIST
#define PBS_PERSIST -1  // classic PBS persistent grid + ticket queue: -1 per-shape default (PbsConfig), 0/1 force
#endif

namespace tfhe_mi355 {

// Workgroups of a kernel resident at once on the current device (CUs x occupancy); the
// persistent PBS grids are capped at this so that every workgroup is running from the start.
inline int resident_blocks(const void *kernel, int threads, size_t lds) {
    int dev = 0, cus = 0, per = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, threads, lds) != hipSuccess || cus <= 0 || per <= 0)
        return 0x7fffffff;
    return cus * per;
}

template <int LOG2N>
__device__ __forceinline__ uint32_t pbs_modulus_switch(uint64_t x) {
    uint64_t o = x >> (64 - LOG2N - 2);
    o += 1;
    o >>= 1;
    return (uint32_t)o;  // in [0, 2N]
}

constexpr int ilog2(int x) { return x <= 1 ? 0 : 1 + ilog2(x / 2); }

struct BlockSync {
    __device__ __forceinline__ void operator()() const { __syncthreads(); }
};
// Orders LDS accesses among the lanes of ONE wavefront: LDS executes a wave's ds_* operations
// in issue order, so a compiler-level fence at wavefront scope is all a wave-private buffer
// (rotation, FFT exchanges) needs -- no s_barrier across the workgroup.
struct WaveLocalSync {
    __device__ __forceinline__ void operator()() const {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
};
// The same sync, telling WaveFft<1024> to recompute its exchange addresses at every call
// (SyncLaunder, fft_device.h) instead of letting them be hoisted out of the caller's loop: for
// kernels at the 256-VGPR limit, where the 32 hoisted XOR addresses were spilled to scratch
// inside the CMUX loop (onchip_cmux_kernel<N, D32, 2>).
template <int Bits>
struct WaveLocalSyncL : WaveLocalSync {
    static constexpr int launder = Bits;
};

// Sync among the (k+1) waves of one ciphertext through LDS flags instead of s_barrier, so the
// ciphertexts sharing a workgroup (and a CU) are not forced into lockstep: their LDS bursts and
// VALU phases drift apart and overlap.  Each wave publishes a per-wave counter after its LDS
// writes (a wave's LDS operations execute in issue order, so a partner that reads the new
// count also sees the data) and polls its partners' counters.  Every wave of a group executes
// the same number of syncs, so every wait ends.
// The store and the poll are asm blocks (memory clobbers keep the compiler from moving LDS
// accesses across them); as C++ atomics in a loop the CMUX loop's register allocation spilled.
template <int W>  // waves in the group
struct GroupSync {
    uint32_t base;      // LDS byte address of the group's first flag word
    uint32_t mine;      // LDS byte address of this wave's flag word
    uint32_t seq = 0;
    __device__ __forceinline__ void operator()() {
        seq++;
        asm volatile("ds_write_b32 %0, %1" ::"v"(mine), "v"(seq) : "memory");
#pragma unroll
        for (int r = 0; r < (W == 2 ? 1 : W); r++) {
            // W = 2: only the partner's word (the group's two words are 8-byte aligned, so it is
            // this wave's address ^ 4); otherwise every word, its own (already published) included
            const uint32_t addr = W == 2 ? (mine ^ 4u) : base + 4u * r;
            uint32_t tmp, stmp;
            asm volatile(
                "1:\n\t"
                "ds_read_b32 %[v], %[a]\n\t"
                "s_waitcnt lgkmcnt(0)\n\t"
                "v_readfirstlane_b32 %[s], %[v]\n\t"
                "s_nop 1\n\t"
                "s_cmp_lt_u32 %[s], %[q]\n\t"
                "s_cbranch_scc0 2f\n\t"
                "s_sleep " PBS_SYNC_SLEEP_STR "\n\t"
                "s_branch 1b\n\t"
                "2:"
                : [v] "=&v"(tmp), [s] "=&s"(stmp)
                : [a] "v"(addr), [q] "s"(seq)
                : "scc", "memory");
        }
    }
};

// digit extraction in 32-bit registers: valid when base_log * level <= 30 (all supported
// parameter sets).  Bit-identical digits to the 64-bit SignedDecomposer (decomposer.rs:99-119,
// iter.rs:134-141): the only divergence is the discarded final state when the rounding
// overflows, where every digit is 0 in both.
template <int L>
__device__ __forceinline__ uint32_t decomp_state32(uint64_t x, int beta) {
    const int shift = 63 - beta * L;  // >= 33
    uint32_t s = (uint32_t)((x >> 32) >> (shift - 32));
    return (s + 1) >> 1;
}
template <int L>
__device__ __forceinline__ uint32_t decomp_state32_hi(uint32_t x_hi, int beta) {
    const int shift = 63 - beta * L;  // >= 33
    return ((x_hi >> (shift - 32)) + 1) >> 1;
}
// L = 1: s = ((x >> (63 - beta)) + 1) >> 1, digit = s mod 2^beta balanced into
// (-2^(beta-1), 2^(beta-1)] -- the SignedDecomposer's carry rule for one level, since the
// state left after the level is 0 or 1 and only 1 when the digit is 0.
// With c = 2^beta - 1, k = 31 - beta and h = 2^(beta-1) - 1 the digit is
// bfe((x_hi >> k) + c, 1, beta) - h; adding c << k before the shift (the low k bits of x_hi
// cannot carry into bit k) turns the bfe into the plain shift by 32 - beta:
// digit = ((x_hi + (c << k)) >> (32 - beta)) - h  -- three VALU ops instead of four.
struct DigitL1 {
    uint32_t ck;  // (2^beta - 1) << (31 - beta)
    int sh;       // 32 - beta
    int32_t h;    // 2^(beta-1) - 1
    __device__ __forceinline__ explicit DigitL1(int beta)
        : ck(((1u << beta) - 1) << (31 - beta)), sh(32 - beta), h((int32_t)(1u << (beta - 1)) - 1) {}
    __device__ __forceinline__ int32_t operator()(uint32_t x_hi) const {
        return (int32_t)((x_hi + ck) >> sh) - h;
    }
};
__device__ __forceinline__ int32_t decomp_digit32(uint32_t &state, int beta, uint32_t mask) {
    uint32_t res = state & mask;
    state >>= beta;
    uint32_t carry = ((res - 1) | state) & res;
    carry >>= beta - 1;
    state += carry;
    return (int32_t)(res - (carry << beta));
}

// Two levels (2 beta <= 30) of two values straight into int16 pairs: the digits of
// decomp_state32<2> + two decomp_digit32 calls, 9 VALU per value instead of 18.  With y = x_hi +
// 2^(31 - 2 beta) (the rounding; a 32-bit wrap only drops the final carry), the state is
// y >> (32 - 2 beta), so with h = 2^(beta-1):
//   a  = state mod 2^beta,  t = bit 31 of y (the state bit the tie rule reads),
//   c  = [a + t > h]  = bit beta of z0 = a + t + h - 1,   d0 = a - c 2^beta,
//   d1 = ((y >> (32 - beta)) + c + h - 1) mod 2^beta - (h - 1)
// (every x_hi and beta = 1..15 checked against decomp_digit32 by scripts/check_digit2.cpp).
struct Digit2 {
    uint32_t k1, mask, hm1, maskx2, hm1x2;
    int s0, s1, beta, nb;
    __device__ __forceinline__ explicit Digit2(int b)
        : k1(1u << (31 - 2 * b)), mask((1u << b) - 1), hm1((1u << (b - 1)) - 1),
          maskx2(((1u << b) - 1) * 0x10001u), hm1x2(((1u << (b - 1)) - 1) * 0x10001u),
          s0(32 - 2 * b), s1(32 - b), beta(b), nb(-(1 << b)) {}
    // digits of the values with hi words xa, xb -> lv0 = level-L pair (xa low half), lv1 = level L-1
    __device__ __forceinline__ void pair(uint32_t xa, uint32_t xb, uint32_t &lv0, uint32_t &lv1) const {
        typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
        uint32_t d0[2], z1[2];
        const uint32_t x[2] = {xa, xb};
#pragma unroll
        for (int e = 0; e < 2; e++) {
            const uint32_t y = x[e] + k1;
            const uint32_t a = __builtin_amdgcn_ubfe(y, s0, beta);
            const uint32_t z0 = a + (y >> 31) + hm1;
            const uint32_t c = __builtin_amdgcn_ubfe(z0, beta, 1);
            d0[e] = a + (uint32_t)__mul24((int)c, nb);  // v_mad_i32_i24 (c is 0 or 1, nb = -2^beta)
            z1[e] = (y >> s1) + c + hm1;
        }
        lv0 = __builtin_amdgcn_perm(d0[1], d0[0], 0x05040100u);
        const u16x2 m = __builtin_bit_cast(u16x2, __builtin_amdgcn_perm(z1[1], z1[0], 0x05040100u) & maskx2);
        lv1 = __builtin_bit_cast(uint32_t, m - __builtin_bit_cast(u16x2, hm1x2));
    }
};

#ifndef PBS_MB_TSKIP_MONO
#define PBS_MB_TSKIP_MONO 0
#endif
#ifndef PBS_MB_SWK
#define PBS_MB_SWK 4   // twist-table swizzle: position r ^ ((r >> SWK) & SWM) (M = 1024)
#endif
#ifndef PBS_MB_SWM
#define PBS_MB_SWM 23
#endif
// Twist table in LDS, shared by the linear twist reads (digits, backward conversion) and the
// keybundle's monomial reads.  A monomial read fetches entry r of t = d (1 - 4 f) mod 2N, lanes
// 16 apart in f stepping t by 4d and the two 16-lane halves of a ds_read_b64 group by 256d.  As one
// [M] double2 array the 32 lanes of a group put 8.1 distinct entries on one bank on average (PMC:
// 56 % of the g = 3 kernel's LDS cycles were conflict cycles, profiles/r03_pmc_mb3.json).  Here re
// and im are two [M] double planes and entry r sits at position r ^ ((r >> SWK) & SWM): 2.09 on
// average, worst 4 (exhaustive over d and slots) with SWK = 4, SWM = 23, the best of every shift
// and 10-bit mask (round 3: r ^ ((r >> 5) & 31), 2.36 / worst 8; scripts/probes/
// twist_swizzle_search.py); same two instructions per monomial read, and a linear read
// (r = lane + 64 b) stays conflict-free (the map is linear: position = 64 b + (lane ^ swz(lane) ^
// swz(64 b))).
// (M = 256, the k = 3 sets: plain planes, no swizzle.)
// (M = 4096, the N = 8192 multi-bit paired sub-block kernel: r ^ ((r >> 6) & 31), the best worst
// case of the shift-mask family for that kernel's read pattern (lanes step t by 16 d R): 2.12
// distinct entries per bank on average, worst 4, against 19.6 / 32 for the plain planes
// (scripts/probes/twist_swizzle_search_8192.py; k = 7 gives 2.10 but worst 6).)
#ifndef PBS_MB8_SWK
#define PBS_MB8_SWK 6
#endif
#ifndef PBS_MB8_SWM
#define PBS_MB8_SWM 31
#endif
template <int M>
struct TwistSwz {
    static constexpr uint32_t K = 0, MASK = 0;
};
template <>
struct TwistSwz<1024> {
    static constexpr uint32_t K = PBS_MB_SWK, MASK = PBS_MB_SWM;
};
template <>
struct TwistSwz<4096> {
    static constexpr uint32_t K = PBS_MB8_SWK, MASK = PBS_MB8_SWM;
};
template <int M>
struct TwistLds {
    static_assert(M == 1024 || M == 256 || M == 4096, "twist table layouts for M = 1024, 4096 (swizzled) and 256");
    static constexpr bool SW = TwistSwz<M>::MASK != 0;
    static constexpr uint32_t IM = 8u * M;  // byte offset of the im plane (table at LDS byte 0)
    static constexpr uint32_t SWK = TwistSwz<M>::K, SWM = TwistSwz<M>::MASK;
    static_assert(!SW || SWM >> (ilog2(M) - SWK) == 0, "the swizzle reads bits of r only (not the quadrant bit)");
    __device__ static uint32_t swz(uint32_t r) { return SW ? (r >> SWK) & SWM : 0u; }
    __device__ static uint32_t pos(uint32_t r) { return r ^ swz(r); }
    __device__ static void fill(double *t, const double2 *twist, int tid, int nt) {
        for (int e = tid; e < M; e += nt) {
            const uint32_t p = pos((uint32_t)e);
            t[p] = twist[e].x;
            t[M + p] = twist[e].y;
        }
    }
    // 8 (lane ^ swz(lane)): position of twist[lane + 64 b] is 64 b + (lane ^ swz(lane) ^ swz(64 b))
    // (swz(64 b) < 64 for every swizzle allowed here)
    __device__ static uint32_t lane_base(int lane) { return 8u * (uint32_t)(SW ? lane ^ swz(lane) : lane); }
    __device__ static cx linear(uint32_t lb, int b) {  // twist[lane + 64 b]; b compile-time: one XOR
        const uint32_t a = (SW ? lb ^ (8u * swz(64u * (uint32_t)b)) : lb) + 512u * (uint32_t)b;
        return {lds_ld_f64(a), lds_ld_f64(a + IM)};
    }
    // i^q twist[r] for t = q M + r (t mod 2^32, bits 0 .. log2 M + 1 used): the swap for odd q is
    // the plane choice of the two reads (re at the returned address, im at address ^ IM), the signs
    // (re: q0 ^ q1, im: q1) are XORed into the high words -- no selects
    __device__ static cx mono(uint32_t t) {
        constexpr int LOG2M = ilog2(M);
        // PBS_MB_TSKIP_MONO (timing-only builds, wrong outputs): every lane reads its own entry, so
        // the monomial reads are conflict-free -- measures what their bank conflicts cost
        const uint32_t are = PBS_MB_TSKIP_MONO ? ((t & (uint32_t)M) | (uint32_t)__lane_id()) << 3
                                               : ((t & (2u * M - 1)) ^ swz(t)) << 3;
        const double re = lds_ld_f64(are), im = lds_ld_f64(are ^ IM);
        const uint32_t sim = t << (30 - LOG2M);  // q1 at bit 31; + 2^30 carries q0 into it
        return {flip_sign(re, sim + 0x40000000u), flip_sign(im, sim)};
    }
};

template <int M>
struct PbsLds {
    using Fft = WaveFft<M>;
    using Tw = typename Fft::Lds;
    static constexpr int XL = Fft::XL;
    // layout (double2 units): [twist M][s1 table][s2 table][exchange: one XL buffer per wave]
    static constexpr int twist_off = 0;
    static constexpr int s1_off = M;
    static constexpr int s2_off = s1_off + Tw::s1_len;
    // M = 1024 exchange buffers start on 1 KiB boundaries (WaveFft<1024> XORs into the address)
    static constexpr int XALIGN = M == 1024 ? 64 : 4;
    static constexpr int xbuf_off = ((s2_off + Tw::s2_len + XALIGN - 1) / XALIGN) * XALIGN;
    static constexpr size_t bytes(int waves) { return sizeof(double2) * (size_t)(xbuf_off + waves * XL); }
};

}  // namespace tfhe_mi355
