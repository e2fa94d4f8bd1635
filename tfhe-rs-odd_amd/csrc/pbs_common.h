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
