// fir_common.h — shared device helpers for the gfx950 FIR kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fir_hip.h"

namespace fir {

constexpr int kWave = 64;
constexpr int kBlock = 256;  // 4 waves: one per SIMD of a CU

// gfx9 DPP wavefront shifts (whole 64-lane wave, not row-limited).
constexpr int kDppWaveShl1 = 0x130;  // lane i <- lane i+1
constexpr int kDppWaveShr1 = 0x138;  // lane i <- lane i-1

// lane i receives lane i-1's `v`; lane 0 (no source) keeps `own`.
__device__ __forceinline__ uint32_t from_prev_lane(uint32_t own, uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)own, (int)v, kDppWaveShr1, 0xF, 0xF, false);
}
// lane i receives lane i+1's `v`; lane 63 keeps `own`.
__device__ __forceinline__ uint32_t from_next_lane(uint32_t own, uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)own, (int)v, kDppWaveShl1, 0xF, 0xF, false);
}

template <typename T>
struct InTraits;
template <>
struct InTraits<uint8_t> {
    static constexpr int kPerDword = 4;
    __device__ static __forceinline__ int32_t get(uint32_t d, int i) { return (int32_t)((d >> (8 * i)) & 0xFFu); }
};
template <>
struct InTraits<int16_t> {
    static constexpr int kPerDword = 2;
    __device__ static __forceinline__ int32_t get(uint32_t d, int i) {
        return i ? ((int32_t)d >> 16) : ((int32_t)(d << 16) >> 16);
    }
};

template <int STAGE>
struct OutTraits;
template <>
struct OutTraits<FIR_OUT_U8_SAT> {
    using T = uint8_t;
};
template <>
struct OutTraits<FIR_OUT_I32> {
    using T = int32_t;
};

// (wrap(acc) + 2^(f-1)) >> f for a 32-bit accumulator; shl = 32 - acc_bits (0..31).
// Overflow-free form of fir_1d_fixed_ref.py:110-120: floor(a / 2^f) + bit (f-1) of a.
__device__ __forceinline__ int32_t round32(uint32_t acc, int shl, int frac) {
    const int32_t a = (int32_t)(acc << shl) >> shl;
    return (a >> frac) + ((a >> (frac - 1)) & 1);
}

// (wrap(acc) + 2^(f-1)) >> f, with the wrap skipped when acc_bits == 32 (ACC32).
template <bool ACC32>
__device__ __forceinline__ int32_t round_acc(uint32_t acc, int shl, int frac) {
    const int32_t a = ACC32 ? (int32_t)acc : (int32_t)(acc << shl) >> shl;
    return (a >> frac) + ((a >> (frac - 1)) & 1);
}

// 64-bit generic form (any acc_bits >= 1, any frac_bits >= 1): `acc` is the sum mod 2^64,
// which is exact for the wrap to acc_bits < 64, and the true sum for acc_bits >= 64 whenever the
// launchers pick this form: only when needs_wide is false, i.e. |sum| < 2^63 is proven for the
// taps and sample range (round128 below carries every other no-wrap sum).  floor((a + 2^(f-1)) /
// 2^f) without overflow: (a >> f) + bit (f-1) of a; for f >= 64 that is 0 for every |a| < 2^63.
__device__ __forceinline__ int64_t round64(int64_t acc, int frac, int acc_bits) {
    if (acc_bits < 64) {
        const int s = 64 - acc_bits;
        acc = (int64_t)((uint64_t)acc << s) >> s;
    }
    if (frac >= 64) return 0;
    return (acc >> frac) + ((acc >> (frac - 1)) & 1);
}

// 128-bit form for sums that may exceed 2^63 (no-wrap calls with huge taps x samples): `acc` is
// the exact sum (|sum| < 2^127 for every legal input: FIR_MAX_TAPS x 2^31 x 2^15), wrapped to
// acc_bits < 128 like the reference's mask-and-sign-restore, then rounded.
__device__ __forceinline__ __int128 round128(__int128 acc, int frac, int acc_bits) {
    if (acc_bits < 128) {
        const int s = 128 - acc_bits;
        acc = (__int128)((unsigned __int128)acc << s) >> s;
    }
    if (frac >= 128) return 0;
    return (acc >> frac) + ((acc >> (frac - 1)) & 1);
}

template <int STAGE>
__device__ __forceinline__ typename OutTraits<STAGE>::T stage_out(int64_t q) {
    if constexpr (STAGE == FIR_OUT_U8_SAT) {
        return (uint8_t)(q < 0 ? 0 : (q > 255 ? 255 : q));
    } else {
        return (int32_t)q;
    }
}

// the stage of a 128-bit result: u8 saturation, or the low 32 bits (as stage_out's int32 cast)
template <int STAGE>
__device__ __forceinline__ typename OutTraits<STAGE>::T stage_out128(__int128 q) {
    if constexpr (STAGE == FIR_OUT_U8_SAT) {
        return (uint8_t)(q < 0 ? 0 : (q > 255 ? 255 : (int)q));
    } else {
        return (int32_t)(uint32_t)(unsigned __int128)q;
    }
}

template <int STAGE>
__device__ __forceinline__ typename OutTraits<STAGE>::T stage_out32(int32_t q) {
    if constexpr (STAGE == FIR_OUT_U8_SAT) {
        return (uint8_t)min(max(q, 0), 255);  // v_med3_i32
    } else {
        return q;
    }
}

// ---- packed integer helpers shared by the 1-D and 2-D register kernels ----

typedef short fir_short2 __attribute__((ext_vector_type(2)));

// v_dot2_i32_i16 (no clamp: wrap-around int32) on raw dwords
__device__ __forceinline__ uint32_t dot2_acc(uint32_t a, uint32_t b, uint32_t c) {
    return (uint32_t)__builtin_amdgcn_sdot2(__builtin_bit_cast(fir_short2, a), __builtin_bit_cast(fir_short2, b),
                                            (int)c, false);
}

// First MAC of a chain without a zero-initialised destination: VOP3P v_dot2_i32_i16 with an
// inline-constant or VGPR addend (hipcc otherwise emits v_dot2c plus a v_mov of the addend).
// Pure VALU, no memory, no hazards: safe as inline asm.
__device__ __forceinline__ uint32_t dot2_from0(uint32_t pair, uint32_t taps) {
    uint32_t d;
    asm("v_dot2_i32_i16 %0, %1, %2, 0" : "=v"(d) : "v"(pair), "s"(taps));
    return d;
}
__device__ __forceinline__ uint32_t dot2_from(uint32_t pair, uint32_t taps, uint32_t c) {
    uint32_t d;
    asm("v_dot2_i32_i16 %0, %1, %2, %3" : "=v"(d) : "v"(pair), "s"(taps), "v"(c));
    return d;
}

// v_mad_i32_i24 d = a[23:0] * b[23:0] + c (|a|, |b| < 2^23 host-checked); as asm because hipcc
// sign-extends a value it cannot range-check (v_bfe_i32) before every __mul24.
__device__ __forceinline__ uint32_t mad_i24(uint32_t a, int32_t b, uint32_t c) {
    uint32_t d;
    asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(d) : "v"(a), "s"(b), "v"(c));
    return d;
}

// bytes k and k+1 of a little-endian byte stream held in dwords s[], zero-extended into the
// two 16-bit halves of one dword (one v_perm_b32).
template <int K>
__device__ __forceinline__ uint32_t pair16(const uint32_t* s) {
    constexpr int d0 = K / 4, b0 = K % 4, d1 = (K + 1) / 4, b1 = (K + 1) % 4;
    if constexpr (d0 == d1) {
        constexpr uint32_t sel = (uint32_t)b0 | (0x0Cu << 8) | ((uint32_t)b1 << 16) | (0x0Cu << 24);
        return __builtin_amdgcn_perm(s[d0], s[d0], sel);
    } else {
        // perm(hi_src, lo_src): bytes 0-3 = lo_src, 4-7 = hi_src
        constexpr uint32_t sel = (uint32_t)b0 | (0x0Cu << 8) | ((uint32_t)(4 + b1) << 16) | (0x0Cu << 24);
        return __builtin_amdgcn_perm(s[d1], s[d0], sel);
    }
}

template <int K0, int N>
struct PairBuilder {
    __device__ static __forceinline__ void run(const uint32_t* s, uint32_t* P) {
        if constexpr (N > 0) {
            P[K0] = pair16<K0>(s);
            PairBuilder<K0 + 1, N - 1>::run(s, P);
        }
    }
};

// One saturated u8 output.  NOWRAP (bias already in acc): clamp to [0, 256*2^f - 1] first,
// then shift -- the same value as sat(acc >> f), in an order hipcc (ROCm 7.2) does not fuse
// into v_ashr_pk_u8_i32: that fusion left bits set above the packed byte pair, which the
// following v_lshl_or merged into the next pixel (measured: wrong byte 2 of every dword).
template <bool NOWRAP>
__device__ __forceinline__ uint32_t sat_u8_pixel(uint32_t acc, int shl, int frac, int32_t sat_hi) {
    if constexpr (NOWRAP) {
        uint32_t c;  // v_med3_i32(acc, 0, hi) == clamp(acc, 0, hi) since hi > 0 (hipcc emits max + min)
        asm("v_med3_i32 %0, %1, 0, %2" : "=v"(c) : "v"(acc), "s"(sat_hi));
        return c >> frac;
    } else {
        return (uint32_t)min(max(round32(acc, shl, frac), 0), 255);
    }
}

// Packed 16-bit pixel-pair arithmetic (v_pk_mad_u16: exact mod 2^16 in each half), shared by
// the 1-D u8 and 2-D packed-16 forms.
typedef unsigned short fir_u16x2 __attribute__((ext_vector_type(2)));
typedef short fir_i16x2 __attribute__((ext_vector_type(2)));

// a * b + c in each 16-bit half, mod 2^16 (v_pk_mad_u16)
__device__ __forceinline__ uint32_t pk_mad16(uint32_t a, uint32_t b, uint32_t c) {
    const fir_u16x2 r = __builtin_bit_cast(fir_u16x2, a) * __builtin_bit_cast(fir_u16x2, b) + __builtin_bit_cast(fir_u16x2, c);
    return __builtin_bit_cast(uint32_t, r);
}
__device__ __forceinline__ uint32_t pk_mul16(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(fir_u16x2, a) * __builtin_bit_cast(fir_u16x2, b));
}
// u8 stage of two packed sums: (V >> k) clamped to [0, 255] in each half (signed or unsigned V)
template <bool SIGNED>
__device__ __forceinline__ uint32_t pk_stage_u8(uint32_t v, uint32_t k2, uint32_t max2) {
    if constexpr (SIGNED) {
        fir_i16x2 a = __builtin_bit_cast(fir_i16x2, v) >> __builtin_bit_cast(fir_i16x2, k2);
        a = __builtin_elementwise_max(a, (fir_i16x2){0, 0});
        a = __builtin_elementwise_min(a, __builtin_bit_cast(fir_i16x2, max2));
        return __builtin_bit_cast(uint32_t, a);
    } else {
        fir_u16x2 a = __builtin_bit_cast(fir_u16x2, v) >> __builtin_bit_cast(fir_u16x2, k2);
        a = __builtin_elementwise_min(a, __builtin_bit_cast(fir_u16x2, max2));
        return __builtin_bit_cast(uint32_t, a);
    }
}

}  // namespace fir
