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

// 64-bit generic form (any acc_bits >= 1, any frac_bits >= 1); |acc| < 2^52.
__device__ __forceinline__ int64_t round64(int64_t acc, int frac, int acc_bits) {
    if (acc_bits < 64) {
        const int s = 64 - acc_bits;
        acc = (int64_t)((uint64_t)acc << s) >> s;
    }
    if (frac > 62) return 0;
    return (acc + ((int64_t)1 << (frac - 1))) >> frac;
}

template <int STAGE>
__device__ __forceinline__ typename OutTraits<STAGE>::T stage_out(int64_t q) {
    if constexpr (STAGE == FIR_OUT_U8_SAT) {
        return (uint8_t)(q < 0 ? 0 : (q > 255 ? 255 : q));
    } else {
        return (int32_t)q;
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

}  // namespace fir
