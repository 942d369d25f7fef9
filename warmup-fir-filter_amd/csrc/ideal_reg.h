// ideal_reg.h — register/DPP f64 "ideal" FIR kernel, shared by the
// library (ideal.hip) and the A/B microbenchmark (tools/microbench/ideal_micro.hip).
//
// A lane owns NV consecutive dwords (4*NV u8 samples); the (L-1)-sample halo is one dword
// from each neighbouring lane by DPP wave shifts (lanes 0 / 63 load it); every sample is
// converted to f64 once and shared by the L outputs that use it; 16-byte f64 stores (8 of
// the 9 bytes per sample of HBM traffic).  Row edges: rows that are a whole number of
// vectors zero the halo dword that lies in the neighbouring row (a +-0.0 product leaves the
// running sum unchanged, exactly as skipping the term does); other widths mask per output.
// Bit-exactness needs the reference's rounding order (fir_1d_ref.py:57-63): every product
// and sum rounded on its own (__dmul_rn / __dadd_rn, -ffp-contract=off), taps in k order.
#pragma once

#include "fir_common.h"

namespace fir {

template <int L>
struct TapsIdeal {
    double h[L];
};

// NV dwords of u8 samples starting at dword index di (zero fill outside [0, total)).
template <int NV, bool NT = false>
__device__ __forceinline__ void load_u8_dwords(const uint8_t* __restrict__ x, int64_t di, int64_t total,
                                               uint32_t (&d)[NV]) {
    const int64_t b0 = di * 4;
    if (di >= 0 && b0 + 4 * NV <= total) {
        typedef uint32_t vN __attribute__((ext_vector_type(NV)));
        if constexpr (NV == 1) {
            d[0] = *reinterpret_cast<const uint32_t*>(x + b0);
        } else {
            const vN* p = reinterpret_cast<const vN*>(x + b0);
            const vN q = NT ? __builtin_nontemporal_load(p) : *p;
#pragma unroll
            for (int i = 0; i < NV; ++i) d[i] = q[i];
        }
    } else {
#pragma unroll
        for (int i = 0; i < NV; ++i) d[i] = 0;
        if (di >= 0 && b0 < total) {
            const int n = (int)min((int64_t)(4 * NV), total - b0);
            for (int j = 0; j < n; ++j) d[j / 4] |= (uint32_t)x[b0 + j] << (8 * (j % 4));
        }
    }
}

// Sum in tap order, every product and sum rounded on its own (fir_1d_ref.py:57-63).
template <int L, int NS, int VEC>
__device__ __forceinline__ void ideal_outputs(const double (&s)[NS], const TapsIdeal<L>& t, double (&q)[VEC]) {
    constexpr int C = L / 2, HLE = L - 1 - C;
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
        double acc = 0.0;
#pragma unroll
        for (int k = 0; k < L; ++k) acc = __dadd_rn(acc, __dmul_rn(t.h[k], s[HLE + j + C - k]));
        q[j] = acc;
    }
}

// COAL: a full wave stages its outputs in LDS and writes them back as whole contiguous
// 1 KiB rows per store instruction (instead of 16 B per lane at a 16*NV-byte stride).
template <int L, int NV, bool COAL = false, bool NTL = false, bool NTS = false>
__global__ __launch_bounds__(kBlock) void fir1d_ideal_reg_kernel(const uint8_t* __restrict__ x,
                                                                 double* __restrict__ y, int64_t total,
                                                                 uint32_t rowlen32, int multi_row, int aligned,
                                                                 TapsIdeal<L> taps) {
    constexpr int VEC = 4 * NV;
    constexpr int C = L / 2, HLE = L - 1 - C, HRE = C;
    static_assert(HLE <= 4 && HRE <= 4, "halo must fit in one dword");
    constexpr int NS = HLE + VEC + HRE;
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t v = (int64_t)blockIdx.x * kBlock + threadIdx.x;  // this lane's vector
    const int64_t wave_v0 = v - lane;
    uint32_t own[NV];
    load_u8_dwords<NV, NTL>(x, v * NV, total, own);
    uint32_t seam = 0;
    if (lane == 0) {
        load_u8_dwords<1>(x, wave_v0 * NV - 1, total, *reinterpret_cast<uint32_t(*)[1]>(&seam));
    } else if (lane == kWave - 1) {
        load_u8_dwords<1>(x, (wave_v0 + kWave) * NV, total, *reinterpret_cast<uint32_t(*)[1]>(&seam));
    }
    uint32_t Wd[NV + 2];
    Wd[0] = from_prev_lane(seam, own[NV - 1]);
#pragma unroll
    for (int i = 0; i < NV; ++i) Wd[1 + i] = own[i];
    Wd[NV + 1] = from_next_lane(seam, own[0]);
    const int64_t g0 = v * VEC;
    const int64_t rowlen = multi_row ? (int64_t)rowlen32 : total;
    const int64_t col0 = multi_row ? (int64_t)((uint32_t)g0 % rowlen32) : g0;
    bool interior = col0 >= HLE && col0 + VEC + HRE <= rowlen;
    if (aligned) {  // whole vectors per row: only the halo dwords can lie in another row
        if (multi_row) {
            Wd[0] = col0 == 0 ? 0u : Wd[0];
            Wd[NV + 1] = col0 + VEC == rowlen ? 0u : Wd[NV + 1];
        }
        interior = true;
    }
    double s[NS];
#pragma unroll
    for (int i = 0; i < NS; ++i) {
        const int b = 4 - HLE + i;  // byte index in the window
        s[i] = (double)((Wd[b / 4] >> (8 * (b % 4))) & 0xFFu);
    }
    double q[VEC];
    if (__builtin_expect(interior, 1)) {
        ideal_outputs<L, NS, VEC>(s, taps, q);
    } else {
        // the vector's row spans window offsets [-a, b), the next row [b, b + r)
        constexpr int64_t kFar = 1 << 24;
        const int a = (int)min(col0, kFar), bb = (int)min(rowlen - col0, kFar), r = (int)min(rowlen, kFar);
        double s1[NS], s2[NS], q1[VEC], q2[VEC];
#pragma unroll
        for (int i = 0; i < NS; ++i) {
            const int o = i - HLE;
            s1[i] = (o >= -a && o < bb) ? s[i] : 0.0;
            s2[i] = (o >= bb && o < bb + r) ? s[i] : 0.0;
        }
        ideal_outputs<L, NS, VEC>(s1, taps, q1);
        ideal_outputs<L, NS, VEC>(s2, taps, q2);
#pragma unroll
        for (int j = 0; j < VEC; ++j) q[j] = j < bb ? q1[j] : q2[j];
    }
    typedef double d2 __attribute__((ext_vector_type(2)));
    if constexpr (COAL) {
        if ((wave_v0 + kWave) * VEC <= total) {  // wave-uniform
            __shared__ d2 sbuf[kBlock * VEC / 2];
            d2* wb = sbuf + (threadIdx.x - lane) * (VEC / 2);
#pragma unroll
            for (int i = 0; i < VEC / 2; ++i) wb[lane * (VEC / 2) + i] = d2{q[2 * i], q[2 * i + 1]};
            __builtin_amdgcn_wave_barrier();  // LDS ops of one wave complete in order
            asm volatile("" ::: "memory");
            d2* yw = reinterpret_cast<d2*>(y + wave_v0 * VEC);
#pragma unroll
            for (int i = 0; i < VEC / 2; ++i) {
                if constexpr (NTS) {  // inline nt store: 352.8 -> 344.2 us vs the builtin (micro_ideal_asm.txt);
                    // the s_nop covers the store-data hazard the compiler cannot see in inline asm
                    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
                    asm volatile("global_store_dwordx4 %0, %1, off nt\n\ts_nop 1" ::"v"(&yw[i * kWave + lane]),
                                 "v"(__builtin_bit_cast(u4, wb[i * kWave + lane])) : "memory");
                } else {
                    yw[i * kWave + lane] = wb[i * kWave + lane];
                }
            }
            return;
        }
    }
    if (g0 >= total) return;
    if (g0 + VEC <= total) {
#pragma unroll
        for (int i = 0; i < VEC / 2; ++i) reinterpret_cast<d2*>(y + g0)[i] = d2{q[2 * i], q[2 * i + 1]};
    } else {
#pragma unroll
        for (int j = 0; j < VEC; ++j)
            if (g0 + j < total) y[g0 + j] = q[j];
    }
}

}  // namespace fir
