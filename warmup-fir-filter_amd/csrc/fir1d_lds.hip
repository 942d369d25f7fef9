// fir1d_lds.hip — the 1-D fixed-point FIR for long filters (10..64 taps), SURVEY §8 a1/a6.
//
// Arithmetic: fir_1d/model/python/fir_1d_fixed_ref.py:95-126 (reference root), as in the
// register kernel: a 32-bit wrap-around accumulator (exact mod 2^32, which is all wrap_acc
// needs for acc_bits <= 32), MACs on packed v_dot2_i32_i16 (int16 taps over int16 samples, or
// over u8 samples zero-extended to int16), wrap to acc_bits, overflow-free rounding, u8 or
// int32 stage.
//
// Beyond 9 taps the register kernel's one-neighbour DPP halo no longer reaches, and the
// generic int64 kernel is VALU-bound (953 us at 10 taps, 3.1 ms at 64 for 2^28 int16 samples,
// profiles/r02/long_taps.txt).  Here a workgroup stages an LDS sliding window of its 2048
// outputs plus the (LP-1)-sample halo as int16 (u8 widened on the way in), and every lane
// reads the LP + 7 samples behind its 8 outputs back as 16-byte LDS rows: the aligned sample
// pairs are window dwords, the odd ones one v_alignbit each (shared by every output that uses
// them), then LP/2 v_dot2 per output.  Filters are padded with zero taps to an even bucket
// length LP in {12, 16, 20, 24, 32, 40, 48, 64}, shifted so the centre sample stays where it was.
// Rows (images): a lane whose window crosses a row edge zeroes the samples of the other row
// before its MACs (a wave-uniform branch, taken by about one wave in eight at 4096-sample rows).
#include <string>

#include "fir_common.h"
#include "fir_launch.h"

namespace fir {

constexpr int kLdsMaxTaps = 64;
constexpr int kLdsVec = 8;                      // outputs per lane
constexpr int kLdsTile = kBlock * kLdsVec;      // outputs per workgroup
constexpr int kLdsPadL = 32;                    // LDS samples before the tile (>= HLE, 8-aligned)
constexpr int kLdsSpan = kLdsPadL + kLdsTile + 40;  // + right halo (<= 32) and read slack

template <int LP>
struct TapsLds {
    uint32_t pk[LP / 2];  // pair p = (h'[LP-1-2p], h'[LP-2-2p]) as two int16 halves
};

// window dword q -> the sample pair starting at window sample s (s even: dword s/2; odd:
// alignbit of dwords (s+1)/2 and (s-1)/2)
template <typename InT, int STAGE, int LP, bool ACC32>
__global__ __launch_bounds__(kBlock) void fir1d_lds_kernel(const InT* __restrict__ x,
                                                           typename OutTraits<STAGE>::T* __restrict__ y,
                                                           int64_t total, int64_t rowlen, TapsLds<LP> taps, int shl,
                                                           int frac) {
    constexpr int HLE = LP - 1 - LP / 2;  // samples left of an output (= LP/2 - 1)
    constexpr int HRE = LP / 2;
    constexpr int OFF = (kLdsPadL - HLE) % 8;            // window start inside its 16-byte LDS row
    constexpr int NS = OFF + kLdsVec + LP - 1;           // samples read per lane
    constexpr int NQ = (NS + 7) / 8;                     // 16-byte LDS rows per lane
    constexpr int ND = NQ * 4;                           // window dwords
    static_assert(HLE <= kLdsPadL && HRE + 8 <= 40, "halo exceeds the LDS padding");
    __shared__ __attribute__((aligned(16))) int16_t win[kLdsSpan];

    const int64_t t0 = (int64_t)blockIdx.x * kLdsTile;  // first output of this workgroup
    // ---- stage samples [t0 - kLdsPadL, t0 + kLdsTile + 40) as int16 (zero outside [0, total))
    {
        const int64_t g = t0 + (int64_t)threadIdx.x * kLdsVec;  // 8 samples per thread
        int16_t v[kLdsVec];
        if (g + kLdsVec <= total) {
            if constexpr (sizeof(InT) == 2) {
                typedef uint32_t u4 __attribute__((ext_vector_type(4)));
                const u4 q = *reinterpret_cast<const u4*>(x + g);
                *reinterpret_cast<u4*>(&win[kLdsPadL + threadIdx.x * kLdsVec]) = q;
            } else {
                typedef uint32_t u2 __attribute__((ext_vector_type(2)));
                const u2 q = *reinterpret_cast<const u2*>(x + g);
                typedef uint32_t u4 __attribute__((ext_vector_type(4)));
                const u4 w = {__builtin_amdgcn_perm(0u, q.x, 0x0C010C00u), __builtin_amdgcn_perm(0u, q.x, 0x0C030C02u),
                              __builtin_amdgcn_perm(0u, q.y, 0x0C010C00u), __builtin_amdgcn_perm(0u, q.y, 0x0C030C02u)};
                *reinterpret_cast<u4*>(&win[kLdsPadL + threadIdx.x * kLdsVec]) = w;
            }
        } else {
#pragma unroll
            for (int j = 0; j < kLdsVec; ++j) v[j] = g + j < total ? (int16_t)x[g + j] : (int16_t)0;
#pragma unroll
            for (int j = 0; j < kLdsVec; ++j) win[kLdsPadL + threadIdx.x * kLdsVec + j] = v[j];
        }
        // the halos: kLdsPadL samples before the tile, 40 after (threads 0..71, one sample each)
        if (threadIdx.x < kLdsPadL + 40) {
            const int i = threadIdx.x;
            const int li = i < kLdsPadL ? i : kLdsPadL + kLdsTile + (i - kLdsPadL);
            const int64_t gi = t0 - kLdsPadL + li;
            win[li] = gi >= 0 && gi < total ? (int16_t)x[gi] : (int16_t)0;
        }
    }
    __syncthreads();

    const int64_t o0 = t0 + (int64_t)threadIdx.x * kLdsVec;  // this lane's first output
    if (o0 >= total) return;
    // ---- the lane's window: samples [o0 - HLE - OFF, ...) as dwords
    uint32_t d[ND];
    {
        typedef uint32_t u4 __attribute__((ext_vector_type(4)));
        const u4* src = reinterpret_cast<const u4*>(&win[kLdsPadL + threadIdx.x * kLdsVec - HLE - OFF]);
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const u4 r = src[q];
            d[4 * q] = r.x;
            d[4 * q + 1] = r.y;
            d[4 * q + 2] = r.z;
            d[4 * q + 3] = r.w;
        }
    }
    if (rowlen > 0) {  // images: zero the samples of a neighbouring row (wave-divergent, rare)
        const int64_t col0 = o0 % rowlen;
        if (col0 < HLE || col0 + kLdsVec + HRE > rowlen) {
            const int64_t ws = o0 - HLE - OFF;  // global sample of window sample 0
            const int64_t rs = o0 - col0;       // this row's first sample (outputs stay in it)
            const int lo = (int)max((int64_t)-1, min(rs - ws, (int64_t)(2 * ND)));
            const int hi = (int)max((int64_t)-1, min(rs + rowlen - ws, (int64_t)(2 * ND)));
#pragma unroll
            for (int q = 0; q < ND; ++q) {
                const uint32_t m = ((2 * q >= lo && 2 * q < hi) ? 0x0000FFFFu : 0u) |
                                   ((2 * q + 1 >= lo && 2 * q + 1 < hi) ? 0xFFFF0000u : 0u);
                d[q] &= m;
            }
        }
    }
    // odd pairs: e[q] = (sample 2q+1, sample 2q+2)
    uint32_t e[ND - 1];
#pragma unroll
    for (int q = 0; q + 1 < ND; ++q) e[q] = __builtin_amdgcn_alignbit(d[q + 1], d[q], 16);
    int32_t qo[kLdsVec];
#pragma unroll
    for (int j = 0; j < kLdsVec; ++j) {
        // output j = sum_m h'[LP-1-m] * win[j + m], window sample index s = OFF + j + m
        uint32_t acc = 0;
#pragma unroll
        for (int p = 0; p < LP / 2; ++p) {
            const int s = OFF + j + 2 * p;  // compile-time after unrolling
            const uint32_t pr = (s % 2 == 0) ? d[s / 2] : e[(s - 1) / 2];
            acc = dot2_acc(pr, taps.pk[p], acc);
        }
        qo[j] = round_acc<ACC32>(acc, shl, frac);
    }
    using OutT = typename OutTraits<STAGE>::T;
    if constexpr (STAGE == FIR_OUT_I32) {
        // a whole wave's 512 int32 outputs go out as two 1 KiB rows through wave-private LDS
        // (lane-strided 32-byte stores cost the register kernel 6 %, profiles/r01)
        const int lane = threadIdx.x & (kWave - 1);
        const int64_t wo = o0 - lane * kLdsVec;  // the wave's first output
        if (wo + kWave * kLdsVec <= total) {     // wave-uniform
            typedef uint32_t u4 __attribute__((ext_vector_type(4)));
            __shared__ u4 sout[kBlock / kWave][kWave * kLdsVec / 4];
            u4* wb = sout[threadIdx.x >> 6];
            wb[2 * lane] = u4{(uint32_t)qo[0], (uint32_t)qo[1], (uint32_t)qo[2], (uint32_t)qo[3]};
            wb[2 * lane + 1] = u4{(uint32_t)qo[4], (uint32_t)qo[5], (uint32_t)qo[6], (uint32_t)qo[7]};
            __builtin_amdgcn_wave_barrier();  // one wave's LDS ops complete in order
            asm volatile("" ::: "memory");
            u4* dst = reinterpret_cast<u4*>(y + wo);
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                const u4 v = wb[r * kWave + lane];
                asm volatile("global_store_dwordx4 %0, %1, off nt\n\ts_nop 1" ::"v"(&dst[r * kWave + lane]), "v"(v)
                             : "memory");
            }
            return;
        }
    }
    if (o0 + kLdsVec <= total) {
        if constexpr (STAGE == FIR_OUT_I32) {
            typedef uint32_t u4 __attribute__((ext_vector_type(4)));
            u4* dst = reinterpret_cast<u4*>(y + o0);
            dst[0] = u4{(uint32_t)qo[0], (uint32_t)qo[1], (uint32_t)qo[2], (uint32_t)qo[3]};
            dst[1] = u4{(uint32_t)qo[4], (uint32_t)qo[5], (uint32_t)qo[6], (uint32_t)qo[7]};
        } else {
            typedef uint32_t u2 __attribute__((ext_vector_type(2)));
            uint32_t w[2];
#pragma unroll
            for (int i = 0; i < 2; ++i)
                w[i] = (uint32_t)stage_out32<STAGE>(qo[4 * i]) | ((uint32_t)stage_out32<STAGE>(qo[4 * i + 1]) << 8) |
                       ((uint32_t)stage_out32<STAGE>(qo[4 * i + 2]) << 16) |
                       ((uint32_t)stage_out32<STAGE>(qo[4 * i + 3]) << 24);
            *reinterpret_cast<u2*>(y + o0) = u2{w[0], w[1]};
        }
    } else {
#pragma unroll
        for (int j = 0; j < kLdsVec; ++j)
            if (o0 + j < total) y[o0 + j] = (OutT)stage_out32<STAGE>(qo[j]);
    }
}

template <typename InT, int STAGE, int LP>
static hipError_t launch_lds_lp(const void* x, void* y, int64_t total, int64_t rowlen, const int32_t* hq, int L,
                                int frac, int acc_bits, hipStream_t s) {
    // zero-padded taps h'[d + k] = h[k], d = LP/2 - L/2: the centre sample does not move
    int32_t hp[LP] = {};
    const int dsh = LP / 2 - L / 2;
    for (int k = 0; k < L; ++k) hp[dsh + k] = hq[k];
    TapsLds<LP> t;
    for (int p = 0; p < LP / 2; ++p)
        t.pk[p] = ((uint32_t)hp[LP - 1 - 2 * p] & 0xFFFFu) | ((uint32_t)hp[LP - 2 - 2 * p] << 16);
    const unsigned blocks = (unsigned)((total + kLdsTile - 1) / kLdsTile);
    using OutT = typename OutTraits<STAGE>::T;
    if (acc_bits == 32)
        hipLaunchKernelGGL((fir1d_lds_kernel<InT, STAGE, LP, true>), dim3(blocks), dim3(kBlock), 0, s, (const InT*)x,
                           (OutT*)y, total, rowlen, t, 0, frac);
    else
        hipLaunchKernelGGL((fir1d_lds_kernel<InT, STAGE, LP, false>), dim3(blocks), dim3(kBlock), 0, s, (const InT*)x,
                           (OutT*)y, total, rowlen, t, 32 - acc_bits, frac);
    return hipGetLastError();
}

template <typename InT, int STAGE>
static hipError_t launch_lds_t(const void* x, void* y, int64_t total, int64_t rowlen, const int32_t* hq, int L,
                               int frac, int acc_bits, hipStream_t s) {
    if (L <= 12) return launch_lds_lp<InT, STAGE, 12>(x, y, total, rowlen, hq, L, frac, acc_bits, s);
    if (L <= 16) return launch_lds_lp<InT, STAGE, 16>(x, y, total, rowlen, hq, L, frac, acc_bits, s);
    if (L <= 20) return launch_lds_lp<InT, STAGE, 20>(x, y, total, rowlen, hq, L, frac, acc_bits, s);
    if (L <= 24) return launch_lds_lp<InT, STAGE, 24>(x, y, total, rowlen, hq, L, frac, acc_bits, s);
    if (L <= 32) return launch_lds_lp<InT, STAGE, 32>(x, y, total, rowlen, hq, L, frac, acc_bits, s);
    if (L <= 40) return launch_lds_lp<InT, STAGE, 40>(x, y, total, rowlen, hq, L, frac, acc_bits, s);
    if (L <= 48) return launch_lds_lp<InT, STAGE, 48>(x, y, total, rowlen, hq, L, frac, acc_bits, s);
    return launch_lds_lp<InT, STAGE, 64>(x, y, total, rowlen, hq, L, frac, acc_bits, s);
}

bool lds_path_ok(const void* x, const void* y, int in_dtype, int64_t rows, int64_t rowlen, int64_t total, int ch,
                 const int32_t* hq, int L, int frac, int acc_bits) {
    bool taps16 = true;
    for (int k = 0; k < L; ++k) taps16 &= hq[k] >= -32768 && hq[k] <= 32767;
    return L >= 2 && L <= kLdsMaxTaps && ch == 1 && taps16 && acc_bits <= 32 && frac <= 31 &&
           (rows == 1 || rowlen % kLdsVec == 0) &&  // a lane's 8 outputs never straddle two rows
           (uintptr_t)x % (in_dtype == FIR_IN_U8 ? 8 : 16) == 0 && (uintptr_t)y % 16 == 0 && total < ((int64_t)1 << 40);
}

hipError_t launch_fir1d_lds(const void* x, int in_dtype, int64_t rows, int64_t rowlen, int64_t total,
                            const int32_t* hq, int L, int frac, int acc_bits, int stage, void* y, hipStream_t s) {
    const int64_t rl = rows > 1 ? rowlen : 0;
    if (in_dtype == FIR_IN_U8)
        return stage == FIR_OUT_U8_SAT ? launch_lds_t<uint8_t, FIR_OUT_U8_SAT>(x, y, total, rl, hq, L, frac, acc_bits, s)
                                       : launch_lds_t<uint8_t, FIR_OUT_I32>(x, y, total, rl, hq, L, frac, acc_bits, s);
    return stage == FIR_OUT_U8_SAT ? launch_lds_t<int16_t, FIR_OUT_U8_SAT>(x, y, total, rl, hq, L, frac, acc_bits, s)
                                   : launch_lds_t<int16_t, FIR_OUT_I32>(x, y, total, rl, hq, L, frac, acc_bits, s);
}

}  // namespace fir
