// fir1d.hip — gfx950 kernels for the row-wise 1-D fixed-point FIR.
//
// Arithmetic restated from fir_1d/model/python/fir_1d_fixed_ref.py:95-126 (reference root):
//   acc = sum_k hq[k] * x[n - k + L/2] (zero outside the row), wrapped to acc_bits,
//   q = (acc + 2^(f-1)) >> f, then saturated to u8 or kept as int32.
//
// Two kernels:
//  * fir1d_reg_kernel (fir1d_reg.h; launchers in fir1d_reg_impl.h, instantiated per
//    configuration by fir1d_reg_inst.hip) — the hot path.  A lane owns one 16-byte vector
//    of samples (16 u8 or 8 int16); a wave owns kRegU chunks of 64 vectors (1 KiB per load
//    instruction).  The (L-1)-sample halo comes from the neighbouring lanes' registers by
//    DPP wave shifts, so every HBM byte is loaded once; only lanes 0 and 63 issue one extra
//    16-byte load for the adjacent tile's edge vector (an L2 hit).  MACs on packed
//    v_dot2_i32_i16 (int16 samples, or u8 byte pairs when no accumulator can wrap) or
//    v_mad_i32_i24, overflow-free rounding, int32 outputs stored through LDS as whole
//    1 KiB rows.  Rows that are a whole number of vectors zero the out-of-row halo and
//    stay on the unmasked path; other widths mask the vectors that straddle a row edge.
//  * fir1d_generic_kernel — every other configuration (any tap count up to FIR_MAX_TAPS,
//    any acc_bits / frac_bits, unaligned buffers, narrow rows, halo segments): a
//    workgroup stages an LDS sliding-window tile of 1024 outputs + (L-1)*channels halo
//    samples, then every thread forms its outputs from LDS with an exact int64 sum.
#include <algorithm>
#include <string>

#include "fir1d_reg_launch.h"
#include "fir_common.h"
#include "fir_launch.h"

// Long filters (beyond the register kernel's 9 taps) take the int8 matrix-core kernel
// (fir1d_mfma.hip) when its layout conditions hold, else the v_dot2 LDS kernel.  Measured at
// 2^28 samples (profiles/r02/long_taps_*.txt): u8 samples 90-97 us on MFMA at every length vs
// 190-425 us on LDS; int16 -> u8 152-163 vs 192-416; int16 -> int32 MFMA 289-291 us flat,
// LDS 249-275 up to 31 taps and 298-405 from 40: int16 -> int32 below FIR_MFMA_MIN_TAPS_I32
// stays on LDS.  Both overridable for A/B builds (65 keeps everything on LDS).
#ifndef FIR_MFMA_MIN_TAPS
#define FIR_MFMA_MIN_TAPS 10
#endif
#ifndef FIR_MFMA_MIN_TAPS_I32
#define FIR_MFMA_MIN_TAPS_I32 40
#endif

namespace fir {

// ---------------------------------------------------------------------------------------
// Generic LDS sliding-window kernel.
constexpr int kGenTile = 1024;
constexpr int kGenMaxHalo = 1024;  // (L-1) * channels

struct TapsG {
    int32_t h[FIR_MAX_TAPS];
};

template <typename InT, int STAGE>
__global__ __launch_bounds__(kBlock) void fir1d_generic_kernel(const InT* __restrict__ x,
                                                               typename OutTraits<STAGE>::T* __restrict__ y,
                                                               int64_t start, int64_t end, int64_t total,
                                                               int64_t rowlen, int multi_row, int ch,
                                                               const InT* __restrict__ halo_l,
                                                               const InT* __restrict__ halo_r, TapsG taps, int L,
                                                               int frac, int acc_bits) {
    __shared__ int32_t s_taps[FIR_MAX_TAPS];
    __shared__ int32_t s_x[kGenTile + kGenMaxHalo];
    const int c = L / 2;
    const int HLE = (L - 1 - c) * ch;
    const int HRE = c * ch;
    const int64_t t0 = start + (int64_t)blockIdx.x * kGenTile;
    const int span = kGenTile + HLE + HRE;

    for (int k = threadIdx.x; k < L; k += kBlock) s_taps[k] = taps.h[k];
    for (int i = threadIdx.x; i < span; i += kBlock) {
        const int64_t gi = t0 - HLE + i;
        int32_t val = 0;
        if (gi >= 0 && gi < total) {
            val = (int32_t)x[gi];
        } else if (gi < 0) {
            if (halo_l && gi >= -HLE) val = (int32_t)halo_l[HLE + gi];
        } else if (halo_r && gi < total + HRE) {
            val = (int32_t)halo_r[gi - total];
        }
        s_x[i] = val;
    }
    __syncthreads();

    for (int i = threadIdx.x; i < kGenTile; i += kBlock) {
        const int64_t gi = t0 + i;
        if (gi >= end) break;
        const int64_t col = multi_row ? gi % rowlen : 0;
        int64_t acc = 0;
        for (int k = 0; k < L; ++k) {
            const int d = (c - k) * ch;
            int32_t xv = s_x[HLE + i + d];
            if (multi_row && (col + d < 0 || col + d >= rowlen)) xv = 0;
            acc += (int64_t)s_taps[k] * xv;
        }
        y[gi] = stage_out<STAGE>(round64(acc, frac, acc_bits));
    }
}

// Both edges of a single-row segment in one launch (multi-GPU step): output j < hle is the
// left edge, j >= hle maps to the right edge total - hre + (j - hle).  Samples left of the
// segment come from halo_l, right of it from halo_r (zeros when NULL).  Exact int64 sums.
template <typename InT, int STAGE>
__global__ __launch_bounds__(kBlock) void fir1d_edges_kernel(const InT* __restrict__ x,
                                                             typename OutTraits<STAGE>::T* __restrict__ y,
                                                             int64_t total, int ch, const InT* __restrict__ halo_l,
                                                             const InT* __restrict__ halo_r, TapsG taps, int L,
                                                             int hle, int hre, int frac, int acc_bits) {
    const int c = L / 2;
    for (int j = threadIdx.x; j < hle + hre; j += kBlock) {
        const int64_t gi = j < hle ? j : total - hre + (j - hle);
        int64_t acc = 0;
        for (int k = 0; k < L; ++k) {
            const int64_t si = gi + (int64_t)(c - k) * ch;
            int32_t v = 0;
            if (si >= 0 && si < total) {
                v = (int32_t)x[si];
            } else if (si < 0) {
                if (halo_l) v = (int32_t)halo_l[hle + si];
            } else if (halo_r) {
                v = (int32_t)halo_r[si - total];
            }
            acc += (int64_t)taps.h[k] * v;
        }
        y[gi] = stage_out<STAGE>(round64(acc, frac, acc_bits));
    }
}

// ---------------------------------------------------------------------------------------
// Host-side launchers.

template <typename InT, int STAGE>
static hipError_t launch_generic(const void* x, void* y, int64_t start, int64_t end, int64_t total,
                                 int64_t rowlen, bool multi_row, int ch, const void* hl, const void* hr,
                                 const int32_t* hq, int L, int frac, int acc_bits, hipStream_t stream) {
    using OutT = typename OutTraits<STAGE>::T;
    if (end <= start) return hipSuccess;
    TapsG t;
    for (int k = 0; k < L; ++k) t.h[k] = hq[k];
    for (int k = L; k < FIR_MAX_TAPS; ++k) t.h[k] = 0;
    const int64_t blocks = (end - start + kGenTile - 1) / kGenTile;
    hipLaunchKernelGGL((fir1d_generic_kernel<InT, STAGE>), dim3((unsigned)blocks), dim3(kBlock), 0, stream,
                       (const InT*)x, (OutT*)y, start, end, total, rowlen, multi_row ? 1 : 0, ch, (const InT*)hl,
                       (const InT*)hr, t, L, frac, acc_bits);
    return hipGetLastError();
}

static hipError_t dispatch_generic(int in_dtype, int stage, const void* x, void* y, int64_t start, int64_t end,
                                   int64_t total, int64_t rowlen, bool multi_row, int ch, const void* hl,
                                   const void* hr, const int32_t* hq, int L, int frac, int acc_bits,
                                   hipStream_t s) {
    if (in_dtype == FIR_IN_U8) {
        return stage == FIR_OUT_U8_SAT
                   ? launch_generic<uint8_t, FIR_OUT_U8_SAT>(x, y, start, end, total, rowlen, multi_row, ch, hl,
                                                             hr, hq, L, frac, acc_bits, s)
                   : launch_generic<uint8_t, FIR_OUT_I32>(x, y, start, end, total, rowlen, multi_row, ch, hl, hr,
                                                          hq, L, frac, acc_bits, s);
    }
    return stage == FIR_OUT_U8_SAT
               ? launch_generic<int16_t, FIR_OUT_U8_SAT>(x, y, start, end, total, rowlen, multi_row, ch, hl, hr,
                                                         hq, L, frac, acc_bits, s)
               : launch_generic<int16_t, FIR_OUT_I32>(x, y, start, end, total, rowlen, multi_row, ch, hl, hr, hq,
                                                      L, frac, acc_bits, s);
}

template <typename InT, int STAGE>
static hipError_t launch_edges(const void* x, void* y, int64_t total, int ch, const void* hl, const void* hr,
                               const TapsG& t, int L, int64_t hle, int64_t hre, int frac, int acc_bits,
                               hipStream_t stream) {
    hipLaunchKernelGGL((fir1d_edges_kernel<InT, STAGE>), dim3(1), dim3(kBlock), 0, stream, (const InT*)x,
                       (typename OutTraits<STAGE>::T*)y, total, ch, (const InT*)hl, (const InT*)hr, t, L, (int)hle,
                       (int)hre, frac, acc_bits);
    return hipGetLastError();
}

static int check_common(int in_dtype, int64_t rows, int64_t width, int ch, const int32_t* hq, int L, int frac,
                        int acc_bits, int stage, std::string* err) {
    if (in_dtype != FIR_IN_U8 && in_dtype != FIR_IN_I16) return *err = "in_dtype must be FIR_IN_U8 or FIR_IN_I16", FIR_EINVAL;
    if (stage != FIR_OUT_U8_SAT && stage != FIR_OUT_I32) return *err = "out_stage must be FIR_OUT_U8_SAT or FIR_OUT_I32", FIR_EINVAL;
    if (rows < 0 || width < 0) return *err = "rows and width must be >= 0", FIR_EINVAL;
    if (ch < 1) return *err = "channels must be >= 1", FIR_EINVAL;
    if (!hq) return *err = "hq must not be NULL", FIR_EINVAL;
    if (L < 1 || L > FIR_MAX_TAPS) return *err = "taps must be in [1, " + std::to_string(FIR_MAX_TAPS) + "]", FIR_EINVAL;
    if ((int64_t)(L - 1) * ch > kGenMaxHalo) return *err = "(taps-1)*channels exceeds 1024", FIR_EINVAL;
    if (frac < 1 || acc_bits < 1) return *err = "frac_bits and acc_bits must be >= 1", FIR_EINVAL;
    return FIR_OK;
}

// Conditions for the register/DPP kernel (otherwise the generic LDS kernel runs).
static bool reg_path_ok(const void* x, const void* y, int in_dtype, int64_t rows, int64_t rowlen, int64_t total,
                        int ch, const int32_t* hq, int nh, int L, int frac, int acc_bits) {
    const int vec = in_dtype == FIR_IN_U8 ? 16 : 8;
    bool taps24 = true;
    for (int k = 0; k < nh; ++k) taps24 &= (hq[k] >= -(1 << 23) && hq[k] < (1 << 23));
    return L <= 9 && (ch == 1 || (ch == 2 && in_dtype == FIR_IN_I16)) && acc_bits <= 32 && frac <= 31 && taps24 &&
           ((uintptr_t)x % 16 == 0) && ((uintptr_t)y % 16 == 0) &&
           (rows == 1 || (rowlen >= vec + (L - 1) * ch && total < ((int64_t)1 << 32)));
}

int launch_fir1d_rows(const void* x, int in_dtype, int64_t rows, int64_t width, int ch, const int32_t* hq, int L,
                      int frac, int acc_bits, int stage, void* y, hipStream_t stream, std::string* err) {
    int rc = check_common(in_dtype, rows, width, ch, hq, L, frac, acc_bits, stage, err);
    if (rc) return rc;
    const int64_t rowlen = width * ch;
    const int64_t total = rows * rowlen;
    if (total == 0) return FIR_OK;
    if (!x || !y) return *err = "x and y must not be NULL", FIR_EINVAL;
    hipError_t e;
    if (reg_path_ok(x, y, in_dtype, rows, rowlen, total, ch, hq, L, L, frac, acc_bits)) {
        if (in_dtype == FIR_IN_U8) {
            e = stage == FIR_OUT_U8_SAT
                    ? launch_reg_taps<uint8_t, FIR_OUT_U8_SAT, 1, 1>(L, x, y, rows, total, rowlen, hq, frac, acc_bits, stream)
                    : launch_reg_taps<uint8_t, FIR_OUT_I32, 1, 1>(L, x, y, rows, total, rowlen, hq, frac, acc_bits, stream);
        } else if (ch == 1) {
            e = stage == FIR_OUT_U8_SAT
                    ? launch_reg_taps<int16_t, FIR_OUT_U8_SAT, 1, 1>(L, x, y, rows, total, rowlen, hq, frac, acc_bits, stream)
                    : launch_reg_taps<int16_t, FIR_OUT_I32, 1, 1>(L, x, y, rows, total, rowlen, hq, frac, acc_bits, stream);
        } else {
            e = stage == FIR_OUT_U8_SAT
                    ? launch_reg_taps<int16_t, FIR_OUT_U8_SAT, 2, 1>(L, x, y, rows, total, rowlen, hq, frac, acc_bits, stream)
                    : launch_reg_taps<int16_t, FIR_OUT_I32, 2, 1>(L, x, y, rows, total, rowlen, hq, frac, acc_bits, stream);
        }
    } else if (L >= (in_dtype == FIR_IN_I16 && stage == FIR_OUT_I32 ? FIR_MFMA_MIN_TAPS_I32 : FIR_MFMA_MIN_TAPS) &&
               mfma_path_ok(x, y, in_dtype, rows, rowlen, total, ch, hq, L, frac, acc_bits)) {
        e = launch_fir1d_mfma(x, in_dtype, rows, rowlen, total, hq, L, frac, acc_bits, stage, y, stream);
    } else if (lds_path_ok(x, y, in_dtype, rows, rowlen, total, ch, hq, L, frac, acc_bits)) {
        e = launch_fir1d_lds(x, in_dtype, rows, rowlen, total, hq, L, frac, acc_bits, stage, y, stream);
    } else {
        e = dispatch_generic(in_dtype, stage, x, y, 0, total, total, rowlen, rows > 1, ch, nullptr, nullptr, hq, L,
                             frac, acc_bits, stream);
    }
    if (e != hipSuccess) return *err = std::string("fir1d launch failed: ") + hipGetErrorString(e), FIR_EHIP;
    return FIR_OK;
}

// u8 images: up to 4 filters per launch share one read of x.
template <int STAGE>
static hipError_t launch_multi_u8(int F, int L, const void* x, void* y, int64_t rows, int64_t total, int64_t rowlen,
                                  const int32_t* hq, int frac, int acc_bits, hipStream_t s) {
    switch (F) {
        case 1: return launch_reg_taps<uint8_t, STAGE, 1, 1>(L, x, y, rows, total, rowlen, hq, frac, acc_bits, s);
        case 2: return launch_reg_taps<uint8_t, STAGE, 1, 2>(L, x, y, rows, total, rowlen, hq, frac, acc_bits, s);
        case 3: return launch_reg_taps<uint8_t, STAGE, 1, 3>(L, x, y, rows, total, rowlen, hq, frac, acc_bits, s);
        case 4: return launch_reg_taps<uint8_t, STAGE, 1, 4>(L, x, y, rows, total, rowlen, hq, frac, acc_bits, s);
        default: return hipErrorInvalidValue;
    }
}

int launch_fir1d_rows_multi(const void* x, int in_dtype, int64_t rows, int64_t width, int ch, const int32_t* hq,
                            int L, int F, int frac, int acc_bits, int stage, void* y, hipStream_t stream,
                            std::string* err) {
    if (F < 1) return *err = "filters must be >= 1", FIR_EINVAL;
    int rc = check_common(in_dtype, rows, width, ch, hq, L, frac, acc_bits, stage, err);
    if (rc) return rc;
    const int64_t rowlen = width * ch;
    const int64_t total = rows * rowlen;
    if (total == 0) return FIR_OK;
    if (!x || !y) return *err = "x and y must not be NULL", FIR_EINVAL;
    const size_t osz = stage == FIR_OUT_I32 ? 4 : 1;
    const bool fused = in_dtype == FIR_IN_U8 && ch == 1 && (total * (int64_t)osz) % 16 == 0 &&
                       reg_path_ok(x, y, in_dtype, rows, rowlen, total, ch, hq, F * L, L, frac, acc_bits);
    for (int f0 = 0; f0 < F;) {
        const int nf = fused ? (F - f0 < 4 ? F - f0 : 4) : 1;
        void* yf = (char*)y + (size_t)f0 * (size_t)total * osz;
        const int32_t* hf = hq + (size_t)f0 * L;
        if (fused) {
            const hipError_t e =
                stage == FIR_OUT_U8_SAT
                    ? launch_multi_u8<FIR_OUT_U8_SAT>(nf, L, x, yf, rows, total, rowlen, hf, frac, acc_bits, stream)
                    : launch_multi_u8<FIR_OUT_I32>(nf, L, x, yf, rows, total, rowlen, hf, frac, acc_bits, stream);
            if (e != hipSuccess) return *err = std::string("fir1d multi launch failed: ") + hipGetErrorString(e), FIR_EHIP;
        } else {
            rc = launch_fir1d_rows(x, in_dtype, rows, width, ch, hf, L, frac, acc_bits, stage, yf, stream, err);
            if (rc) return rc;
        }
        f0 += nf;
    }
    return FIR_OK;
}

// One shard of a longer single-row signal with its halos (fir1d_fixed_segment_dev): ONE launch
// of the register kernel with the halos standing in for the zero padding when the segment is
// a whole number of wave tiles (512 int16 / 4096 u8 samples), else the bulk pass then the edge
// kernel.
int launch_fir1d_segment(const void* x, int in_dtype, int64_t n, int ch, const int32_t* hq, int L, int frac,
                         int acc_bits, int stage, const void* hl, const void* hr, void* y, hipStream_t stream,
                         std::string* err) {
    int rc = check_common(in_dtype, 1, n, ch, hq, L, frac, acc_bits, stage, err);
    if (rc) return rc;
    const int64_t total = n * ch;
    if (total == 0) return FIR_OK;
    if (!x || !y) return *err = "x and y must not be NULL", FIR_EINVAL;
    if (total % reg_tile_samples(in_dtype == FIR_IN_U8) == 0 &&
        reg_path_ok(x, y, in_dtype, 1, total, total, ch, hq, L, L, frac, acc_bits)) {
        hipError_t e;
        if (in_dtype == FIR_IN_U8)
            e = stage == FIR_OUT_U8_SAT
                    ? launch_reg_taps<uint8_t, FIR_OUT_U8_SAT, 1, 1>(L, x, y, 1, total, total, hq, frac, acc_bits, stream, hl, hr)
                    : launch_reg_taps<uint8_t, FIR_OUT_I32, 1, 1>(L, x, y, 1, total, total, hq, frac, acc_bits, stream, hl, hr);
        else if (ch == 1)
            e = stage == FIR_OUT_U8_SAT
                    ? launch_reg_taps<int16_t, FIR_OUT_U8_SAT, 1, 1>(L, x, y, 1, total, total, hq, frac, acc_bits, stream, hl, hr)
                    : launch_reg_taps<int16_t, FIR_OUT_I32, 1, 1>(L, x, y, 1, total, total, hq, frac, acc_bits, stream, hl, hr);
        else
            e = stage == FIR_OUT_U8_SAT
                    ? launch_reg_taps<int16_t, FIR_OUT_U8_SAT, 2, 1>(L, x, y, 1, total, total, hq, frac, acc_bits, stream, hl, hr)
                    : launch_reg_taps<int16_t, FIR_OUT_I32, 2, 1>(L, x, y, 1, total, total, hq, frac, acc_bits, stream, hl, hr);
        if (e != hipSuccess) return *err = std::string("fir1d segment launch failed: ") + hipGetErrorString(e), FIR_EHIP;
        return FIR_OK;
    }
    rc = launch_fir1d_rows(x, in_dtype, 1, n, ch, hq, L, frac, acc_bits, stage, y, stream, err);
    if (rc) return rc;
    return launch_fir1d_edges(x, in_dtype, n, ch, hq, L, frac, acc_bits, stage, hl, hr, y, stream, err);
}

int launch_fir1d_edges(const void* x, int in_dtype, int64_t n, int ch, const int32_t* hq, int L, int frac,
                       int acc_bits, int stage, const void* hl, const void* hr, void* y, hipStream_t stream,
                       std::string* err) {
    int rc = check_common(in_dtype, 1, n, ch, hq, L, frac, acc_bits, stage, err);
    if (rc) return rc;
    const int64_t total = n * ch;
    if (total == 0) return FIR_OK;
    if (!x || !y) return *err = "x and y must not be NULL", FIR_EINVAL;
    const int c = L / 2;
    const int64_t hle = (int64_t)(L - 1 - c) * ch, hre = (int64_t)c * ch;
    hipError_t e = hipSuccess;
    if (total <= hle + hre) {  // the whole segment is edge
        e = dispatch_generic(in_dtype, stage, x, y, 0, total, total, total, false, ch, hl, hr, hq, L, frac, acc_bits,
                             stream);
    } else if (hle + hre > 0) {  // both edges, one launch
        TapsG t;
        for (int k = 0; k < FIR_MAX_TAPS; ++k) t.h[k] = k < L ? hq[k] : 0;
        if (in_dtype == FIR_IN_U8)
            e = stage == FIR_OUT_U8_SAT
                    ? launch_edges<uint8_t, FIR_OUT_U8_SAT>(x, y, total, ch, hl, hr, t, L, hle, hre, frac, acc_bits, stream)
                    : launch_edges<uint8_t, FIR_OUT_I32>(x, y, total, ch, hl, hr, t, L, hle, hre, frac, acc_bits, stream);
        else
            e = stage == FIR_OUT_U8_SAT
                    ? launch_edges<int16_t, FIR_OUT_U8_SAT>(x, y, total, ch, hl, hr, t, L, hle, hre, frac, acc_bits, stream)
                    : launch_edges<int16_t, FIR_OUT_I32>(x, y, total, ch, hl, hr, t, L, hle, hre, frac, acc_bits, stream);
    }
    if (e != hipSuccess) return *err = std::string("fir1d edge launch failed: ") + hipGetErrorString(e), FIR_EHIP;
    return FIR_OK;
}

}  // namespace fir
