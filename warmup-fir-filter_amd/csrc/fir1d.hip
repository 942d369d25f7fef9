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
//    any channel count, any acc_bits / frac_bits, unaligned buffers, narrow rows, halo
//    segments): a workgroup owns 1024 outputs and walks the taps (read from HBM) in chunks,
//    staging each chunk's taps and window in LDS; exact 64-bit sums (128-bit when a no-wrap
//    call's sum could reach 2^63).
#include <algorithm>
#include <string>
#include <type_traits>
#include <vector>

#include "fir1d_reg_launch.h"
#include "fir_common.h"
#include "fir_launch.h"

// Long filters (beyond the register kernel's 9 taps) take the int8 matrix-core kernel
// (fir1d_mfma.hip) when its layout conditions hold, else the v_dot2 LDS kernel.  Measured at
// 2^28 samples (profiles/r02/long_taps_*.txt): u8 samples 90-97 us on MFMA at every length vs
// 190-425 us on LDS; int16 -> u8 152-163 vs 192-416; int16 -> int32 MFMA 289-291 us flat,
// LDS 249-275 up to 31 taps and 298-405 from 40: int16 -> int32 below kMfmaMinTapsI32 stays on LDS.

namespace fir {

constexpr int kMfmaMinTaps = 10, kMfmaMinTapsI32 = 40;

// ---------------------------------------------------------------------------------------
// Generic LDS sliding-window kernel: any tap count, any channel count.  A workgroup owns
// kGenTile consecutive outputs; the taps (device memory) are taken kc at a time: each chunk
// stages its kc taps and the kGenTile + (kc-1)*ch samples they touch in LDS, and every thread
// adds the chunk's products to its outputs' sums (uint64: exact mod 2^64, which is all the
// wrap to acc_bits <= 64 needs, and the exact value while |sum| < 2^63, host-checked).
constexpr int kGenTile = 1024;
constexpr int kGenWin = 4096;       // LDS window samples
constexpr int kGenTapChunk = 1024;  // taps per LDS chunk
constexpr int kGenPer = kGenTile / kBlock;

// taps per chunk for `ch` interleaved channels: the window kGenTile + (kc-1)*ch fits kGenWin
static int gen_tap_chunk(int L, int64_t ch) {
    const int64_t kc = (kGenWin - kGenTile) / ch + 1;
    return (int)std::min<int64_t>(std::min<int64_t>(kc, kGenTapChunk), L);
}

// sample gi of a segment [0, total) with optional halos before / after it (zeros otherwise)
template <typename InT>
__device__ __forceinline__ int32_t seg_sample(const InT* __restrict__ x, int64_t gi, int64_t total,
                                              const InT* __restrict__ halo_l, int64_t hle,
                                              const InT* __restrict__ halo_r, int64_t hre) {
    if (gi >= 0 && gi < total) return (int32_t)x[gi];
    if (gi < 0) return halo_l && gi >= -hle ? (int32_t)halo_l[hle + gi] : 0;
    return halo_r && gi < total + hre ? (int32_t)halo_r[gi - total] : 0;
}

// WIDE: 128-bit sums (a no-wrap call whose sum may exceed 2^63: int16 samples with huge taps, or
// more taps than 2^24), else 64-bit ones.
template <typename InT, int STAGE, bool WIDE>
__global__ __launch_bounds__(kBlock) void fir1d_generic_kernel(const InT* __restrict__ x,
                                                               typename OutTraits<STAGE>::T* __restrict__ y,
                                                               int64_t start, int64_t end, int64_t total,
                                                               int64_t rowlen, int multi_row, int64_t ch,
                                                               const InT* __restrict__ halo_l,
                                                               const InT* __restrict__ halo_r,
                                                               const int32_t* __restrict__ taps, int L, int KC,
                                                               int frac, int acc_bits) {
    __shared__ int32_t s_taps[kGenTapChunk];
    __shared__ int32_t s_x[kGenWin];
    const int c = L / 2;
    const int64_t HLE = (int64_t)(L - 1 - c) * ch, HRE = (int64_t)c * ch;
    const int64_t t0 = start + (int64_t)blockIdx.x * kGenTile;
    using Acc = typename std::conditional<WIDE, unsigned __int128, uint64_t>::type;
    using SAcc = typename std::conditional<WIDE, __int128, int64_t>::type;
    Acc acc[kGenPer] = {};
    int64_t col[kGenPer];
#pragma unroll
    for (int j = 0; j < kGenPer; ++j) col[j] = multi_row ? (t0 + threadIdx.x + j * kBlock) % rowlen : 0;

    for (int k0 = 0; k0 < L; k0 += KC) {
        const int kc = min(KC, L - k0);
        // outputs t0 + i use samples t0 + i + (c - k) * ch, k in [k0, k0 + kc): window from
        // w0 = t0 + (c - k0 - kc + 1) * ch, output i's tap k at window index i + (kc - 1 - (k - k0)) * ch
        const int64_t w0 = t0 + (int64_t)(c - k0 - kc + 1) * ch;
        const int span = kGenTile + (kc - 1) * (int)ch;
        __syncthreads();  // the previous chunk's reads are done
        for (int k = threadIdx.x; k < kc; k += kBlock) s_taps[k] = taps[k0 + k];
        for (int i = threadIdx.x; i < span; i += kBlock) s_x[i] = seg_sample(x, w0 + i, total, halo_l, HLE, halo_r, HRE);
        __syncthreads();
#pragma unroll
        for (int j = 0; j < kGenPer; ++j) {
            const int i = threadIdx.x + j * kBlock;
            for (int k = 0; k < kc; ++k) {
                int32_t xv = s_x[i + (kc - 1 - k) * (int)ch];
                if (multi_row) {
                    const int64_t d = (int64_t)(c - k0 - k) * ch;
                    if (col[j] + d < 0 || col[j] + d >= rowlen) xv = 0;
                }
                acc[j] += (Acc)(SAcc)((int64_t)s_taps[k] * xv);
            }
        }
    }
#pragma unroll
    for (int j = 0; j < kGenPer; ++j) {
        const int64_t gi = t0 + threadIdx.x + j * kBlock;
        if (gi < end) {
            if constexpr (WIDE)
                y[gi] = stage_out128<STAGE>(round128((__int128)acc[j], frac, acc_bits));
            else
                y[gi] = stage_out<STAGE>(round64((int64_t)acc[j], frac, acc_bits));
        }
    }
}

// Both edges of a single-row segment in one launch (multi-GPU step): output j < hle is the
// left edge, j >= hle maps to the right edge total - hre + (j - hle).  Samples left of the
// segment come from halo_l, right of it from halo_r (zeros when NULL).  Exact 64-bit sums.
template <typename InT, int STAGE, bool WIDE>
__global__ __launch_bounds__(kBlock) void fir1d_edges_kernel(const InT* __restrict__ x,
                                                             typename OutTraits<STAGE>::T* __restrict__ y,
                                                             int64_t total, int64_t ch, const InT* __restrict__ halo_l,
                                                             const InT* __restrict__ halo_r,
                                                             const int32_t* __restrict__ taps, int L, int64_t hle,
                                                             int64_t hre, int frac, int acc_bits) {
    const int c = L / 2;
    for (int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x; j < hle + hre; j += (int64_t)gridDim.x * kBlock) {
        const int64_t gi = j < hle ? j : total - hre + (j - hle);
        using Acc = typename std::conditional<WIDE, unsigned __int128, uint64_t>::type;
        using SAcc = typename std::conditional<WIDE, __int128, int64_t>::type;
        Acc acc = 0;
        for (int k = 0; k < L; ++k)
            acc += (Acc)(SAcc)((int64_t)taps[k] * seg_sample(x, gi + (int64_t)(c - k) * ch, total, halo_l, hle, halo_r, hre));
        if constexpr (WIDE)
            y[gi] = stage_out128<STAGE>(round128((__int128)acc, frac, acc_bits));
        else
            y[gi] = stage_out<STAGE>(round64((int64_t)acc, frac, acc_bits));
    }
}

// ---------------------------------------------------------------------------------------
// Host-side launchers.

// A no-wrap call (acc_bits >= 64) whose exact sum could reach 2^63: the 128-bit generic kernels
// (the reference's sum is an unbounded Python int, fir_1d_fixed_ref.py:94-115).  A wrap to
// acc_bits < 64 is exact mod 2^64, and |sum| < 2^63 is exact in 64 bits.
static bool needs_wide(int in_dtype, const int32_t* hq, int L, int acc_bits) {
    if (acc_bits < 64) return false;
    unsigned __int128 habs = 0;
    for (int k = 0; k < L; ++k) habs += (unsigned __int128)(hq[k] < 0 ? -(int64_t)hq[k] : (int64_t)hq[k]);
    const unsigned __int128 xmax = in_dtype == FIR_IN_U8 ? 255 : 32768;
    return habs * xmax >= ((unsigned __int128)1 << 63);
}

template <typename InT, int STAGE>
static hipError_t launch_generic(const void* x, void* y, int64_t start, int64_t end, int64_t total,
                                 int64_t rowlen, bool multi_row, int ch, const void* hl, const void* hr,
                                 const int32_t* hq, int L, int frac, int acc_bits, hipStream_t stream) {
    using OutT = typename OutTraits<STAGE>::T;
    if (end <= start) return hipSuccess;
    std::string err;
    const int32_t* td = (const int32_t*)device_table(hq, sizeof(int32_t) * (size_t)L, &err);
    if (!td) return hipErrorOutOfMemory;
    TableHold hold(td, stream);
    const int64_t blocks = (end - start + kGenTile - 1) / kGenTile;
    if (blocks >= ((int64_t)1 << 31)) return hipErrorInvalidValue;
    if (needs_wide(sizeof(InT) == 1 ? FIR_IN_U8 : FIR_IN_I16, hq, L, acc_bits))
        hipLaunchKernelGGL((fir1d_generic_kernel<InT, STAGE, true>), dim3((unsigned)blocks), dim3(kBlock), 0, stream,
                           (const InT*)x, (OutT*)y, start, end, total, rowlen, multi_row ? 1 : 0, (int64_t)ch,
                           (const InT*)hl, (const InT*)hr, td, L, gen_tap_chunk(L, ch), frac, acc_bits);
    else
        hipLaunchKernelGGL((fir1d_generic_kernel<InT, STAGE, false>), dim3((unsigned)blocks), dim3(kBlock), 0, stream,
                           (const InT*)x, (OutT*)y, start, end, total, rowlen, multi_row ? 1 : 0, (int64_t)ch,
                           (const InT*)hl, (const InT*)hr, td, L, gen_tap_chunk(L, ch), frac, acc_bits);
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
                               const int32_t* td, int L, int64_t hle, int64_t hre, int frac, int acc_bits, bool wide,
                               hipStream_t stream) {
    const int64_t blocks = std::min<int64_t>((hle + hre + kBlock - 1) / kBlock, 1024);
    if (wide)
        hipLaunchKernelGGL((fir1d_edges_kernel<InT, STAGE, true>), dim3((unsigned)blocks), dim3(kBlock), 0, stream,
                           (const InT*)x, (typename OutTraits<STAGE>::T*)y, total, (int64_t)ch, (const InT*)hl,
                           (const InT*)hr, td, L, hle, hre, frac, acc_bits);
    else
        hipLaunchKernelGGL((fir1d_edges_kernel<InT, STAGE, false>), dim3((unsigned)blocks), dim3(kBlock), 0, stream,
                           (const InT*)x, (typename OutTraits<STAGE>::T*)y, total, (int64_t)ch, (const InT*)hl,
                           (const InT*)hr, td, L, hle, hre, frac, acc_bits);
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
    } else if (L >= (in_dtype == FIR_IN_I16 && stage == FIR_OUT_I32 ? kMfmaMinTapsI32 : kMfmaMinTaps) &&
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
    // u8 output planes start where the previous one ends, at any byte (the reference's 4499 x 2999
    // image: plane f at f * 13492501): the fused kernel's 16-byte stores then run unaligned, which
    // gfx950 performs in the unaligned-access mode ROCm sets for compute queues (byte-aligned store
    // types, fir1d_reg.h), so for the u8 stage no plane's alignment is a condition, plane 0's
    // included; the int32 planes keep whole-dword row staging and stay on 16-byte plane starts
    const bool u8out = stage == FIR_OUT_U8_SAT;
    const bool fused = in_dtype == FIR_IN_U8 && ch == 1 && (u8out || (total * (int64_t)osz) % 16 == 0) &&
                       reg_path_ok(x, u8out ? x : y, in_dtype, rows, rowlen, total, ch, hq, F * L, L, frac, acc_bits);
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

template <int F>
static hipError_t launch_batch_u8(int L, int n, const RegImage* im, const int32_t* hq, int frac, int acc_bits,
                                  hipStream_t s) {
    return launch_reg_batch_taps<uint8_t, FIR_OUT_U8_SAT, 1, F>(L, n, im, hq, frac, acc_bits, s);
}

int launch_fir1d_images_multi(int n, const void* const* xs, const int64_t* rows, const int64_t* widths, int in_dtype,
                              int ch, const int32_t* hq, int L, int F, int frac, int acc_bits, int stage,
                              void* const* planes, hipStream_t stream, std::string* err) {
    if (n < 0) return *err = "images must be >= 0", FIR_EINVAL;
    if (n == 0) return FIR_OK;
    if (!xs || !planes || !rows || !widths) return *err = "image arrays must not be NULL", FIR_EINVAL;
    if (F < 1) return *err = "filters must be >= 1", FIR_EINVAL;
    for (int i = 0; i < n; ++i) {  // the whole call is refused before anything runs
        int rc = check_common(in_dtype, rows[i], widths[i], ch, hq, L, frac, acc_bits, stage, err);
        if (rc) return *err = "image " + std::to_string(i) + ": " + *err, rc;
        bool null = !xs[i];
        for (int f = 0; f < F; ++f) null |= !planes[(size_t)i * F + f];
        if (rows[i] * widths[i] != 0 && null)
            return *err = "image " + std::to_string(i) + ": x and its output planes must not be NULL", FIR_EINVAL;
    }
    std::vector<int> batch;  // images on the batch kernel
    for (int i = 0; i < n; ++i) {
        const int64_t total = rows[i] * widths[i] * ch;
        if (total == 0) continue;
        void* const* yp = planes + (size_t)i * F;
        // u8 planes may start at any byte, each of them (see launch_fir1d_rows_multi): only the
        // image's own alignment and shape decide
        if (in_dtype == FIR_IN_U8 && ch == 1 && stage == FIR_OUT_U8_SAT &&
            reg_path_ok(xs[i], xs[i], in_dtype, rows[i], widths[i], total, ch, hq, F * L, L, frac, acc_bits)) {
            batch.push_back(i);
            continue;
        }
        for (int f = 0; f < F; ++f) {
            int rc = launch_fir1d_rows(xs[i], in_dtype, rows[i], widths[i], ch, hq + (size_t)f * L, L, frac, acc_bits,
                                       stage, yp[f], stream, err);
            if (rc) return rc;
        }
    }
    // largest images first: their waves start first and the small images' waves fill the launch's
    // tail (the 7 golden images: 15.3 vs 16.0 us per stage in their file order; tools/batch_ab.py)
    std::stable_sort(batch.begin(), batch.end(),
                     [&](int a, int b) { return rows[a] * widths[a] > rows[b] * widths[b]; });
    for (size_t i0 = 0; i0 < batch.size(); i0 += kRegBatch) {
        const int nb = (int)std::min<size_t>(kRegBatch, batch.size() - i0);
        for (int f0 = 0; f0 < F; f0 += 4) {
            const int nf = F - f0 < 4 ? F - f0 : 4;
            RegImage im[kRegBatch];
            for (int j = 0; j < nb; ++j) {
                const int i = batch[i0 + j];
                im[j].x = xs[i];
                im[j].rows = rows[i];
                im[j].rowlen = widths[i];
                for (int f = 0; f < 4; ++f) im[j].y[f] = f < nf ? planes[(size_t)i * F + f0 + f] : nullptr;
            }
            const int32_t* hf = hq + (size_t)f0 * L;
            hipError_t e;
            switch (nf) {
                case 1: e = launch_batch_u8<1>(L, nb, im, hf, frac, acc_bits, stream); break;
                case 2: e = launch_batch_u8<2>(L, nb, im, hf, frac, acc_bits, stream); break;
                case 3: e = launch_batch_u8<3>(L, nb, im, hf, frac, acc_bits, stream); break;
                default: e = launch_batch_u8<4>(L, nb, im, hf, frac, acc_bits, stream); break;
            }
            if (e != hipSuccess) return *err = std::string("fir1d batch launch failed: ") + hipGetErrorString(e), FIR_EHIP;
        }
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
        const int32_t* td = (const int32_t*)device_table(hq, sizeof(int32_t) * (size_t)L, err);
        if (!td) return FIR_ENOMEM;
        TableHold hold(td, stream);
        const bool wide = needs_wide(in_dtype, hq, L, acc_bits);
        if (in_dtype == FIR_IN_U8)
            e = stage == FIR_OUT_U8_SAT
                    ? launch_edges<uint8_t, FIR_OUT_U8_SAT>(x, y, total, ch, hl, hr, td, L, hle, hre, frac, acc_bits, wide, stream)
                    : launch_edges<uint8_t, FIR_OUT_I32>(x, y, total, ch, hl, hr, td, L, hle, hre, frac, acc_bits, wide, stream);
        else
            e = stage == FIR_OUT_U8_SAT
                    ? launch_edges<int16_t, FIR_OUT_U8_SAT>(x, y, total, ch, hl, hr, td, L, hle, hre, frac, acc_bits, wide, stream)
                    : launch_edges<int16_t, FIR_OUT_I32>(x, y, total, ch, hl, hr, td, L, hle, hre, frac, acc_bits, wide, stream);
    }
    if (e != hipSuccess) return *err = std::string("fir1d edge launch failed: ") + hipGetErrorString(e), FIR_EHIP;
    return FIR_OK;
}

}  // namespace fir
