// fir2d.hip — gfx950 kernels for the 2-D fixed-point FIR.
//
// y[i,j] = stage(round(wrap(sum_m sum_n hq[m][n] * x[i - m + R/2][j - n + C/2]))), zero padded:
// the 2-D extension of the reference's centre-aligned 1-D rule
// (fir_1d/model/python/fir_1d_fixed_ref.py:95-126, fir_1d/docs/fir_1d_golden_spec_v1.md:65-74).
//
// fir2d_reg_kernel (fir2d_reg.h) reuses the 1-D template: a lane owns kVec2d horizontally
// adjacent pixels, the horizontal (C-1)-pixel halo arrives from the neighbouring lanes by
// DPP wave shifts, and the vertical (R-1)-row halo is carried in a register ring of R
// partial-output rows (input-stationary, no LDS, no re-read inside a strip).
// fir2d_generic_kernel handles every other shape/width/alignment.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <string>
#include <type_traits>

#include "fir2d_pk16.h"
#include "fir2d_reg.h"
#include "fir_common.h"
#include "fir_launch.h"

namespace fir {

// Shape chosen by the A/B microbenchmark (tools/microbench/fir2d_micro.hip, profiles/).
// Every launch stores non-temporally and remaps blocks XCD-major (fir2d_reg_kernel's NTS / XCD):
// 4 HBM-resident 8192^2 frames per launch, packed-16 separable 26.5 -> 21.8 us per frame,
// general packed-16 38.5 -> 35.8 us (profiles/r02/micro2d_nts_sweep.txt).
constexpr int kVec2d = 16;       // separable path: 16 pixels per lane, 16-row strips
constexpr int kStrip2dSep = 16;
constexpr int kVec2dGen = 8;     // general (dot2) path: 8 pixels per lane, 16-row strips, <= 128
constexpr int kStrip2dGen = 16;  // VGPRs (4 waves/SIMD): 45.8 vs 48.5 us for 16 px x 8 rows
// input rows loaded this many rows ahead (8192^2 frame: separable 32.9 -> 31.0 us at 3,
// packed-16 25.7 -> 23.9 us at 3, general dot2 45.5 -> 43.9 us at 2; profiles/r01/micro2d_pk16.txt)
constexpr int kPdSep = 3;
constexpr int kPdGen = 2;
// packed-16 form: 32-row strips, rows 4 ahead (23.5 vs 24.3 us for 16 rows / 3 ahead; a
// memory-only twin of the same loop takes 21.1 us, profiles/r01/micro2d_copy.txt)
constexpr int kStrip2dPk = 32;
constexpr int kPdPk = 4;
constexpr int kMinwPk = 1;  // waves per SIMD the register allocation must allow

// The separable packed-16 form on fir2d_pk16_strip_kernel (frames below 2^31 pixels; larger ones
// keep the unrolled 32-row fir2d_reg_kernel strip): strips of about kPkRows rows (whole turns of U
// input rows).  Short strips keep the two neighbours
// that share R - 1 rows in step with each other (see the kernel's walk directions): 16-26 rows
// measured 79.7-81.3 us per 4 frames, 6 rows 97, 36 rows 86, one resident round (56 rows) 85.5
// (profiles/r03/ab2d_pk16_rows.txt).
constexpr int kPkRows = 16;
template <int R, int C, int MODE>
static hipError_t launch_pk16_rolled(const uint8_t* x, uint8_t* y, int64_t frames, int64_t H, int64_t W,
                                     const Taps2<R, C>& t, hipStream_t s) {
    constexpr int PD = kPdPk, U = p16_lcm(R, PD + 1);
    auto kern = fir2d_pk16_strip_kernel<R, C, PD, MODE, kMinwPk>;
    const int64_t gx = (W / 16 + kBlock - 1) / kBlock;
    int64_t rows = kPkRows;
    // whole turns of U input rows per strip (S + R - 1 a multiple of U), and at most 65535 strips
    rows = std::max<int64_t>(rows, (H + 65534) / 65535);
    const int64_t lo = rows;
    rows = std::max<int64_t>((rows + R - 1 + U / 2) / U, 1) * U - (R - 1);  // nearest whole turns (U >= R)
    if ((H + rows - 1) / rows > 65535) rows = ((lo + R - 1 + U - 1) / U) * U - (R - 1);
    if (rows > H) rows = H;  // one strip: the kernel stops at its last row (t < T), not at a turn
    const int64_t nstrips = (H + rows - 1) / rows;
    hipLaunchKernelGGL(kern, dim3((unsigned)gx, (unsigned)nstrips, (unsigned)frames), dim3(kBlock), 0, s, x, y, H, W,
                       t, (int)rows);
    return hipGetLastError();
}
// general packed-16 form: 16-row strips (a 32-row strip's R*C MACs per row exceed the forced
// unroll budget: the loop stays rolled and its ring spills to scratch)
constexpr int kVec2dPkGen = 16;
constexpr int kStrip2dPkGen = 16;
// prefetch depth: rows 2 ahead for 5x5-size kernels (0.5-3 % faster than depth 3 over two A/B
// runs), 3 ahead for smaller ones (3x3: 21.9 vs 22.3 us at depth 2; profiles/r01/ab2d_pk16_general.txt)
template <int R, int C>
constexpr int pd_pk_gen() { return R * C >= 20 ? 2 : 3; }

// Generic: one output per thread, exact 64-bit sum (mod 2^64, see round64), global loads (L1/L2
// absorb the reuse), taps of any count from HBM; rows grid-strided (any height).
template <int STAGE, bool WIDE>  // WIDE: 128-bit sums (a no-wrap call whose sum could reach 2^63)
__global__ __launch_bounds__(kBlock) void fir2d_generic_kernel(const uint8_t* __restrict__ x,
                                                               typename OutTraits<STAGE>::T* __restrict__ y,
                                                               int64_t H, int64_t W, const int32_t* __restrict__ taps,
                                                               int R, int C, int frac, int acc_bits) {
    const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (j >= W) return;
    x += (int64_t)blockIdx.z * H * W;  // frame blockIdx.z of a batch stored back to back
    y += (int64_t)blockIdx.z * H * W;
    const int cr = R / 2, cc = C / 2;
    for (int64_t i = blockIdx.y; i < H; i += gridDim.y) {
        using Acc = typename std::conditional<WIDE, unsigned __int128, uint64_t>::type;
        using SAcc = typename std::conditional<WIDE, __int128, int64_t>::type;
        Acc acc = 0;
        for (int m = 0; m < R; ++m) {
            const int64_t ii = i - m + cr;
            if (ii < 0 || ii >= H) continue;
            for (int n = 0; n < C; ++n) {
                const int64_t jj = j - n + cc;
                if (jj < 0 || jj >= W) continue;
                acc += (Acc)(SAcc)((int64_t)taps[(int64_t)m * C + n] * (int64_t)x[ii * W + jj]);
            }
        }
        if constexpr (WIDE)
            y[i * W + j] = stage_out128<STAGE>(round128((__int128)acc, frac, acc_bits));
        else
            y[i * W + j] = stage_out<STAGE>(round64((int64_t)acc, frac, acc_bits));
    }
}

// Exact integer rank-1 factorisation h[m][n] == col[m] * row[n] (row taps int16), if any.
static bool rank1_factor(const int32_t* hq, int R, int C, int32_t* col, int32_t* row) {
    int r0 = -1, n0 = -1;
    for (int m = 0; m < R && r0 < 0; ++m)
        for (int n = 0; n < C; ++n)
            if (hq[m * C + n] != 0) {
                r0 = m;
                n0 = n;
                break;
            }
    if (r0 < 0) return false;  // all-zero kernel: the general path is exact and cheap enough
    int64_t g = 0;
    for (int n = 0; n < C; ++n) {
        int64_t v = hq[r0 * C + n] < 0 ? -(int64_t)hq[r0 * C + n] : hq[r0 * C + n];
        while (v) {
            const int64_t t = g % v;
            g = v;
            v = t;
        }
    }
    for (int n = 0; n < C; ++n) {
        const int64_t b = hq[r0 * C + n] / g;
        if (b < -32768 || b > 32767) return false;
        row[n] = (int32_t)b;
    }
    for (int m = 0; m < R; ++m) {
        const int64_t num = hq[m * C + n0];
        if (num % row[n0]) return false;
        const int64_t a = num / row[n0];
        for (int n = 0; n < C; ++n)
            if ((int64_t)hq[m * C + n] != a * row[n]) return false;
        col[m] = (int32_t)a;
    }
    return true;
}

template <int R, int C, int STAGE>
static hipError_t launch2d_reg(const uint8_t* x, void* y, int64_t frames, int64_t H, int64_t W, const int32_t* hq,
                               int frac, int acc_bits, hipStream_t s) {
    using OutT = typename OutTraits<STAGE>::T;
    Taps2<R, C> t = {};
    for (int m = 0; m < R; ++m)
        for (int n = 0; n < C; ++n) t.h[m][n] = hq[m * C + n];
    pack_taps2(t);  // packed v_dot2_i32_i16 taps: two MACs per instruction (taps are int16 here)
    // no wrap possible: 255 * sum|h| + 2^(f-1) below the acc_bits limit (u8 samples >= 0)
    int64_t habs = 0;
    for (int k = 0; k < R * C; ++k) habs += hq[k] < 0 ? -(int64_t)hq[k] : hq[k];
    const bool nowrap = frac <= 22 && 255 * habs + ((int64_t)1 << (frac - 1)) < ((int64_t)1 << (acc_bits - 1));
    int32_t rowt[C];
    bool sep = R > 1 && C > 1 && rank1_factor(hq, R, C, t.col, rowt);
    if (sep) {  // the row sums must fit the 24-bit multiplier: 255 * sum|row| < 2^23, |col| < 2^23
        int64_t sr = 0;
        for (int n = 0; n < C; ++n) sr += rowt[n] < 0 ? -(int64_t)rowt[n] : rowt[n];
        sep = 255 * sr < (1 << 23);
        for (int m = 0; m < R; ++m) sep &= t.col[m] >= -(1 << 23) && t.col[m] < (1 << 23);
    }
    if (sep) {
        const dim3 grid = fir2d_reg_grid<kVec2d, kStrip2dSep>(H, W, frames);
        // separable: R + (C+1)/2 instructions per pixel-row instead of R * (C+1)/2
        for (int p = 0; p < (C + 1) / 2; ++p) {
            const int lo = rowt[C - 1 - 2 * p];
            const int hi = C - 2 - 2 * p >= 0 ? rowt[C - 2 - 2 * p] : 0;
            t.rowp[p] = ((uint32_t)lo & 0xFFFFu) | ((uint32_t)hi << 16);
        }
        // int16 row sums (255 * sum|row| <= 32767) and int16 column taps: the column pass packs
        // two rows' sums per dword and runs on v_dot2 too
        int64_t sr = 0;
        for (int n = 0; n < C; ++n) sr += rowt[n] < 0 ? -(int64_t)rowt[n] : rowt[n];
        bool sep16 = 255 * sr <= 32767;
        for (int m = 0; m < R; ++m) sep16 &= t.col[m] >= -32768 && t.col[m] <= 32767;
        for (int p = 0; p < (R + 1) / 2; ++p) {
            const int lo = t.col[2 * p];
            const int hi = 2 * p + 1 < R ? t.col[2 * p + 1] : 0;
            t.colp[p] = ((uint32_t)lo & 0xFFFFu) | ((uint32_t)hi << 16);
        }
        constexpr int S16 = kMode2dSep | kMode2dSep16;
        constexpr int SNW = kMode2dSep | kMode2dNoWrap;
        // packed 16-bit pixel pairs when the whole sum provably fits 16 bits (u8 stage only)
        if constexpr (STAGE == FIR_OUT_U8_SAT) {
            const int pk = nowrap ? plan_pk16(t, t.col, rowt, frac) : 0;
            if (H * W < ((int64_t)1 << 31)) {
                if (pk == (kMode2dPk16 | kMode2dPkHi8))
                    return launch_pk16_rolled<R, C, kMode2dPk16 | kMode2dPkHi8>(x, (uint8_t*)y, frames, H, W, t, s);
                if (pk == kMode2dPk16) return launch_pk16_rolled<R, C, kMode2dPk16>(x, (uint8_t*)y, frames, H, W, t, s);
                if (pk == (kMode2dPk16 | kMode2dPkSigned))
                    return launch_pk16_rolled<R, C, kMode2dPk16 | kMode2dPkSigned>(x, (uint8_t*)y, frames, H, W, t, s);
            }
            const dim3 gpk = fir2d_reg_grid<kVec2d, kStrip2dPk>(H, W, frames);
            if (pk == (kMode2dPk16 | kMode2dPkHi8)) {
                hipLaunchKernelGGL((fir2d_reg_kernel<R, C, STAGE, kVec2d, kStrip2dPk, SNW | kMode2dPk16 | kMode2dPkHi8, kMinwPk, kPdPk, false, true, true>),
                                   gpk, dim3(kBlock), 0, s, x, (OutT*)y, H, W, t, 32 - acc_bits, frac);
                return hipGetLastError();
            }
            if (pk == kMode2dPk16) {
                hipLaunchKernelGGL((fir2d_reg_kernel<R, C, STAGE, kVec2d, kStrip2dPk, SNW | kMode2dPk16, kMinwPk, kPdPk, false, true, true>), gpk,
                                   dim3(kBlock), 0, s, x, (OutT*)y, H, W, t, 32 - acc_bits, frac);
                return hipGetLastError();
            }
            if (pk == (kMode2dPk16 | kMode2dPkSigned)) {
                hipLaunchKernelGGL((fir2d_reg_kernel<R, C, STAGE, kVec2d, kStrip2dPk, SNW | kMode2dPk16 | kMode2dPkSigned, kMinwPk, kPdPk, false, true, true>),
                                   gpk, dim3(kBlock), 0, s, x, (OutT*)y, H, W, t, 32 - acc_bits, frac);
                return hipGetLastError();
            }
        }
        if (sep16 && nowrap)
            hipLaunchKernelGGL((fir2d_reg_kernel<R, C, STAGE, kVec2d, kStrip2dSep, S16 | kMode2dNoWrap, 1, kPdSep, false, true, true>), grid,
                               dim3(kBlock), 0, s, x, (OutT*)y, H, W, t, 32 - acc_bits, frac);
        else if (sep16)
            hipLaunchKernelGGL((fir2d_reg_kernel<R, C, STAGE, kVec2d, kStrip2dSep, S16, 1, kPdSep, false, true, true>), grid, dim3(kBlock), 0, s, x,
                               (OutT*)y, H, W, t, 32 - acc_bits, frac);
        else if (nowrap)
            hipLaunchKernelGGL((fir2d_reg_kernel<R, C, STAGE, kVec2d, kStrip2dSep, kMode2dSep | kMode2dNoWrap, 1, kPdSep, false, true, true>), grid,
                               dim3(kBlock), 0, s, x, (OutT*)y, H, W, t, 32 - acc_bits, frac);
        else
            hipLaunchKernelGGL((fir2d_reg_kernel<R, C, STAGE, kVec2d, kStrip2dSep, kMode2dSep, 1, kPdSep, false, true, true>), grid, dim3(kBlock), 0, s,
                               x, (OutT*)y, H, W, t, 32 - acc_bits, frac);
    } else {
        // packed 16-bit pixel pairs when the whole sum provably fits 16 bits (u8 stage only)
        if constexpr (STAGE == FIR_OUT_U8_SAT) {
            constexpr int GNW = kMode2dDot2 | kMode2dNoWrap | kMode2dPk16, ST = kStrip2dPkGen, PD = pd_pk_gen<R, C>();
            const int pk = nowrap ? plan_pk16_gen(t, hq, frac) : 0;
            const dim3 gpk = fir2d_reg_grid<kVec2dPkGen, ST>(H, W, frames);
            if (pk == (kMode2dPk16 | kMode2dPkHi8)) {
                hipLaunchKernelGGL((fir2d_reg_kernel<R, C, STAGE, kVec2dPkGen, ST, GNW | kMode2dPkHi8, 1, PD, false, true, true>), gpk,
                                   dim3(kBlock), 0, s, x, (OutT*)y, H, W, t, 32 - acc_bits, frac);
                return hipGetLastError();
            }
            if (pk == kMode2dPk16) {
                hipLaunchKernelGGL((fir2d_reg_kernel<R, C, STAGE, kVec2dPkGen, ST, GNW, 1, PD, false, true, true>), gpk, dim3(kBlock), 0, s, x,
                                   (OutT*)y, H, W, t, 32 - acc_bits, frac);
                return hipGetLastError();
            }
            if (pk == (kMode2dPk16 | kMode2dPkSigned)) {
                hipLaunchKernelGGL((fir2d_reg_kernel<R, C, STAGE, kVec2dPkGen, ST, GNW | kMode2dPkSigned, 1, PD, false, true, true>), gpk,
                                   dim3(kBlock), 0, s, x, (OutT*)y, H, W, t, 32 - acc_bits, frac);
                return hipGetLastError();
            }
        }
        const dim3 grid = fir2d_reg_grid<kVec2dGen, kStrip2dGen>(H, W, frames);
        if (nowrap)
            hipLaunchKernelGGL((fir2d_reg_kernel<R, C, STAGE, kVec2dGen, kStrip2dGen, kMode2dDot2 | kMode2dNoWrap, 4, kPdGen, false, true, true>),
                               grid, dim3(kBlock), 0, s, x, (OutT*)y, H, W, t, 32 - acc_bits, frac);
        else
            hipLaunchKernelGGL((fir2d_reg_kernel<R, C, STAGE, kVec2dGen, kStrip2dGen, kMode2dDot2, 4, kPdGen, false, true, true>), grid,
                               dim3(kBlock), 0, s, x, (OutT*)y, H, W, t, 32 - acc_bits, frac);
    }
    return hipGetLastError();
}

template <int STAGE>
static hipError_t launch2d_reg_shape(int R, int C, const uint8_t* x, void* y, int64_t frames, int64_t H, int64_t W,
                                     const int32_t* hq, int frac, int acc_bits, hipStream_t s) {
#define FIR2D_CASE(r, c) \
    if (R == r && C == c) return launch2d_reg<r, c, STAGE>(x, y, frames, H, W, hq, frac, acc_bits, s);
    FIR2D_CASE(1, 1) FIR2D_CASE(1, 3) FIR2D_CASE(1, 5) FIR2D_CASE(3, 1) FIR2D_CASE(3, 3) FIR2D_CASE(3, 5)
    FIR2D_CASE(5, 1) FIR2D_CASE(5, 3) FIR2D_CASE(5, 5)
#undef FIR2D_CASE
    return hipErrorInvalidValue;
}

static bool reg2d_shape(int R, int C) { return (R == 1 || R == 3 || R == 5) && (C == 1 || C == 3 || C == 5); }

// rank-1 kernels have a register form with R + C/2 MACs per pixel; measured against the MFMA path
// in profiles/r02 (the default dispatch keeps the faster one)
static bool sep2d_register_form(const int32_t* hq, int R, int C) {
    if (!reg2d_shape(R, C)) return false;
    int32_t col[5], row[5];
    return R > 1 && C > 1 && rank1_factor(hq, R, C, col, row);
}

int launch_fir2d(const uint8_t* x, int64_t frames, int64_t H, int64_t W, const int32_t* hq, int R, int C, int frac,
                 int acc_bits, int stage, void* y, hipStream_t stream, std::string* err) {
    if (stage != FIR_OUT_U8_SAT && stage != FIR_OUT_I32) return *err = "out_stage must be FIR_OUT_U8_SAT or FIR_OUT_I32", FIR_EINVAL;
    if (H < 0 || W < 0 || frames < 0) return *err = "frames, height and width must be >= 0", FIR_EINVAL;
    if (frames > 65535) return *err = "frames must be <= 65535 per call", FIR_EINVAL;
    if (!hq) return *err = "hq must not be NULL", FIR_EINVAL;
    if (R < 1 || C < 1 || (int64_t)R * C > FIR_MAX_TAPS)
        return *err = "tap_rows*tap_cols must be in [1, " + std::to_string(FIR_MAX_TAPS) + "]", FIR_EINVAL;
    if (frac < 1 || acc_bits < 1) return *err = "frac_bits and acc_bits must be >= 1", FIR_EINVAL;
    const int64_t ntaps = (int64_t)R * C;
    bool wide = false;  // a no-wrap call whose exact sum could reach 2^63: 128-bit sums
    if (acc_bits >= 64) {
        unsigned __int128 habs = 0;
        for (int64_t k = 0; k < ntaps; ++k) habs += (unsigned __int128)(hq[k] < 0 ? -(int64_t)hq[k] : (int64_t)hq[k]);
        wide = habs * 255 >= ((unsigned __int128)1 << 63);
    }
    if (H == 0 || W == 0 || frames == 0) return FIR_OK;
    if (!x || !y) return *err = "x and y must not be NULL", FIR_EINVAL;
    bool taps16 = true;  // the register kernel multiplies on v_dot2_i32_i16
    for (int64_t k = 0; k < ntaps && taps16; ++k) taps16 &= (hq[k] >= -32768 && hq[k] <= 32767);
    // the register kernel's grid holds a strip of rows per blockIdx.y
    const bool fast = reg2d_shape(R, C) && W % kVec2d == 0 && (uintptr_t)x % 16 == 0 && (uintptr_t)y % 16 == 0 &&
                      acc_bits <= 32 && frac <= 31 && taps16 && W >= kVec2d && H <= 65535 * (int64_t)kStrip2dSep;
    hipError_t e = hipErrorNotSupported;
    // matrix-core path (fir2d_mfma.hip) unless FIR2D_PATH=reg; rank-1 kernels keep the separable
    // register kernels by default (faster there: 79.3 vs 83.7 us for the bench's separable 5x5 per
    // 4-frame launch).  Since the MFMA kernel's strips walk both ways it also beats the general
    // packed-16 register form of a 3x3 sharpen (82.6 vs 83.8 us; round 2 had 86.9 vs 82.7;
    // profiles/r03/ab2d_paths.txt).  FIR2D_PATH=mfma takes the MFMA path for rank-1 kernels too.
    const char* path = getenv("FIR2D_PATH");
    const bool force = path && !strcmp(path, "mfma"), off = path && !strcmp(path, "reg");
    if (!off && (force || !sep2d_register_form(hq, R, C)))
        e = launch_fir2d_mfma(x, frames, H, W, hq, R, C, frac, acc_bits, stage, y, stream);
    if (e != hipErrorNotSupported) {
        // launched (or failed to launch) on the matrix cores
    } else if (fast) {
        e = stage == FIR_OUT_U8_SAT ? launch2d_reg_shape<FIR_OUT_U8_SAT>(R, C, x, y, frames, H, W, hq, frac, acc_bits, stream)
                                    : launch2d_reg_shape<FIR_OUT_I32>(R, C, x, y, frames, H, W, hq, frac, acc_bits, stream);
    } else {
        if ((W + kBlock - 1) / kBlock >= ((int64_t)1 << 31)) return *err = "width too large", FIR_EINVAL;
        const int32_t* td = (const int32_t*)device_table(hq, sizeof(int32_t) * (size_t)ntaps, err);
        if (!td) return FIR_ENOMEM;
        TableHold hold(td, stream);
        dim3 grid((unsigned)((W + kBlock - 1) / kBlock), (unsigned)std::min<int64_t>(H, 65535), (unsigned)frames);
        if (stage == FIR_OUT_U8_SAT && wide)
            hipLaunchKernelGGL((fir2d_generic_kernel<FIR_OUT_U8_SAT, true>), grid, dim3(kBlock), 0, stream, x, (uint8_t*)y,
                               H, W, td, R, C, frac, acc_bits);
        else if (stage == FIR_OUT_U8_SAT)
            hipLaunchKernelGGL((fir2d_generic_kernel<FIR_OUT_U8_SAT, false>), grid, dim3(kBlock), 0, stream, x, (uint8_t*)y,
                               H, W, td, R, C, frac, acc_bits);
        else if (wide)
            hipLaunchKernelGGL((fir2d_generic_kernel<FIR_OUT_I32, true>), grid, dim3(kBlock), 0, stream, x, (int32_t*)y,
                               H, W, td, R, C, frac, acc_bits);
        else
            hipLaunchKernelGGL((fir2d_generic_kernel<FIR_OUT_I32, false>), grid, dim3(kBlock), 0, stream, x, (int32_t*)y,
                               H, W, td, R, C, frac, acc_bits);
        e = hipGetLastError();
    }
    if (e != hipSuccess) return *err = std::string("fir2d launch failed: ") + hipGetErrorString(e), FIR_EHIP;
    return FIR_OK;
}

}  // namespace fir
