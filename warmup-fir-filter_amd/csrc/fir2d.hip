// fir2d.hip — gfx950 kernels for the 2-D fixed-point FIR.
//
// y[i,j] = stage(round(wrap(sum_m sum_n hq[m][n] * x[i - m + R/2][j - n + C/2]))), zero padded:
// the 2-D extension of the reference's centre-aligned 1-D rule
// (fir_1d/model/python/fir_1d_fixed_ref.py:95-126, fir_1d/docs/fir_1d_golden_spec_v1.md:65-74).
//
// fir2d_reg_kernel reuses the 1-D template: a thread owns 16 horizontally adjacent pixels
// (one 16-byte load per input row), the horizontal (C-1)-pixel halo arrives from the
// neighbouring lanes by DPP wave shifts, and the vertical (R-1)-row halo is carried in a
// register ring of R partial-output rows: every input row is loaded once per strip and
// scattered into the R output rows it contributes to (input-stationary), so no LDS and
// no re-read inside a strip.  Strips of kStrip output rows overlap by R-1 input rows
// (L2 hits).  fir2d_generic_kernel handles every other shape/width/alignment.
#include <string>

#include "fir_common.h"
#include "fir_launch.h"

namespace fir {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int R, int C>
struct Taps2 {
    int32_t h[R][C];
};

constexpr int kStrip = 32;  // output rows per thread

__device__ __forceinline__ void load_row16(const uint8_t* __restrict__ x, int64_t row, int64_t H, int64_t W,
                                           int64_t col, uint32_t (&d)[4]) {
    if (row >= 0 && row < H && col >= 0 && col < W) {
        const u32x4 q = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(x + row * W + col));
        d[0] = q.x;
        d[1] = q.y;
        d[2] = q.z;
        d[3] = q.w;
    } else {
        d[0] = d[1] = d[2] = d[3] = 0;
    }
}

template <int R, int C, int STAGE>
__global__ __launch_bounds__(kBlock) void fir2d_reg_kernel(const uint8_t* __restrict__ x,
                                                           typename OutTraits<STAGE>::T* __restrict__ y, int64_t H,
                                                           int64_t W, Taps2<R, C> taps, int shl, int frac) {
    using OutT = typename OutTraits<STAGE>::T;
    constexpr int VEC = 16;
    constexpr int CC = C / 2, CR = R / 2;
    constexpr int HLE = C - 1 - CC, HRE = CC;  // horizontal halo
    constexpr int TOP = R - 1 - CR;            // input rows needed above an output row
    static_assert(HLE <= 4 && HRE <= 4, "horizontal halo must fit in one dword");
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t vecs_per_row = W / VEC;
    const int64_t v = (int64_t)blockIdx.x * kBlock + threadIdx.x;  // vector column index
    const int64_t col0 = v * VEC;
    const int64_t r0 = (int64_t)blockIdx.y * kStrip;
    const bool active = v < vecs_per_row;

    uint32_t acc[R][VEC];  // wrap-around (mod 2^32) partial sums
#pragma unroll
    for (int s = 0; s < R; ++s)
#pragma unroll
        for (int j = 0; j < VEC; ++j) acc[s][j] = 0;

    // input rows ii = r0 - TOP + t, t in [0, kStrip + R - 1)
    constexpr int T = kStrip + R - 1;
    constexpr int TU = ((T + R - 1) / R) * R;
    uint32_t cur[4], hcur[4] = {0, 0, 0, 0};
    load_row16(x, r0 - TOP, H, active ? W : 0, col0, cur);
    if (lane == 0) load_row16(x, r0 - TOP, H, W, col0 - VEC, hcur);
    else if (lane == kWave - 1) load_row16(x, r0 - TOP, H, W, col0 + VEC, hcur);

    for (int tb = 0; tb < TU; tb += R) {
#pragma unroll
        for (int s = 0; s < R; ++s) {
            const int t = tb + s;
            // prefetch the next input row
            uint32_t nxt[4], hnxt[4] = {0, 0, 0, 0};
            const int64_t nrow = r0 - TOP + t + 1;
            const bool more = t + 1 < T;
            load_row16(x, more ? nrow : -1, H, active ? W : 0, col0, nxt);
            if (lane == 0) load_row16(x, more ? nrow : -1, H, W, col0 - VEC, hnxt);
            else if (lane == kWave - 1) load_row16(x, more ? nrow : -1, H, W, col0 + VEC, hnxt);

            // horizontal window of this input row
            int32_t w[HLE + VEC + HRE];
            if constexpr (HLE > 0) {
                const uint32_t p = from_prev_lane(hcur[3], cur[3]);
#pragma unroll
                for (int i = 0; i < HLE; ++i) w[i] = (int32_t)((p >> (8 * (4 - HLE + i))) & 0xFFu);
            }
#pragma unroll
            for (int j = 0; j < VEC; ++j) w[HLE + j] = (int32_t)((cur[j / 4] >> (8 * (j % 4))) & 0xFFu);
            if constexpr (HRE > 0) {
                const uint32_t nx = from_next_lane(hcur[0], cur[0]);
#pragma unroll
                for (int i = 0; i < HRE; ++i) w[HLE + VEC + i] = (int32_t)((nx >> (8 * i)) & 0xFFu);
            }
            // scatter into the R output rows o = t - (R-1) + m (ring slot (s + 1 + m) % R)
#pragma unroll
            for (int m = 0; m < R; ++m) {
                const int slot = (s + 1 + m) % R;
#pragma unroll
                for (int j = 0; j < VEC; ++j) {
                    uint32_t a = acc[slot][j];
#pragma unroll
                    for (int n = 0; n < C; ++n) a += (uint32_t)__mul24(taps.h[m][n], w[HLE + j + CC - n]);
                    acc[slot][j] = a;
                }
            }
            // output row o = t - (R-1) is complete: slot (s + 1) % R
            {
                const int slot = (s + 1) % R;
                const int o = t - (R - 1);
                const int64_t orow = r0 + o;
                if (active && o >= 0 && o < kStrip && orow < H) {
                    int32_t q[VEC];
#pragma unroll
                    for (int j = 0; j < VEC; ++j) q[j] = round32(acc[slot][j], shl, frac);
                    OutT* dst = y + orow * W + col0;
                    if constexpr (STAGE == FIR_OUT_U8_SAT) {
                        uint32_t o4[4];
#pragma unroll
                        for (int i = 0; i < 4; ++i)
                            o4[i] = (uint32_t)stage_out32<STAGE>(q[4 * i]) |
                                    ((uint32_t)stage_out32<STAGE>(q[4 * i + 1]) << 8) |
                                    ((uint32_t)stage_out32<STAGE>(q[4 * i + 2]) << 16) |
                                    ((uint32_t)stage_out32<STAGE>(q[4 * i + 3]) << 24);
                        u32x4 val = {o4[0], o4[1], o4[2], o4[3]};
                        __builtin_nontemporal_store(val, reinterpret_cast<u32x4*>(dst));
                    } else {
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            u32x4 val = {(uint32_t)q[4 * i], (uint32_t)q[4 * i + 1], (uint32_t)q[4 * i + 2],
                                         (uint32_t)q[4 * i + 3]};
                            __builtin_nontemporal_store(val, reinterpret_cast<u32x4*>(dst) + i);
                        }
                    }
                }
#pragma unroll
                for (int j = 0; j < VEC; ++j) acc[slot][j] = 0;
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                cur[i] = nxt[i];
                hcur[i] = hnxt[i];
            }
        }
    }
}

// Generic: one output per thread, exact int64 sum, global loads (L1/L2 absorb the reuse).
struct Taps2G {
    int32_t h[FIR_MAX_TAPS];
};

template <int STAGE>
__global__ __launch_bounds__(kBlock) void fir2d_generic_kernel(const uint8_t* __restrict__ x,
                                                               typename OutTraits<STAGE>::T* __restrict__ y,
                                                               int64_t H, int64_t W, Taps2G taps, int R, int C,
                                                               int frac, int acc_bits) {
    const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const int64_t i = blockIdx.y;
    if (j >= W) return;
    const int cr = R / 2, cc = C / 2;
    int64_t acc = 0;
    for (int m = 0; m < R; ++m) {
        const int64_t ii = i - m + cr;
        if (ii < 0 || ii >= H) continue;
        for (int n = 0; n < C; ++n) {
            const int64_t jj = j - n + cc;
            if (jj < 0 || jj >= W) continue;
            acc += (int64_t)taps.h[m * C + n] * (int64_t)x[ii * W + jj];
        }
    }
    y[i * W + j] = stage_out<STAGE>(round64(acc, frac, acc_bits));
}

template <int R, int C, int STAGE>
static hipError_t launch2d_reg(const uint8_t* x, void* y, int64_t H, int64_t W, const int32_t* hq, int frac,
                               int acc_bits, hipStream_t s) {
    using OutT = typename OutTraits<STAGE>::T;
    Taps2<R, C> t;
    for (int m = 0; m < R; ++m)
        for (int n = 0; n < C; ++n) t.h[m][n] = hq[m * C + n];
    const int64_t vecs = W / 16;
    dim3 grid((unsigned)((vecs + kBlock - 1) / kBlock), (unsigned)((H + kStrip - 1) / kStrip));
    hipLaunchKernelGGL((fir2d_reg_kernel<R, C, STAGE>), grid, dim3(kBlock), 0, s, x, (OutT*)y, H, W, t,
                       32 - acc_bits, frac);
    return hipGetLastError();
}

template <int STAGE>
static hipError_t launch2d_reg_shape(int R, int C, const uint8_t* x, void* y, int64_t H, int64_t W,
                                     const int32_t* hq, int frac, int acc_bits, hipStream_t s) {
#define FIR2D_CASE(r, c) \
    if (R == r && C == c) return launch2d_reg<r, c, STAGE>(x, y, H, W, hq, frac, acc_bits, s);
    FIR2D_CASE(1, 1) FIR2D_CASE(1, 3) FIR2D_CASE(1, 5) FIR2D_CASE(3, 1) FIR2D_CASE(3, 3) FIR2D_CASE(3, 5)
    FIR2D_CASE(5, 1) FIR2D_CASE(5, 3) FIR2D_CASE(5, 5)
#undef FIR2D_CASE
    return hipErrorInvalidValue;
}

static bool reg2d_shape(int R, int C) { return (R == 1 || R == 3 || R == 5) && (C == 1 || C == 3 || C == 5); }

int launch_fir2d(const uint8_t* x, int64_t H, int64_t W, const int32_t* hq, int R, int C, int frac, int acc_bits,
                 int stage, void* y, hipStream_t stream, std::string* err) {
    if (stage != FIR_OUT_U8_SAT && stage != FIR_OUT_I32) return *err = "out_stage must be FIR_OUT_U8_SAT or FIR_OUT_I32", FIR_EINVAL;
    if (H < 0 || W < 0) return *err = "height and width must be >= 0", FIR_EINVAL;
    if (!hq) return *err = "hq must not be NULL", FIR_EINVAL;
    if (R < 1 || C < 1 || (int64_t)R * C > FIR_MAX_TAPS) return *err = "tap_rows*tap_cols must be in [1, 256]", FIR_EINVAL;
    if (frac < 1 || acc_bits < 1) return *err = "frac_bits and acc_bits must be >= 1", FIR_EINVAL;
    if (H == 0 || W == 0) return FIR_OK;
    if (!x || !y) return *err = "x and y must not be NULL", FIR_EINVAL;
    if (H > 65535 * (int64_t)kStrip) return *err = "height too large", FIR_EINVAL;
    bool taps24 = true;
    for (int k = 0; k < R * C; ++k) taps24 &= (hq[k] >= -(1 << 23) && hq[k] < (1 << 23));
    const bool fast = reg2d_shape(R, C) && W % 16 == 0 && (uintptr_t)x % 16 == 0 && (uintptr_t)y % 16 == 0 &&
                      acc_bits <= 32 && frac <= 31 && taps24 && W >= 16;
    hipError_t e;
    if (fast) {
        e = stage == FIR_OUT_U8_SAT ? launch2d_reg_shape<FIR_OUT_U8_SAT>(R, C, x, y, H, W, hq, frac, acc_bits, stream)
                                    : launch2d_reg_shape<FIR_OUT_I32>(R, C, x, y, H, W, hq, frac, acc_bits, stream);
    } else {
        if (H > 65535) return *err = "height > 65535 needs the fast path (W % 16 == 0)", FIR_EINVAL;
        Taps2G t;
        for (int k = 0; k < FIR_MAX_TAPS; ++k) t.h[k] = k < R * C ? hq[k] : 0;
        dim3 grid((unsigned)((W + kBlock - 1) / kBlock), (unsigned)H);
        if (stage == FIR_OUT_U8_SAT)
            hipLaunchKernelGGL((fir2d_generic_kernel<FIR_OUT_U8_SAT>), grid, dim3(kBlock), 0, stream, x, (uint8_t*)y, H,
                               W, t, R, C, frac, acc_bits);
        else
            hipLaunchKernelGGL((fir2d_generic_kernel<FIR_OUT_I32>), grid, dim3(kBlock), 0, stream, x, (int32_t*)y, H,
                               W, t, R, C, frac, acc_bits);
        e = hipGetLastError();
    }
    if (e != hipSuccess) return *err = std::string("fir2d launch failed: ") + hipGetErrorString(e), FIR_EHIP;
    return FIR_OK;
}

}  // namespace fir
