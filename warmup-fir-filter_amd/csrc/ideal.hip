// ideal.hip — float64 "ideal" model.
//
// Restates fir_1d/model/python/fir_1d_ref.py:43-65 per row (as driven by
// fir_1d/sim/vector/gen_ideal_output.py:37-50): acc = 0.0; for k in order:
// acc += h[k] * x[n - k + L/2] over in-row samples; no output clamp.  Bit-exactness
// needs the reference's rounding order: every product and every sum is rounded on its
// own (__dmul_rn / __dadd_rn, and the library is built with -ffp-contract=off), taps
// are summed in k order, and out-of-row terms contribute +0.0 (identical to skipping
// them: the running sum is never -0.0 because samples are >= 0).
//
// fir1d_ideal_reg_kernel (ideal_reg.h; L <= 9, aligned buffers): register/DPP layout.
// fir1d_ideal_kernel (any L, any alignment): 1024 outputs per workgroup, the taps walked in
// LDS chunks of 1024 (taps in HBM) with each output's running sum kept across chunks.
#include <string>

#include "fir_common.h"
#include "fir_launch.h"
#include "ideal_reg.h"

namespace fir {

constexpr int kIdealTile = 1024;
constexpr int kIdealChunk = 1024;  // taps (and window halo) per LDS chunk
constexpr int kIdealPer = kIdealTile / kBlock;

// Any L: the taps (device memory) are walked in chunks of kIdealChunk; each chunk stages its
// taps and the kIdealTile + kc - 1 samples they touch in LDS, and each thread carries its
// outputs' running sums across the chunks, so every sum is still formed in k order.
__global__ __launch_bounds__(kBlock) void fir1d_ideal_kernel(const uint8_t* __restrict__ x, double* __restrict__ y,
                                                             int64_t total, int64_t rowlen, int multi_row,
                                                             const double* __restrict__ taps, int L) {
    __shared__ double s_h[kIdealChunk];
    __shared__ int32_t s_x[kIdealTile + kIdealChunk];
    const int c = L / 2;
    const int64_t t0 = (int64_t)blockIdx.x * kIdealTile;
    const int64_t rl = multi_row ? rowlen : total;
    double acc[kIdealPer];
    int64_t col[kIdealPer];
#pragma unroll
    for (int j = 0; j < kIdealPer; ++j) {
        acc[j] = 0.0;
        const int64_t gi = t0 + threadIdx.x + j * kBlock;
        col[j] = multi_row ? gi % rowlen : gi;
    }
    for (int k0 = 0; k0 < L; k0 += kIdealChunk) {
        const int kc = min(kIdealChunk, L - k0);
        const int64_t w0 = t0 + (c - k0 - kc + 1);  // output i's tap k at window index i + kc - 1 - (k - k0)
        __syncthreads();
        for (int k = threadIdx.x; k < kc; k += kBlock) s_h[k] = taps[k0 + k];
        for (int i = threadIdx.x; i < kIdealTile + kc - 1; i += kBlock) {
            const int64_t gi = w0 + i;
            s_x[i] = (gi >= 0 && gi < total) ? (int32_t)x[gi] : 0;
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < kIdealPer; ++j) {
            const int i = threadIdx.x + j * kBlock;
            double a = acc[j];
            for (int k = 0; k < kc; ++k) {
                const int64_t d = c - k0 - k;
                const bool ok = col[j] + d >= 0 && col[j] + d < rl;
                const double xv = ok ? (double)s_x[i + kc - 1 - k] : 0.0;
                a = __dadd_rn(a, __dmul_rn(s_h[k], xv));
            }
            acc[j] = a;
        }
    }
#pragma unroll
    for (int j = 0; j < kIdealPer; ++j) {
        const int64_t gi = t0 + threadIdx.x + j * kBlock;
        if (gi < total) y[gi] = acc[j];
    }
}

// dwords (x4 u8 samples) per lane, outputs through LDS as whole 1 KiB non-temporal rows
// (394.5 -> 352.5 us, profiles/r01/micro_ideal_nts.txt).  One dword per lane (a wave: 256 B in,
// 2 KiB out) beats two (512 B in, 4 KiB out): 347.6 -> 337.6 us (profiles/r02/micro_ideal_nv1.txt);
// short waves keep more of the store stream in flight.
constexpr int kIdealNV = 1;

template <int L>
static hipError_t launch_ideal_reg(const uint8_t* x, double* y, int64_t rows, int64_t width, const double* h,
                                   hipStream_t stream) {
    TapsIdeal<L> t;
    for (int k = 0; k < L; ++k) t.h[k] = h[k];
    const int64_t total = rows * width;
    constexpr int VEC = 4 * kIdealNV;
    const int64_t vecs = (total + VEC - 1) / VEC;
    const int aligned = rows == 1 || width % VEC == 0;
    hipLaunchKernelGGL((fir1d_ideal_reg_kernel<L, kIdealNV, true, false, true>), dim3((unsigned)((vecs + kBlock - 1) / kBlock)),
                       dim3(kBlock), 0, stream, x, y, total, (uint32_t)(rows > 1 ? width : 0), rows > 1 ? 1 : 0,
                       aligned, t);
    return hipGetLastError();
}

int launch_fir1d_ideal(const uint8_t* x, int64_t rows, int64_t width, const double* h, int L, double* y,
                       hipStream_t stream, std::string* err) {
    if (rows < 0 || width < 0) return *err = "rows and width must be >= 0", FIR_EINVAL;
    if (!h) return *err = "h must not be NULL", FIR_EINVAL;
    if (L < 1 || L > FIR_MAX_TAPS) return *err = "taps must be in [1, " + std::to_string(FIR_MAX_TAPS) + "]", FIR_EINVAL;
    const int64_t total = rows * width;
    if (total == 0) return FIR_OK;
    if (!x || !y) return *err = "x and y must not be NULL", FIR_EINVAL;
    const bool reg = L <= 9 && (uintptr_t)x % (4 * kIdealNV) == 0 && (uintptr_t)y % 16 == 0 &&
                     (rows == 1 || (width >= 4 * kIdealNV + L - 1 && total < ((int64_t)1 << 32))) &&
                     (total + 4 * kIdealNV - 1) / (4 * kIdealNV) / kBlock < ((int64_t)1 << 31);
    if (reg) {
        hipError_t e = hipErrorInvalidValue;
        switch (L) {
            case 1: e = launch_ideal_reg<1>(x, y, rows, width, h, stream); break;
            case 2: e = launch_ideal_reg<2>(x, y, rows, width, h, stream); break;
            case 3: e = launch_ideal_reg<3>(x, y, rows, width, h, stream); break;
            case 4: e = launch_ideal_reg<4>(x, y, rows, width, h, stream); break;
            case 5: e = launch_ideal_reg<5>(x, y, rows, width, h, stream); break;
            case 6: e = launch_ideal_reg<6>(x, y, rows, width, h, stream); break;
            case 7: e = launch_ideal_reg<7>(x, y, rows, width, h, stream); break;
            case 8: e = launch_ideal_reg<8>(x, y, rows, width, h, stream); break;
            case 9: e = launch_ideal_reg<9>(x, y, rows, width, h, stream); break;
        }
        if (e != hipSuccess) return *err = std::string("ideal launch failed: ") + hipGetErrorString(e), FIR_EHIP;
        return FIR_OK;
    }
    const double* td = (const double*)device_table(h, sizeof(double) * (size_t)L, err);
    if (!td) return FIR_ENOMEM;
    TableHold hold(td, stream);
    const int64_t blocks = (total + kIdealTile - 1) / kIdealTile;
    if (blocks >= ((int64_t)1 << 31)) return *err = "too many samples for one launch", FIR_EINVAL;
    hipLaunchKernelGGL(fir1d_ideal_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, stream, x, y, total, width,
                       rows > 1 ? 1 : 0, td, L);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return *err = std::string("ideal launch failed: ") + hipGetErrorString(e), FIR_EHIP;
    return FIR_OK;
}

}  // namespace fir
