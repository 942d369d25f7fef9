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
// fir1d_ideal_reg_kernel (L <= 9, aligned buffers): the fixed kernel's register/DPP layout.
// A lane owns NV consecutive dwords (4*NV u8 samples); the (L-1)-sample halo is one dword
// from each neighbouring lane by DPP wave shifts (lanes 0 / 63 load it); every sample is
// converted to f64 once and shared by the L outputs that use it; 16-byte f64 stores (8 of
// the 9 bytes per sample of HBM traffic).  Row edges: rows that are a whole number of
// vectors zero the halo dword that lies in the neighbouring row (a +-0.0 product leaves the
// running sum unchanged, exactly as skipping the term does); other widths mask per output.
// fir1d_ideal_kernel (any L, any alignment): LDS tile of 1024 outputs plus the halo.
#include <string>

#include "fir_common.h"
#include "fir_launch.h"

namespace fir {

constexpr int kIdealTile = 1024;

struct TapsF64 {
    double h[FIR_MAX_TAPS];
};

__global__ __launch_bounds__(kBlock) void fir1d_ideal_kernel(const uint8_t* __restrict__ x, double* __restrict__ y,
                                                             int64_t total, int64_t rowlen, int multi_row,
                                                             TapsF64 taps, int L) {
    __shared__ double s_h[FIR_MAX_TAPS];
    __shared__ int32_t s_x[kIdealTile + FIR_MAX_TAPS];
    const int c = L / 2;
    const int HLE = L - 1 - c, HRE = c;
    const int64_t t0 = (int64_t)blockIdx.x * kIdealTile;
    const int span = kIdealTile + HLE + HRE;
    for (int k = threadIdx.x; k < L; k += kBlock) s_h[k] = taps.h[k];
    for (int i = threadIdx.x; i < span; i += kBlock) {
        const int64_t gi = t0 - HLE + i;
        s_x[i] = (gi >= 0 && gi < total) ? (int32_t)x[gi] : 0;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kIdealTile; i += kBlock) {
        const int64_t gi = t0 + i;
        if (gi >= total) break;
        const int64_t col = multi_row ? gi % rowlen : gi;
        const int64_t rl = multi_row ? rowlen : total;
        double acc = 0.0;
        for (int k = 0; k < L; ++k) {
            const int d = c - k;
            const bool ok = col + d >= 0 && col + d < rl;
            const double xv = ok ? (double)s_x[HLE + i + d] : 0.0;
            acc = __dadd_rn(acc, __dmul_rn(s_h[k], xv));
        }
        y[gi] = acc;
    }
}

constexpr int kIdealNV = 1;  // dwords (x4 u8 samples) per lane

template <int L>
struct TapsIdeal {
    double h[L];
};

// NV dwords of u8 samples starting at dword index di (zero fill outside [0, total)).
template <int NV>
__device__ __forceinline__ void load_u8_dwords(const uint8_t* __restrict__ x, int64_t di, int64_t total,
                                               uint32_t (&d)[NV]) {
    const int64_t b0 = di * 4;
    if (di >= 0 && b0 + 4 * NV <= total) {
        typedef uint32_t vN __attribute__((ext_vector_type(NV)));
        if constexpr (NV == 1) {
            d[0] = *reinterpret_cast<const uint32_t*>(x + b0);
        } else {
            const vN q = *reinterpret_cast<const vN*>(x + b0);
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

template <int L, int NV>
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
    load_u8_dwords<NV>(x, v * NV, total, own);
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
    if (g0 >= total) return;
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
    if (g0 + VEC <= total) {
        typedef double d2 __attribute__((ext_vector_type(2)));
#pragma unroll
        for (int i = 0; i < VEC / 2; ++i) reinterpret_cast<d2*>(y + g0)[i] = d2{q[2 * i], q[2 * i + 1]};
    } else {
#pragma unroll
        for (int j = 0; j < VEC; ++j)
            if (g0 + j < total) y[g0 + j] = q[j];
    }
}

template <int L>
static hipError_t launch_ideal_reg(const uint8_t* x, double* y, int64_t rows, int64_t width, const double* h,
                                   hipStream_t stream) {
    TapsIdeal<L> t;
    for (int k = 0; k < L; ++k) t.h[k] = h[k];
    const int64_t total = rows * width;
    constexpr int VEC = 4 * kIdealNV;
    const int64_t vecs = (total + VEC - 1) / VEC;
    const int aligned = rows == 1 || width % VEC == 0;
    hipLaunchKernelGGL((fir1d_ideal_reg_kernel<L, kIdealNV>), dim3((unsigned)((vecs + kBlock - 1) / kBlock)),
                       dim3(kBlock), 0, stream, x, y, total, (uint32_t)(rows > 1 ? width : 0), rows > 1 ? 1 : 0,
                       aligned, t);
    return hipGetLastError();
}

int launch_fir1d_ideal(const uint8_t* x, int64_t rows, int64_t width, const double* h, int L, double* y,
                       hipStream_t stream, std::string* err) {
    if (rows < 0 || width < 0) return *err = "rows and width must be >= 0", FIR_EINVAL;
    if (!h) return *err = "h must not be NULL", FIR_EINVAL;
    if (L < 1 || L > FIR_MAX_TAPS) return *err = "taps must be in [1, 256]", FIR_EINVAL;
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
    TapsF64 t;
    for (int k = 0; k < FIR_MAX_TAPS; ++k) t.h[k] = k < L ? h[k] : 0.0;
    const int64_t blocks = (total + kIdealTile - 1) / kIdealTile;
    hipLaunchKernelGGL(fir1d_ideal_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, stream, x, y, total, width,
                       rows > 1 ? 1 : 0, t, L);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return *err = std::string("ideal launch failed: ") + hipGetErrorString(e), FIR_EHIP;
    return FIR_OK;
}

}  // namespace fir
