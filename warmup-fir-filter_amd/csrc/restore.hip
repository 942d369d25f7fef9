// restore.hip — f64 -> u8 image conversions of the restore stage.
//
// Restates fir_1d/sim/vector/restore_images.py:51-64:
//   clip       np.clip(np.rint(a), 0, 255).astype(np.uint8)                      (:51-54)
//   normalize  lo, hi = a.min(), a.max(); zeros if hi <= lo, else
//              np.rint(np.clip((a - lo) * (255.0 / (hi - lo)), 0, 255)).astype(np.uint8)  (:57-64)
// rint is round-half-even (v_rndne_f64); for finite inputs rint-then-clip and
// clip-then-rint give the same byte, so one converter serves both.  (a - lo) and the
// product are rounded separately as in NumPy (-ffp-contract=off); the scale 255/(hi-lo)
// is formed once on the device.  NaN maps to 0 (NumPy's cast of NaN is unspecified).
//
// HBM layout: a wave converts 128*K consecutive doubles with whole-wave 1 KiB non-temporal
// loads (lane-interleaved 16-byte pairs, K = 2 per lane), then transposes its result bytes
// through LDS so every store instruction writes one contiguous row.  normalize adds a
// min/max pass (grid-stride, per-block tree, one final block) ahead of the same map.
#include <algorithm>
#include <string>

#include "fir_common.h"
#include "fir_launch.h"

namespace fir {

constexpr int kRestoreBlocks = 1024;
// 2 non-temporal 16-byte loads per lane (256 doubles, 256 result bytes per wave): many short
// waves keep more of the read stream in flight than few long ones.  Same-process A/B over
// 2^28 doubles (profiles/r02/ab_restore_metrics.txt): 16 loads 372-397 us, 8: 366, 4: 361-376,
// 2: 354-363, 1: 389; the 2 GiB read-only ceiling is 301 us at 1-2 loads per lane
// (profiles/r02/read_ceiling_2gib.txt).  The result bytes are stored plainly (non-temporal
// stores: 394 -> 415 us, profiles/r01/nts_ab_benches.txt).
constexpr int kRestoreLoads = 2;
static_assert(kRestoreLoads <= 4 || kRestoreLoads % 8 == 0, "restore loads per lane");
constexpr int kRestorePerWave = 2 * kWave * kRestoreLoads;

struct RestoreParams {
    double lo, scale;
    int zero;  // hi <= lo: all zeros
};

__device__ __forceinline__ uint32_t to_u8(double v) {
    if (!(v == v)) return 0u;
    const double r = __builtin_rint(fmin(fmax(v, 0.0), 255.0));
    return (uint32_t)(int)r;
}

__device__ __forceinline__ uint32_t conv(double a, bool norm, const RestoreParams& p) {
    if (!norm) return to_u8(a);
    if (p.zero) return 0u;
    return to_u8(__dmul_rn(__dsub_rn(a, p.lo), p.scale));
}

template <bool NORM>
__global__ __launch_bounds__(kBlock) void restore_map_kernel(const double* __restrict__ a, int64_t n,
                                                             uint8_t* __restrict__ out,
                                                             const RestoreParams* __restrict__ pp) {
    typedef double d2 __attribute__((ext_vector_type(2)));
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    constexpr int K = kRestoreLoads;
    RestoreParams p{0.0, 1.0, 0};
    if (NORM) p = *pp;
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t base = ((int64_t)blockIdx.x * (kBlock / kWave) + (threadIdx.x >> 6)) * kRestorePerWave;
    if (base >= n) return;
    if (base + kRestorePerWave <= n) {
        __shared__ uint16_t sb[kBlock * K];
        uint16_t* wb = sb + (threadIdx.x - lane) * K;
        const d2* src = reinterpret_cast<const d2*>(a + base);
        d2 v[K];
#pragma unroll
        for (int i = 0; i < K; ++i) v[i] = __builtin_nontemporal_load(src + i * kWave + lane);  // read once
#pragma unroll
        for (int i = 0; i < K; ++i)
            wb[i * kWave + lane] = (uint16_t)(conv(v[i].x, NORM, p) | (conv(v[i].y, NORM, p) << 8));
        __builtin_amdgcn_wave_barrier();  // one wave's LDS ops complete in order
        asm volatile("" ::: "memory");
        // the wave's 128*K result bytes as whole rows: 16 (K >= 8), 8, 4 or 2 (K = 4, 2, 1) bytes per lane
        if constexpr (K >= 8) {
#pragma unroll
            for (int i = 0; i < K / 8; ++i) {  // plain stores: non-temporal ones measured 394 -> 415 us
                u32x4* dst = reinterpret_cast<u32x4*>(out + base) + i * kWave + lane;
                const u32x4 val = reinterpret_cast<const u32x4*>(wb)[i * kWave + lane];
                *dst = val;
            }
        } else if constexpr (K == 4) {
            typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
            reinterpret_cast<u32x2*>(out + base)[lane] = reinterpret_cast<const u32x2*>(wb)[lane];
        } else if constexpr (K == 2) {
            reinterpret_cast<uint32_t*>(out + base)[lane] = reinterpret_cast<const uint32_t*>(wb)[lane];
        } else {
            static_assert(K == 1, "restore loads per lane");
            reinterpret_cast<uint16_t*>(out + base)[lane] = wb[lane];
        }
    } else {
        for (int64_t e = base + lane; e < n; e += kWave) out[e] = (uint8_t)conv(a[e], NORM, p);
    }
}

__global__ __launch_bounds__(kBlock) void restore_minmax_kernel(const double* __restrict__ a, int64_t n,
                                                                double* __restrict__ parts) {
    __shared__ double smin[kBlock], smax[kBlock];
    double lo = __builtin_inf(), hi = -__builtin_inf();
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
        const double v = a[i];
        lo = fmin(lo, v);
        hi = fmax(hi, v);
    }
    smin[threadIdx.x] = lo;
    smax[threadIdx.x] = hi;
    __syncthreads();
    for (int w = kBlock / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w) {
            smin[threadIdx.x] = fmin(smin[threadIdx.x], smin[threadIdx.x + w]);
            smax[threadIdx.x] = fmax(smax[threadIdx.x], smax[threadIdx.x + w]);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        parts[2 * blockIdx.x] = smin[0];
        parts[2 * blockIdx.x + 1] = smax[0];
    }
}

__global__ __launch_bounds__(kBlock) void restore_params_kernel(const double* __restrict__ parts, int nparts,
                                                                RestoreParams* __restrict__ pp) {
    __shared__ double smin[kBlock], smax[kBlock];
    double lo = __builtin_inf(), hi = -__builtin_inf();
    for (int i = threadIdx.x; i < nparts; i += kBlock) {
        lo = fmin(lo, parts[2 * i]);
        hi = fmax(hi, parts[2 * i + 1]);
    }
    smin[threadIdx.x] = lo;
    smax[threadIdx.x] = hi;
    __syncthreads();
    for (int w = kBlock / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w) {
            smin[threadIdx.x] = fmin(smin[threadIdx.x], smin[threadIdx.x + w]);
            smax[threadIdx.x] = fmax(smax[threadIdx.x], smax[threadIdx.x + w]);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const double l = smin[0], h = smax[0];
        pp->lo = l;
        pp->zero = !(h > l);
        pp->scale = h > l ? __ddiv_rn(255.0, __dsub_rn(h, l)) : 1.0;
    }
}

size_t restore_work_bytes() { return 256 + (size_t)kRestoreBlocks * 2 * sizeof(double); }

int launch_restore_u8(const double* a, int64_t n, int policy, uint8_t* out, void* work, hipStream_t stream,
                      std::string* err) {
    if (n < 0) return *err = "n must be >= 0", FIR_EINVAL;
    if (policy != FIR_RESTORE_CLIP && policy != FIR_RESTORE_NORMALIZE)
        return *err = "policy must be FIR_RESTORE_CLIP or FIR_RESTORE_NORMALIZE", FIR_EINVAL;
    if (n == 0) return FIR_OK;
    if (!a || !out) return *err = "a and out must not be NULL", FIR_EINVAL;
    if ((uintptr_t)a % 16 || (uintptr_t)out % 16) return *err = "a and out must be 16-byte aligned", FIR_EINVAL;
    const int64_t waves = (n + kRestorePerWave - 1) / kRestorePerWave;
    const dim3 grid((unsigned)((waves + kBlock / kWave - 1) / (kBlock / kWave)));
    if (policy == FIR_RESTORE_CLIP) {
        hipLaunchKernelGGL((restore_map_kernel<false>), grid, dim3(kBlock), 0, stream, a, n, out, nullptr);
    } else {
        if (!work) return *err = "work must not be NULL for FIR_RESTORE_NORMALIZE", FIR_EINVAL;
        RestoreParams* pp = reinterpret_cast<RestoreParams*>(work);
        double* parts = reinterpret_cast<double*>((char*)work + 256);
        const int nb = (int)std::min<int64_t>(kRestoreBlocks, (n + kBlock - 1) / kBlock);
        hipLaunchKernelGGL(restore_minmax_kernel, dim3(nb), dim3(kBlock), 0, stream, a, n, parts);
        hipLaunchKernelGGL(restore_params_kernel, dim3(1), dim3(kBlock), 0, stream, parts, nb, pp);
        hipLaunchKernelGGL((restore_map_kernel<true>), grid, dim3(kBlock), 0, stream, a, n, out, pp);
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return *err = std::string("restore launch failed: ") + hipGetErrorString(e), FIR_EHIP;
    return FIR_OK;
}

}  // namespace fir
