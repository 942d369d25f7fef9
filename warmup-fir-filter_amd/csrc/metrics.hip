// metrics.hip — fixed-vs-ideal comparison metrics in one pass over HBM.
//
// Restates fir_1d/sim/vector/gen_3tap_compare_report.py:67-112 (_compute_metrics): with
// d = fixed - ideal (float64), it needs max|d|, sum|d|, sum d^2, sum d, #(fixed == 0),
// #(fixed == 255) and #(ideal < 0 or ideal > 255).  The reference takes each from a
// separate NumPy reduction (seven passes over 9 bytes/sample); here one kernel reads
// each sample once.  Sums are float64: plain per 8-sample tile, Neumaier-compensated across
// tiles per thread, then a fixed reduction order (per-block tree, then one block over the
// partials), so results are deterministic run to run; they differ from NumPy's pairwise
// summation only in the last bits (tests use a 1e-12 relative tolerance).  Counts and
// max|d| are exact.
#include <string>

#include "fir_common.h"
#include "fir_launch.h"

namespace fir {

// 2048 blocks (8192 waves, 32 per CU) over 4096: 359 -> 356 / 369 -> 362 us in two same-process
// A/Bs; 1024 blocks, 8 or 4 loads per tile, the next tile's loads issued before the arithmetic
// (+3-5 %), and the fixed bytes as whole rows through LDS gained nothing
// (profiles/r02/ab_restore_metrics.txt).  FIR_METRIC_*: A/B builds only.
#ifndef FIR_METRIC_BLOCKS
#define FIR_METRIC_BLOCKS 2048
#endif
#ifndef FIR_METRIC_LOADS
#define FIR_METRIC_LOADS 16
#endif

constexpr int kMetricBlocks = FIR_METRIC_BLOCKS;

struct Part {
    double sabs, cabs, ssq, csq, sd, cd, mx;
    unsigned long long lo, hi, clip;
};

__device__ __forceinline__ void neu_add(double& s, double& c, double v) {
    const double t = __dadd_rn(s, v);
    c = __dadd_rn(c, fabs(s) >= fabs(v) ? __dadd_rn(__dsub_rn(s, t), v) : __dadd_rn(__dsub_rn(v, t), s));
    s = t;
}

__device__ void reduce_block(Part& p) {
    __shared__ Part sh[kBlock];
    sh[threadIdx.x] = p;
    __syncthreads();
    for (int w = kBlock / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w) {
            Part& a = sh[threadIdx.x];
            const Part& b = sh[threadIdx.x + w];
            neu_add(a.sabs, a.cabs, b.sabs);
            a.cabs = __dadd_rn(a.cabs, b.cabs);
            neu_add(a.ssq, a.csq, b.ssq);
            a.csq = __dadd_rn(a.csq, b.csq);
            neu_add(a.sd, a.cd, b.sd);
            a.cd = __dadd_rn(a.cd, b.cd);
            a.mx = fmax(a.mx, b.mx);
            a.lo += b.lo;
            a.hi += b.hi;
            a.clip += b.clip;
        }
        __syncthreads();
    }
    p = sh[0];
}

// One sample's terms: |d| and d^2 and d into the tile partials, max and the three counts.
__device__ __forceinline__ void metrics_term(double id, uint32_t fx, double& sabs, double& ssq, double& sd,
                                             double& mx, uint32_t& lo, uint32_t& hi, uint32_t& clip) {
    const double d = __dsub_rn((double)fx, id);
    const double ad = fabs(d);
    sabs = __dadd_rn(sabs, ad);
    ssq = __dadd_rn(ssq, __dmul_rn(d, d));
    sd = __dadd_rn(sd, d);
    mx = fmax(mx, ad);
    lo += fx == 0;
    hi += fx == 255;
    clip += (id < 0.0) | (id > 255.0);
}

// VEC (ideal 16-byte and fixed 2-byte aligned): a wave reads tiles of kMetricTile samples as
// whole 1 KiB f64 rows plus 128 B u8 rows, 16 non-temporal f64 loads in flight per lane
// (the read-stream A/B, tools/microbench/read_micro.hip); each lane sums its 32 samples of
// a tile plainly and adds the tile partials into its Neumaier-compensated accumulators
// (a compensated add per sample made the kernel latency-bound).  The ragged tail and
// unaligned inputs take the per-sample grid-stride loop.
constexpr int kMetricLoads = FIR_METRIC_LOADS;
constexpr int kMetricTile = kMetricLoads * kWave * 2;

template <bool VEC>
__global__ __launch_bounds__(kBlock) void metrics_pass1(const double* __restrict__ ideal,
                                                        const uint8_t* __restrict__ fixed, int64_t n,
                                                        Part* __restrict__ parts) {
    typedef double d2 __attribute__((ext_vector_type(2)));
    Part p{0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    double mx = 0.0;
    uint32_t lo = 0, hi = 0, clip = 0;
    int64_t start = 0;
    if constexpr (VEC) {
        const int lane = threadIdx.x & (kWave - 1);
        const int64_t ntile = n / kMetricTile;
        const int64_t nwaves = (int64_t)gridDim.x * (kBlock / kWave);
        auto load_tile = [&](int64_t t, d2 (&a)[kMetricLoads], uint32_t (&f)[kMetricLoads]) {
            const d2* pi = reinterpret_cast<const d2*>(ideal + t * kMetricTile);
            const uint16_t* pf = reinterpret_cast<const uint16_t*>(fixed + t * kMetricTile);
#pragma unroll
            for (int i = 0; i < kMetricLoads; ++i) {
                a[i] = __builtin_nontemporal_load(pi + i * kWave + lane);
                f[i] = __builtin_nontemporal_load(pf + i * kWave + lane);
            }
        };
        auto tile_sums = [&](const d2 (&a)[kMetricLoads], const uint32_t (&f)[kMetricLoads]) {
            double sabs = 0.0, ssq = 0.0, sd = 0.0;
#pragma unroll
            for (int i = 0; i < kMetricLoads; ++i) {
                metrics_term(a[i].x, f[i] & 0xFFu, sabs, ssq, sd, mx, lo, hi, clip);
                metrics_term(a[i].y, f[i] >> 8, sabs, ssq, sd, mx, lo, hi, clip);
            }
            neu_add(p.sabs, p.cabs, sabs);
            neu_add(p.ssq, p.csq, ssq);
            neu_add(p.sd, p.cd, sd);
        };
        for (int64_t t = (int64_t)blockIdx.x * (kBlock / kWave) + (threadIdx.x >> 6); t < ntile; t += nwaves) {
            d2 a[kMetricLoads];
            uint32_t f[kMetricLoads];
            load_tile(t, a, f);
            tile_sums(a, f);
        }
        start = ntile * kMetricTile;
    }
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t i = start + (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
        double sabs = 0.0, ssq = 0.0, sd = 0.0;
        metrics_term(ideal[i], fixed[i], sabs, ssq, sd, mx, lo, hi, clip);
        neu_add(p.sabs, p.cabs, sabs);
        neu_add(p.ssq, p.csq, ssq);
        neu_add(p.sd, p.cd, sd);
    }
    p.mx = mx;
    p.lo = lo;
    p.hi = hi;
    p.clip = clip;
    reduce_block(p);
    if (threadIdx.x == 0) parts[blockIdx.x] = p;
}

// out: [max_abs, sum_abs, sum_sq, sum_d, n_low, n_high, n_clip, n, 0]
__global__ __launch_bounds__(kBlock) void metrics_pass2(const Part* __restrict__ parts, int nparts, int64_t n,
                                                        double* __restrict__ out) {
    Part p{0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = threadIdx.x; i < nparts; i += kBlock) {  // fixed order per thread
        const Part& b = parts[i];
        neu_add(p.sabs, p.cabs, b.sabs);
        p.cabs = __dadd_rn(p.cabs, b.cabs);
        neu_add(p.ssq, p.csq, b.ssq);
        p.csq = __dadd_rn(p.csq, b.csq);
        neu_add(p.sd, p.cd, b.sd);
        p.cd = __dadd_rn(p.cd, b.cd);
        p.mx = fmax(p.mx, b.mx);
        p.lo += b.lo;
        p.hi += b.hi;
        p.clip += b.clip;
    }
    reduce_block(p);
    if (threadIdx.x == 0) {
        out[0] = p.mx;
        out[1] = __dadd_rn(p.sabs, p.cabs);
        out[2] = __dadd_rn(p.ssq, p.csq);
        out[3] = __dadd_rn(p.sd, p.cd);
        out[4] = (double)p.lo;
        out[5] = (double)p.hi;
        out[6] = (double)p.clip;
        out[7] = (double)n;
        out[8] = 0.0;
    }
}

size_t metrics_work_bytes() { return sizeof(Part) * kMetricBlocks; }

int launch_metrics(const double* ideal, const uint8_t* fixed, int64_t n, double* out, void* work,
                   hipStream_t stream, std::string* err) {
    if (n < 0) return *err = "n must be >= 0", FIR_EINVAL;
    if (!out || !work || (n > 0 && (!ideal || !fixed))) return *err = "null pointer argument", FIR_EINVAL;
    int64_t want = (n + kBlock - 1) / kBlock;
    const int blocks = (int)(want < 1 ? 1 : (want > kMetricBlocks ? kMetricBlocks : want));
    if ((uintptr_t)ideal % 16 == 0 && (uintptr_t)fixed % 2 == 0)
        hipLaunchKernelGGL(metrics_pass1<true>, dim3(blocks), dim3(kBlock), 0, stream, ideal, fixed, n, (Part*)work);
    else
        hipLaunchKernelGGL(metrics_pass1<false>, dim3(blocks), dim3(kBlock), 0, stream, ideal, fixed, n, (Part*)work);
    hipLaunchKernelGGL(metrics_pass2, dim3(1), dim3(kBlock), 0, stream, (const Part*)work, blocks, n, out);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return *err = std::string("metrics launch failed: ") + hipGetErrorString(e), FIR_EHIP;
    return FIR_OK;
}

}  // namespace fir
