// metrics.hip — fixed-vs-ideal comparison metrics in one pass over HBM.
//
// Restates fir_1d/sim/vector/gen_3tap_compare_report.py:67-112 (_compute_metrics): with
// d = fixed - ideal (float64), it needs max|d|, sum|d|, sum d^2, sum d, #(fixed == 0),
// #(fixed == 255) and #(ideal < 0 or ideal > 255).  The reference takes each from a
// separate NumPy reduction (seven passes over 9 bytes/sample); here one kernel reads
// each sample once.  Sums are float64 with Neumaier compensation per thread and a fixed
// reduction order (per-block tree, then one block over the partials), so results are
// deterministic run to run; they differ from NumPy's pairwise summation only in the last
// bits (tests use a 1e-12 relative tolerance).  Counts and max|d| are exact.
#include <string>

#include "fir_common.h"
#include "fir_launch.h"

namespace fir {

constexpr int kMetricBlocks = 1024;

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

__global__ __launch_bounds__(kBlock) void metrics_pass1(const double* __restrict__ ideal,
                                                        const uint8_t* __restrict__ fixed, int64_t n,
                                                        Part* __restrict__ parts) {
    Part p{0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
        const double id = ideal[i];
        const uint8_t fx = fixed[i];
        const double d = __dsub_rn((double)fx, id);
        const double ad = fabs(d);
        neu_add(p.sabs, p.cabs, ad);
        neu_add(p.ssq, p.csq, __dmul_rn(d, d));
        neu_add(p.sd, p.cd, d);
        p.mx = fmax(p.mx, ad);
        p.lo += fx == 0;
        p.hi += fx == 255;
        p.clip += (id < 0.0) | (id > 255.0);
    }
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
    hipLaunchKernelGGL(metrics_pass1, dim3(blocks), dim3(kBlock), 0, stream, ideal, fixed, n, (Part*)work);
    hipLaunchKernelGGL(metrics_pass2, dim3(1), dim3(kBlock), 0, stream, (const Part*)work, blocks, n, out);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return *err = std::string("metrics launch failed: ") + hipGetErrorString(e), FIR_EHIP;
    return FIR_OK;
}

}  // namespace fir
