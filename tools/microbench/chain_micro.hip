// chain_micro.hip — dependent float64 add chains on one wave (dev tool for metrics.hip's
// in-order block-sum chain): ns per dependent add, plain VGPR operand vs v_readlane-fed SGPR.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(e)                                                                              \
    do {                                                                                   \
        hipError_t _e = (e);                                                               \
        if (_e != hipSuccess) {                                                            \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(_e));      \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

constexpr int kN = 1 << 16;

__device__ double lane_d(double v, int j) {
    const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b, j);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b >> 32), j);
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

template <int MODE>
__global__ void chain(const double* x, double* out) {
    __shared__ double sh[64];
    const int lane = threadIdx.x;
    double s = 0.0, s2 = 0.0, s3 = 0.0;
    const double v = x[lane];
    sh[lane] = v;
    __syncthreads();
    for (int it = 0; it < kN / 64; ++it) {
#pragma unroll
        for (int j = 0; j < 64; ++j) {
            if constexpr (MODE == 0) s = __dadd_rn(s, v);            // VGPR operand
            if constexpr (MODE == 1) s = __dadd_rn(s, lane_d(v, j));  // readlane-fed
            if constexpr (MODE == 2) {                                // three chains
                const double w = lane_d(v, j);
                s = __dadd_rn(s, w), s2 = __dadd_rn(s2, w * 2.0), s3 = __dadd_rn(s3, w * 3.0);
            }
            if constexpr (MODE == 3) s = (double)((float)s + (float)v);  // f32 reference
            if constexpr (MODE == 4) s = __dadd_rn(s, sh[j]);           // LDS broadcast-fed
        }
    }
    out[lane] = s + s2 + s3;
}

template <int MODE>
float run(const double* x, double* o) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(chain<MODE>, dim3(1), dim3(64), 0, 0, x, o);
    CK(hipEventRecord(a, 0));
    hipLaunchKernelGGL(chain<MODE>, dim3(1), dim3(64), 0, 0, x, o);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms * 1e6f / kN;
}

int main() {
    double *x, *o;
    CK(hipMalloc(&x, 64 * sizeof(double)));
    CK(hipMalloc(&o, 64 * sizeof(double)));
    CK(hipMemset(x, 0, 64 * sizeof(double)));
    printf("ns per dependent step: f64 VGPR %.2f, f64 readlane-fed %.2f, 3 chains readlane-fed %.2f, f32-ish %.2f, "
           "f64 LDS-broadcast-fed %.2f\n", run<0>(x, o), run<1>(x, o), run<2>(x, o), run<3>(x, o), run<4>(x, o));
    return 0;
}
