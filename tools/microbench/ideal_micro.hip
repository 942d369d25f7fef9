// ideal_micro.hip — A/B microbenchmark for the f64 ideal kernel (dev tool, not the product).
// Variants of fir1d_ideal_reg_kernel<5, NV> (dwords per lane) on 2^28 u8 samples in rows of
// 4096, batches of back-to-back launches interleaved round-robin; each variant's full output
// is checked bit-exactly against a CPU evaluation in the reference's rounding order.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "ideal_reg.h"

using namespace fir;

#define CK(e)                                                                              \
    do {                                                                                   \
        hipError_t _e = (e);                                                               \
        if (_e != hipSuccess) {                                                            \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #e, hipGetErrorString(_e)); \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

static const double kH[5] = {-1.0 / 16, -4.0 / 16, 26.0 / 16, -4.0 / 16, -1.0 / 16};
static const int64_t kW = 4096;

template <int NV, bool COAL, bool NTL = false, bool NTS = false>
static void launch(const uint8_t* x, double* y, int64_t total, hipStream_t s) {
    TapsIdeal<5> t;
    for (int k = 0; k < 5; ++k) t.h[k] = kH[k];
    const int64_t vecs = (total + 4 * NV - 1) / (4 * NV);
    hipLaunchKernelGGL((fir1d_ideal_reg_kernel<5, NV, COAL, NTL, NTS>), dim3((unsigned)((vecs + kBlock - 1) / kBlock)),
                       dim3(kBlock), 0, s, x, y, total, (uint32_t)kW, 1, 1, t);
}

// Store-only ceilings: 4 doubles per lane, lane-strided (as the kernel) or wave-contiguous.
template <bool COAL>
__global__ __launch_bounds__(kBlock) void store_only(double* __restrict__ y, int64_t total) {
    typedef double d2 __attribute__((ext_vector_type(2)));
    const int64_t v = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const int lane = threadIdx.x & 63;
    const double a = (double)v;
    d2* p = reinterpret_cast<d2*>(y);
    if (COAL) {
        const int64_t w0 = (v - lane) * 2;
        p[w0 + lane] = d2{a, a};
        p[w0 + 64 + lane] = d2{a, a};
    } else {
        p[2 * v] = d2{a, a};
        p[2 * v + 1] = d2{a, a};
    }
}
template <bool COAL>
static void launch_store(const uint8_t*, double* y, int64_t total, hipStream_t s) {
    hipLaunchKernelGGL((store_only<COAL>), dim3((unsigned)(total / 4 / kBlock)), dim3(kBlock), 0, s, y, total);
}

struct V {
    std::string name;
    void (*fn)(const uint8_t*, double*, int64_t, hipStream_t);
    std::vector<float> us;
};

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 15;
    const int64_t total = (int64_t)1 << 28, rows = total / kW;
    std::vector<uint8_t> hx(total);
    uint64_t s = 88172645463325252ull;
    for (auto& v : hx) {
        s ^= s << 13, s ^= s >> 7, s ^= s << 17;
        v = (uint8_t)s;
    }
    std::vector<double> ref(total), got(total);
    for (int64_t r = 0; r < rows; ++r)
        for (int64_t n = 0; n < kW; ++n) {
            volatile double acc = 0.0;
            for (int k = 0; k < 5; ++k) {
                const int64_t j = n - k + 2;
                volatile double p = kH[k] * (j >= 0 && j < kW ? (double)hx[r * kW + j] : 0.0);
                acc = acc + p;
            }
            ref[r * kW + n] = acc;
        }
    uint8_t* dx;
    double* dy;
    CK(hipMalloc(&dx, total));
    CK(hipMalloc(&dy, total * 8));
    CK(hipMemcpy(dx, hx.data(), total, hipMemcpyHostToDevice));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    std::vector<V> vs = {{"NV2 coal ntst (lib)", launch<2, true, false, true>, {}},
                         {"NV1 coal ntst", launch<1, true, false, true>, {}},
                         {"NV1 coal ntld+st", launch<1, true, true, true>, {}},
                         {"NV1 coal", launch<1, true>, {}},
                         {"NV2 coal ntst (lib) b", launch<2, true, false, true>, {}},
                         {"store-only strided", launch_store<false>, {}},
                         {"store-only coal", launch_store<true>, {}}};
    const size_t nchecked = 5;
    for (size_t vi = 0; vi < nchecked; ++vi) {
        auto& v = vs[vi];
        CK(hipMemset(dy, 0xFF, total * 8));
        v.fn(dx, dy, total, st);
        CK(hipStreamSynchronize(st));
        CK(hipMemcpy(got.data(), dy, total * 8, hipMemcpyDeviceToHost));
        int64_t bad = 0;
        for (int64_t i = 0; i < total; ++i) bad += memcmp(&got[i], &ref[i], 8) != 0;
        printf("check %s %s (%lld bad)\n", v.name.c_str(), bad ? "FAIL" : "ok", (long long)bad);
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int w = 0; w < 60; ++w) vs[w % vs.size()].fn(dx, dy, total, st);
    const int batch = 20;
    for (int r = 0; r < rounds; ++r)
        for (auto& v : vs) {
            CK(hipEventRecord(e0, st));
            for (int b = 0; b < batch; ++b) v.fn(dx, dy, total, st);
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            v.us.push_back(ms * 1e3f / batch);
        }
    printf("%-20s %10s %10s %10s\n", "variant", "median_us", "min_us", "GB/s(alg)");
    for (auto& v : vs) {
        std::sort(v.us.begin(), v.us.end());
        const double med = v.us[v.us.size() / 2];
        printf("%-20s %10.1f %10.1f %10.1f\n", v.name.c_str(), med, v.us[0], total * 9.0 / med / 1e3);
    }
    return 0;
}
