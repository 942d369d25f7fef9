// read_micro.hip — read-stream ceilings for the f64-input kernels (restore, metrics): dev
// tool, not the product.  2^28 doubles (2 GiB) read per launch with K 16-byte loads per
// lane in flight (whole-wave 1 KiB rows), nothing written; plus the restore
// kernel's own shape (8 loads, LDS byte transpose, 16-byte store) for comparison.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CK(e)                                                                              \
    do {                                                                                   \
        hipError_t _e = (e);                                                               \
        if (_e != hipSuccess) {                                                            \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #e, hipGetErrorString(_e)); \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

typedef double d2 __attribute__((ext_vector_type(2)));
constexpr int kBlock = 256;

template <int K, bool NT>
__global__ __launch_bounds__(kBlock) void read_k(const double* __restrict__ a, double* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
    const d2* p = reinterpret_cast<const d2*>(a) + wave * (64 * K);
    d2 v[K];
#pragma unroll
    for (int i = 0; i < K; ++i) v[i] = NT ? __builtin_nontemporal_load(p + i * 64 + lane) : p[i * 64 + lane];
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < K; ++i) s += v[i].x + v[i].y;
    if (s == 1234.5) out[threadIdx.x] = s;  // never true (a is zero): keeps the loads, writes nothing
}

template <int K, bool NT>
static void launch_read(const double* a, double* out, int64_t n, hipStream_t s) {
    const int64_t waves = n / (128 * K);
    hipLaunchKernelGGL((read_k<K, NT>), dim3((unsigned)(waves * 64 / kBlock)), dim3(kBlock), 0, s, a, out);
}

struct V {
    std::string name;
    void (*fn)(const double*, double*, int64_t, hipStream_t);
    std::vector<float> us;
};

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 15;
    const int64_t n = (int64_t)1 << 28;
    double *a, *out;
    CK(hipMalloc(&a, n * 8));
    CK(hipMalloc(&out, kBlock * sizeof(double)));  // written only under a never-true condition
    CK(hipMemset(a, 0, n * 8));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    std::vector<V> vs = {{"read K1", launch_read<1, false>, {}},   {"read K1 nt", launch_read<1, true>, {}},
                         {"read K2", launch_read<2, false>, {}},   {"read K2 nt", launch_read<2, true>, {}},
                         {"read K4 nt", launch_read<4, true>, {}},
                         {"read K4", launch_read<4, false>, {}},   {"read K8", launch_read<8, false>, {}},
                         {"read K16", launch_read<16, false>, {}}, {"read K32", launch_read<32, false>, {}},
                         {"read K8 nt", launch_read<8, true>, {}}, {"read K16 nt", launch_read<16, true>, {}}};
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int w = 0; w < 60; ++w) vs[w % vs.size()].fn(a, out, n, st);
    const int batch = 20;
    for (int r = 0; r < rounds; ++r)
        for (auto& v : vs) {
            CK(hipEventRecord(e0, st));
            for (int b = 0; b < batch; ++b) v.fn(a, out, n, st);
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            v.us.push_back(ms * 1e3f / batch);
        }
    printf("%-16s %10s %10s %10s %8s\n", "variant", "median_us", "min_us", "GB/s", "%8TB/s");
    for (auto& v : vs) {
        std::sort(v.us.begin(), v.us.end());
        const double med = v.us[v.us.size() / 2];
        printf("%-16s %10.1f %10.1f %10.1f %8.1f\n", v.name.c_str(), med, v.us[0], n * 8.0 / med / 1e3,
               n * 8.0 / med / 1e3 / 80.0);
    }
    return 0;
}
