// fir_u8_micro.hip — A/B microbenchmark for the 1:1 u8 -> sat-u8 path (dev tool, not the
// product): fir1d_reg_kernel<u8, U8_SAT, 5> with U chunks per wave over 2^28 samples in
// 4096-sample rows, next to plain 16-byte copies with the same layouts and hipMemcpy; and
// the fused 4-filter 3-tap bank (1 B in, 4 B out per sample), byte-pair v_dot2 vs the
// per-filter packed-16 form.  Every FIR variant's full output is checked against a CPU evaluation.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "fir1d_reg.h"

using namespace fir;

#define CK(e)                                                                              \
    do {                                                                                   \
        hipError_t _e = (e);                                                               \
        if (_e != hipSuccess) {                                                            \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #e, hipGetErrorString(_e)); \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

static const int32_t kTaps[5] = {-256, -1024, 6656, -1024, -256};
static const int64_t kW = 4096;

template <int U, int FLAGS, bool ONEROW = false>
static void launch_fir(const uint8_t* x, uint8_t* y, int64_t n, hipStream_t s) {
    RowGeom g{n, ONEROW ? 0u : (uint32_t)kW, ONEROW ? 0 : 1, 1};
    TapsN<5> t;
    for (int k = 0; k < 5; ++k) t.h[0][k] = kTaps[k];
    pack_taps(t);
    if ((FLAGS & kU8Pk16) && plan_u8_pk16(t, 12) != (FLAGS & (kU8Pk16 | kU8PkHi8))) {
        fprintf(stderr, "pk16 plan mismatch\n");
        exit(1);
    }
    int64_t ntiles, blocks;
    reg_launch_geometry<uint8_t, U, FLAGS>(n, 2048, &ntiles, &blocks);
    hipLaunchKernelGGL((fir1d_reg_kernel<uint8_t, FIR_OUT_U8_SAT, 5, 1, U, FLAGS>), dim3((unsigned)blocks),
                       dim3(kBlock), 0, s, x, y, g, t, 0, 12, ntiles);
}

// BANK3 of the reference (h_coeff.py): moving_avg, simple_lp, edge, sharpen in Q4.12
static const int32_t kBank[4][3] = {{1365, 1365, 1365}, {1024, 2048, 1024}, {-4096, 0, 4096}, {-512, 5120, -512}};

template <int U, int FLAGS>
static void launch_bank(const uint8_t* x, uint8_t* y, int64_t n, hipStream_t s) {
    RowGeom g{n, (uint32_t)kW, 1, 1};
    TapsN<3, 4> t;
    for (int f = 0; f < 4; ++f)
        for (int k = 0; k < 3; ++k) t.h[f][k] = kBank[f][k];
    pack_taps(t);
    if ((FLAGS & kU8Pk16) && plan_u8_pk16(t, 12) != kU8Pk16) {
        fprintf(stderr, "bank pk16 plan mismatch\n");
        exit(1);
    }
    int64_t ntiles, blocks;
    reg_launch_geometry<uint8_t, U, FLAGS>(n, 2048, &ntiles, &blocks);
    hipLaunchKernelGGL((fir1d_reg_kernel<uint8_t, FIR_OUT_U8_SAT, 3, 1, U, FLAGS, 4>), dim3((unsigned)blocks),
                       dim3(kBlock), 0, s, x, y, g, t, 0, 12, ntiles);
}

template <int U, bool NT = false>
__global__ __launch_bounds__(kBlock) void copy16(const uint8_t* __restrict__ x, uint8_t* __restrict__ y, int64_t nvec) {
    typedef uint32_t v4 __attribute__((ext_vector_type(4)));
    const int lane = threadIdx.x & 63;
    const int64_t w = ((int64_t)blockIdx.x * kBlock + threadIdx.x - lane) * U;  // wave's first vector
    v4 d[U];
#pragma unroll
    for (int u = 0; u < U; ++u) d[u] = reinterpret_cast<const v4*>(x)[w + u * 64 + lane];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        v4* p = reinterpret_cast<v4*>(y) + w + u * 64 + lane;
        if (NT) __builtin_nontemporal_store(d[u], p); else *p = d[u];
    }
}
template <int U, bool NT = false>
static void launch_copy(const uint8_t* x, uint8_t* y, int64_t n, hipStream_t s) {
    const int64_t nvec = n / 16;
    hipLaunchKernelGGL((copy16<U, NT>), dim3((unsigned)(nvec / U / kBlock)), dim3(kBlock), 0, s, x, y, nvec);
}

static void launch_memcpy(const uint8_t* x, uint8_t* y, int64_t n, hipStream_t s) {
    CK(hipMemcpyAsync(y, x, n, hipMemcpyDeviceToDevice, s));
}

struct V {
    std::string name;
    int kind;  // 0 copy (unchecked), 1 single filter, 2 four-filter bank
    void (*fn)(const uint8_t*, uint8_t*, int64_t, hipStream_t);
    std::vector<float> us;
};

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 15;
    const int64_t n = (int64_t)1 << 28;
    std::vector<uint8_t> hx(n), ref(n), refb(4 * n), got(4 * n);
    uint64_t s = 88172645463325252ull;
    for (auto& v : hx) {
        s ^= s << 13, s ^= s >> 7, s ^= s << 17;
        v = (uint8_t)s;
    }
    auto fir = [&](const int32_t* h, int L, int64_t i) {
        const int64_t r = i / kW, c = i % kW;
        int64_t acc = 0;
        for (int k = 0; k < L; ++k) {
            const int64_t j = c - k + L / 2;
            if (j >= 0 && j < kW) acc += (int64_t)h[k] * hx[r * kW + j];
        }
        const int64_t q = (acc + 2048) >> 12;
        return (uint8_t)(q < 0 ? 0 : q > 255 ? 255 : q);
    };
    for (int64_t i = 0; i < n; ++i) {
        ref[i] = fir(kTaps, 5, i);
        for (int f = 0; f < 4; ++f) refb[f * n + i] = fir(kBank[f], 3, i);
    }
    uint8_t *dx, *dy;
    CK(hipMalloc(&dx, n));
    CK(hipMalloc(&dy, 4 * n));
    CK(hipMemcpy(dx, hx.data(), n, hipMemcpyHostToDevice));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    constexpr int PK = kU8Dot2 | kU8Pk16;
    constexpr int NS = kU8Dot2 | kNtStore;
    std::vector<V> vs = {{"fir U4 ntst (lib)", 1, launch_fir<4, NS>, {}},
                         {"fir U4 ntst pk16", 1, launch_fir<4, NS | kU8Pk16>, {}},
                         {"fir U4 ntst pk16 edw", 1, launch_fir<4, NS | kU8Pk16 | kEdgeDword>, {}},
                         {"fir U2 ntst pk16 edw", 1, launch_fir<2, NS | kU8Pk16 | kEdgeDword>, {}},
                         {"fir U1 ntst pk16 edw", 1, launch_fir<1, NS | kU8Pk16 | kEdgeDword>, {}},
                         {"fir U4 ntst pk16 edw xcd", 1, launch_fir<4, NS | kU8Pk16 | kEdgeDword | kXcd>, {}},
                         {"fir U4 ntst (lib) b", 1, launch_fir<4, NS>, {}},
                         {"fir U4 ntst pk16 b", 1, launch_fir<4, NS | kU8Pk16>, {}},
                         {"copy16 U1 nt", 0, launch_copy<1, true>, {}},
                         {"copy16 U4 nt", 0, launch_copy<4, true>, {}}};
    for (auto& v : vs) {
        if (v.kind == 0) continue;
        const int64_t nb = v.kind == 2 ? 4 * n : n;
        CK(hipMemset(dy, 0x5A, nb));
        CK(hipDeviceSynchronize());  // the memset runs on the null stream, st is non-blocking
        v.fn(dx, dy, n, st);
        CK(hipStreamSynchronize(st));
        CK(hipMemcpy(got.data(), dy, nb, hipMemcpyDeviceToHost));
        const uint8_t* r = v.kind == 2 ? refb.data() : ref.data();
        int64_t bad = 0;
        for (int64_t i = 0; i < nb; ++i)
            if (got[i] != r[i] && bad++ < 6)
                printf("  %s: [%lld] plane %lld col %lld: got %d want %d\n", v.name.c_str(), (long long)i,
                       (long long)(i / n), (long long)(i % n % kW), got[i], r[i]);
        printf("check %-16s %s (%lld bad)\n", v.name.c_str(), bad ? "FAIL" : "ok", (long long)bad);
        if (bad) return 1;
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int w = 0; w < 80; ++w) vs[w % vs.size()].fn(dx, dy, n, st);
    const int batch = 20;
    for (int r = 0; r < rounds; ++r)
        for (auto& v : vs) {
            CK(hipEventRecord(e0, st));
            for (int b = 0; b < batch; ++b) v.fn(dx, dy, n, st);
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            v.us.push_back(ms * 1e3f / batch);
        }
    printf("%-20s %10s %10s %10s %8s\n", "variant", "median_us", "min_us", "GB/s", "%8TB/s");
    for (auto& v : vs) {
        std::sort(v.us.begin(), v.us.end());
        const double med = v.us[v.us.size() / 2];
        const double bytes = (v.kind == 2 ? 5.0 : 2.0) * n;
        printf("%-20s %10.1f %10.1f %10.1f %8.1f\n", v.name.c_str(), med, v.us[0], bytes / med / 1e3,
               bytes / med / 1e3 / 80.0);
    }
    return 0;
}
