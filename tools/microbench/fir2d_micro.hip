// fir2d_micro.hip — A/B microbenchmark for the 2-D kernel (dev tool, not the product).
// Variants of fir2d_reg_kernel<5,5,u8> (pixels per lane, strip height) on an 8192x8192 u8
// frame, batches of back-to-back launches interleaved round-robin; each variant is checked
// against a CPU evaluation on sampled pixels (all four borders included).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "fir2d_reg.h"

using namespace fir;

#define CK(e)                                                                              \
    do {                                                                                   \
        hipError_t _e = (e);                                                               \
        if (_e != hipSuccess) {                                                            \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #e, hipGetErrorString(_e)); \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

static int32_t g_h[5][5];

static int32_t g_col[5], g_row[5];

// Memory-only twin of the strip loop: the same row loads (PD ahead, + the halo dword) and
// output-row stores, no arithmetic (output row o = input row o, XOR of the halo dword so the
// loads stay live).  Bounds the 2-D kernel's memory time for this access pattern.
template <int VEC, int STRIP, int PD, bool HALO>
__global__ __launch_bounds__(kBlock) void copy2d_kernel(const uint8_t* __restrict__ x, uint8_t* __restrict__ y,
                                                         int64_t H, int64_t W) {
    constexpr int ND = VEC / 4, T = STRIP + 4;
    typedef uint32_t vN __attribute__((ext_vector_type(ND)));
    const int lane = threadIdx.x & 63;
    const int64_t col0 = ((int64_t)blockIdx.x * kBlock + threadIdx.x) * VEC;
    const int64_t r0 = (int64_t)blockIdx.y * STRIP;
    const int64_t hcol = lane == 0 ? (col0 >= 4 ? col0 - 4 : col0) : (lane == 63 && col0 + VEC < W ? col0 + VEC : col0);
    vN rows[T];
    uint32_t hr[T];
    auto rp = [&](int t) { int64_t r = r0 - 2 + t; return x + (r < 0 ? 0 : (r >= H ? H - 1 : r)) * W; };
    auto load = [&](int t) {
        rows[t] = *reinterpret_cast<const vN*>(rp(t) + col0);
        hr[t] = HALO ? *reinterpret_cast<const uint32_t*>(rp(t) + hcol) : 0u;
    };
#pragma unroll
    for (int t = 0; t < PD; ++t) load(t);
#pragma unroll
    for (int t = 0; t < T; ++t) {
        if (t + PD < T) load(t + PD);
        const int o = t - 4;
        if (o >= 0 && r0 + o < H) {
            vN v = rows[t];
            v[0] ^= hr[t];
            *reinterpret_cast<vN*>(y + (r0 + o) * W + col0) = v;
        }
    }
}

template <int VEC, int STRIP, int PD, bool HALO>
static void launch_copy2d(const uint8_t* x, uint8_t* y, int64_t H, int64_t W, hipStream_t s) {
    const dim3 grid = fir2d_reg_grid<VEC, STRIP>(H, W);
    hipLaunchKernelGGL((copy2d_kernel<VEC, STRIP, PD, HALO>), grid, dim3(kBlock), 0, s, x, y, H, W);
}

static void launch_memcpy2d(const uint8_t* x, uint8_t* y, int64_t H, int64_t W, hipStream_t s) {
    CK(hipMemcpyAsync(y, x, H * W, hipMemcpyDeviceToDevice, s));
}

template <int VEC, int STRIP, int MODE, int MINW = 1, int PD = 1, bool NTL = false>
static void launch(const uint8_t* x, uint8_t* y, int64_t H, int64_t W, hipStream_t s) {
    Taps2<5, 5> t = {};
    for (int m = 0; m < 5; ++m)
        for (int n = 0; n < 5; ++n) t.h[m][n] = g_h[m][n];
    pack_taps2(t);
    for (int m = 0; m < 5; ++m) t.col[m] = g_col[m];
    for (int p = 0; p < 3; ++p)
        t.rowp[p] = ((uint32_t)g_row[4 - 2 * p] & 0xFFFFu) | ((uint32_t)(3 - 2 * p >= 0 ? g_row[3 - 2 * p] : 0) << 16);
    for (int p = 0; p < 3; ++p)
        t.colp[p] = ((uint32_t)g_col[2 * p] & 0xFFFFu) | ((uint32_t)(2 * p + 1 < 5 ? g_col[2 * p + 1] : 0) << 16);
    if ((MODE & kMode2dPk16) && !(plan_pk16(t, g_col, g_row, 12) & kMode2dPk16)) {
        fprintf(stderr, "pk16 not applicable\n");
        exit(1);
    }
    const dim3 grid = fir2d_reg_grid<VEC, STRIP>(H, W);
    hipLaunchKernelGGL((fir2d_reg_kernel<5, 5, FIR_OUT_U8_SAT, VEC, STRIP, MODE, MINW, PD, NTL>), grid, dim3(kBlock), 0, s, x, y, H,
                       W, t, 0, 12);
}

struct V {
    std::string name;
    bool check;
    void (*fn)(const uint8_t*, uint8_t*, int64_t, int64_t, hipStream_t);
    std::vector<float> us;
};

int main(int argc, char** argv) {
    const int64_t H = 8192, W = 8192;
    const int rounds = argc > 1 ? atoi(argv[1]) : 15;
    const int h1[5] = {256, 1024, 1536, 1024, 256};
    for (int m = 0; m < 5; ++m)
        for (int n = 0; n < 5; ++n) g_h[m][n] = h1[m] * h1[n] / 4096;  // rank 1: (h1/256) x (h1/16)
    for (int m = 0; m < 5; ++m) g_col[m] = h1[m] / 16;
    for (int n = 0; n < 5; ++n) g_row[n] = h1[n] / 256;
    std::vector<uint8_t> hx(H * W), hy(H * W);
    uint64_t s = 88172645463325252ull;
    for (auto& v : hx) {
        s ^= s << 13;
        s ^= s >> 7;
        s ^= s << 17;
        v = (uint8_t)(s >> 33);
    }
    uint8_t *dx, *dy;
    CK(hipMalloc(&dx, H * W));
    CK(hipMalloc(&dy, H * W));
    CK(hipMemcpy(dx, hx.data(), H * W, hipMemcpyHostToDevice));
    hipStream_t st;
    CK(hipStreamCreate(&st));
    std::vector<V> vs = {
        {"pk16hi8 v16 s32 pd4 (lib)", true, launch<16, 32, kMode2dSep | kMode2dPk16 | kMode2dPkHi8 | kMode2dNoWrap, 1, 4>, {}},
        {"pk16hi8 v16 s32 pd6", true, launch<16, 32, kMode2dSep | kMode2dPk16 | kMode2dPkHi8 | kMode2dNoWrap, 1, 6>, {}},
        {"pk16hi8 v16 s32 pd8", true, launch<16, 32, kMode2dSep | kMode2dPk16 | kMode2dPkHi8 | kMode2dNoWrap, 1, 8>, {}},
        {"pk16hi8 v16 s32 pd12", true, launch<16, 32, kMode2dSep | kMode2dPk16 | kMode2dPkHi8 | kMode2dNoWrap, 1, 12>, {}},
        {"pk16hi8 v16 s16 pd6", true, launch<16, 16, kMode2dSep | kMode2dPk16 | kMode2dPkHi8 | kMode2dNoWrap, 1, 6>, {}},
        {"pk16hi8 v16 s16 pd8", true, launch<16, 16, kMode2dSep | kMode2dPk16 | kMode2dPkHi8 | kMode2dNoWrap, 1, 8>, {}},
        {"pk16hi8 v8 s32 pd8", true, launch<8, 32, kMode2dSep | kMode2dPk16 | kMode2dPkHi8 | kMode2dNoWrap, 1, 8>, {}},
        {"pk16hi8 v8 s16 pd8", true, launch<8, 16, kMode2dSep | kMode2dPk16 | kMode2dPkHi8 | kMode2dNoWrap, 1, 8>, {}},
        {"pk16hi8 v16 s32 pd4 (lib) b", true, launch<16, 32, kMode2dSep | kMode2dPk16 | kMode2dPkHi8 | kMode2dNoWrap, 1, 4>, {}},
        {"copy2d v16 s16 pd3", false, launch_copy2d<16, 16, 3, true>, {}},
        {"copy2d v16 s16 pd3 nohalo", false, launch_copy2d<16, 16, 3, false>, {}},
        {"copy2d v16 s32 pd3", false, launch_copy2d<16, 32, 3, true>, {}},
        {"copy2d v16 s64 pd4", false, launch_copy2d<16, 64, 4, true>, {}},
        {"copy2d v8 s16 pd3", false, launch_copy2d<8, 16, 3, true>, {}},
        {"hipMemcpy D2D", false, launch_memcpy2d, {}},
    };
    auto ref = [&](int64_t i, int64_t j) {
        uint32_t a = 0;
        for (int m = 0; m < 5; ++m)
            for (int n = 0; n < 5; ++n) {
                const int64_t ii = i - m + 2, jj = j - n + 2;
                if (ii >= 0 && ii < H && jj >= 0 && jj < W) a += (uint32_t)(g_h[m][n] * (int32_t)hx[ii * W + jj]);
            }
        const int32_t q = ((int32_t)a >> 12) + (((int32_t)a >> 11) & 1);
        return (uint8_t)std::min(std::max(q, 0), 255);
    };
    bool any_bad = false;
    for (auto& v : vs) {
        if (!v.check) continue;
        CK(hipMemset(dy, 0xA5, H * W));
        v.fn(dx, dy, H, W, st);
        CK(hipGetLastError());
        CK(hipStreamSynchronize(st));
        CK(hipMemcpy(hy.data(), dy, H * W, hipMemcpyDeviceToHost));
        int64_t bad = 0, n = 0;
        for (int64_t i = 0; i < H; ++i) {
            const bool edge_row = i < 3 || i >= H - 3 || i % 31 == 0 || i % 32 < 3;
            for (int64_t j = 0; j < W; j += (edge_row || j < 3 || j >= W - 3) ? 1 : 61) {
                ++n;
                if (hy[i * W + j] != ref(i, j) && bad++ < 3)
                    fprintf(stderr, "%s: (%lld,%lld) %d vs %d\n", v.name.c_str(), (long long)i, (long long)j,
                            hy[i * W + j], ref(i, j));
            }
        }
        printf("check %-16s %s (%lld px, %lld bad)\n", v.name.c_str(), bad ? "FAIL" : "ok", (long long)n,
               (long long)bad);
        any_bad |= bad != 0;
    }
    if (any_bad) return 1;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int r = 0; r < rounds; ++r)
        for (auto& v : vs) {
            CK(hipEventRecord(a, st));
            for (int i = 0; i < 10; ++i) v.fn(dx, dy, H, W, st);
            CK(hipEventRecord(b, st));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            v.us.push_back(ms * 100.f);
        }
    printf("%-16s %10s %10s %10s %9s\n", "variant", "median_us", "min_us", "Gpx/s", "GB/s(alg)");
    for (auto& v : vs) {
        std::sort(v.us.begin(), v.us.end());
        const double med = v.us[v.us.size() / 2];
        printf("%-16s %10.1f %10.1f %10.1f %9.1f\n", v.name.c_str(), med, v.us[0], H * W / med / 1e3,
               2.0 * H * W / med / 1e3);
    }
    return 0;
}
