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
static int32_t g_hg[5][5];  // a non-separable kernel for the general packed-16 variants

// Memory-only twin of the strip loop: the same row loads (PD ahead, + the halo dword) and
// output-row stores, no arithmetic (output row o = input row o, XOR of the halo dword so the
// loads stay live).  Bounds the 2-D kernel's memory time for this access pattern.
template <int VEC, int STRIP, int PD, bool HALO, bool NTS = false, bool XCD = false>
__global__ __launch_bounds__(kBlock) void copy2d_kernel(const uint8_t* __restrict__ x, uint8_t* __restrict__ y,
                                                         int64_t H, int64_t W) {
    constexpr int ND = VEC / 4, T = STRIP + 4;
    typedef uint32_t vN __attribute__((ext_vector_type(ND)));
    int64_t bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
    if constexpr (XCD) {  // same remap as fir2d_reg_kernel<..., XCD = true>
        const int64_t gx = gridDim.x, gy = gridDim.y, nb = gx * gy * gridDim.z;
        const int64_t b = bx + gx * (by + gy * bz), q = nb / 8;
        const int64_t p = b < q * 8 ? (b % 8) * q + b / 8 : b;
        bx = p % gx;
        by = (p / gx) % gy;
        bz = p / (gx * gy);
    }
    x += bz * H * W;  // batched launches: frame bz
    y += bz * H * W;
    const int lane = threadIdx.x & 63;
    const int64_t col0 = (bx * kBlock + threadIdx.x) * VEC;
    const int64_t r0 = by * STRIP;
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
            vN* d = reinterpret_cast<vN*>(y + (r0 + o) * W + col0);
            if constexpr (NTS) __builtin_nontemporal_store(v, d);
            else *d = v;
        }
    }
}

// Contiguous copy with the 1-D u8 kernel's shape: a wave moves K consecutive 1 KiB chunks,
// non-temporal stores.  The ceiling for the same bytes without the strip pattern.
template <int K>
__global__ __launch_bounds__(kBlock) void copy1d_nt_kernel(const uint8_t* __restrict__ x, uint8_t* __restrict__ y, int64_t n) {
    typedef uint32_t v4 __attribute__((ext_vector_type(4)));
    const int64_t wave = ((int64_t)blockIdx.x * kBlock + threadIdx.x) / 64, lane = threadIdx.x & 63;
    const int64_t base = wave * K * 1024 + lane * 16;
    v4 d[K];
#pragma unroll
    for (int k = 0; k < K; ++k) d[k] = base + k * 1024 < n ? *reinterpret_cast<const v4*>(x + base + k * 1024) : v4{};
#pragma unroll
    for (int k = 0; k < K; ++k)
        if (base + k * 1024 < n) __builtin_nontemporal_store(d[k], reinterpret_cast<v4*>(y + base + k * 1024));
}

template <int VEC, int STRIP, int PD, bool HALO>
static void launch_copy2d(const uint8_t* x, uint8_t* y, int64_t H, int64_t W, hipStream_t s) {
    const dim3 grid = fir2d_reg_grid<VEC, STRIP>(H, W);
    hipLaunchKernelGGL((copy2d_kernel<VEC, STRIP, PD, HALO>), grid, dim3(kBlock), 0, s, x, y, H, W);
}

static void launch_memcpy2d(const uint8_t* x, uint8_t* y, int64_t H, int64_t W, hipStream_t s) {
    CK(hipMemcpyAsync(y, x, H * W, hipMemcpyDeviceToDevice, s));
}

static const uint8_t* g_bx;  // frame-batch base pointers (set in main)
static uint8_t* g_by;
template <int VEC, int STRIP, int PD, bool NTS = false, bool XCD = false>
static void launch_copy2d_x4(const uint8_t*, uint8_t*, int64_t H, int64_t W, hipStream_t s) {
    dim3 grid = fir2d_reg_grid<VEC, STRIP>(H, W);
    grid.z = 4;
    hipLaunchKernelGGL((copy2d_kernel<VEC, STRIP, PD, true, NTS, XCD>), grid, dim3(kBlock), 0, s, g_bx, g_by, H, W);
}
template <int K>
static void launch_copy1d_x4(const uint8_t*, uint8_t*, int64_t H, int64_t W, hipStream_t s) {
    const int64_t n = 4 * H * W, waves = (n + K * 1024 - 1) / (K * 1024);
    hipLaunchKernelGGL((copy1d_nt_kernel<K>), dim3((unsigned)((waves + 3) / 4)), dim3(kBlock), 0, s, g_bx, g_by, n);
}
static void launch_memcpy_x4(const uint8_t*, uint8_t*, int64_t H, int64_t W, hipStream_t s) {
    CK(hipMemcpyAsync(g_by, g_bx, 4 * H * W, hipMemcpyDeviceToDevice, s));
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
    int frames = 1;  // frames per launch (batched variants run on g_x / g_y from frame 0)
    bool gen = false;  // checked against g_hg instead of g_h
};

static const uint8_t* g_x;
static uint8_t* g_y;
template <int VEC, int STRIP, int MODE, int PD, int NF, bool NTS = false, bool XCD = false>
static void launch_batch(const uint8_t*, uint8_t*, int64_t H, int64_t W, hipStream_t s) {
    Taps2<5, 5> t = {};
    for (int m = 0; m < 5; ++m)
        for (int n = 0; n < 5; ++n) t.h[m][n] = g_h[m][n];
    pack_taps2(t);
    if (!(plan_pk16(t, g_col, g_row, 12) & kMode2dPk16)) exit(1);
    dim3 grid = fir2d_reg_grid<VEC, STRIP>(H, W);
    grid.z = NF;
    hipLaunchKernelGGL((fir2d_reg_kernel<5, 5, FIR_OUT_U8_SAT, VEC, STRIP, MODE, 1, PD, false, NTS, XCD>), grid, dim3(kBlock),
                       0, s, g_x, g_y, H, W, t, 0, 12);
}

template <int VEC, int STRIP, int MODE, int PD, bool NTS, bool XCD>
static void launch_batch_gen(const uint8_t*, uint8_t*, int64_t H, int64_t W, hipStream_t s) {
    Taps2<5, 5> t = {};
    for (int m = 0; m < 5; ++m)
        for (int n = 0; n < 5; ++n) t.h[m][n] = g_hg[m][n];
    pack_taps2(t);
    if (plan_pk16_gen(t, &g_hg[0][0], 12) != (MODE & (kMode2dPk16 | kMode2dPkSigned | kMode2dPkHi8))) exit(2);
    dim3 grid = fir2d_reg_grid<VEC, STRIP>(H, W);
    grid.z = 4;
    hipLaunchKernelGGL((fir2d_reg_kernel<5, 5, FIR_OUT_U8_SAT, VEC, STRIP, MODE, 1, PD, false, NTS, XCD>), grid, dim3(kBlock),
                       0, s, g_x, g_y, H, W, t, 0, 12);
}

// Reads n 16-byte words grid-stride; writes one word only if a never-true condition holds.
typedef uint32_t ev_u4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void evict_read(const ev_u4* __restrict__ p, size_t n, uint32_t* __restrict__ sink) {
    uint32_t acc = 0;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const ev_u4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

int main(int argc, char** argv) {
    const int64_t H = 8192, W = 8192;
    const int rounds = argc > 1 ? atoi(argv[1]) : 15;
    const int h1[5] = {256, 1024, 1536, 1024, 256};
    for (int m = 0; m < 5; ++m)
        for (int n = 0; n < 5; ++n) g_h[m][n] = h1[m] * h1[n] / 4096;  // rank 1: (h1/256) x (h1/16)
    for (int m = 0; m < 5; ++m) g_col[m] = h1[m] / 16;
    for (int n = 0; n < 5; ++n) g_row[n] = h1[n] / 256;
    {  // tests/test_gpu_fir2d_ideal.py GEN_PK_KERNELS-like: signed taps in [-4, 4], Laplacian-ish centre
        const int32_t hg[5][5] = {{1, -2, 3, -1, 0}, {-3, 4, 2, -4, 1}, {2, 1, 4, 1, 2}, {0, -4, 2, 4, -3}, {-1, 3, -2, 1, 2}};
        for (int m = 0; m < 5; ++m)
            for (int n = 0; n < 5; ++n) g_hg[m][n] = hg[m][n];
    }
    std::vector<uint8_t> hx(H * W), hy(H * W);
    uint64_t s = 88172645463325252ull;
    for (auto& v : hx) {
        s ^= s << 13;
        s ^= s >> 7;
        s ^= s << 17;
        v = (uint8_t)(s >> 33);
    }
    uint8_t *dx, *dy;
    // kFrames distinct frames (in and out): the timed batches cycle through them so every launch
    // streams from HBM (one 64 MiB frame would stay in the 256 MB Infinity Cache)
    constexpr int kFrames = 4;
    CK(hipMalloc(&dx, kFrames * H * W));
    CK(hipMalloc(&dy, kFrames * H * W));
    for (int f = 0; f < kFrames; ++f) CK(hipMemcpy(dx + f * H * W, hx.data(), H * W, hipMemcpyHostToDevice));
    g_x = dx;
    g_y = dy;
    g_bx = dx;
    g_by = dy;
    hipStream_t st;
    CK(hipStreamCreate(&st));
    constexpr int PKM = kMode2dSep | kMode2dPk16 | kMode2dPkHi8 | kMode2dNoWrap;
    constexpr int GKM = kMode2dDot2 | kMode2dNoWrap | kMode2dPk16 | kMode2dPkSigned;
    std::vector<V> vs = {
        {"x4 v16 s32 pd4 (lib)", true, launch_batch<16, 32, PKM, 4, 4>, {}, 4},
        {"x4 v16 s32 pd4 nts", true, launch_batch<16, 32, PKM, 4, 4, true>, {}, 4},
        {"x4 v16 s32 pd4 nts xcd", true, launch_batch<16, 32, PKM, 4, 4, true, true>, {}, 4},
        {"x4 v16 s32 pd3 nts xcd", true, launch_batch<16, 32, PKM, 3, 4, true, true>, {}, 4},
        {"x4 v16 s32 pd6 nts xcd", true, launch_batch<16, 32, PKM, 6, 4, true, true>, {}, 4},
        {"x4 v16 s16 pd4 nts", true, launch_batch<16, 16, PKM, 4, 4, true>, {}, 4},
        {"x4 v16 s16 pd4 nts xcd", true, launch_batch<16, 16, PKM, 4, 4, true, true>, {}, 4},
        {"x4 v16 s16 pd3 nts xcd", true, launch_batch<16, 16, PKM, 3, 4, true, true>, {}, 4},
        {"x4 v16 s16 pd6 nts xcd", true, launch_batch<16, 16, PKM, 6, 4, true, true>, {}, 4},
        {"x4 v16 s24 pd4 nts xcd", true, launch_batch<16, 24, PKM, 4, 4, true, true>, {}, 4},
        {"x4 v16 s8 pd4 nts xcd", true, launch_batch<16, 8, PKM, 4, 4, true, true>, {}, 4},
        {"x4 v16 s12 pd4 nts xcd", true, launch_batch<16, 12, PKM, 4, 4, true, true>, {}, 4},
        {"x4 gen v16 s16 pd2 (lib)", true, launch_batch_gen<16, 16, GKM, 2, false, false>, {}, 4, true},
        {"x4 gen v16 s16 pd2 nts", true, launch_batch_gen<16, 16, GKM, 2, true, false>, {}, 4, true},
        {"x4 gen v16 s16 pd2 nts xcd", true, launch_batch_gen<16, 16, GKM, 2, true, true>, {}, 4, true},
        {"x4 gen v16 s8 pd2 nts xcd", true, launch_batch_gen<16, 8, GKM, 2, true, true>, {}, 4, true},
        {"x4 gen v16 s12 pd2 nts xcd", true, launch_batch_gen<16, 12, GKM, 2, true, true>, {}, 4, true},
        {"x4 gen v8 s16 pd3 nts xcd", true, launch_batch_gen<8, 16, GKM, 3, true, true>, {}, 4, true},
        {"x4 copy2d v16 s32 pd3 nts xcd", false, launch_copy2d_x4<16, 32, 3, true, true>, {}, 4},
        {"x4 copy2d v16 s16 pd4 nts xcd", false, launch_copy2d_x4<16, 16, 4, true, true>, {}, 4},
        {"x4 copy1d nt K1", false, launch_copy1d_x4<1>, {}, 4},
        {"x4 hipMemcpy D2D", false, launch_memcpy_x4, {}, 4},
    };
    auto ref = [&](int64_t i, int64_t j, bool gen) {
        uint32_t a = 0;
        for (int m = 0; m < 5; ++m)
            for (int n = 0; n < 5; ++n) {
                const int64_t ii = i - m + 2, jj = j - n + 2;
                const int32_t h = gen ? g_hg[m][n] : g_h[m][n];
                if (ii >= 0 && ii < H && jj >= 0 && jj < W) a += (uint32_t)(h * (int32_t)hx[ii * W + jj]);
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
                if (hy[i * W + j] != ref(i, j, v.gen) && bad++ < 3)
                    fprintf(stderr, "%s: (%lld,%lld) %d vs %d\n", v.name.c_str(), (long long)i, (long long)j,
                            hy[i * W + j], ref(i, j, v.gen));
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
            for (int i = 0; i < 12; ++i) v.fn(dx + (i % kFrames) * H * W, dy + (i % kFrames) * H * W, H, W, st);
            // batched variants filter v.frames frames per launch: time per frame below
            CK(hipEventRecord(b, st));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            v.us.push_back(ms * 1000.f / 12 / v.frames);
        }
    // Cold runs: the frame (64 MiB in + 64 MiB out) fits the 256 MB Infinity Cache, so the
    // back-to-back batches above may be served partly from it.  Here every launch follows a
    // 1 GiB READ sweep that evicts it (and the L2s) with clean lines, so no dirty write-back
    // lands in the timed launch; events around the single launch.
    {
        uint8_t *junk, *dy2;
        CK(hipMalloc(&junk, (size_t)1 << 30));
        CK(hipMalloc(&dy2, 256));
        CK(hipMemset(junk, 1, (size_t)1 << 30));
        CK(hipDeviceSynchronize());
        std::vector<std::string> cold_names = {vs[0].name, "copy2d v16 s32 pd3", "hipMemcpy D2D"};
        for (const auto& cn : cold_names) {
            V* vp = nullptr;
            for (auto& v : vs)
                if (v.name == cn) vp = &v;
            if (!vp) continue;
            std::vector<float> t;
            for (int r = 0; r < 20; ++r) {
                hipLaunchKernelGGL(evict_read, dim3(4096), dim3(256), 0, st, reinterpret_cast<const ev_u4*>(junk),
                                   ((size_t)1 << 30) / 16, reinterpret_cast<uint32_t*>(dy2));
                CK(hipEventRecord(a, st));
                vp->fn(dx, dy, H, W, st);
                CK(hipEventRecord(b, st));
                CK(hipEventSynchronize(b));
                float ms;
                CK(hipEventElapsedTime(&ms, a, b));
                t.push_back(ms * 1000.f);
            }
            std::sort(t.begin(), t.end());
            printf("cold %-28s median %7.1f us  min %7.1f us\n", cn.c_str(), t[t.size() / 2], t[0]);
        }
        CK(hipFree(junk));
        CK(hipFree(dy2));
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
