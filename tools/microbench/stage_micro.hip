// stage_micro.hip — memory twins of the configs[0] stage launch (dev tool, not the product).
//
// The stage: the 7 golden images (16,993,813 u8 pixels, shapes of SURVEY Appendix A) through a
// 4-filter bank, every (image, filter) output plane its own allocation, as the bench lays them out.
// These kernels move exactly the stage's bytes with the batch kernel's dispatch (a wave finds its
// image from tile prefix sums, one 1 KiB chunk of input per wave, 4 planes stored non-temporally)
// but compute nothing, so their time is the ceiling of a launch of this size and shape:
//   copy4 U=1/2/4     1/2/4 KiB of input per wave, each plane a copy of the input
//   write4 only       the 68 MB of stores alone;  read only: the 17 MB of loads alone
//   one plane copy    17 MB in, 17 MB out (a quarter of the store traffic)
// Each variant runs HBM-streaming (4 rotated buffer sets, 340 MB > the 256 MB Infinity Cache) and
// MALL-resident (one set replayed).  Variants are interleaved round-robin in one process.
//
// Build: make -C tools/microbench stage_micro     Run: tools/microbench/stage_micro [rounds]
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

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kImg = 7;
constexpr int kF = 4;
// (rows, width) of the golden images, largest first as the launcher orders them
constexpr int kShape[kImg][2] = {{2999, 4499}, {854, 1280}, {853, 1280}, {641, 1280},
                                 {762, 640},   {64, 64},    {64, 64}};

struct Batch {
    const uint8_t* x[8];
    uint8_t* y[8][4];
    int64_t total[8];
    int64_t tile0[9];
    int n;
};

// store cache policy: 0 nt (the product's), 1 plain, 2 sc0 sc1, 3 sc1, 4 nt sc1
template <int POL>
__device__ __forceinline__ void st_pol(void* p, u32x4 v) {
    if constexpr (POL == 0) asm volatile("global_store_dwordx4 %0, %1, off nt\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
    else if constexpr (POL == 1) asm volatile("global_store_dwordx4 %0, %1, off\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
    else if constexpr (POL == 2) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
    else if constexpr (POL == 3) asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
    else asm volatile("global_store_dwordx4 %0, %1, off nt sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}

// MODE 0: copy to F planes; 1: stores only; 2: loads only (one sink store per wave if a value
// matches a pattern no input has); 3: copy to one plane.  U chunks of 64 vectors per wave.
template <int MODE, int U, int POL = 0>
__global__ __launch_bounds__(256) void twin(Batch b) {
    const int64_t tile = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    int i = 0;
#pragma unroll
    for (int k = 1; k < 8; ++k) i += k < b.n && tile >= b.tile0[k] ? 1 : 0;
    const int64_t lt = tile - b.tile0[i];
    if (tile >= b.tile0[b.n]) return;
    const int lane = threadIdx.x & 63;
    const int64_t total = b.total[i];
    const int64_t nvec = (total + 15) / 16;
    u32x4 d[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int64_t v = (lt * U + u) * 64 + lane;
        if constexpr (MODE == 1) {
            d[u] = u32x4{(uint32_t)v, 1u, 2u, 3u};
        } else {
            // full vectors only; the image's last (partial) vector is copied byte by byte below
            d[u] = 16 * v + 16 <= total ? *reinterpret_cast<const u32x4*>(b.x[i] + 16 * v) : u32x4{0u, 0u, 0u, 0u};
        }
    }
    if constexpr (MODE == 2) {
        uint32_t s = 0;
#pragma unroll
        for (int u = 0; u < U; ++u) s ^= d[u].x ^ d[u].y ^ d[u].z ^ d[u].w;
        if (s == 0x9E3779B9u) b.y[i][0][lane] = (uint8_t)s;
        return;
    }
    constexpr int NF = MODE == 3 ? 1 : kF;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int64_t v = (lt * U + u) * 64 + lane;
        if (v >= nvec) continue;
#pragma unroll
        for (int f = 0; f < NF; ++f) {
            uint8_t* p = b.y[i][f] + 16 * v;
            if (16 * v + 16 <= total)
                st_pol<POL>(p, d[u] + (uint32_t)f);
            else if (MODE == 1)
                for (int k = 0; k < (int)(total - 16 * v); ++k) p[k] = (uint8_t)k;
            else
                for (int k = 0; k < (int)(total - 16 * v); ++k) p[k] = b.x[i][16 * v + k];
        }
    }
}

static Batch make_batch(uint8_t* const* x, uint8_t* const (*y)[kF], int U) {
    Batch b{};
    b.n = kImg;
    int64_t tiles = 0;
    for (int i = 0; i < kImg; ++i) {
        b.x[i] = x[i];
        for (int f = 0; f < kF; ++f) b.y[i][f] = y[i][f];
        b.total[i] = (int64_t)kShape[i][0] * kShape[i][1];
        b.tile0[i] = tiles;
        tiles += ((b.total[i] + 15) / 16 + 64 * U - 1) / (64 * U);
    }
    b.tile0[kImg] = tiles;
    return b;
}

struct V {
    std::string name;
    int mode, u, pol;
    double bytes;
    std::vector<float> hbm, mall;
};

template <int MODE, int U, int POL = 0>
static void launch(const Batch& b, hipStream_t s) {
    const int64_t blocks = (b.tile0[b.n] + 3) / 4;
    hipLaunchKernelGGL((twin<MODE, U, POL>), dim3((unsigned)blocks), dim3(256), 0, s, b);
}

static void run(const V& v, const Batch& b, hipStream_t s) {
    switch (v.pol * 100 + v.mode * 10 + v.u) {
        case 1: launch<0, 1>(b, s); break;
        case 2: launch<0, 2>(b, s); break;
        case 4: launch<0, 4>(b, s); break;
        case 11: launch<1, 1>(b, s); break;
        case 21: launch<2, 1>(b, s); break;
        case 24: launch<2, 4>(b, s); break;
        case 31: launch<3, 1>(b, s); break;
        case 101: launch<0, 1, 1>(b, s); break;
        case 201: launch<0, 1, 2>(b, s); break;
        case 301: launch<0, 1, 3>(b, s); break;
        case 401: launch<0, 1, 4>(b, s); break;
        case 111: launch<1, 1, 1>(b, s); break;
        case 211: launch<1, 1, 2>(b, s); break;
        default: fprintf(stderr, "bad variant\n"); exit(1);
    }
}

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 15;
    constexpr int kSets = 4;
    int64_t px = 0;
    for (auto& s : kShape) px += (int64_t)s[0] * s[1];
    uint8_t* x[kSets][kImg];
    uint8_t* y[kSets][kImg][kF];
    std::vector<uint8_t> host;
    for (int s = 0; s < kSets; ++s)
        for (int i = 0; i < kImg; ++i) {
            const int64_t n = (int64_t)kShape[i][0] * kShape[i][1];
            CK(hipMalloc(&x[s][i], n));
            host.resize(n);
            uint32_t r = 12345u + 7u * i + 1000u * s;
            for (auto& c : host) {
                r = r * 1664525u + 1013904223u;
                c = (uint8_t)(r >> 24);
            }
            CK(hipMemcpy(x[s][i], host.data(), n, hipMemcpyHostToDevice));
            for (int f = 0; f < kF; ++f) CK(hipMalloc(&y[s][i][f], n));
        }
    // sets x U
    Batch bs[kSets][3];
    for (int s = 0; s < kSets; ++s)
        for (int k = 0; k < 3; ++k) bs[s][k] = make_batch(x[s], y[s], 1 << k);
    std::vector<V> vs = {
        {"copy4 U=1 (batch layout)", 0, 1, 0, px * 5.0, {}, {}},
        {"copy4 U=2", 0, 2, 0, px * 5.0, {}, {}},
        {"copy4 U=4", 0, 4, 0, px * 5.0, {}, {}},
        {"write4 only", 1, 1, 0, px * 4.0, {}, {}},
        {"read only U=1", 2, 1, 0, px * 1.0, {}, {}},
        {"read only U=4", 2, 4, 0, px * 1.0, {}, {}},
        {"copy to one plane", 3, 1, 0, px * 2.0, {}, {}},
        {"copy4 U=1 plain stores", 0, 1, 1, px * 5.0, {}, {}},
        {"copy4 U=1 sc0 sc1 stores", 0, 1, 2, px * 5.0, {}, {}},
        {"copy4 U=1 sc1 stores", 0, 1, 3, px * 5.0, {}, {}},
        {"copy4 U=1 nt sc1 stores", 0, 1, 4, px * 5.0, {}, {}},
        {"write4 only plain", 1, 1, 1, px * 4.0, {}, {}},
        {"write4 only sc0 sc1", 1, 1, 2, px * 4.0, {}, {}},
    };
    auto bidx = [](int u) { return u == 1 ? 0 : (u == 2 ? 1 : 2); };
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    // check copy4 (every U) against the input on set 0
    for (int u : {1, 2, 4}) {
        for (int i = 0; i < kImg; ++i)
            for (int f = 0; f < kF; ++f)
                CK(hipMemset(y[0][i][f], 0xA5, (int64_t)kShape[i][0] * kShape[i][1]));
        CK(hipDeviceSynchronize());
        run(vs[bidx(u)], bs[0][bidx(u)], st);
        CK(hipStreamSynchronize(st));
        int64_t bad = 0;
        for (int i = 0; i < kImg; ++i) {
            const int64_t n = (int64_t)kShape[i][0] * kShape[i][1];
            std::vector<uint8_t> hx(n), hy(n);
            CK(hipMemcpy(hx.data(), x[0][i], n, hipMemcpyDeviceToHost));
            for (int f = 0; f < kF; ++f) {
                CK(hipMemcpy(hy.data(), y[0][i][f], n, hipMemcpyDeviceToHost));
                for (int64_t k = 0; k < n; ++k) {
                    // full vectors carry +f in each dword's low byte position of the u32 add
                    const bool full = (k / 16) * 16 + 16 <= n;
                    uint8_t want = hx[k];
                    if (full && f) {
                        const int64_t w0 = (k / 4) * 4;
                        uint32_t wv = (uint32_t)hx[w0] | (uint32_t)hx[w0 + 1] << 8 | (uint32_t)hx[w0 + 2] << 16 |
                                      (uint32_t)hx[w0 + 3] << 24;
                        wv += (uint32_t)f;
                        want = (uint8_t)(wv >> (8 * (k - w0)));
                    }
                    bad += hy[k] != want;
                }
            }
        }
        printf("copy4 U=%d check: %lld wrong bytes\n", u, (long long)bad);
        if (bad) return 1;
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int w = 0; w < 400; ++w) run(vs[w % vs.size()], bs[w % kSets][bidx(vs[w % vs.size()].u)], st);
    const int batch = 40;
    for (int rr = 0; rr < rounds; ++rr)
        for (auto& v : vs)
            for (int mall = 0; mall < 2; ++mall) {
                CK(hipEventRecord(e0, st));
                for (int i = 0; i < batch; ++i) run(v, bs[mall ? 0 : i % kSets][bidx(v.u)], st);
                CK(hipEventRecord(e1, st));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                (mall ? v.mall : v.hbm).push_back(ms * 1e3f / batch);
            }
    printf("stage shape: %d images, %lld px, 4 planes each (own allocations); %d rounds x %d launches\n", kImg,
           (long long)px, rounds, batch);
    printf("%-28s %9s %9s %8s | %9s %8s\n", "variant", "hbm_med", "hbm_min", "%8TB/s", "mall_med", "%8TB/s");
    for (auto& v : vs) {
        std::sort(v.hbm.begin(), v.hbm.end());
        std::sort(v.mall.begin(), v.mall.end());
        const double h = v.hbm[v.hbm.size() / 2], m = v.mall[v.mall.size() / 2];
        printf("%-28s %9.2f %9.2f %8.1f | %9.2f %8.1f\n", v.name.c_str(), h, v.hbm[0], v.bytes / h / 1e3 / 80.0, m,
               v.bytes / m / 1e3 / 80.0);
    }
    return 0;
}
