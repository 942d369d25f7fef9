// fir_micro.hip — A/B microbenchmark for the hot 1-D kernel (dev tool, not the product).
//
// Times variants of fir1d_reg_kernel<int16, int32, 5 taps> (chunks per wave U, NT flags,
// persistent grid) interleaved round-robin in ONE process (guide §5.4 rule 24), next to
// "widen copy" kernels that move the same bytes (2 B in, 4 B out per sample) with no math,
// which bound what the FIR can reach on this traffic mix.  Every FIR variant is checked
// against a CPU evaluation at ~270k sampled positions plus both ends.
//
// Build: make -C tools/microbench     Run: tools/microbench/fir_micro [log2n] [rounds]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "fir1d_reg.h"
#include "old_fir1d_reg.h"  // r01f version (before the multi-filter template), A/B only

using namespace fir;

#define CK(e)                                                                              \
    do {                                                                                   \
        hipError_t _e = (e);                                                               \
        if (_e != hipSuccess) {                                                            \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #e, hipGetErrorString(_e)); \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

template <int U, int FLAGS>
__global__ __launch_bounds__(kBlock) void widen_copy(const int16_t* __restrict__ x, int32_t* __restrict__ y,
                                                     int64_t nvec, int64_t ntiles) {
    constexpr int WPB = kBlock / kWave;
    const int lane = threadIdx.x & 63;
    const int64_t stride = (FLAGS & kPersist) ? (int64_t)gridDim.x * WPB : ntiles;
    for (int64_t tile = (int64_t)blockIdx.x * WPB + (threadIdx.x >> 6); tile < ntiles; tile += stride) {
        u32x4 d[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t v = tile * 64 * U + u * 64 + lane;
            const u32x4* p = reinterpret_cast<const u32x4*>(x) + v;
            d[u] = v < nvec ? ((FLAGS & kNtLoad) ? __builtin_nontemporal_load(p) : *p) : u32x4{0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t v = tile * 64 * U + u * 64 + lane;
            if (v >= nvec) continue;
            u32x4 a = {(uint32_t)(int32_t)(int16_t)d[u].x, (uint32_t)((int32_t)d[u].x >> 16),
                       (uint32_t)(int32_t)(int16_t)d[u].y, (uint32_t)((int32_t)d[u].y >> 16)};
            u32x4 b = {(uint32_t)(int32_t)(int16_t)d[u].z, (uint32_t)((int32_t)d[u].z >> 16),
                       (uint32_t)(int32_t)(int16_t)d[u].w, (uint32_t)((int32_t)d[u].w >> 16)};
            u32x4* q = reinterpret_cast<u32x4*>(y + v * 8);
            if (FLAGS & kNtStore) {
                __builtin_nontemporal_store(a, q);
                __builtin_nontemporal_store(b, q + 1);
            } else {
                q[0] = a;
                q[1] = b;
            }
        }
    }
}

// Same bytes, but every store instruction writes 1 KiB contiguous: lane i handles samples
// [4i, 4i+4) of each 256-sample half-chunk (8-byte loads, 16-byte stores).
template <int U>
__global__ __launch_bounds__(kBlock) void widen_copy_split(const int16_t* __restrict__ x, int32_t* __restrict__ y,
                                                           int64_t n, int64_t ntiles) {
    const int lane = threadIdx.x & 63;
    const int64_t tile = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (tile >= ntiles) return;
    u32x2 d[2 * U];
#pragma unroll
    for (int h = 0; h < 2 * U; ++h) {
        const int64_t i = tile * 512 * U + h * 256 + 4 * lane;
        d[h] = i + 4 <= n ? *reinterpret_cast<const u32x2*>(x + i) : u32x2{0, 0};
    }
#pragma unroll
    for (int h = 0; h < 2 * U; ++h) {
        const int64_t i = tile * 512 * U + h * 256 + 4 * lane;
        if (i + 4 > n) continue;
        u32x4 a = {(uint32_t)(int32_t)(int16_t)d[h].x, (uint32_t)((int32_t)d[h].x >> 16),
                   (uint32_t)(int32_t)(int16_t)d[h].y, (uint32_t)((int32_t)d[h].y >> 16)};
        *reinterpret_cast<u32x4*>(y + i) = a;
    }
}

// widen copy whose int32 stores go through LDS as whole 1 KiB rows (the kCoal store path)
__global__ __launch_bounds__(kBlock) void widen_copy_coal(const int16_t* __restrict__ x, int32_t* __restrict__ y,
                                                          int64_t nvec) {
    __shared__ u32x4 sb[kBlock * 2];
    const int lane = threadIdx.x & 63;
    const int64_t v = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const int64_t w0 = v - lane;
    if (w0 + 64 > nvec) return;
    const u32x4 d = reinterpret_cast<const u32x4*>(x)[v];
    u32x4* wb = sb + (threadIdx.x - lane) * 2;
    wb[2 * lane] = u32x4{(uint32_t)(int32_t)(int16_t)d.x, (uint32_t)((int32_t)d.x >> 16),
                         (uint32_t)(int32_t)(int16_t)d.y, (uint32_t)((int32_t)d.y >> 16)};
    wb[2 * lane + 1] = u32x4{(uint32_t)(int32_t)(int16_t)d.z, (uint32_t)((int32_t)d.z >> 16),
                             (uint32_t)(int32_t)(int16_t)d.w, (uint32_t)((int32_t)d.w >> 16)};
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    u32x4* yw = reinterpret_cast<u32x4*>(y + w0 * 8);
    yw[lane] = wb[lane];
    yw[64 + lane] = wb[64 + lane];
}

static void launch_copy_coal(const int16_t* x, int32_t* y, int64_t n, hipStream_t s, int) {
    const int64_t nvec = n / 8;
    hipLaunchKernelGGL(widen_copy_coal, dim3((unsigned)((nvec + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, x, y, nvec);
}

template <int U>
static void launch_copy_split(const int16_t* x, int32_t* y, int64_t n, hipStream_t s, int) {
    const int64_t ntiles = (n + 512 * U - 1) / (512 * U);
    hipLaunchKernelGGL((widen_copy_split<U>), dim3((unsigned)((ntiles + 3) / 4)), dim3(kBlock), 0, s, x, y, n, ntiles);
}

// Buffer-op copy with explicit cache-policy bits (gfx950: 1 = sc0, 2 = nt, 16 = sc1).
template <int LAUX, int SAUX>
__global__ __launch_bounds__(kBlock) void widen_copy_policy(const int16_t* __restrict__ x, int32_t* __restrict__ y,
                                                            int64_t nvec) {
    const int64_t blk0 = (int64_t)blockIdx.x * kBlock;  // first vector of this block
    if (blk0 >= nvec) return;
    const int lane_v = threadIdx.x;
    const int64_t v = blk0 + lane_v;
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)(x + blk0 * 8), 0, kBlock * 16, 0x00020000);
    const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc((void*)(y + blk0 * 8), 0, kBlock * 32, 0x00020000);
    if (v >= nvec) return;
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    v4u d = __builtin_amdgcn_raw_buffer_load_b128(rx, lane_v * 16, 0, LAUX);
    v4u a = {(uint32_t)(int32_t)(int16_t)d.x, (uint32_t)((int32_t)d.x >> 16), (uint32_t)(int32_t)(int16_t)d.y,
             (uint32_t)((int32_t)d.y >> 16)};
    v4u b = {(uint32_t)(int32_t)(int16_t)d.z, (uint32_t)((int32_t)d.z >> 16), (uint32_t)(int32_t)(int16_t)d.w,
             (uint32_t)((int32_t)d.w >> 16)};
    __builtin_amdgcn_raw_buffer_store_b128(a, ry, lane_v * 32, 0, SAUX);
    __builtin_amdgcn_raw_buffer_store_b128(b, ry, lane_v * 32 + 16, 0, SAUX);
}

template <int LAUX, int SAUX>
static void launch_copy_policy(const int16_t* x, int32_t* y, int64_t n, hipStream_t s, int) {
    const int64_t nvec = n / 8;
    hipLaunchKernelGGL((widen_copy_policy<LAUX, SAUX>), dim3((unsigned)((nvec + kBlock - 1) / kBlock)), dim3(kBlock), 0, s,
                       x, y, nvec);
}

static const int32_t kTaps[5] = {-256, -1024, 6656, -1024, -256};

// Lean single-row int16 -> int32 kernel (acc_bits 32, int16 taps on v_dot2): a lane owns 4
// samples (8 B), a wave 256 samples, ONE 1 KiB store row per wave straight from registers; the
// two edge dwords come from one branch-free 4-byte load (lane 0: the dword before the wave,
// lane 63: the dword after it, other lanes re-read their own first dword, unused).  Needs
// whole waves: nvec % 64 == 0.
template <int L, bool NTS>
__global__ __launch_bounds__(kBlock) void fir1d_i16_lean(const int16_t* __restrict__ x, int32_t* __restrict__ y,
                                                         int64_t nvec, TapsN<L> taps, int frac) {
    constexpr int HLE = L - 1 - L / 2, HRE = L / 2;
    static_assert(HLE <= 2 && HRE <= 2, "halo of one dword per side");
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t v = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (v >= nvec) return;  // wave-uniform
    const u32x2 d = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(x) + v);
    const int64_t ei = lane == 0 ? 2 * v - 1 : (lane == kWave - 1 ? 2 * v + 2 : 2 * v);
    const bool eok = ei >= 0 && ei < 2 * nvec;
    const uint32_t ev = reinterpret_cast<const uint32_t*>(x)[eok ? ei : 2 * v];
    const uint32_t e = eok ? ev : 0u;
    uint32_t Wd[4];
    Wd[0] = from_prev_lane(e, d.y);
    Wd[1] = d.x;
    Wd[2] = d.y;
    Wd[3] = from_next_lane(e, d.x);
    int32_t q[4];
    Dot2Vec<1, 4, L, 0, 4, true>::run(Wd, taps.pk[0], 0, frac, q);
    u32x4* dst = reinterpret_cast<u32x4*>(y) + v;
    const u32x4 val = {(uint32_t)q[0], (uint32_t)q[1], (uint32_t)q[2], (uint32_t)q[3]};
    if constexpr (NTS) store16_nt(dst, val); else *dst = val;
}

template <bool NTS>
static void launch_lean(const int16_t* x, int32_t* y, int64_t n, hipStream_t s, int) {
    TapsN<5> t;
    for (int k = 0; k < 5; ++k) t.h[0][k] = kTaps[k];
    pack_taps(t);
    const int64_t nvec = n / 4;
    hipLaunchKernelGGL((fir1d_i16_lean<5, NTS>), dim3((unsigned)((nvec + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, x,
                       y, nvec, t, 12);
}

struct Variant {
    std::string name;
    bool is_fir;
    void (*launch)(const int16_t*, int32_t*, int64_t, hipStream_t, int);
    int blocks_arg;
    std::vector<float> us;
};

template <int U, int FLAGS>
static void launch_fir(const int16_t* x, int32_t* y, int64_t n, hipStream_t s, int pblocks) {
    RowGeom g{n, 0, 0, 1};
    TapsN<5> t;
    for (int k = 0; k < 5; ++k) t.h[0][k] = kTaps[k];
    pack_taps(t);
    int64_t ntiles, blocks;
    reg_launch_geometry<int16_t, U, FLAGS>(n, pblocks, &ntiles, &blocks);
    hipLaunchKernelGGL((fir1d_reg_kernel<int16_t, FIR_OUT_I32, 5, 1, U, FLAGS>), dim3((unsigned)blocks),
                       dim3(kBlock), 0, s, x, y, g, t, 0, 12, ntiles);
}

template <int U, int FLAGS>
static void launch_fir_old(const int16_t* x, int32_t* y, int64_t n, hipStream_t s, int pblocks) {
    fir_old::RowGeom g{n, 0, 0};
    fir_old::TapsN<5> t;
    for (int k = 0; k < 5; ++k) t.h[k] = kTaps[k];
    int64_t ntiles, blocks;
    fir_old::reg_launch_geometry<int16_t, U, FLAGS>(n, pblocks, &ntiles, &blocks);
    hipLaunchKernelGGL((fir_old::fir1d_reg_kernel<int16_t, FIR_OUT_I32, 5, 1, U, FLAGS>), dim3((unsigned)blocks),
                       dim3(kBlock), 0, s, x, y, g, t, 0, 12, ntiles);
}

template <int U, int FLAGS>
static void launch_copy(const int16_t* x, int32_t* y, int64_t n, hipStream_t s, int pblocks) {
    const int64_t nvec = n / 8;
    const int64_t ntiles = (nvec + 64 * U - 1) / (64 * U);
    int64_t blocks = (ntiles + 3) / 4;
    if (FLAGS & kPersist) blocks = std::min<int64_t>(blocks, pblocks);
    hipLaunchKernelGGL((widen_copy<U, FLAGS>), dim3((unsigned)blocks), dim3(kBlock), 0, s, x, y, nvec, ntiles);
}

static int32_t ref_at(const std::vector<int16_t>& x, int64_t n) {
    uint32_t acc = 0;
    for (int k = 0; k < 5; ++k) {
        const int64_t i = n - k + 2;
        if (i >= 0 && i < (int64_t)x.size()) acc += (uint32_t)(kTaps[k] * (int32_t)x[i]);
    }
    const int32_t a = (int32_t)acc;
    return (a >> 12) + ((a >> 11) & 1);
}

int main(int argc, char** argv) {
    const int log2n = argc > 1 ? atoi(argv[1]) : 28;
    const int rounds = argc > 2 ? atoi(argv[2]) : 12;
    const int64_t n = (int64_t)1 << log2n;
    std::vector<int16_t> hx(n);
    uint64_t s = 0x9E3779B97F4A7C15ull;
    for (int64_t i = 0; i < n; ++i) {
        s ^= s << 13;
        s ^= s >> 7;
        s ^= s << 17;
        hx[i] = (int16_t)(s >> 17);
    }
    int16_t* dx;
    int32_t* dy;
    CK(hipMalloc(&dx, n * 2));
    CK(hipMalloc(&dy, n * 4));
    CK(hipMemcpy(dx, hx.data(), n * 2, hipMemcpyHostToDevice));
    hipStream_t st;
    CK(hipStreamCreate(&st));

    std::vector<Variant> vs = {
        {"fir U1 coal ntst (lib)", true, launch_fir<1, kDot2 | kAcc32 | kCoal | kNtStore>, 0, {}},
        {"fir U1 coal ntst edw", true, launch_fir<1, kDot2 | kAcc32 | kCoal | kNtStore | kEdgeDword>, 0, {}},
        {"fir U1 coal ntst (lib) b", true, launch_fir<1, kDot2 | kAcc32 | kCoal | kNtStore>, 0, {}},
        {"fir U1 coal ntst edw b", true, launch_fir<1, kDot2 | kAcc32 | kCoal | kNtStore | kEdgeDword>, 0, {}},
        {"copy U1 coal (LDS)", false, launch_copy_coal, 0, {}},
    };

    // correctness (FIR variants): sampled positions + both ends
    std::vector<int32_t> hy(n);
    for (auto& v : vs) {
        if (!v.is_fir) continue;
        CK(hipMemsetAsync(dy, 0x5A, n * 4, st));
        v.launch(dx, dy, n, st, v.blocks_arg);
        CK(hipGetLastError());
        CK(hipStreamSynchronize(st));
        CK(hipMemcpy(hy.data(), dy, n * 4, hipMemcpyDeviceToHost));
        int64_t bad = 0, checked = 0;
        for (int64_t i = 0; i < n; i += (i < 4096 || i > n - 4096) ? 1 : 997) {
            ++checked;
            if (hy[i] != ref_at(hx, i)) {
                if (bad < 3) fprintf(stderr, "%s: mismatch at %lld: %d vs %d\n", v.name.c_str(), (long long)i, hy[i], ref_at(hx, i));
                ++bad;
            }
        }
        printf("check %-28s %s (%lld positions)\n", v.name.c_str(), bad ? "FAIL" : "ok", (long long)checked);
        if (bad) return 1;
    }

    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (auto& v : vs)  // warm
        for (int i = 0; i < 3; ++i) v.launch(dx, dy, n, st, v.blocks_arg);
    CK(hipStreamSynchronize(st));
    // Steady state: each sample is a batch of kBatch back-to-back launches (events around the
    // batch), so deferred write-back of the previous launch's dirty lines is paid inside the
    // timed window, as in bench.py.  Variants interleave round-robin.
    const int kBatch = 10;
    for (int r = 0; r < rounds; ++r) {
        for (auto& v : vs) {
            CK(hipEventRecord(a, st));
            for (int i = 0; i < kBatch; ++i) v.launch(dx, dy, n, st, v.blocks_arg);
            CK(hipEventRecord(b, st));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            v.us.push_back(ms * 1000.f / kBatch);
        }
    }
    const double bytes = (double)n * 6.0;
    printf("%-28s %10s %10s %10s %8s\n", "variant", "median_us", "min_us", "GB/s(med)", "%8TB/s");
    for (auto& v : vs) {
        std::sort(v.us.begin(), v.us.end());
        const double med = v.us[v.us.size() / 2], mn = v.us[0];
        printf("%-28s %10.1f %10.1f %10.1f %8.1f\n", v.name.c_str(), med, mn, bytes / med / 1e3, bytes / med / 1e3 / 80.0);
    }
    // D2D memcpy of the same byte count (read + write counted)
    {
        std::vector<float> t;
        for (int i = 0; i < 10; ++i) {
            CK(hipEventRecord(a, st));
            CK(hipMemcpyAsync(dy, dx, n * 2, hipMemcpyDeviceToDevice, st));
            CK(hipEventRecord(b, st));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            t.push_back(ms * 1000.f);
        }
        std::sort(t.begin(), t.end());
        printf("%-28s %10.1f %10.1f %10.1f %8.1f\n", "hipMemcpy D2D (2B*n r+w)", t[5], t[0], 2.0 * n * 2 / t[5] / 1e3,
               2.0 * n * 2 / t[5] / 1e3 / 80.0);
    }
    return 0;
}
