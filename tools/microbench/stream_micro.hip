// stream_micro.hip — HBM stream ceilings for the headline kernel's traffic (dev tool, not the
// product): 2^28 int16 read, 2^28 int32 written (the 5-tap int16 -> int32 FIR's bytes), with
// the read side as register loads or LDS-DMA (global_load_lds_dwordx4), default or
// non-temporal policy, and the store side's shape and cache policy; plus read-only and write-only
// ceilings of the same sizes.  Variants interleaved round-robin in one process; the widen
// copies are checked against the CPU.
//
// Build: make -C tools/microbench     Run: tools/microbench/stream_micro [rounds]
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
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
constexpr int kAuxNt = 2;  // CPol NT on gfx94x/gfx950

__device__ __forceinline__ void st_nt(u32x4* p, u32x4 v) {
    asm volatile("global_store_dwordx4 %0, %1, off nt\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}

__device__ __forceinline__ void glds16(const void* g, void* lds_wave_base, bool nt) {
    if (nt)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                         (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, kAuxNt);
    else
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                         (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

__device__ __forceinline__ u32x4 widen_lo(u32x2 d) {  // 4 int16 -> 4 int32
    return u32x4{(uint32_t)(int32_t)(int16_t)d.x, (uint32_t)((int32_t)d.x >> 16), (uint32_t)(int32_t)(int16_t)d.y,
                 (uint32_t)((int32_t)d.y >> 16)};
}

template <int N>
__device__ __forceinline__ void vmcnt_n() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

// ---- widen copies: K KiB of int16 per wave -> 2K KiB of int32 ---------------------------
// Register path: lane loads 16 B per KiB, LDS transpose, 1 KiB nt row stores (the FIR's shape).
template <int K, int BLOCK>
__global__ __launch_bounds__(BLOCK) void widen_reg(const int16_t* __restrict__ x, int32_t* __restrict__ y) {
    __shared__ u32x4 sb[BLOCK / 64][K * 64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t wave = (int64_t)blockIdx.x * (BLOCK / 64) + w;
    const u32x4* src = reinterpret_cast<const u32x4*>(x) + wave * (64 * K);
    u32x4 d[K];
#pragma unroll
    for (int k = 0; k < K; ++k) d[k] = __builtin_nontemporal_load(src + k * 64 + lane);
#pragma unroll
    for (int k = 0; k < K; ++k) sb[w][k * 64 + lane] = d[k];
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    const u32x2* s2 = reinterpret_cast<const u32x2*>(&sb[w][0]);
    u32x4* dst = reinterpret_cast<u32x4*>(y) + wave * (128 * K);
#pragma unroll
    for (int r = 0; r < 2 * K; ++r) st_nt(dst + r * 64 + lane, widen_lo(s2[r * 64 + lane]));
}

// LDS-DMA path: K global_load_lds_dwordx4 (1 KiB each) per wave, vmcnt(0), then rows as above.
template <int K, int BLOCK, bool NT>
__global__ __launch_bounds__(BLOCK) void widen_glds(const int16_t* __restrict__ x, int32_t* __restrict__ y) {
    __shared__ u32x4 sb[BLOCK / 64][K * 64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t wave = (int64_t)blockIdx.x * (BLOCK / 64) + w;
    const u32x4* src = reinterpret_cast<const u32x4*>(x) + wave * (64 * K);
#pragma unroll
    for (int k = 0; k < K; ++k) glds16(src + k * 64 + lane, &sb[w][k * 64], NT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const u32x2* s2 = reinterpret_cast<const u32x2*>(&sb[w][0]);
    u32x4* dst = reinterpret_cast<u32x4*>(y) + wave * (128 * K);
#pragma unroll
    for (int r = 0; r < 2 * K; ++r) st_nt(dst + r * 64 + lane, widen_lo(s2[r * 64 + lane]));
}

// ---- read-only / write-only ceilings ---------------------------------------------------
template <int K, int BLOCK>
__global__ __launch_bounds__(BLOCK) void read_reg(const int16_t* __restrict__ x, int32_t* __restrict__ sink) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * BLOCK + threadIdx.x) >> 6;
    const u32x4* src = reinterpret_cast<const u32x4*>(x) + wave * (64 * K);
    u32x4 d[K];
#pragma unroll
    for (int k = 0; k < K; ++k) d[k] = __builtin_nontemporal_load(src + k * 64 + lane);
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) s ^= d[k].x ^ d[k].y ^ d[k].z ^ d[k].w;
    if (s == 0x9E3779B9u) sink[lane] = (int32_t)s;  // keeps the loads
}

template <int K, int BLOCK, bool NT>
__global__ __launch_bounds__(BLOCK) void read_glds(const int16_t* __restrict__ x, int32_t* __restrict__ sink) {
    __shared__ u32x4 sb[BLOCK / 64][K * 64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t wave = (int64_t)blockIdx.x * (BLOCK / 64) + w;
    const u32x4* src = reinterpret_cast<const u32x4*>(x) + wave * (64 * K);
#pragma unroll
    for (int k = 0; k < K; ++k) glds16(src + k * 64 + lane, &sb[w][k * 64], NT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const u32x4 v = sb[w][lane];
    if ((v.x ^ v.w) == 0x9E3779B9u) sink[lane] = 1;
}

template <int K, int BLOCK>
__global__ __launch_bounds__(BLOCK) void write_nt(int32_t* __restrict__ y) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * BLOCK + threadIdx.x) >> 6;
    u32x4* dst = reinterpret_cast<u32x4*>(y) + wave * (64 * K);
#pragma unroll
    for (int k = 0; k < K; ++k) st_nt(dst + k * 64 + lane, u32x4{(uint32_t)lane, (uint32_t)k, 0u, 1u});
}

// Store patterns, R KiB per wave: P=0 whole 1 KiB rows (lane i -> bytes 16i of each row),
// P=1 each lane 32 contiguous bytes per 2 KiB (two adjacent dwordx4), P=2 64 contiguous bytes
// per 4 KiB.  POL: 0 plain, 1 nt, 2 sc0 sc1, 3 sc1.
template <int POL>
__device__ __forceinline__ void st16(u32x4* p, u32x4 v) {
    if constexpr (POL == 0) asm volatile("global_store_dwordx4 %0, %1, off\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
    else if constexpr (POL == 1) asm volatile("global_store_dwordx4 %0, %1, off nt\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
    else if constexpr (POL == 2) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
    else asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}
// Widen copies with the store side varied: H=1 a wave loads 512 B (8 B per lane) and stores one
// 1 KiB row; H=0 a wave loads 1 KiB and stores (P=0) two rows through LDS or (P=1) each lane's
// own 32 output bytes straight from registers.  POL as st16.
template <int H, int P, int POL, int BLOCK>
__global__ __launch_bounds__(BLOCK) void widen_pat(const int16_t* __restrict__ x, int32_t* __restrict__ y) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t wave = (int64_t)blockIdx.x * (BLOCK / 64) + w;
    if constexpr (H == 1) {
        const u32x2* src = reinterpret_cast<const u32x2*>(x) + wave * 64;
        const u32x2 d = __builtin_nontemporal_load(src + lane);
        st16<POL>(reinterpret_cast<u32x4*>(y) + wave * 64 + lane, widen_lo(d));
    } else if constexpr (P == 1) {
        const u32x4* src = reinterpret_cast<const u32x4*>(x) + wave * 64;
        const u32x4 d = __builtin_nontemporal_load(src + lane);
        u32x4* dst = reinterpret_cast<u32x4*>(y) + wave * 128 + 2 * lane;
        st16<POL>(dst, widen_lo(u32x2{d.x, d.y}));
        st16<POL>(dst + 1, widen_lo(u32x2{d.z, d.w}));
    } else {
        __shared__ u32x4 sb[BLOCK / 64][64];
        const u32x4* src = reinterpret_cast<const u32x4*>(x) + wave * 64;
        sb[w][lane] = __builtin_nontemporal_load(src + lane);
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");
        const u32x2* s2 = reinterpret_cast<const u32x2*>(&sb[w][0]);
        u32x4* dst = reinterpret_cast<u32x4*>(y) + wave * 128;
        st16<POL>(dst + lane, widen_lo(s2[lane]));
        st16<POL>(dst + 64 + lane, widen_lo(s2[64 + lane]));
    }
}

// widen_pat H=1 plus what the FIR adds per wave: E=1 one more 4-byte load per lane (branch-free,
// lanes 0/63 the dwords around the wave, the rest their own), E=2 that plus the two DPP moves,
// E=3 the halo through LDS instead: each wave publishes its edge dwords, one block barrier,
// lanes 0/63 read the neighbours' (block edges load from memory).
// Producer/consumer widen: wave 0 of a block only LOADS (LDS-DMA, so its vmcnt counts nothing
// but its own loads, in order) and keeps D phase-groups of 3 tiles in flight; waves 1-3 only
// read LDS, widen and STORE (nothing to wait for).  One s_barrier per phase; G = D + 1 LDS
// groups of 3 x 1 KiB.  Each block walks a contiguous range of tiles.
template <int D, bool NT>
__global__ __launch_bounds__(256) void widen_pc(const int16_t* __restrict__ x, int32_t* __restrict__ y,
                                                int64_t ntiles, int64_t per_block) {
    constexpr int G = D + 1;
    __shared__ u32x4 ring[G][3][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t t0 = (int64_t)blockIdx.x * per_block;
    const int64_t t1 = t0 + per_block < ntiles ? t0 + per_block : ntiles;
    const int64_t nph = (t1 - t0 + 2) / 3;  // phases of 3 tiles
    const u32x4* src = reinterpret_cast<const u32x4*>(x);
    u32x4* dst = reinterpret_cast<u32x4*>(y);
    auto issue = [&](int64_t p) {  // loader: the 3 tiles of phase p into group p % G
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            int64_t t = t0 + 3 * p + c;
            t = t < t1 ? t : t1 - 1;  // the last phase may be short: re-read a valid tile
            glds16(src + t * 64 + lane, &ring[p % G][c][0], NT);
        }
    };
    if (w == 0) {
        for (int64_t p = 0; p < D && p < nph; ++p) issue(p);
    }
    for (int64_t p = 0; p < nph; ++p) {
        if (w == 0) {
            if (p + D < nph) {
                issue(p + D);
                vmcnt_n<3 * D>();  // phase p's 3 loads landed (3*D younger loads may be in flight)
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
        }
        __builtin_amdgcn_s_barrier();  // phase p's group is in LDS for every wave
        asm volatile("" ::: "memory");
        if (w > 0) {
            const int64_t t = t0 + 3 * p + (w - 1);
            if (t < t1) {
                const u32x2* s2 = reinterpret_cast<const u32x2*>(&ring[p % G][w - 1][0]);
                const u32x2 a = s2[lane], b = s2[64 + lane];
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                st_nt(dst + t * 128 + lane, widen_lo(a));
                st_nt(dst + t * 128 + 64 + lane, widen_lo(b));
            }
        }
        // the group read in phase p is reloaded in phase p + G - D = p + 1 only after the next
        // barrier, by which time every consumer has read it (the reads finish before the stores)
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    }
}

template <int E>
__global__ __launch_bounds__(256) void widen_half_edge(const int16_t* __restrict__ x, int32_t* __restrict__ y,
                                                       int64_t nvec) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const u32x2 d = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(x) + v);
    uint32_t e = 0;
    if constexpr (E == 1 || E == 2) {
        const int64_t ei = lane == 0 ? 2 * v - 1 : (lane == 63 ? 2 * v + 2 : 2 * v);
        const bool ok = ei >= 0 && ei < 2 * nvec;
        const uint32_t ev = reinterpret_cast<const uint32_t*>(x)[ok ? ei : 2 * v];
        e = ok ? ev : 0u;
    } else if constexpr (E == 3) {
        __shared__ uint32_t edge[4][2];
        if (lane == 0) edge[w][0] = d.x;
        if (lane == 63) edge[w][1] = d.y;
        uint32_t ev = 0;
        const bool outer = (lane == 0 && w == 0) || (lane == 63 && w == 3);
        if (outer) {
            const int64_t ei = lane == 0 ? 2 * v - 1 : 2 * v + 2;
            if (ei >= 0 && ei < 2 * nvec) ev = reinterpret_cast<const uint32_t*>(x)[ei];
        }
        __syncthreads();
        if (!outer) ev = lane == 0 ? edge[w - 1][1] : (lane == 63 ? edge[w + 1][0] : 0u);
        e = ev;
    }
    uint32_t a = d.x, b = d.y;
    if constexpr (E >= 2) {
        a ^= (uint32_t)__builtin_amdgcn_update_dpp((int)e, (int)d.y, 0x138, 0xF, 0xF, false) & 0x80000000u;
        b ^= (uint32_t)__builtin_amdgcn_update_dpp((int)e, (int)d.x, 0x130, 0xF, 0xF, false) & 0x80000000u;
    } else {
        a ^= e & 0x80000000u & (uint32_t)(lane == 64);
    }
    (void)a;
    st16<1>(reinterpret_cast<u32x4*>(y) + v, widen_lo(u32x2{E >= 2 ? a ^ (a & 0x80000000u) ^ (d.x & 0x80000000u) : d.x, E >= 2 ? b ^ (b & 0x80000000u) ^ (d.y & 0x80000000u) : d.y}));
}

template <int P, int R, int POL, int BLOCK>
__global__ __launch_bounds__(BLOCK) void write_pat(int32_t* __restrict__ y) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * BLOCK + threadIdx.x) >> 6;
    u32x4* dst = reinterpret_cast<u32x4*>(y) + wave * (64 * R);
    constexpr int G = P == 0 ? 1 : (P == 1 ? 2 : 4);  // contiguous 16-B pieces per lane
#pragma unroll
    for (int k = 0; k < R / G; ++k)
#pragma unroll
        for (int g = 0; g < G; ++g)
            st16<POL>(dst + k * 64 * G + lane * G + g, u32x4{(uint32_t)lane, (uint32_t)k, (uint32_t)g, 1u});
}

// ---------------------------------------------------------------------------------------
struct Bufs {
    int16_t* x;
    int32_t* y;
    int64_t n;
};

struct V {
    std::string name;
    void (*fn)(const Bufs&, hipStream_t);
    double bytes;   // per launch
    bool widen;     // output checkable
    std::vector<float> us;
};

template <int K, int BLOCK>
void l_widen_reg(const Bufs& b, hipStream_t s) {
    hipLaunchKernelGGL((widen_reg<K, BLOCK>), dim3((unsigned)(b.n / (512 * K) / (BLOCK / 64))), dim3(BLOCK), 0, s,
                       b.x, b.y);
}
template <int K, int BLOCK, bool NT>
void l_widen_glds(const Bufs& b, hipStream_t s) {
    hipLaunchKernelGGL((widen_glds<K, BLOCK, NT>), dim3((unsigned)(b.n / (512 * K) / (BLOCK / 64))), dim3(BLOCK), 0,
                       s, b.x, b.y);
}
template <int K, int BLOCK>
void l_read_reg(const Bufs& b, hipStream_t s) {
    hipLaunchKernelGGL((read_reg<K, BLOCK>), dim3((unsigned)(b.n / (512 * K) / (BLOCK / 64))), dim3(BLOCK), 0, s, b.x,
                       b.y);
}
template <int K, int BLOCK, bool NT>
void l_read_glds(const Bufs& b, hipStream_t s) {
    hipLaunchKernelGGL((read_glds<K, BLOCK, NT>), dim3((unsigned)(b.n / (512 * K) / (BLOCK / 64))), dim3(BLOCK), 0,
                       s, b.x, b.y);
}
template <int K, int BLOCK>
void l_write(const Bufs& b, hipStream_t s) {
    hipLaunchKernelGGL((write_nt<K, BLOCK>), dim3((unsigned)(b.n / (256 * K) / (BLOCK / 64))), dim3(BLOCK), 0, s,
                       b.y);
}

template <int P, int R, int POL, int BLOCK>
void l_wpat(const Bufs& b, hipStream_t s) {
    hipLaunchKernelGGL((write_pat<P, R, POL, BLOCK>), dim3((unsigned)(b.n / (256 * R) / (BLOCK / 64))), dim3(BLOCK),
                       0, s, b.y);
}

template <int H, int P, int POL, int BLOCK>
void l_wdpat(const Bufs& b, hipStream_t s) {
    hipLaunchKernelGGL((widen_pat<H, P, POL, BLOCK>), dim3((unsigned)(b.n / (H ? 256 : 512) / (BLOCK / 64))),
                       dim3(BLOCK), 0, s, b.x, b.y);
}

template <int D, bool NT, int BPC>
void l_pc(const Bufs& b, hipStream_t s) {
    const int64_t ntiles = b.n / 512, blocks = 256 * BPC;
    hipLaunchKernelGGL((widen_pc<D, NT>), dim3((unsigned)blocks), dim3(256), 0, s, b.x, b.y, ntiles,
                       (ntiles + blocks - 1) / blocks);
}

// widen_pat H=1 with the output moved OFF bytes past the allocation start (HBM channel phase
// of the write stream relative to the read stream)
template <int64_t OFF>
void l_wdpat_off(const Bufs& b, hipStream_t s) {
    hipLaunchKernelGGL((widen_pat<1, 0, 1, 256>), dim3((unsigned)(b.n / 256 / 4)), dim3(256), 0, s, b.x,
                       reinterpret_cast<int32_t*>(reinterpret_cast<char*>(b.y) + OFF));
}
// 1:1 copy of the int16 input into the output buffer (16 B per lane, one 1 KiB nt store per wave)
__global__ __launch_bounds__(256) void copy_nt(const u32x4* __restrict__ x, u32x4* __restrict__ y) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    st16<1>(y + i, __builtin_nontemporal_load(x + i));
}
void l_copy(const Bufs& b, hipStream_t s) {
    hipLaunchKernelGGL(copy_nt, dim3((unsigned)(b.n * 2 / 16 / 256)), dim3(256), 0, s, reinterpret_cast<const u32x4*>(b.x),
                       reinterpret_cast<u32x4*>(b.y));
}

// int16 -> u8 narrowing copies (the i16 -> u8 FIR's bytes: 2 B in, 1 B out per sample): a wave
// reads K KiB (K 16-byte loads per lane, each a contiguous 1 KiB) and writes K/2 KiB (the high
// bytes), as 8-byte (K = 1) or 16-byte stores per lane; POL as st16 (0 plain, 1 nt).
template <int K, int POL>
__global__ __launch_bounds__(256) void narrow_copy(const u32x4* __restrict__ x, uint8_t* __restrict__ y) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
    const u32x4* src = x + wave * (64 * K);
    u32x4 d[K];
#pragma unroll
    for (int k = 0; k < K; ++k) d[k] = __builtin_nontemporal_load(src + k * 64 + lane);
    uint32_t h[2 * K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        h[2 * k] = __builtin_amdgcn_perm(d[k].y, d[k].x, 0x07050301u);
        h[2 * k + 1] = __builtin_amdgcn_perm(d[k].w, d[k].z, 0x07050301u);
    }
    if constexpr (K == 1) {
        u32x2* dst = reinterpret_cast<u32x2*>(y) + wave * 64 + lane;
        if constexpr (POL == 1) __builtin_nontemporal_store(u32x2{h[0], h[1]}, dst);
        else *dst = u32x2{h[0], h[1]};
    } else {
        // two input rows' high bytes per 1 KiB of output, as two 512-byte row stores (a traffic
        // ceiling: the byte order differs from the input's and is not checked)
#pragma unroll
        for (int j = 0; j < K / 2; ++j) {
            u32x2* dst = reinterpret_cast<u32x2*>(y) + wave * (64 * K) + 128 * j;
            if constexpr (POL == 1) {
                __builtin_nontemporal_store(u32x2{h[4 * j], h[4 * j + 1]}, dst + lane);
                __builtin_nontemporal_store(u32x2{h[4 * j + 2], h[4 * j + 3]}, dst + 64 + lane);
            } else {
                dst[lane] = u32x2{h[4 * j], h[4 * j + 1]};
                dst[64 + lane] = u32x2{h[4 * j + 2], h[4 * j + 3]};
            }
        }
    }
}
template <int K, int POL>
void l_narrow(const Bufs& b, hipStream_t s) {
    hipLaunchKernelGGL((narrow_copy<K, POL>), dim3((unsigned)(b.n / (512 * K) / 4)), dim3(256), 0, s,
                       reinterpret_cast<const u32x4*>(b.x), reinterpret_cast<uint8_t*>(b.y));
}

// The long-filter MFMA kernel's memory pattern, rebuilt step by step from narrow_copy (dev
// ladder): persistent waves walk 1024-sample tiles grid-stride (2048 blocks of 4 waves), read a
// tile's window and write its 1 KiB of u8.  W: 0 = the tile's 2 KiB, 1 = the MFMA kernel's
// window (1088 samples from 16 before the tile, 3 loads per lane, lanes past it re-load its last
// vector).  PF: window of the next tile loaded before this tile's store (1 in flight).  LDS:
// the window goes through wave-private LDS as two byte planes, read back as 16-byte fragments.
template <int W, bool PF, bool LDS>
__global__ __launch_bounds__(256, 4) void mfpat(const int16_t* __restrict__ x, uint8_t* __restrict__ y, uint32_t ntiles) {
    constexpr int NIT = W ? 3 : 2;
    __shared__ __attribute__((aligned(16))) uint8_t lds[4][2 * 1632];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t step = gridDim.x * 4;
    uint32_t tile = blockIdx.x * 4 + wv;
    u32x4 raw[NIT];
    auto load = [&](uint32_t t) {
        const int64_t w0 = (int64_t)t * 1024 - (W ? 16 : 0);
#pragma unroll
        for (int it = 0; it < NIT; ++it) {
            int v = it * 64 + lane;
            if (W) v = v < 136 ? v : 135;
            int64_t g = w0 + 8 * v;
            g = g < 0 ? 0 : (g > (int64_t)ntiles * 1024 - 8 ? (int64_t)ntiles * 1024 - 8 : g);  // stay inside x
            raw[it] = *reinterpret_cast<const u32x4*>(x + g);
        }
    };
    if (tile < ntiles) load(tile);
    for (; tile < ntiles; tile += step) {
        uint32_t hv[4];
        if constexpr (LDS) {
            uint8_t* ph = lds[wv];
            uint8_t* pl = lds[wv] + 1632;
#pragma unroll
            for (int it = 0; it < NIT; ++it) {
                const int v = it * 64 + lane;
                if (v < 136) {
                    const int pos = 8 * v + ((8 * v) >> 5) * 16;
                    *reinterpret_cast<u32x2*>(&ph[pos]) = u32x2{__builtin_amdgcn_perm(raw[it].y, raw[it].x, 0x07050301u),
                                                                __builtin_amdgcn_perm(raw[it].w, raw[it].z, 0x07050301u)};
                    *reinterpret_cast<u32x2*>(&pl[pos]) = u32x2{__builtin_amdgcn_perm(raw[it].y, raw[it].x, 0x06040200u),
                                                                __builtin_amdgcn_perm(raw[it].w, raw[it].z, 0x06040200u)};
                }
            }
            __builtin_amdgcn_wave_barrier();
            asm volatile("" ::: "memory");
            const int r = lane & 31, hf = lane >> 5;
            u32x4 acc = {0u, 0u, 0u, 0u};
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                const int i = 32 * r + 32 * s + 16 * hf, pos = i + (i >> 5) * 16;
                acc ^= *reinterpret_cast<const u32x4*>(&ph[pos]);
                acc ^= *reinterpret_cast<const u32x4*>(&pl[pos]);
            }
            __builtin_amdgcn_wave_barrier();
            asm volatile("" ::: "memory");
            hv[0] = acc.x, hv[1] = acc.y, hv[2] = acc.z, hv[3] = acc.w;
        } else {
            hv[0] = __builtin_amdgcn_perm(raw[0].y, raw[0].x, 0x07050301u);
            hv[1] = __builtin_amdgcn_perm(raw[0].w, raw[0].z, 0x07050301u);
            hv[2] = __builtin_amdgcn_perm(raw[1].y, raw[1].x, 0x07050301u);
            hv[3] = __builtin_amdgcn_perm(raw[1].w, raw[1].z, 0x07050301u);
        }
        const uint32_t nxt = tile + step < ntiles ? tile + step : tile;
        if constexpr (PF) load(nxt);
        __builtin_nontemporal_store(u32x4{hv[0], hv[1], hv[2], hv[3]}, reinterpret_cast<u32x4*>(y + (int64_t)tile * 1024) + lane);
        if constexpr (!PF) load(nxt);
    }
}
template <int W, bool PF, bool LDS>
void l_mfpat(const Bufs& b, hipStream_t s) {
    hipLaunchKernelGGL((mfpat<W, PF, LDS>), dim3(2048), dim3(256), 0, s, b.x, reinterpret_cast<uint8_t*>(b.y),
                       (uint32_t)(b.n / 1024));
}
// The same tile loop (2 KiB aligned read, 1 KiB store, next tile prefetched) with the work split
// varied: BLOCKS grid-stride blocks (0 = one tile per wave), ORDER 0 = tile += all waves, 1 = each
// wave a contiguous run of tiles, 2 = each XCD (blocks b % 8) a contiguous eighth, walked
// grid-stride by its own waves; MINB = blocks per CU the registers must allow.
template <int ORDER, int MINB, bool NTL = false, bool ST2 = false>
__global__ __launch_bounds__(256, MINB) void mfsplit(const int16_t* __restrict__ x, uint8_t* __restrict__ y,
                                                     uint32_t ntiles) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t nw = gridDim.x * 4, w = blockIdx.x * 4 + wv;
    uint32_t t0, t1, step;
    if constexpr (ORDER == 0 || ORDER == 3) {
        t0 = w, t1 = ntiles, step = nw;
    } else if constexpr (ORDER == 1) {
        const uint32_t per = (ntiles + nw - 1) / nw;
        t0 = w * per, t1 = min(t0 + per, ntiles), step = 1;
    } else {
        const uint32_t x8 = blockIdx.x % 8, per = (ntiles + 7) / 8, lo = x8 * per;
        t0 = lo + (blockIdx.x / 8) * 4 + wv, t1 = min(lo + per, ntiles), step = nw / 8;
    }
    u32x4 raw[2];
    auto load = [&](uint32_t t) {
        const u32x4* src = reinterpret_cast<const u32x4*>(x + (int64_t)t * 1024);
        if constexpr (NTL) {
            raw[0] = __builtin_nontemporal_load(src + lane);
            raw[1] = __builtin_nontemporal_load(src + 64 + lane);
        } else {
            raw[0] = src[lane];
            raw[1] = src[64 + lane];
        }
    };
    if (t0 < t1) load(t0);
    for (uint32_t t = t0; t < t1; t += step) {
        const u32x4 h = {__builtin_amdgcn_perm(raw[0].y, raw[0].x, 0x07050301u), __builtin_amdgcn_perm(raw[0].w, raw[0].z, 0x07050301u),
                         __builtin_amdgcn_perm(raw[1].y, raw[1].x, 0x07050301u), __builtin_amdgcn_perm(raw[1].w, raw[1].z, 0x07050301u)};
        if (ORDER != 3 || t + step < t1) load(t + step < t1 ? t + step : t);  // ORDER 3: no reload past the end
        if constexpr (ST2) {  // two 512-byte row stores (8 bytes per lane each)
            u32x2* d2 = reinterpret_cast<u32x2*>(y + (int64_t)t * 1024);
            __builtin_nontemporal_store(u32x2{h.x, h.y}, d2 + lane);
            __builtin_nontemporal_store(u32x2{h.z, h.w}, d2 + 64 + lane);
        } else {
            __builtin_nontemporal_store(h, reinterpret_cast<u32x4*>(y + (int64_t)t * 1024) + lane);
        }
    }
}
// contiguous runs of RUN tiles per wave over a grid sized to cover them once (dispatch order keeps
// the active region compact)
template <int RUN, int MINB>
void l_mfrun(const Bufs& b, hipStream_t s) {
    const uint32_t nt = (uint32_t)(b.n / 1024);
    hipLaunchKernelGGL((mfsplit<1, MINB, false>), dim3(nt / (4 * RUN)), dim3(256), 0, s, b.x,
                       reinterpret_cast<uint8_t*>(b.y), nt);
}
template <int BLOCKS, int ORDER, int MINB, bool NTL = false, bool ST2 = false>
void l_mfsplit(const Bufs& b, hipStream_t s) {
    const uint32_t nt = (uint32_t)(b.n / 1024);
    hipLaunchKernelGGL((mfsplit<ORDER, MINB, NTL, ST2>), dim3(BLOCKS ? BLOCKS : nt / 4), dim3(256), 0, s, b.x,
                       reinterpret_cast<uint8_t*>(b.y), nt);
}

// Round 3b: persistent grid-stride with BIG steps: a wave reads TPS consecutive 1024-sample int16
// tiles (2 TPS loads of 16 B per lane, all issued together) plus one 16-byte halo vector per lane
// (the next step's first 1 KiB, as a long filter's window needs), converts, and writes TPS KiB of
// u8; the next step's loads are issued right after the conversion (one step in flight while the
// stores go).  LDS: the high bytes pass through wave-private LDS (write + read back) as the MFMA
// kernel's byte planes do.  WALK > 0: each wave instead walks a contiguous run of WALK steps.
template <int TPS, bool LDS, int WALK>
__global__ __launch_bounds__(256, 4) void mfbig(const int16_t* __restrict__ x, uint8_t* __restrict__ y, uint32_t nsteps) {
    constexpr int NL = 2 * TPS;
    __shared__ __attribute__((aligned(16))) uint8_t lds[4][LDS ? 1024 * TPS + 64 : 16];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t step = gridDim.x * 4, s0 = blockIdx.x * 4 + wv, s1 = nsteps;
    if constexpr (WALK > 0) {
        s0 = (blockIdx.x * 4 + wv) * WALK, s1 = min(s0 + WALK, nsteps), step = 1;
    }
    u32x4 raw[NL], halo;
    auto load = [&](uint32_t t) {
        const u32x4* src = reinterpret_cast<const u32x4*>(x + (int64_t)t * 1024 * TPS);
#pragma unroll
        for (int k = 0; k < NL; ++k) raw[k] = src[64 * k + lane];
        halo = t + 1 < nsteps ? src[64 * NL + (lane & 7)] : u32x4{0u, 0u, 0u, 0u};
    };
    if (s0 < s1) load(s0);
    for (uint32_t t = s0; t < s1; t += step) {
        uint32_t h[2 * NL];
#pragma unroll
        for (int k = 0; k < NL; ++k) {
            h[2 * k] = __builtin_amdgcn_perm(raw[k].y, raw[k].x, 0x07050301u);
            h[2 * k + 1] = __builtin_amdgcn_perm(raw[k].w, raw[k].z, 0x07050301u) ^ halo.x;
        }
        if constexpr (LDS) {
            uint8_t* p = lds[wv];
#pragma unroll
            for (int k = 0; k < NL; ++k) *reinterpret_cast<u32x2*>(&p[512 * k + 8 * lane]) = u32x2{h[2 * k], h[2 * k + 1]};
            __builtin_amdgcn_wave_barrier();
            asm volatile("" ::: "memory");
#pragma unroll
            for (int k = 0; k < TPS; ++k) {
                const u32x4 q = *reinterpret_cast<const u32x4*>(&p[1024 * k + 16 * lane]);
                h[4 * k] = q.x, h[4 * k + 1] = q.y, h[4 * k + 2] = q.z, h[4 * k + 3] = q.w;
            }
            __builtin_amdgcn_wave_barrier();
            asm volatile("" ::: "memory");
        }
        load(t + step < s1 ? t + step : t);
#pragma unroll
        for (int k = 0; k < TPS; ++k)
            __builtin_nontemporal_store(u32x4{h[4 * k], h[4 * k + 1], h[4 * k + 2], h[4 * k + 3]},
                                        reinterpret_cast<u32x4*>(y + ((int64_t)t * TPS + k) * 1024) + lane);
    }
}
// The same big-step copy with DYNAMIC step order: each wave takes its next step from a global
// ticket counter (one atomic per step, taken one step ahead), so the steps in flight stay a
// compact, in-order window of addresses as in a one-shot grid.  NTL: non-temporal body loads.
__device__ unsigned g_ticket;
template <int TPS, bool NTL>
__global__ __launch_bounds__(256, 4) void mfticket(const int16_t* __restrict__ x, uint8_t* __restrict__ y, uint32_t nsteps) {
    constexpr int NL = 2 * TPS;
    const int lane = threadIdx.x & 63;
    u32x4 raw[NL], halo;
    auto load = [&](uint32_t t) {
        const u32x4* src = reinterpret_cast<const u32x4*>(x + (int64_t)t * 1024 * TPS);
#pragma unroll
        for (int k = 0; k < NL; ++k) raw[k] = NTL ? __builtin_nontemporal_load(src + 64 * k + lane) : src[64 * k + lane];
        halo = t + 1 < nsteps ? src[64 * NL + (lane & 7)] : u32x4{0u, 0u, 0u, 0u};
    };
    auto take = [&]() {
        unsigned v = 0;
        if (lane == 0) v = atomicAdd(&g_ticket, 1u);
        return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
    };
    uint32_t t = take();
    if (t >= nsteps) return;
    load(t);
    uint32_t nx = take();
    for (;;) {
        uint32_t h[2 * NL];
#pragma unroll
        for (int k = 0; k < NL; ++k) {
            h[2 * k] = __builtin_amdgcn_perm(raw[k].y, raw[k].x, 0x07050301u);
            h[2 * k + 1] = __builtin_amdgcn_perm(raw[k].w, raw[k].z, 0x07050301u) ^ halo.x;
        }
        const uint32_t cur = t;
        t = nx;
        if (t < nsteps) {
            load(t);
            nx = take();
        }
#pragma unroll
        for (int k = 0; k < TPS; ++k)
            __builtin_nontemporal_store(u32x4{h[4 * k], h[4 * k + 1], h[4 * k + 2], h[4 * k + 3]},
                                        reinterpret_cast<u32x4*>(y + ((int64_t)cur * TPS + k) * 1024) + lane);
        if (t >= nsteps) break;
    }
}
template <int TPS, bool NTL, int BLOCKS>
void l_mfticket(const Bufs& b, hipStream_t s) {
    const unsigned zero = 0;
    (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(g_ticket), &zero, sizeof(zero), 0, hipMemcpyHostToDevice, s);
    hipLaunchKernelGGL((mfticket<TPS, NTL>), dim3(BLOCKS), dim3(256), 0, s, b.x, reinterpret_cast<uint8_t*>(b.y),
                       (uint32_t)(b.n / 1024 / TPS));
}

template <int TPS, bool LDS, int BLOCKS, int WALK = 0>
void l_mfbig(const Bufs& b, hipStream_t s) {
    const uint32_t ns = (uint32_t)(b.n / 1024 / TPS);
    const unsigned blocks = WALK ? (ns / WALK + 3) / 4 : BLOCKS;
    hipLaunchKernelGGL((mfbig<TPS, LDS, WALK>), dim3(blocks), dim3(256), 0, s, b.x, reinterpret_cast<uint8_t*>(b.y), ns);
}

template <int E>
void l_whe(const Bufs& b, hipStream_t s) {
    hipLaunchKernelGGL((widen_half_edge<E>), dim3((unsigned)(b.n / 4 / 256)), dim3(256), 0, s, b.x, b.y, b.n / 4);
}

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 15;
    Bufs b;
    b.n = (int64_t)1 << 28;
    // STREAM_ALLOC=1: output fine-grained, 3: output uncached (hipExtMallocWithFlags), 0: hipMalloc
    const int alloc = getenv("STREAM_ALLOC") ? atoi(getenv("STREAM_ALLOC")) : 0;
    CK(hipMalloc(&b.x, b.n * 2));
    if (alloc)
        CK(hipExtMallocWithFlags((void**)&b.y, b.n * 4, alloc == 1 ? hipDeviceMallocFinegrained : hipDeviceMallocUncached));
    else
        CK(hipMalloc(&b.y, b.n * 4 + (8 << 20)));  // + room for the output-offset variants
    printf("output allocation: %s\n", alloc == 1 ? "fine-grained" : (alloc == 3 ? "uncached" : "hipMalloc"));
    std::vector<int16_t> hx(b.n);
    uint32_t r = 12345;
    for (auto& v : hx) {
        r = r * 1664525u + 1013904223u;
        v = (int16_t)(r >> 16);
    }
    CK(hipMemcpy(b.x, hx.data(), b.n * 2, hipMemcpyHostToDevice));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    const double rw = b.n * 6.0, rd = b.n * 2.0, wr = b.n * 4.0;
    std::vector<V> vs = {
        {"widen half row nt", l_wdpat<1, 0, 1, 256>, rw, true, {}},
        {"copy 1:1 int16 nt", l_copy, b.n * 4.0, false, {}},
        {"narrow i16->u8 K2 nt", l_narrow<2, 1>, b.n * 3.0, false, {}},
        {"narrow i16->u8 K4 nt", l_narrow<4, 1>, b.n * 3.0, false, {}},
        {"split one-shot", l_mfsplit<0, 0, 4>, b.n * 3.0, false, {}},
        {"oneshot ntl", l_mfsplit<0, 3, 4, true>, b.n * 3.0, false, {}},
        {"mfpat win pf lds", l_mfpat<1, true, true>, b.n * 3.0, false, {}},
        {"ticket1 b1k", l_mfticket<1, false, 1024>, b.n * 3.0, false, {}},
        {"ticket1 ntl b1k", l_mfticket<1, true, 1024>, b.n * 3.0, false, {}},
        {"ticket2 ntl b1k", l_mfticket<2, true, 1024>, b.n * 3.0, false, {}},
        {"ticket2 ntl b2k", l_mfticket<2, true, 2048>, b.n * 3.0, false, {}},
        {"ticket4 ntl b1k", l_mfticket<4, true, 1024>, b.n * 3.0, false, {}},
        {"big1 b1k", l_mfbig<1, false, 1024>, b.n * 3.0, false, {}},
        {"big2 b1k", l_mfbig<2, false, 1024>, b.n * 3.0, false, {}},
        {"big4 b1k", l_mfbig<4, false, 1024>, b.n * 3.0, false, {}},
        {"big2 b2k", l_mfbig<2, false, 2048>, b.n * 3.0, false, {}},
        {"big4 b2k", l_mfbig<4, false, 2048>, b.n * 3.0, false, {}},
        {"big2 lds b1k", l_mfbig<2, true, 1024>, b.n * 3.0, false, {}},
        {"big4 lds b1k", l_mfbig<4, true, 1024>, b.n * 3.0, false, {}},
        {"big4 lds b2k", l_mfbig<4, true, 2048>, b.n * 3.0, false, {}},
        {"big4 lds oneshot", l_mfbig<4, true, 0, 1>, b.n * 3.0, false, {}},
        {"big2 lds walk4", l_mfbig<2, true, 0, 4>, b.n * 3.0, false, {}},
        {"read reg K1 b256", l_read_reg<1, 256>, rd, false, {}},
        {"write nt rows R1", l_wpat<0, 1, 1, 256>, wr, false, {}},
    };
    // correctness of every widen variant (sampled)
    std::vector<int32_t> hy(b.n);
    for (auto& v : vs) {
        if (!v.widen) continue;
        CK(hipMemset(b.y, 0xA5, b.n * 4));
        CK(hipDeviceSynchronize());  // the memset runs on the null stream; st is non-blocking
        v.fn(b, st);
        CK(hipStreamSynchronize(st));
        CK(hipMemcpy(hy.data(), b.y, b.n * 4, hipMemcpyDeviceToHost));
        int64_t nbad = 0, nunw = 0, first = -1;
        for (int64_t i = 0; i < b.n; ++i)
            if (hy[i] != (int32_t)hx[i]) {
                if (first < 0) first = i;
                ++nbad;
                nunw += hy[i] == (int32_t)0xA5A5A5A5;
            }
        if (nbad) {
            printf("MISMATCH %-24s %lld wrong (%lld never written), first at %lld (tile %lld): %d != %d\n",
                   v.name.c_str(), (long long)nbad, (long long)nunw, (long long)first, (long long)(first / 512),
                   hy[first], (int)hx[first]);
            v.widen = false;
            v.name += " [WRONG]";
        }
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int w = 0; w < 100; ++w) vs[w % vs.size()].fn(b, st);
    const int batch = 20;
    for (int rr = 0; rr < rounds; ++rr)
        for (auto& v : vs) {
            CK(hipEventRecord(e0, st));
            for (int i = 0; i < batch; ++i) v.fn(b, st);
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            v.us.push_back(ms * 1e3f / batch);
        }
    printf("%-26s %10s %10s %10s %8s\n", "variant", "median_us", "min_us", "GB/s", "%8TB/s");
    for (auto& v : vs) {
        std::sort(v.us.begin(), v.us.end());
        const double med = v.us[v.us.size() / 2];
        printf("%-26s %10.1f %10.1f %10.1f %8.1f\n", v.name.c_str(), med, v.us[0], v.bytes / med / 1e3,
               v.bytes / med / 1e3 / 80.0);
    }
    return 0;
}
