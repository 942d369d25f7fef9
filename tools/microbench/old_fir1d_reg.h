// fir1d_reg.h — the register/DPP 1-D FIR kernel template (hot path), shared by the library
// (fir1d.hip) and the A/B microbenchmark (tools/microbench).
//
// Work unit: a wave owns a "tile" of U chunks; chunk u is 64 consecutive 16-byte vectors,
// one per lane, so every load instruction is 1 KiB contiguous.  The (L-1)-sample halo of a
// lane comes from its neighbours' registers by DPP wave shifts; at chunk seams lane 0 / 63
// take lane 63 / 0 of the adjacent chunk through wave rotates, so only the tile's two
// outer edges cost an extra (L2-served) 16-byte load, issued by lane 0 and lane 63.
//
// Arithmetic: fir_1d/model/python/fir_1d_fixed_ref.py:95-126 (reference root) with a
// 32-bit accumulator: wrap-around MACs on v_mad_i32_i24 (taps < 2^23 checked on the
// host), wrap to acc_bits by shl/ashr, overflow-free round (floor(a/2^f) + bit f-1),
// saturate (u8) or keep (int32).
#pragma once

#include "fir_common.h"

namespace fir_old {
using namespace fir;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

enum RegFlags : int {
    kNtLoad = 1,   // non-temporal 16-byte loads (streamed once)
    kNtStore = 2,  // non-temporal stores
    kPersist = 4,  // grid-stride over tiles with the next tile's loads issued early
};

constexpr int kDppWaveRol1 = 0x134;  // lane i <- lane i+1, lane 63 <- lane 0
constexpr int kDppWaveRor1 = 0x13C;  // lane i <- lane i-1, lane 0 <- lane 63

__device__ __forceinline__ uint32_t dpp_rol1(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kDppWaveRol1, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t dpp_ror1(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kDppWaveRor1, 0xF, 0xF, false);
}

template <int L>
struct TapsN {
    int32_t h[L];
};

struct RowGeom {
    int64_t total;      // samples in the buffer (rows * width * channels)
    uint32_t rowlen32;  // width * channels, valid when multi_row
    int multi_row;      // rows > 1 (then total < 2^32 is guaranteed by the host)
};

// Load vector `v` (VEC samples) into 4 dwords: one 16-byte load when wholly in range,
// element-wise with zero fill at the ragged end, zeros past the end / before 0.
template <typename InT, bool NT>
__device__ __forceinline__ void load_vec(const InT* __restrict__ x, int64_t v, int64_t nvec, int64_t total,
                                         uint32_t (&d)[4]) {
    constexpr int EPD = InTraits<InT>::kPerDword;
    constexpr int VEC = 4 * EPD;
    if (v >= 0 && v < nvec) {
        const u32x4* p = reinterpret_cast<const u32x4*>(x + v * VEC);
        const u32x4 q = NT ? __builtin_nontemporal_load(p) : *p;
        d[0] = q.x;
        d[1] = q.y;
        d[2] = q.z;
        d[3] = q.w;
    } else {
        d[0] = d[1] = d[2] = d[3] = 0;
        const int64_t base = v * VEC;
        if (v >= 0 && base < total) {
            const int n = (int)min((int64_t)VEC, total - base);
            for (int j = 0; j < n; ++j) {
                const uint32_t e = (uint32_t)x[base + j] & (EPD == 4 ? 0xFFu : 0xFFFFu);
                d[j / EPD] |= e << ((32 / EPD) * (j % EPD));
            }
        }
    }
}

template <int STAGE, int VEC, bool NT>
__device__ __forceinline__ void store_vec(typename OutTraits<STAGE>::T* __restrict__ y, int64_t g0, int64_t total,
                                          bool full, const int32_t (&q)[VEC]) {
    if (full) {
        if constexpr (STAGE == FIR_OUT_U8_SAT) {
            uint32_t o[VEC / 4];
#pragma unroll
            for (int i = 0; i < VEC / 4; ++i)
                o[i] = (uint32_t)stage_out32<STAGE>(q[4 * i]) | ((uint32_t)stage_out32<STAGE>(q[4 * i + 1]) << 8) |
                       ((uint32_t)stage_out32<STAGE>(q[4 * i + 2]) << 16) |
                       ((uint32_t)stage_out32<STAGE>(q[4 * i + 3]) << 24);
            if constexpr (VEC == 16) {
                const u32x4 val = {o[0], o[1], o[2], o[3]};
                u32x4* p = reinterpret_cast<u32x4*>(y + g0);
                if (NT) __builtin_nontemporal_store(val, p); else *p = val;
            } else {
                const u32x2 val = {o[0], o[1]};
                u32x2* p = reinterpret_cast<u32x2*>(y + g0);
                if (NT) __builtin_nontemporal_store(val, p); else *p = val;
            }
        } else {
#pragma unroll
            for (int i = 0; i < VEC / 4; ++i) {
                const u32x4 val = {(uint32_t)q[4 * i], (uint32_t)q[4 * i + 1], (uint32_t)q[4 * i + 2],
                                   (uint32_t)q[4 * i + 3]};
                u32x4* p = reinterpret_cast<u32x4*>(y + g0) + i;
                if (NT) __builtin_nontemporal_store(val, p); else *p = val;
            }
        }
    } else if (g0 < total) {
        const int n = (int)min((int64_t)VEC, total - g0);
#pragma unroll
        for (int j = 0; j < VEC; ++j)
            if (j < n) y[g0 + j] = stage_out32<STAGE>(q[j]);
    }
}

// Compute the VEC outputs of one vector from its window (left halo | own | right halo).
template <typename InT, int L, int CH>
__device__ __forceinline__ void fir_vector(const int32_t* w, int64_t col0, int64_t rowlen, const TapsN<L>& taps,
                                           int shl, int frac, int32_t* q) {
    constexpr int VEC = 4 * InTraits<InT>::kPerDword;
    constexpr int C = L / 2;
    constexpr int HLE = (L - 1 - C) * CH;
    constexpr int HRE = C * CH;
    const bool interior = col0 >= HLE && col0 + VEC + HRE <= rowlen;
    if (interior) {
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
            uint32_t acc = 0;
#pragma unroll
            for (int k = 0; k < L; ++k) acc += (uint32_t)__mul24(taps.h[k], w[HLE + j + (C - k) * CH]);
            q[j] = round32(acc, shl, frac);
        }
    } else {
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
            int64_t cj = col0 + j;
            if (cj >= rowlen) cj -= rowlen;  // the vector crossed into the next row
            uint32_t acc = 0;
#pragma unroll
            for (int k = 0; k < L; ++k) {
                const int64_t p = cj + (C - k) * CH;
                const uint32_t t = (uint32_t)__mul24(taps.h[k], w[HLE + j + (C - k) * CH]);
                acc += (p >= 0 && p < rowlen) ? t : 0u;
            }
            q[j] = round32(acc, shl, frac);
        }
    }
}

template <typename InT, int STAGE, int L, int CH, int U, int FLAGS>
__global__ __launch_bounds__(kBlock) void fir1d_reg_kernel(const InT* __restrict__ x,
                                                           typename OutTraits<STAGE>::T* __restrict__ y,
                                                           RowGeom g, TapsN<L> taps, int shl, int frac,
                                                           int64_t ntiles) {
    using IT = InTraits<InT>;
    constexpr int EPD = IT::kPerDword;
    constexpr int VEC = 4 * EPD;
    constexpr int C = L / 2;
    constexpr int HLE = (L - 1 - C) * CH;  // samples needed left of a vector
    constexpr int HRE = C * CH;            // samples needed right of a vector
    static_assert(HLE <= VEC && HRE <= VEC, "halo must fit in one neighbouring vector");
    constexpr int NDL = (HLE + EPD - 1) / EPD;  // dwords shifted in from lane-1
    constexpr int NDR = (HRE + EPD - 1) / EPD;  // dwords shifted in from lane+1
    constexpr bool NTL = FLAGS & kNtLoad, NTS = FLAGS & kNtStore, PERSIST = FLAGS & kPersist;
    constexpr int WPB = kBlock / kWave;

    const int lane = threadIdx.x & (kWave - 1);
    const int64_t total = g.total;
    const int64_t nvec = total / VEC;
    const int64_t stride = PERSIST ? (int64_t)gridDim.x * WPB : ntiles;
    int64_t tile = (int64_t)blockIdx.x * WPB + (threadIdx.x >> 6);  // wave-uniform

    uint32_t own[U][4];
    if (tile < ntiles) {
#pragma unroll
        for (int u = 0; u < U; ++u) load_vec<InT, NTL>(x, tile * (kWave * U) + u * kWave + lane, nvec, total, own[u]);
    }
    for (; tile < ntiles; tile += stride) {
        const int64_t vb = tile * (kWave * U);
        uint32_t hv[4] = {0, 0, 0, 0};
        if (lane == 0) {
            if (NDL > 0) load_vec<InT, false>(x, vb - 1, nvec, total, hv);
        } else if (lane == kWave - 1) {
            if (NDR > 0) load_vec<InT, false>(x, vb + kWave * U, nvec, total, hv);
        }
        uint32_t nxt[U][4];
        if constexpr (PERSIST) {  // next tile's loads go out before this tile's math and stores
            const int64_t nt = tile + stride;
            if (nt < ntiles) {
#pragma unroll
                for (int u = 0; u < U; ++u) load_vec<InT, NTL>(x, nt * (kWave * U) + u * kWave + lane, nvec, total, nxt[u]);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t v = vb + u * kWave + lane;
            const int64_t g0 = v * VEC;
            int32_t w[HLE + VEC + HRE];
            if constexpr (NDL > 0) {
                uint32_t prev[4];
#pragma unroll
                for (int qd = 4 - NDL; qd < 4; ++qd) {
                    const uint32_t seam = u == 0 ? hv[qd] : dpp_ror1(own[u - 1][qd]);
                    prev[qd] = from_prev_lane(seam, own[u][qd]);
                }
#pragma unroll
                for (int i = 0; i < HLE; ++i) {
                    constexpr int base = VEC - HLE;
                    w[i] = IT::get(prev[(base + i) / EPD], (base + i) % EPD);
                }
            }
#pragma unroll
            for (int j = 0; j < VEC; ++j) w[HLE + j] = IT::get(own[u][j / EPD], j % EPD);
            if constexpr (NDR > 0) {
                uint32_t next[4];
#pragma unroll
                for (int qd = 0; qd < NDR; ++qd) {
                    const uint32_t seam = u == U - 1 ? hv[qd] : dpp_rol1(own[u + 1][qd]);
                    next[qd] = from_next_lane(seam, own[u][qd]);
                }
#pragma unroll
                for (int i = 0; i < HRE; ++i) w[HLE + VEC + i] = IT::get(next[i / EPD], i % EPD);
            }
            if (g0 < total) {
                int64_t col0, rowlen;
                if (g.multi_row) {
                    rowlen = g.rowlen32;
                    col0 = (uint32_t)g0 % g.rowlen32;
                } else {
                    rowlen = total;
                    col0 = g0;
                }
                int32_t q[VEC];
                fir_vector<InT, L, CH>(w, col0, rowlen, taps, shl, frac, q);
                store_vec<STAGE, VEC, NTS>(y, g0, total, v < nvec, q);
            }
        }
        if constexpr (PERSIST) {
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int i = 0; i < 4; ++i) own[u][i] = nxt[u][i];
        }
    }
}

// Tiles and grid for a launch of fir1d_reg_kernel<.., U, FLAGS>.
template <typename InT, int U, int FLAGS>
inline void reg_launch_geometry(int64_t total, int persist_blocks, int64_t* ntiles, int64_t* blocks) {
    constexpr int VEC = 4 * InTraits<InT>::kPerDword;
    const int64_t vecs = (total + VEC - 1) / VEC;
    *ntiles = (vecs + (int64_t)kWave * U - 1) / ((int64_t)kWave * U);
    const int64_t need = (*ntiles + (kBlock / kWave) - 1) / (kBlock / kWave);
    *blocks = (FLAGS & kPersist) ? (need < persist_blocks ? need : persist_blocks) : need;
}

}  // namespace fir
