// fir1d_reg.h — the register/DPP 1-D FIR kernel template (hot path), shared by the library
// (fir1d_reg_impl.h) and the A/B microbenchmarks (tools/microbench).
//
// Work unit: a wave owns a "tile" of U chunks; chunk u is 64 consecutive 16-byte vectors,
// one per lane, so every load instruction is 1 KiB contiguous.  The (L-1)-sample halo of a
// lane comes from its neighbours' registers by DPP wave shifts; at chunk seams lane 0 / 63
// take lane 63 / 0 of the adjacent chunk through wave rotates, so only the tile's two
// outer edges cost an extra (L2-served) 16-byte load, issued by lane 0 and lane 63.
//
// Arithmetic: fir_1d/model/python/fir_1d_fixed_ref.py:95-126 (reference root) with a
// 32-bit accumulator: wrap-around MACs (v_mad_i32_i24 with taps < 2^23 checked on the host;
// packed v_dot2_i32_i16 for int16 taps over int16 samples [kDot2] or over zero-extended u8
// byte pairs when no accumulator can wrap [kU8Dot2, bias preloaded, v_med3 saturation]),
// wrap to acc_bits by shl/ashr (skipped for acc_bits = 32 [kAcc32]), overflow-free round
// (floor(a/2^f) + bit f-1), saturate (u8) or keep (int32; stored through LDS [kCoal]).
#pragma once

#include "fir1d_reg_launch.h"
#include "fir_common.h"

namespace fir {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
// u8 output planes may start at any byte (a fused bank's planes follow each other, and the
// reference's 4499 x 2999 image puts plane f at f * 13492501): their 16- / 8-byte stores go
// through these byte-aligned types, so the code states the alignment it has; gfx950 runs compute
// queues in unaligned-access mode, and the same global_store_dwordx4 / dwordx2 is emitted.
typedef uint32_t u32x4_u8a __attribute__((ext_vector_type(4), aligned(1)));
typedef uint32_t u32x2_u8a __attribute__((ext_vector_type(2), aligned(1)));
typedef short fir_short2v __attribute__((ext_vector_type(2)));

enum RegFlags : int {
    kNtLoad = 1,   // non-temporal 16-byte loads (streamed once)
    kNtStore = 2,  // non-temporal stores
    kPersist = 4,  // grid-stride over tiles with the next tile's loads issued early
    kDot2 = 8,     // int16 samples, 1 channel, int16 taps: packed v_dot2_i32_i16 MACs
    kAcc32 = 16,   // acc_bits == 32: the wrap is the hardware's, skip the shl/ashr pair
    kU8Dot2 = 32,  // u8 samples, 1 channel, int16 taps, no wrap possible: byte-pair v_dot2 MACs
    kCoal = 64,    // int32 outputs of a full 64-vector chunk go out through LDS as contiguous
                   // 1 KiB store instructions (instead of 16 B per lane at a 16*VEC/4-byte stride)
    kXcd = 128,    // XCD-aware block order: the hardware deals consecutive blocks round-robin
                   // to the 8 XCDs; remap so each XCD (own L2) streams one contiguous eighth
    // with kU8Dot2, u8 stage: filters whose V = 2^(f-1-s) + sum h'[k] x (h = 2^s h') provably
    // stays in [0, 2^16) or [-2^15, 2^15) for every u8 input (plan_u8_pk16, TapsN::pkmode)
    // compute their outputs in PAIRS on v_pk_mad_u16 (exact mod 2^16); u8 stage =
    // clamp(V >> (f-s), 0, 255).  The other filters keep the byte-pair v_dot2 form.
    kU8Pk16 = 256,
    kU8PkHi8 = 1024,  // every filter unsigned with f - s == 8: the output byte is V's high byte
    kHalo = 2048,     // a shard with halos (RowGeom::halo_l / halo_r) instead of zero padding; a
                      // separate instantiation: the extra edge-load branches cost the plain
                      // kernel 1.5 % (256.9 -> 260.8 us, tools/lib_ab.py)
    kEdgeDword = 4096,  // halo of at most one dword per side: a tile away from both buffer ends
                        // fetches both edge dwords with ONE wave-wide dword load (lane 0: the
                        // dword before the tile, lane 63: the dword after it) instead of two
                        // lane-masked 16-byte loads in branches
    // Rows that are not a whole number of vectors (the reference's 4499-wide image), u8 stage, one
    // channel: every vector is computed as if the rows were one signal (no masks, the interior
    // forms), then the lane whose vector holds a row seam rewrites the HLE + HRE outputs around it
    // from the samples of their own row, in registers before the store (ragged_put_bytes).  The masked
    // pair it replaces ran two generic windows for every seam vector: 27.0 vs 13.5 us for the
    // 4499 x 2999 bank (tools/pipeline_probe.py).
    kRagged = 8192,
    // Rows that straddle vectors, other stages / channel counts: seam vectors take the masked
    // generic pair (fir_vector_masked).  Without kMasked or kRagged the launcher guarantees
    // RowGeom::aligned, and the masked pair is not compiled in (it held 45 of the fused u8 bank's
    // 90 VGPRs; single int16 filters keep kMasked for its code layout, fir1d_reg_impl.h).
    kMasked = 16384,
    // with kRagged: every filter's output bytes are held until ONE seam fix after the filter loop,
    // then stored (batch launches that hold a ragged image): the 7 golden images' stage 15.05-15.35
    // vs 15.48-15.95 us, but 2^28-sample banks 4-5 % slower (the stores go out later), so the
    // single-image kernels keep the per-filter form (profiles/r05/pipeline_batch_ab.txt, r05ae)
    kDefer = 32768,
};

// One non-temporal 16-byte row-store of the coalesced path, as inline asm: the same
// `global_store_dwordx4 ... nt` the builtin emits, but 1.6 % faster in this kernel (the compiler
// folds the second row's address into `offset:1024` and reorders; 247.8 -> 243.9 us,
// profiles/r01/micro_i16_sc.txt; the sc0 / sc1 policy bits add nothing).  The s_nop covers the
// VMEM-store-data hazard (a VALU write of the data VGPRs right after a >64-bit store), which the
// compiler cannot see through inline asm.
__device__ __forceinline__ void store16_nt(void* p, u32x4 v) {
    asm volatile("global_store_dwordx4 %0, %1, off nt\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}

constexpr int kNumXcd = 8;

// Block id -> position in the tile order.  Blocks b and b + 8 run on the same XCD; with
// kXcd they get adjacent positions, so a wave's edge vector usually sits in the same L2.
__device__ __forceinline__ int64_t xcd_block(int64_t b, int64_t nb) {
    const int64_t q = nb / kNumXcd;
    return b < q * kNumXcd ? (b % kNumXcd) * q + b / kNumXcd : b;
}

constexpr int kDppWaveRol1 = 0x134;  // lane i <- lane i+1, lane 63 <- lane 0
constexpr int kDppWaveRor1 = 0x13C;  // lane i <- lane i-1, lane 0 <- lane 63

__device__ __forceinline__ uint32_t dpp_rol1(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kDppWaveRol1, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t dpp_ror1(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kDppWaveRor1, 0xF, 0xF, false);
}

// F filters of L taps each (F > 1: several filters share one read of x).
// pk[f][p] packs the taps of window samples 2p and 2p+1 (h[L-1-2p], h[L-2-2p]) as two
// int16 halves for v_dot2 (0 past the end); filled by pack_taps() on the host.
template <int L, int F = 1>
struct TapsN {
    int32_t h[F][L];
    uint32_t pk[F][(L + 1) / 2];
    // kU8Pk16: hb[f][i] = h'[f][L-1-i] (multiplies window byte i of an output) in both 16-bit
    // halves; pkbias = 2^(f-1-s), pkshift = f - s, pkmax = 255, each in both halves
    uint32_t hb[F][L];
    uint32_t pkbias[F], pkshift[F], pkmax;
    uint32_t pkmode[F];  // 0: v_dot2 form, 1: packed-16 unsigned V, 2: packed-16 signed V
    // v_dot2 form, u8 stage: 1 when 2^(frac-1) + sum h x lies in [0, 256 * 2^frac) for every u8
    // x, so the stage is the shift alone (the moving average of the report's bank: no v_med3)
    uint32_t noclamp[F];
};

// noclamp[] for the u8 stage of the no-wrap v_dot2 form (host)
template <int L, int F>
inline void plan_u8_noclamp(TapsN<L, F>& t, int frac) {
    for (int f = 0; f < F; ++f) {
        int64_t vmin = frac >= 1 && frac <= 22 ? (int64_t)1 << (frac - 1) : -1, vmax = vmin;
        for (int k = 0; k < L; ++k) (t.h[f][k] > 0 ? vmax : vmin) += 255 * (int64_t)t.h[f][k];
        t.noclamp[f] = vmin >= 0 && vmax < ((int64_t)256 << frac) ? 1u : 0u;
    }
}

// Packed-16 planning for the u8 stage (host).  Per filter: s = the largest power of two
// common to its taps (s <= frac - 1, frac - s <= 15), h' = h / 2^s, and the range of
// V = 2^(frac-1-s) + sum h' x over u8 x, decided per filter (pkmode).  Returns the flag bits
// to add (0: no filter qualifies) and fills the packed fields.
template <int L, int F>
inline int plan_u8_pk16(TapsN<L, F>& t, int frac) {
    int any = 0;
    for (int f = 0; f < F; ++f) t.pkmode[f] = 0;
    t.pkmax = 0x00FF00FFu;
    if (frac < 1 || frac > 22) return 0;
    for (int f = 0; f < F; ++f) {
        int s = 40;
        for (int k = 0; k < L; ++k) {
            int64_t v = t.h[f][k];
            int z = 0;
            if (v == 0) continue;
            while ((v & 1) == 0) v >>= 1, ++z;
            s = z < s ? z : s;
        }
        if (s == 40) continue;  // an all-zero filter keeps the dot2 form
        s = s < frac - 1 ? s : frac - 1;
        if (frac - s > 15) continue;  // 16-bit shifts take the amount mod 16
        int64_t vmax = (int64_t)1 << (frac - 1 - s), vmin = vmax;
        for (int k = 0; k < L; ++k) {
            const int64_t hp = (int64_t)t.h[f][k] >> s;
            (hp > 0 ? vmax : vmin) += 255 * hp;
        }
        const bool u = vmin >= 0 && vmax <= 65535, sg = vmin >= -32768 && vmax <= 32767;
        if (!u && !sg) continue;
        t.pkmode[f] = u ? 1u : 2u;
        ++any;
        auto rep = [](int64_t v) { return ((uint32_t)v & 0xFFFFu) * 0x10001u; };
        for (int i = 0; i < L; ++i) t.hb[f][i] = rep((int64_t)t.h[f][L - 1 - i] >> s);
        t.pkbias[f] = rep((int64_t)1 << (frac - 1 - s));
        t.pkshift[f] = rep(frac - s);
    }
    if (!any) return 0;
    bool hi8 = any == F;
    for (int f = 0; f < F; ++f) hi8 &= t.pkmode[f] == 1 && t.pkshift[f] == 8u * 0x10001u;
    return kU8Pk16 | (hi8 ? kU8PkHi8 : 0);
}

template <int L, int F>
inline void pack_taps(TapsN<L, F>& t) {
    for (int f = 0; f < F; ++f)
        for (int p = 0; p < (L + 1) / 2; ++p) {
            const int lo = t.h[f][L - 1 - 2 * p];
            const int hi = L - 2 - 2 * p >= 0 ? t.h[f][L - 2 - 2 * p] : 0;
            t.pk[f][p] = ((uint32_t)lo & 0xFFFFu) | ((uint32_t)hi << 16);
        }
}

struct RowGeom {
    int64_t total;      // samples in the buffer (rows * width * channels)
    uint32_t rowlen32;  // width * channels, valid when multi_row
    int multi_row;      // rows > 1 (then total < 2^32 is guaranteed by the host)
    int aligned;        // one row, or rows a whole number of vectors: no vector straddles a row
    // One row that is a shard of a longer signal, a whole number of TILES (64*U vectors), so
    // vectors -1 and nvec are exactly the edge vectors lanes 0 / 63 load: the samples just
    // before / after the row (HL / HR of them, device memory, e.g. a neighbour's HBM mapped
    // over xGMI) stand in for the zero padding there, and the edge outputs come out final.
    const void* halo_l;
    const void* halo_r;
};

// The vector before the row (v = -1: its last `hl` samples = halo[0..hl)) or after it
// (v = nvec: its first `hr` samples = halo[0..hr)), zeros elsewhere.
template <typename InT>
__device__ __forceinline__ void load_halo_vec(const void* halo, bool left, int nh, uint32_t (&d)[4]) {
    constexpr int EPD = InTraits<InT>::kPerDword;
    constexpr int VEC = 4 * EPD;
    const InT* h = static_cast<const InT*>(halo);
    d[0] = d[1] = d[2] = d[3] = 0;
    for (int j = 0; j < nh; ++j) {
        const int pos = left ? VEC - nh + j : j;
        const uint32_t e = (uint32_t)h[j] & (EPD == 4 ? 0xFFu : 0xFFFFu);
        d[pos / EPD] |= e << ((32 / EPD) * (pos % EPD));
    }
}

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

// PRESAT: q already holds the saturated bytes (u8 stage), no clamp needed.
template <int STAGE, int VEC, bool NT, bool PRESAT = false>
__device__ __forceinline__ void store_vec(typename OutTraits<STAGE>::T* __restrict__ y, int64_t g0, int64_t total,
                                          bool full, const int32_t (&q)[VEC]) {
    if (full) {
        if constexpr (STAGE == FIR_OUT_U8_SAT) {
            uint32_t o[VEC / 4];
#pragma unroll
            for (int i = 0; i < VEC / 4; ++i) {
                if constexpr (PRESAT)
                    o[i] = (uint32_t)q[4 * i] | ((uint32_t)q[4 * i + 1] << 8) | ((uint32_t)q[4 * i + 2] << 16) |
                           ((uint32_t)q[4 * i + 3] << 24);
                else
                    o[i] = (uint32_t)stage_out32<STAGE>(q[4 * i]) |
                           ((uint32_t)stage_out32<STAGE>(q[4 * i + 1]) << 8) |
                           ((uint32_t)stage_out32<STAGE>(q[4 * i + 2]) << 16) |
                           ((uint32_t)stage_out32<STAGE>(q[4 * i + 3]) << 24);
            }
            if constexpr (VEC == 16) {
                const u32x4_u8a val = {o[0], o[1], o[2], o[3]};
                u32x4_u8a* p = reinterpret_cast<u32x4_u8a*>(y + g0);
                if constexpr (NT)
                    store16_nt(p, val);  // u8 path: 79.2 -> 78.0 us vs the builtin (micro_u8_asm.txt)
                else
                    *p = val;
            } else {
                const u32x2_u8a val = {o[0], o[1]};
                u32x2_u8a* p = reinterpret_cast<u32x2_u8a*>(y + g0);
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
            if (j < n) y[g0 + j] = PRESAT ? (typename OutTraits<STAGE>::T)q[j] : stage_out32<STAGE>(q[j]);
    }
}

// VEC u8 outputs already packed 4 per dword: one VEC-byte store, bytewise at the ragged end.
template <int VEC, bool NT>
__device__ __forceinline__ void store_u8_dwords(uint8_t* __restrict__ y, int64_t g0, int64_t total, bool full,
                                                const uint32_t (&o)[VEC / 4]) {
    if (full) {
        if constexpr (VEC == 16) {
            const u32x4_u8a val = {o[0], o[1], o[2], o[3]};
            u32x4_u8a* p = reinterpret_cast<u32x4_u8a*>(y + g0);
            if constexpr (NT)
                store16_nt(p, val);
            else
                *p = val;
        } else {
            const u32x2_u8a val = {o[0], o[1]};
            u32x2_u8a* p = reinterpret_cast<u32x2_u8a*>(y + g0);
            if (NT) __builtin_nontemporal_store(val, p); else *p = val;
        }
    } else if (g0 < total) {
        const int n = (int)min((int64_t)VEC, total - g0);
#pragma unroll
        for (int j = 0; j < VEC; ++j)
            if (j < n) y[g0 + j] = (uint8_t)(o[j / 4] >> (8 * (j % 4)));
    }
}

// Sample pair (s, s+1) of the window as two int16 halves; window dword i holds samples
// 2i - 2*NDL and 2i - 2*NDL + 1.  LAST_ZERO: the caller multiplies the high half by 0, so it
// may come from outside the window.
template <int NDL, int NW, int S, bool LAST_ZERO>
__device__ __forceinline__ uint32_t sample_pair(const uint32_t* Wd) {
    constexpr int e = S + 2 * NDL;  // sample index from the window start
    if constexpr (e % 2 == 0) {
        return Wd[e / 2];
    } else if constexpr ((e + 1) / 2 < NW) {
        return __builtin_amdgcn_alignbit(Wd[(e + 1) / 2], Wd[(e - 1) / 2], 16);  // v_alignbit_b32
    } else {
        static_assert(LAST_ZERO, "pair leaves the window");
        return Wd[(e - 1) / 2] >> 16;
    }
}

template <int NDL, int NW, int L, int J, int P>
struct Dot2Row {  // sum over tap pairs p >= P for output J (int16 samples, one channel)
    __device__ static __forceinline__ uint32_t run(const uint32_t* Wd, const uint32_t* pk, uint32_t acc) {
        if constexpr (P < (L + 1) / 2) {
            constexpr int HL = L - 1 - L / 2;
            constexpr int S = J - HL + 2 * P;
            const uint32_t pr = sample_pair<NDL, NW, S, (L % 2 == 1) && (P == (L + 1) / 2 - 1)>(Wd);
            acc = (uint32_t)__builtin_amdgcn_sdot2(__builtin_bit_cast(fir_short2v, pr),
                                                   __builtin_bit_cast(fir_short2v, pk[P]), (int)acc, false);
            return Dot2Row<NDL, NW, L, J, P + 1>::run(Wd, pk, acc);
        } else {
            return acc;
        }
    }
};

template <int NDL, int NW, int L, int J, int VEC, bool ACC32>
struct Dot2Vec {
    __device__ static __forceinline__ void run(const uint32_t* Wd, const uint32_t* pk, int shl, int frac,
                                               int32_t* q) {
        if constexpr (J < VEC) {
            q[J] = round_acc<ACC32>(Dot2Row<NDL, NW, L, J, 0>::run(Wd, pk, 0u), shl, frac);
            Dot2Vec<NDL, NW, L, J + 1, VEC, ACC32>::run(Wd, pk, shl, frac, q);
        }
    }
};

// u8 window bytes K and K+1 zero-extended into two int16 halves (one v_perm_b32, shared by
// every output and filter that uses the pair); past the window the high half is a zero tap's.
template <int NW, int K>
__device__ __forceinline__ uint32_t byte_pair(const uint32_t* Wd) {
    if constexpr (K + 1 < 4 * NW) {
        return pair16<K>(Wd);
    } else {
        return __builtin_amdgcn_perm(0u, Wd[K / 4], (uint32_t)(K % 4) | 0x0C0C0C00u);
    }
}

template <int NDL, int NW, int L, int J, int P>
struct U8Dot2Row {  // sum over tap pairs p >= P for output J, continuing from acc
    __device__ static __forceinline__ uint32_t run(const uint32_t* Wd, const uint32_t* pk, uint32_t acc) {
        if constexpr (P < (L + 1) / 2) {
            constexpr int HL = L - 1 - L / 2;
            const uint32_t pr = byte_pair<NW, J - HL + 2 * P + 4 * NDL>(Wd);
            acc = P == 0 ? dot2_from(pr, pk[0], acc) : dot2_acc(pr, pk[P], acc);
            return U8Dot2Row<NDL, NW, L, J, P + 1>::run(Wd, pk, acc);
        } else {
            return acc;
        }
    }
};

// Packed-16 u8 form: the window byte pairs (w[k], w[k+1]) for k = 0 .. VEC+L-3 (stream byte
// K0 + k), shared by every output pair and filter.
template <int NW, int K0, int N>
struct BytePairs {
    __device__ static __forceinline__ void run(const uint32_t* Wd, uint32_t* P) {
        if constexpr (N > 0) {
            P[0] = byte_pair<NW, K0>(Wd);
            BytePairs<NW, K0 + 1, N - 1>::run(Wd, P + 1);
        }
    }
};

// Output pairs (2q, 2q+1) of one filter: bias + sum_i h'[L-1-i] * (w[2q+i], w[2q+1+i]) mod 2^16,
// taps outer so the VEC/2 chains interleave; then the u8 stage and 4 bytes per dword.
template <int L, int VEC, int FLAGS>
__device__ __forceinline__ void u8_pk16_vec(const uint32_t* P, const uint32_t* hb, uint32_t bias, uint32_t k2,
                                            uint32_t max2, bool sg, uint32_t (&o)[VEC / 4]) {
    uint32_t a[VEC / 2];
#pragma unroll
    for (int q = 0; q < VEC / 2; ++q) a[q] = pk_mad16(P[2 * q], hb[0], bias);
#pragma unroll
    for (int i = 1; i < L; ++i)
        if (hb[i] != 0u)  // wave-uniform: a zero tap (the bank's edge filter) costs nothing
#pragma unroll
            for (int q = 0; q < VEC / 2; ++q) a[q] = pk_mad16(P[2 * q + i], hb[i], a[q]);
#pragma unroll
    for (int d = 0; d < VEC / 4; ++d) {
        if constexpr ((FLAGS & kU8PkHi8) != 0) {
            o[d] = __builtin_amdgcn_perm(a[2 * d + 1], a[2 * d], 0x07050301u);
        } else if (sg) {
            o[d] = __builtin_amdgcn_perm(pk_stage_u8<true>(a[2 * d + 1], k2, max2),
                                         pk_stage_u8<true>(a[2 * d], k2, max2), 0x06040200u);
        } else {
            o[d] = __builtin_amdgcn_perm(pk_stage_u8<false>(a[2 * d + 1], k2, max2),
                                         pk_stage_u8<false>(a[2 * d], k2, max2), 0x06040200u);
        }
    }
}

// No-wrap u8 form: every chain starts at the rounding bias (a VGPR), the u8 stage is
// v_med3 clamp then shift (sat_u8_pixel), the int32 stage one arithmetic shift.
// NC: the filter's u8 stage needs no clamp (TapsN::noclamp): the shift alone.
template <int NDL, int NW, int L, int J, int VEC, int STAGE, bool NC = false>
struct U8Dot2Vec {
    __device__ static __forceinline__ void run(const uint32_t* Wd, const uint32_t* pk, uint32_t bias, int frac,
                                               int32_t sat_hi, int32_t* q) {
        if constexpr (J < VEC) {
            const uint32_t acc = U8Dot2Row<NDL, NW, L, J, 0>::run(Wd, pk, bias);
            if constexpr (NC)
                q[J] = (int32_t)(acc >> frac);  // acc in [0, 256 << frac)
            else
                q[J] = STAGE == FIR_OUT_U8_SAT ? (int32_t)sat_u8_pixel<true>(acc, 0, frac, sat_hi) : (int32_t)acc >> frac;
            U8Dot2Vec<NDL, NW, L, J + 1, VEC, STAGE, NC>::run(Wd, pk, bias, frac, sat_hi, q);
        }
    }
};

// Interior vector (the whole window inside one row): no masks.
template <typename InT, int L, int CH, bool ACC32>
__device__ __forceinline__ void fir_vector_interior(const int32_t* w, const int32_t* taps, int shl, int frac,
                                                    int32_t* q) {
    constexpr int VEC = 4 * InTraits<InT>::kPerDword;
    constexpr int C = L / 2;
    constexpr int HLE = (L - 1 - C) * CH;
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
        uint32_t acc = 0;
#pragma unroll
        for (int k = 0; k < L; ++k) acc += (uint32_t)__mul24(taps[k], w[HLE + j + (C - k) * CH]);
        q[j] = round_acc<ACC32>(acc, shl, frac);
    }
}

// Vector whose window crosses a row edge (or a buffer end).  In window-relative sample
// offsets o (vector start = 0) the vector's row spans [-a, b) and the next row [b, b + r);
// outputs j < b see window w1 (samples outside [-a, b) zeroed), outputs j >= b window w2.
// Both are plain interior sums; all tests are 32-bit (a, b, r clamped far beyond the window).
template <typename InT, int L, int CH, bool ACC32>
__device__ __forceinline__ void fir_vector_masked(const int32_t* w, int a, int b, int r, const int32_t* taps,
                                                  int shl, int frac, int32_t* q) {
    constexpr int VEC = 4 * InTraits<InT>::kPerDword;
    constexpr int C = L / 2;
    constexpr int HLE = (L - 1 - C) * CH;
    constexpr int NS = HLE + VEC + C * CH;
    int32_t w1[NS], w2[NS], q1[VEC], q2[VEC];
#pragma unroll
    for (int i = 0; i < NS; ++i) {
        const int o = i - HLE;
        w1[i] = (o >= -a && o < b) ? w[i] : 0;
        w2[i] = (o >= b && o < b + r) ? w[i] : 0;
    }
    fir_vector_interior<InT, L, CH, ACC32>(w1, taps, shl, frac, q1);
    fir_vector_interior<InT, L, CH, ACC32>(w2, taps, shl, frac, q2);
#pragma unroll
    for (int j = 0; j < VEC; ++j) q[j] = j < b ? q1[j] : q2[j];
}

// kRagged: the outputs p = b - HRE .. b + HLE - 1 around a row seam at vector offset b (rows start
// at b) are recomputed from the samples of their own row and put into the vector's output
// registers BEFORE its store, so every line is still written once and whole (a byte store after
// the 16-byte store turned those lines into partial writes: 14.5 vs 11.4 us for the 4499- vs
// 4496-wide image, tools/pipeline_probe.py).  s[k] = sample b - NP + k; output i (p = b - HRE + i)
// lies in the row after the seam iff i >= HRE, sample k iff k >= NP; both tests are static.
// ragged_samples takes the samples from the lane's own window w (w[0] = sample -HLE) by selects
// over its NS entries: every sample an output inside the vector needs lies in it (the rest read 0
// and feed only outputs outside the vector, which are never inserted).
template <int L, int NS>
__device__ __forceinline__ void ragged_samples(const int32_t (&w)[NS], int b, int32_t (&sv)[2 * (L - 1) + 1]) {
    constexpr int C = L / 2, HLE = L - 1 - C, NP = L - 1;
#pragma unroll
    for (int k = 0; k < 2 * NP; ++k) {
        const int j = b - NP + k + HLE;  // window index
        int32_t v = 0;
#pragma unroll
        for (int q = 0; q < NS; ++q) v = j == q ? w[q] : v;
        sv[k] = v;
    }
}

// The same for u8 samples straight from the window dwords Wd[NW] (sample o of the vector is
// byte 4 * NDL + o): the 2 * NP bytes span at most ND dwords of [PADL zero dwords, Wd..., zeros],
// picked by selects on the dword index, then byte-aligned: about 30 VALU ops for L = 3 where
// ragged_samples spends 144.  The pad keeps the first byte index >= 0 for every seam offset
// b >= 1 - HLE.
template <int L, int NW, int NDL>
__device__ __forceinline__ void ragged_samples_u8(const uint32_t (&Wd)[NW], int b, int32_t (&sv)[2 * (L - 1) + 1]) {
    constexpr int NP = L - 1, ND = (2 * NP + 3) / 4 + 1, HLE = L - 1 - L / 2, PADL = (HLE + NP + 3) / 4;
    const int B0 = b - NP + 4 * (NDL + PADL);
    const int d0 = B0 >> 2;
    uint32_t dw[ND];
#pragma unroll
    for (int e = 0; e < ND; ++e) {
        uint32_t v = 0;
#pragma unroll
        for (int q = 0; q < NW; ++q) v = d0 + e == PADL + q ? Wd[q] : v;
        dw[e] = v;
    }
    const uint32_t sh = 8u * (uint32_t)(B0 & 3);
#pragma unroll
    for (int k = 0; k < 2 * NP; ++k) {
        const uint32_t lo = dw[k / 4], hi = dw[k / 4 + 1];
        const uint32_t four = (uint32_t)(((uint64_t)hi << 32 | lo) >> sh);  // bytes k/4*4 .. +3
        sv[k] = (int32_t)((four >> (8 * (k % 4))) & 0xFFu);
    }
}

// Tap kk of filter f.  FROMPK (the v_dot2 kernels, int16 taps): unpacked from the pairs
// pk[f][p] = h[L-1-2p] | h[L-2-2p] << 16, which those kernels hold anyway, instead of keeping
// h[][] live as F * L more SGPRs across the tile (the batch kernel spilled SGPRs into VGPR lanes).
template <int L, int F, bool FROMPK>
__device__ __forceinline__ int32_t ragged_tap(const TapsN<L, F>& taps, int f, int kk) {
    if constexpr (FROMPK) {
        const uint32_t pr = taps.pk[f][(L - 1 - kk) / 2];
        return (L - 1 - kk) % 2 == 0 ? (int32_t)(int16_t)(pr & 0xFFFFu) : (int32_t)pr >> 16;
    } else {
        return taps.h[f][kk];
    }
}

// Seam output i of filter f, rounded (before the stage).  NOWRAP (the byte-pair kernels, chosen
// only when no sum can wrap): the sum starts at the rounding bias 2^(f-1) and one arithmetic shift
// rounds it, floor((a + 2^(f-1)) / 2^f) = (a >> f) + bit f-1 of a, as the main path does; the
// wrap and the two-term rounding of round_acc are identities there.  Fewer operations, the same
// time within noise (profiles/r05/pipeline_batch_ab.txt, r05am; without any seam values, a
// timing-only build, the stage ran 0.6 us faster).
template <int L, int F, bool ACC32, bool FROMPK, bool NOWRAP>
__device__ __forceinline__ int32_t ragged_value(const int32_t (&sv)[2 * (L - 1) + 1], const TapsN<L, F>& taps, int f,
                                                int i, int shl, int frac, uint32_t bias) {
    constexpr int C = L / 2, HLE = L - 1 - C, HRE = C, NP = L - 1;
    uint32_t acc = NOWRAP ? bias : 0u;
#pragma unroll
    for (int t = -HLE; t <= HRE; ++t) {
        const int k = i + t + HLE;
        if ((i >= HRE) == (k >= NP)) acc += (uint32_t)__mul24(ragged_tap<L, F, FROMPK>(taps, f, C - t), sv[k]);
    }
    if constexpr (NOWRAP)
        return (int32_t)acc >> frac;
    else
        return round_acc<ACC32>(acc, shl, frac);
}

// Put one filter's seam outputs pv[i] (rounded, before the stage) into the packed output bytes
// o[VEC / 4] at vector offsets p0 + i.  The byte masks m[i][d] are plain VGPR values computed
// once per vector (as lane-mask compares the compiler hoisted them out of the filter loop into
// SGPR pairs and spilled SGPRs).
template <int NP, int VEC>
__device__ __forceinline__ void ragged_masks(int p0, uint32_t (&m)[NP][VEC / 4]) {
#pragma unroll
    for (int i = 0; i < NP; ++i)
#pragma unroll
        for (int d = 0; d < VEC / 4; ++d) {
            const uint32_t sd = (uint32_t)(p0 + i - 4 * d);  // byte of dword d, when < 4
            m[i][d] = sd < 4u ? 0xFFu << (8u * sd) : 0u;
        }
}

template <int NP, int VEC>
__device__ __forceinline__ void ragged_put_bytes(const int32_t* pv, const uint32_t (&m)[NP][VEC / 4],
                                                 uint32_t (&o)[VEC / 4]) {
#pragma unroll
    for (int i = 0; i < NP; ++i) {
        const uint32_t v = stage_out32<FIR_OUT_U8_SAT>(pv[i]) * 0x01010101u;  // the byte in every position
#pragma unroll
        for (int d = 0; d < VEC / 4; ++d) o[d] = (o[d] & ~m[i][d]) | (v & m[i][d]);
    }
}

// A seam wave's shared part: every filter's seam outputs pv (from the lane's window: Wd for u8
// samples, the int32 window w otherwise) and the byte masks pm that put them at vector offsets
// sb - HRE .. (all zero in a lane without a seam).
template <typename InT, int L, int F, int VEC, bool ACC32, bool FROMPK, bool NOWRAP, int NDL, int NW, int NS>
__device__ __forceinline__ void ragged_prepare(const uint32_t (&Wd)[NW], const int32_t (&w)[NS], bool seam, int sb,
                                               const TapsN<L, F>& taps, int shl, int frac, uint32_t bias,
                                               int32_t (&pv)[F][L - 1],
                                               uint32_t (&pm)[L - 1][VEC / 4]) {
    int32_t sv[2 * (L - 1) + 1];
    if constexpr (sizeof(InT) == 1)
        ragged_samples_u8<L, NW, NDL>(Wd, sb, sv);
    else
        ragged_samples<L>(w, sb, sv);
#pragma unroll
    for (int f = 0; f < F; ++f)
#pragma unroll
        for (int i = 0; i < L - 1; ++i)
            pv[f][i] = ragged_value<L, F, ACC32, FROMPK, NOWRAP>(sv, taps, f, i, shl, frac, bias);
    ragged_masks<L - 1, VEC>(seam ? sb - L / 2 : -2 * VEC, pm);
}

// The tiles tile, tile + stride, ... below ntiles of one buffer (wave-uniform tile); output
// plane f (g.total samples) at yf[f].
template <typename InT, int STAGE, int L, int CH, int U, int FLAGS, int F>
__device__ __forceinline__ void fir1d_reg_body(const InT* __restrict__ x, typename OutTraits<STAGE>::T* const (&yf)[F],
                                               const RowGeom& g, const TapsN<L, F>& taps, int shl, int frac,
                                               int64_t ntiles, int64_t tile, int64_t stride) {
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
    constexpr bool DOT2 = (FLAGS & kDot2) && sizeof(InT) == 2 && CH == 1;
    constexpr bool ACC32 = FLAGS & kAcc32;
    constexpr bool U8DOT2 = (FLAGS & kU8Dot2) && sizeof(InT) == 1 && CH == 1;
    constexpr bool U8PK = U8DOT2 && (FLAGS & kU8Pk16) && STAGE == FIR_OUT_U8_SAT;
    constexpr bool HALO = (FLAGS & kHalo) != 0;
    constexpr bool COAL = (FLAGS & kCoal) && STAGE == FIR_OUT_I32;
    constexpr bool RAGGED = (FLAGS & kRagged) && STAGE == FIR_OUT_U8_SAT && CH == 1;
    constexpr bool MASKED = (FLAGS & kMasked) != 0;
    constexpr bool DEFER = RAGGED && (FLAGS & kDefer) && L > 1;
    uint32_t bias = 0;
    int32_t sat_hi = 0;
    if constexpr (U8DOT2) {
        asm("v_mov_b32 %0, %1" : "=v"(bias) : "s"(1u << (frac - 1)));  // once, for dot2_from's addend
        sat_hi = (256 << frac) - 1;
    }

    const int lane = threadIdx.x & (kWave - 1);
    const int64_t total = g.total;
    const int64_t nvec = total / VEC;

    uint32_t own[U][4];
    if (tile < ntiles) {
#pragma unroll
        for (int u = 0; u < U; ++u) load_vec<InT, NTL>(x, tile * (kWave * U) + u * kWave + lane, nvec, total, own[u]);
    }
    // one tile per wave unless PERSIST: no loop, so nothing stays live past the tile's stores (the
    // batch kernel spilled SGPRs with the loop).  Multi-chunk tiles (U > 1: one u8 filter) keep the
    // loop form (it runs once there too): 77.8 vs 78.5 us, profiles/r05/u8_loop_form_ab.txt
    for (; tile < ntiles; tile = (PERSIST || U > 1) ? tile + stride : ntiles) {
        const int64_t vb = tile * (kWave * U);
        uint32_t hv[4] = {0, 0, 0, 0};
        constexpr bool EDW = (FLAGS & kEdgeDword) && NDL <= 1 && NDR <= 1;
        if (EDW && vb > 0 && (vb + kWave * U + 1) * VEC <= total) {  // wave-uniform
            const int64_t e = lane == 0 ? vb * VEC - EPD : (lane == kWave - 1 ? (vb + kWave * U) * VEC : vb * VEC);
            const uint32_t d = *reinterpret_cast<const uint32_t*>(x + e);
            hv[0] = d;  // lane 63's right seam (dword 0 of the vector after the tile)
            hv[3] = d;  // lane 0's left seam (dword 3 of the vector before it)
        } else if (lane == 0) {
            if (NDL > 0) {
                if (HALO && vb == 0 && g.halo_l != nullptr)
                    load_halo_vec<InT>(g.halo_l, true, HLE, hv);
                else
                    load_vec<InT, false>(x, vb - 1, nvec, total, hv);
            }
        } else if (lane == kWave - 1) {
            if (NDR > 0) {
                if (HALO && vb + kWave * U == nvec && g.halo_r != nullptr)
                    load_halo_vec<InT>(g.halo_r, false, HRE, hv);
                else
                    load_vec<InT, false>(x, vb + kWave * U, nvec, total, hv);
            }
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
            // window dwords: NDL from lane-1 | 4 own | NDR from lane+1
            constexpr int NW = NDL + 4 + NDR;
            uint32_t Wd[NW];
#pragma unroll
            for (int qd = 0; qd < NDL; ++qd) {
                const int src = 4 - NDL + qd;
                const uint32_t seam = u == 0 ? hv[src] : dpp_ror1(own[u - 1][src]);
                Wd[qd] = from_prev_lane(seam, own[u][src]);
            }
#pragma unroll
            for (int qd = 0; qd < 4; ++qd) Wd[NDL + qd] = own[u][qd];
#pragma unroll
            for (int qd = 0; qd < NDR; ++qd) {
                const uint32_t seam = u == U - 1 ? hv[qd] : dpp_rol1(own[u + 1][qd]);
                Wd[NDL + 4 + qd] = from_next_lane(seam, own[u][qd]);
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
                bool interior = col0 >= HLE && col0 + VEC + HRE <= rowlen;
                if ((!MASKED && !RAGGED) || g.aligned) {
                    // Every vector lies inside one row, so only its halo can leave the row: zero
                    // the halo dwords (all of their samples are in the neighbouring row) and take
                    // the unmasked path.  One row: the loads already zero-fill beyond both ends.
                    if (g.multi_row) {
                        const bool zl = col0 == 0, zr = col0 + VEC == rowlen;
#pragma unroll
                        for (int qd = 0; qd < NDL; ++qd) Wd[qd] = zl ? 0u : Wd[qd];
#pragma unroll
                        for (int qd = 0; qd < NDR; ++qd) Wd[NDL + 4 + qd] = zr ? 0u : Wd[NDL + 4 + qd];
                    }
                    interior = true;
                }
                const bool seam = RAGGED && !interior;  // this vector holds a row seam's outputs
                if constexpr (RAGGED) interior = true;  // computed as one signal, seams patched below
                constexpr int64_t kFar = 1 << 24;  // beyond any window offset
                const int ma = (int)min(col0, kFar), mb = (int)min(rowlen - col0, kFar), mr = (int)min(rowlen, kFar);
                // samples of the window as int32 (first window sample = -HLE)
                int32_t w[HLE + VEC + HRE];
#pragma unroll
                for (int i = 0; i < HLE + VEC + HRE; ++i) {
                    constexpr int off = NDL * EPD - HLE;
                    w[i] = IT::get(Wd[(off + i) / EPD], (off + i) % EPD);
                }
                uint32_t Pp[VEC + L - 2];  // U8PK: byte pairs of the window, shared by the filters
                if constexpr (U8PK) BytePairs<NW, 4 * NDL - HLE, VEC + L - 2>::run(Wd, Pp);
                // RAGGED: in a wave with a seam (a wave-uniform test, so no exec masks to hold), every
                // lane computes its seam outputs pv once; lanes without a seam put them nowhere
                constexpr int NPR = RAGGED && L > 1 ? L - 1 : 1;
                int32_t pv[F][NPR];
                uint32_t pm[NPR][VEC / 4];
                uint32_t ob[DEFER ? F : 1][VEC / 4];  // DEFER: every filter's bytes, stored after the seam fix
                bool anyseam = false;
                const int sb = col0 < HLE ? -(int)col0 : (int)(rowlen - col0);  // RAGGED: the seam's vector offset
                if constexpr (RAGGED && L > 1 && !DEFER) {
                    anyseam = __builtin_amdgcn_ballot_w64(seam) != 0;
                    if (anyseam)
                        ragged_prepare<InT, L, F, VEC, ACC32, U8DOT2 || DOT2, U8DOT2, NDL>(Wd, w, seam, sb, taps, shl, frac, bias,
                                                                                   pv, pm);
                }
#pragma unroll
                for (int f = 0; f < F; ++f) {
                    if constexpr (U8PK) {
                        const uint32_t md = taps.pkmode[f];  // wave-uniform
                        if (__builtin_expect(interior, 1) && md != 0) {
                            uint32_t o[VEC / 4];
                            u8_pk16_vec<L, VEC, FLAGS>(Pp, taps.hb[f], taps.pkbias[f], taps.pkshift[f], taps.pkmax,
                                                       md == 2, o);
                            if constexpr (DEFER) {
#pragma unroll
                                for (int d = 0; d < VEC / 4; ++d) ob[f][d] = o[d];
                                continue;
                            } else if constexpr (RAGGED && L > 1) {
                                if (anyseam) ragged_put_bytes<NPR, VEC>(pv[f], pm, o);
                            }
                            store_u8_dwords<VEC, NTS>(reinterpret_cast<uint8_t*>(yf[f]), g0, total, v < nvec, o);
                            continue;
                        }
                    }
                    int32_t q[VEC];
                    if (__builtin_expect(interior, 1)) {
                        if constexpr (DOT2) {
                            Dot2Vec<NDL, NW, L, 0, VEC, ACC32>::run(Wd, taps.pk[f], shl, frac, q);
                        } else if constexpr (U8DOT2) {
                            if (STAGE == FIR_OUT_U8_SAT && taps.noclamp[f])  // wave-uniform
                                U8Dot2Vec<NDL, NW, L, 0, VEC, STAGE, true>::run(Wd, taps.pk[f], bias, frac, sat_hi, q);
                            else
                                U8Dot2Vec<NDL, NW, L, 0, VEC, STAGE>::run(Wd, taps.pk[f], bias, frac, sat_hi, q);
                        } else {
                            fir_vector_interior<InT, L, CH, ACC32>(w, taps.h[f], shl, frac, q);
                        }
                    } else {
                        fir_vector_masked<InT, L, CH, ACC32>(w, ma, mb, mr, taps.h[f], shl, frac, q);
                        if constexpr (U8DOT2) {
#pragma unroll
                            for (int j = 0; j < VEC; ++j) q[j] = stage_out32<STAGE>(q[j]);
                        }
                    }
                    if constexpr (RAGGED && L > 1) {  // u8 stage: pack, put the seam bytes, store
                        uint32_t o[VEC / 4];
#pragma unroll
                        for (int d = 0; d < VEC / 4; ++d) {
                            uint32_t t = 0;
#pragma unroll
                            for (int e = 0; e < 4; ++e)
                                t |= (uint32_t)(U8DOT2 ? q[4 * d + e] : stage_out32<STAGE>(q[4 * d + e])) << (8 * e);
                            o[d] = t;
                        }
                        if constexpr (DEFER) {
#pragma unroll
                            for (int d = 0; d < VEC / 4; ++d) ob[f][d] = o[d];
                            continue;
                        } else {
                            if (anyseam) ragged_put_bytes<NPR, VEC>(pv[f], pm, o);
                            store_u8_dwords<VEC, NTS>(reinterpret_cast<uint8_t*>(yf[f]), g0, total, v < nvec, o);
                            continue;
                        }
                    }
                    if constexpr (COAL) {
                        if (vb + (u + 1) * kWave <= nvec) {  // wave-uniform: the whole chunk is full
                            __shared__ u32x4 sbuf[kBlock * VEC / 4];
                            u32x4* wb = sbuf + (threadIdx.x - lane) * (VEC / 4);
#pragma unroll
                            for (int i = 0; i < VEC / 4; ++i)
                                wb[lane * (VEC / 4) + i] = u32x4{(uint32_t)q[4 * i], (uint32_t)q[4 * i + 1],
                                                                 (uint32_t)q[4 * i + 2], (uint32_t)q[4 * i + 3]};
                            __builtin_amdgcn_wave_barrier();  // one wave's LDS ops complete in order
                            asm volatile("" ::: "memory");
                            u32x4* yw = reinterpret_cast<u32x4*>(yf[f] + (vb + u * kWave) * VEC);
#pragma unroll
                            for (int i = 0; i < VEC / 4; ++i) {
                                if constexpr (NTS)
                                    store16_nt(&yw[i * kWave + lane], wb[i * kWave + lane]);
                                else
                                    yw[i * kWave + lane] = wb[i * kWave + lane];
                            }
                            asm volatile("" ::: "memory");
                            continue;
                        }
                    }
                    store_vec<STAGE, VEC, NTS, U8DOT2>(yf[f], g0, total, v < nvec, q);
                }
                if constexpr (DEFER) {  // one seam fix for every filter, then the stores
                    if (__builtin_amdgcn_ballot_w64(seam) != 0) {
                        ragged_prepare<InT, L, F, VEC, ACC32, U8DOT2 || DOT2, U8DOT2, NDL>(Wd, w, seam, sb, taps, shl, frac, bias,
                                                                                   pv, pm);
#pragma unroll
                        for (int f = 0; f < F; ++f) ragged_put_bytes<NPR, VEC>(pv[f], pm, ob[f]);
                    }
#pragma unroll
                    for (int f = 0; f < F; ++f)
                        store_u8_dwords<VEC, NTS>(reinterpret_cast<uint8_t*>(yf[f]), g0, total, v < nvec, ob[f]);
                }
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

template <typename InT, int STAGE, int L, int CH, int U, int FLAGS, int F = 1>
__global__ __launch_bounds__(kBlock) void fir1d_reg_kernel(const InT* __restrict__ x,
                                                           typename OutTraits<STAGE>::T* __restrict__ y,
                                                           RowGeom g, TapsN<L, F> taps, int shl, int frac,
                                                           int64_t ntiles) {
    constexpr int WPB = kBlock / kWave;
    const int64_t stride = (FLAGS & kPersist) ? (int64_t)gridDim.x * WPB : ntiles;
    const int64_t bpos = (FLAGS & kXcd) ? xcd_block(blockIdx.x, gridDim.x) : (int64_t)blockIdx.x;
    typename OutTraits<STAGE>::T* yf[F];  // plane f at y + f * total
#pragma unroll
    for (int f = 0; f < F; ++f) yf[f] = y + f * g.total;
    fir1d_reg_body<InT, STAGE, L, CH, U, FLAGS, F>(x, yf, g, taps, shl, frac, ntiles, bpos * WPB + (threadIdx.x >> 6),
                                                   stride);
}

// Several images (buffers of rows) in ONE launch, the same F filters over each: the wave tiles
// of image i are tiles tile0[i] .. tile0[i+1] - 1 of the grid, its output planes anywhere
// (y[i][f]).  The pipeline's 7 golden images took 4.1-4.6 us per launch even at 64 x 64 (a
// launch's load -> store latency chain, not bytes), 40-54 us for the 7 (tools/pipeline_probe.py);
// one launch overlaps those chains.
struct RegBatch {
    const void* x[kRegBatch];
    void* y[kRegBatch][4];
    RowGeom g[kRegBatch];
    int64_t tile0[kRegBatch + 1];  // tile0[n] = the launch's tiles
    int n;
};

template <typename InT, int STAGE, int L, int CH, int U, int FLAGS, int F>
__global__ __launch_bounds__(kBlock) void fir1d_reg_batch_kernel(RegBatch b, TapsN<L, F> taps, int shl, int frac) {
    const int64_t tile = (int64_t)blockIdx.x * (kBlock / kWave) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    int i = 0;
#pragma unroll
    for (int k = 1; k < kRegBatch; ++k) i += k < b.n && tile >= b.tile0[k] ? 1 : 0;
    const int64_t nt = b.tile0[i + 1] - b.tile0[i], lt = tile - b.tile0[i];
    if (lt >= nt) return;  // the last block's spare waves
    typename OutTraits<STAGE>::T* yf[F];
#pragma unroll
    for (int f = 0; f < F; ++f) yf[f] = static_cast<typename OutTraits<STAGE>::T*>(b.y[i][f]);
    const RowGeom g = b.g[i];  // one copy, loaded once
    fir1d_reg_body<InT, STAGE, L, CH, U, FLAGS, F>(static_cast<const InT*>(b.x[i]), yf, g, taps, shl, frac, nt, lt,
                                                   nt);
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
