// fir1d_mfma.hip — long 1-D fixed-point filters (10 taps and up) on the matrix cores, SURVEY §8 a1/a6.
//
// Arithmetic: fir_1d/model/python/fir_1d_fixed_ref.py:95-126 (reference root): y[n] =
// sum_t h[t] x[n - t + L/2] wrapped to acc_bits, rounded, staged (u8 saturate or int32).
//
// Why MFMA: past ~20 taps the v_dot2 kernel (fir1d_lds.hip) is VALU-bound (L/2 dot2 per output:
// 432 us for 64 taps over 2^28 int16, 47 % of HBM peak).  A FIR is a Toeplitz product: with
// tile outputs y[ts + 32n + r] (n = block 0..31, r = offset 0..31),
//     Y[r][n] = sum_k A[r][k] * B[k][n],   A[r][k] = h[r + L/2 + P - k],   B[k][n] = x[ts + 32n + k - P],
// one 32x32 output tile per wave of v_mfma_i32_32x32x32_i8 over K = 32 + L/2 + P (P = the left
// halo rounded up to 8) in KS steps of 32.  The products are exact integers, so the split into
// signed bytes only has to be exact too:
//   samples: u8 x = xs + 128 (xs = x ^ 0x80); int16 x = 256 xh + xls + 128 (xh the high byte,
//            xls = low byte ^ 0x80); zero padding is x = 0 (xs = -128) like every other sample;
//   taps:    h = 256 hh + hl, hl = ((h + 128) & 255) - 128, hh = (h - hl) / 256 (a signed byte for
//            h <= 32639; larger taps stay on the v_dot2 kernel);
//   sum h x = 65536 sum hh xh + 256 (sum hl xh + sum hh xls) + sum hl xls + 128 sum h   (int16)
//   sum h x = 256 sum hh xs + sum hl xs + 128 sum h                                   (u8)
// with int32 accumulators combined mod 2^32: the reference's wrap-around sum bit for bit.
//
// Per wave and tile: the 1024 + K - 32 window samples are loaded one tile ahead (branch-free
// 16-/8-byte vectors), split into signed-byte planes on the way into wave-private LDS (u8: one
// XOR per 4 samples; int16: 6 VALU per 8), read back as B fragments (one ds_read_b128 per plane
// and step); the tap fragments (a function of r - k only) sit in VGPRs for the whole grid-stride
// loop.  Outputs go back through the same LDS as whole 1 KiB rows.  Rows (images) whose length
// is a multiple of 8 are tiled row by row, samples of other rows zeroed while staging.
#include <string>
#include <type_traits>
#include <vector>

#include "fir_common.h"
#include "fir_launch.h"

namespace fir {

constexpr int kMfTile = 1024;        // outputs per wave tile (32 B columns x 32 A rows)
constexpr int kMfWaves = kBlock / kWave;
// grid-stride blocks: 2048 (two resident rounds at 4 blocks per CU) rather than one round, 1-5 %
// faster for u8 input (u8 -> u8 at 31 taps 95.7 -> 91.5 us, u8 -> int32 196.5 -> 193.3 us;
// 3072 / 4096 within noise of 2048; profiles/r02/long_taps_mfma_grid.txt)
#ifndef FIR_MFMA_MAXBLOCKS
#define FIR_MFMA_MAXBLOCKS 2048
#endif
constexpr int kMfMaxBlocks = FIR_MFMA_MAXBLOCKS;
#ifndef FIR_MFMA_SCHED               // A/B builds: a scheduling barrier at each tile
#define FIR_MFMA_SCHED 0
#endif
#ifndef FIR_MFMA_MINB                // blocks per CU the register allocation must allow (A/B builds)
#define FIR_MFMA_MINB 4
#endif
#ifndef FIR_MFMA_DEPTH               // windows in flight per wave (1 or 2; A/B builds)
#define FIR_MFMA_DEPTH 1
#endif
#ifndef FIR_MFMA_ACC3                // int16: one middle accumulator for both cross products (A/B)
#define FIR_MFMA_ACC3 0
#endif
#ifndef FIR_MFMA_XCD                 // XCD-major tile order (A/B)
#define FIR_MFMA_XCD 0
#endif
#ifndef FIR_MFMA_LONG_FROM           // filters longer than this take the chunked kernels (A/B: lower);
#define FIR_MFMA_LONG_FROM 65        // 65 taps still fit the step kernel's 3 k-steps (K = 96)
#endif
#ifndef FIR_MR                       // 0: u8 long filters on fir1d_mfma_long_kernel (A/B)
#define FIR_MR 1
#endif
#ifndef FIR_MFMA_MAX_TAPS            // longest filter on the matrix cores (fragment table <= 4 MiB)
#define FIR_MFMA_MAX_TAPS 65536
#endif
#ifndef FIR_MFMA_LONG_BLOCKS         // grid-stride blocks of the chunked kernel
#define FIR_MFMA_LONG_BLOCKS 2048
#endif
#ifndef FIR_MFMA_PIN_A               // keep the tap fragments in registers (A/B)
#define FIR_MFMA_PIN_A 0
#endif
#ifndef FIR_MFMA_EXACT_LOADS         // lanes past a window issue no memory request (A/B)
#define FIR_MFMA_EXACT_LOADS 0
#endif
#ifndef FIR_MFMA_LDAUX               // cache policy of the window loads (2 = non-temporal; A/B)
#define FIR_MFMA_LDAUX 0
#endif
#ifndef FIR_MFMA_TPW                 // > 0: one-shot grid, each wave a run of TPW consecutive tiles with
#define FIR_MFMA_TPW 0               // its tap fragments loaded from a device table (A/B)
#endif
#ifndef FIR_MFMA_TWIN                // A/B twins: 1 = no MFMAs (memory + staging only), 2 = no window loads
#define FIR_MFMA_TWIN 0
#endif

// Tap fragments by diagonal: entry e holds a signed byte of h[d + L/2 + P], d = 31 - e (d = r - k
// of A[r][k]), 0 outside the filter.  Lane (r, h) of k-step s reads entries
// e = 31 - r + 32 s + 16 h + j, j = 0..15 (straight from the kernarg segment, once per wave).
struct MfmaTaps {
    int8_t hi[128];  // hh
    int8_t lo[128];  // hl
};

typedef int mf_i32x4 __attribute__((ext_vector_type(4)));
typedef int mf_i32x16 __attribute__((ext_vector_type(16)));

// LDS byte of window sample i: a 16-byte pad per 32 samples (48-byte rows keep the 32 lanes of a
// B-fragment read on distinct banks)
__host__ __device__ constexpr int mf_pos(int i) { return i + (i >> 5) * 16; }

// Buffer descriptor over [p, p + bytes): loads outside it return 0, stores outside it are dropped
// (the range check is per dword; every row or tile edge here is 8-sample aligned).  Built from
// wave-uniform values only, so the buffer ops need no waterfall loop.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t mf_rsrc(const void* p, uint32_t bytes) {
    const uint64_t a = (uint64_t)(uintptr_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    void* q = (void*)(uintptr_t)(((uint64_t)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(q, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}
constexpr int kMfAuxNt = 2;  // non-temporal cache policy of a buffer op (gfx950)
constexpr uint32_t kMfOff = 0x80000000u;  // a voffset far outside every descriptor (zero padding)

struct MfTile {
    int64_t rs, re, ts;
};

// tile -> row bounds and start; tile and tiles_per_row are wave-uniform and the tile count is
// below 2^32 (mfma_path_ok), so this is one 32-bit scalar division per tile, not a 64-bit VALU one
__device__ __forceinline__ MfTile mf_tile(uint32_t tile, int64_t rowlen, uint32_t tiles_per_row) {
    const uint32_t row = __builtin_amdgcn_readfirstlane(tile / tiles_per_row);
    const uint32_t tr = __builtin_amdgcn_readfirstlane(tile - row * tiles_per_row);
    MfTile t;
    t.rs = (int64_t)row * rowlen;
    t.re = t.rs + rowlen;
    t.ts = t.rs + (int64_t)tr * kMfTile;
    return t;
}

template <typename InT, int STAGE, int KS, bool ACC32, bool FAST>
__global__ __launch_bounds__(kBlock, FIR_MFMA_MINB) void fir1d_mfma_kernel(const InT* __restrict__ x,
                                                            typename OutTraits<STAGE>::T* __restrict__ y,
                                                            int64_t rowlen, int64_t tiles_per_row, int64_t ntiles,
                                                            MfmaTaps taps, const mf_i32x4* __restrict__ frag,
                                                            int P, uint32_t bias, int shl, int frac) {
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    typedef uint32_t u2 __attribute__((ext_vector_type(2)));
    constexpr bool I16 = sizeof(InT) == 2;
    constexpr int WL = 32 * 31 + 32 * KS;  // window samples (from tile start - P)
    constexpr int NV = WL / 8;              // 8-sample vectors
    constexpr int NIT = (NV + kWave - 1) / kWave;
    constexpr int PLANE = mf_pos(WL);       // bytes per byte plane
    constexpr int WBYTES = (I16 ? 2 * PLANE : PLANE) > 4608 ? (I16 ? 2 * PLANE : PLANE) : 4608;  // + int32 output image
    static_assert(WL <= 1088, "window exceeds the planes");
    __shared__ __attribute__((aligned(16))) uint8_t lds[kMfWaves][WBYTES];

    const int lane = threadIdx.x & (kWave - 1);
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform
    const int r = lane & 31, hf = lane >> 5;  // A row / B column, lane half
    uint8_t* pl = lds[wv];             // xs (u8) or xls (int16) plane
    uint8_t* ph = lds[wv] + PLANE;     // xh plane (int16)

    // tap fragments A[r][32 s + 16 hf + j], j = 0..15
    mf_i32x4 a_lo[KS], a_hi[KS];
#pragma unroll
    for (int s = 0; s < KS; ++s) {
        if constexpr (FIR_MFMA_TPW > 0) {  // from the device table: one coalesced 1 KiB load each
            a_lo[s] = frag[(2 * s) * kWave + lane];
            a_hi[s] = frag[(2 * s + 1) * kWave + lane];
            continue;
        }
        uint32_t lo[4] = {0u, 0u, 0u, 0u}, hi[4] = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int e = 31 - r + 32 * s + 16 * hf + j;
            lo[j / 4] |= (uint32_t)(uint8_t)taps.lo[e] << (8 * (j % 4));
            hi[j / 4] |= (uint32_t)(uint8_t)taps.hi[e] << (8 * (j % 4));
        }
        a_lo[s] = mf_i32x4{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3]};
        a_hi[s] = mf_i32x4{(int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
#if FIR_MFMA_PIN_A
        // opaque from here on: under register pressure hipcc otherwise re-packs these fragments
        // from their bytes inside the tile loop (~100 VALU per tile, the int16 kernels' VALU bound)
        asm volatile("" : "+v"(a_lo[s]), "+v"(a_hi[s]));
#endif
    }
    // FAST u8 stage: clamp the biased sum, then shift (FAST implies frac <= 22; unused otherwise)
    const int32_t sat_hi = FAST ? (int32_t)((256u << (frac & 31)) - 1u) : 0;

    uint32_t step = gridDim.x * kMfWaves, nt32 = (uint32_t)ntiles;
    const uint32_t tpr = (uint32_t)tiles_per_row;
    uint32_t tile = blockIdx.x * kMfWaves + wv;
    if constexpr (FIR_MFMA_TPW > 0) {  // a run of consecutive tiles per wave, grid covering them once
        tile = (blockIdx.x * kMfWaves + wv) * FIR_MFMA_TPW;
        step = 1;
        nt32 = tile + FIR_MFMA_TPW < nt32 ? tile + FIR_MFMA_TPW : nt32;
    }
#if FIR_MFMA_XCD
    // XCD-major tiles: blocks b, b + 8, ... share an XCD (round-robin dispatch); give each XCD one
    // contiguous eighth of the tiles, walked grid-stride by its own waves
    if (gridDim.x % 8 == 0) {
        const uint32_t x8 = blockIdx.x % 8, per = (nt32 + 7) / 8, lo = x8 * per;
        step = gridDim.x / 8 * kMfWaves;
        tile = lo + (blockIdx.x / 8) * kMfWaves + wv;
        nt32 = lo + per < nt32 ? lo + per : nt32;
    }
#endif
    // the window of a tile: 8-sample vectors v (lanes past the window re-load its last one),
    // through a descriptor over the tile's part of its row; other rows' samples read as zeros
    uint32_t rawA[NIT][4], rawB[NIT][4];  // rawB: the second window in flight (DEPTH 2)
    auto load_window = [&](const MfTile& t, uint32_t(&raw)[NIT][4]) __attribute__((always_inline)) {
        const int64_t w0 = t.ts - P, base = w0 > t.rs ? w0 : t.rs, end = t.re < w0 + WL ? t.re : w0 + WL;
        const __amdgpu_buffer_rsrc_t rs = mf_rsrc(x + base, (uint32_t)((end - base) * (int64_t)sizeof(InT)));
#pragma unroll
        for (int it = 0; it < NIT; ++it) {
            const int v = min(it * kWave + lane, NV - 1);
            const int64_t g = w0 + 8 * v;
            uint32_t off = g >= base ? (uint32_t)((g - base) * (int64_t)sizeof(InT)) : kMfOff;
#if FIR_MFMA_EXACT_LOADS
            if (NV % kWave != 0 && it * kWave + lane >= NV) off = kMfOff;  // lanes past the window: no request
#endif
            if constexpr (FIR_MFMA_TWIN == 2) {  // no window loads: synthetic samples
                raw[it][0] = off, raw[it][1] = off + 1, raw[it][2] = off + 2, raw[it][3] = off + 3;
            } else if constexpr (I16) {
                const mf_i32x4 q = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, FIR_MFMA_LDAUX);
                raw[it][0] = q.x, raw[it][1] = q.y, raw[it][2] = q.z, raw[it][3] = q.w;
            } else {
                typedef int i32x2 __attribute__((ext_vector_type(2)));
                const i32x2 q = __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, FIR_MFMA_LDAUX);
                raw[it][0] = q.x, raw[it][1] = q.y, raw[it][2] = 0u, raw[it][3] = 0u;
            }
        }
    };
    constexpr int DEPTH = FIR_MFMA_DEPTH;
    if (tile < nt32) load_window(mf_tile(tile, rowlen, tpr), rawA);  // the first tile's window
    if constexpr (DEPTH > 1) {  // and the second's (past the end: the first again)
        if (tile < nt32) load_window(mf_tile(tile + step < nt32 ? tile + step : tile, rowlen, tpr), rawB);
    }

    // A tile's outputs leave LDS into registers at the end of its iteration and are stored one
    // iteration later, right AFTER the next window's conversion: hipcc's wait for a prefetched
    // window does not count stores issued after it (it drains them: vmcnt(2) with 4 stores
    // younger), so stores placed between a window's loads and its use would be waited for
    // every tile.  In this order the wait covers the window and older stores only.
    constexpr int NST = STAGE == FIR_OUT_I32 ? 4 : 1;  // 16-byte stores per lane and tile
    u4 pend[NST];
    __amdgpu_buffer_rsrc_t pend_rd;
    auto flush = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int k = 0; k < NST; ++k)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(mf_i32x4, pend[k]), pend_rd,
                                                   STAGE == FIR_OUT_I32 ? (uint32_t)(256 * k + 4 * lane) * 4u
                                                                        : (uint32_t)(16 * lane),
                                                   0, kMfAuxNt);
    };

    // One tile: convert its prefetched window, store the previous tile, prefetch the next window,
    // MFMA, stage the outputs.
    auto body = [&](uint32_t tile, bool first, uint32_t(&raw)[NIT][4]) __attribute__((always_inline)) {
#if FIR_MFMA_SCHED
        __builtin_amdgcn_sched_barrier(0);  // A/B: keep each tile's instructions in place
#endif
        const MfTile t = mf_tile(tile, rowlen, tpr);
        const int m = (int)min((int64_t)kMfTile, t.re - t.ts);  // outputs of this tile

        // ---- the window as signed-byte planes in LDS
#pragma unroll
        for (int it = 0; it < NIT; ++it) {
            const int v = it * kWave + lane;
            if (NV % kWave == 0 || v < NV) {
                const uint32_t* d = raw[it];
                if constexpr (I16) {  // samples 2q, 2q+1 in dword q: high bytes (1, 3), low bytes (0, 2)
                    *reinterpret_cast<u2*>(&ph[mf_pos(8 * v)]) =
                        u2{__builtin_amdgcn_perm(d[1], d[0], 0x07050301u), __builtin_amdgcn_perm(d[3], d[2], 0x07050301u)};
                    *reinterpret_cast<u2*>(&pl[mf_pos(8 * v)]) =
                        u2{__builtin_amdgcn_perm(d[1], d[0], 0x06040200u) ^ 0x80808080u,
                           __builtin_amdgcn_perm(d[3], d[2], 0x06040200u) ^ 0x80808080u};
                } else {
                    *reinterpret_cast<u2*>(&pl[mf_pos(8 * v)]) = u2{d[0] ^ 0x80808080u, d[1] ^ 0x80808080u};
                }
            }
        }
        if (!first) flush();  // the previous tile's outputs
        // ---- the next tile's window goes out now, its latency hidden behind this tile's math
        // (unconditional: past the last tile it re-loads this one, so every path into the loop
        // header has the same memory operations in flight and the compiler's wait there stays exact)
        if constexpr (FIR_MFMA_TPW != 1)  // one tile per wave: nothing to prefetch
            load_window(mf_tile(tile + DEPTH * step < nt32 ? tile + DEPTH * step : tile, rowlen, tpr), raw);
        __builtin_amdgcn_wave_barrier();  // one wave's LDS ops complete in order
        asm volatile("" ::: "memory");

        // ---- Y = A B over KS k-steps: B[32 s + 16 hf + j][n = r] = window sample 32 r + 32 s + 16 hf + j
        // one accumulator per product: each MFMA's C comes from the one issued 2 (u8) or 4 (int16)
        // MFMAs earlier, never from the one just before it (a back-to-back dependent 32x32 MFMA
        // stalls the wave for the whole latency: one shared middle accumulator cost int16 ~20 %)
        mf_i32x16 acc_ll = {}, acc_mid = {}, acc_m2 = {}, acc_hh = {};
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const int i = mf_pos(32 * r + 32 * s + 16 * hf);
            const mf_i32x4 b_l = *reinterpret_cast<const mf_i32x4*>(&pl[i]);
#if FIR_MFMA_TWIN == 1
            acc_ll[s] += b_l.x ^ a_lo[s].y;  // memory-only twin: keep the B reads, drop the MFMAs
            if constexpr (I16) acc_hh[s] += (*reinterpret_cast<const mf_i32x4*>(&ph[i])).z;
            continue;
#endif
            acc_ll = __builtin_amdgcn_mfma_i32_32x32x32_i8(a_lo[s], b_l, acc_ll, 0, 0, 0);
            acc_mid = __builtin_amdgcn_mfma_i32_32x32x32_i8(a_hi[s], b_l, acc_mid, 0, 0, 0);
            if constexpr (I16) {
                const mf_i32x4 b_h = *reinterpret_cast<const mf_i32x4*>(&ph[i]);
                acc_hh = __builtin_amdgcn_mfma_i32_32x32x32_i8(a_hi[s], b_h, acc_hh, 0, 0, 0);
                if constexpr (FIR_MFMA_ACC3)  // two MFMAs (acc_hh) after the first write of acc_mid
                    acc_mid = __builtin_amdgcn_mfma_i32_32x32x32_i8(a_lo[s], b_h, acc_mid, 0, 0, 0);
                else
                    acc_m2 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a_lo[s], b_h, acc_m2, 0, 0, 0);
            }
        }
        // u8: acc_mid = sum hh xs, acc_ll = sum hl xs; int16: acc_hh = sum hh xh,
        // acc_mid + acc_m2 = sum hh xls + sum hl xh, acc_ll = sum hl xls

        // ---- combine (mod 2^32), wrap, round; C[row][col = r]: register i is tile output
        // 32 r + (i & 3) + 8 (i >> 2) + 4 hf.  FAST (host-proven: no wrap, no overflow of the
        // rounding add): the bias already holds 2^(frac-1), the round is one shift.
        int32_t q[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            uint32_t a;
            if constexpr (I16)
                a = ((uint32_t)(acc_mid[i] + acc_m2[i]) << 8) + (uint32_t)acc_ll[i] + ((uint32_t)acc_hh[i] << 16) + bias;
            else
                a = ((uint32_t)acc_mid[i] << 8) + (uint32_t)acc_ll[i] + bias;
            if constexpr (FAST)
                q[i] = STAGE == FIR_OUT_U8_SAT ? min(max((int32_t)a, 0), sat_hi) : (int32_t)a >> frac;
            else
                q[i] = round_acc<ACC32>(a, shl, frac);
        }
        __builtin_amdgcn_wave_barrier();  // every B read of this tile is done before LDS is reused
        asm volatile("" ::: "memory");
        if constexpr (STAGE == FIR_OUT_I32) {
            // LDS image: block n at dwords [36 n, 36 n + 32) (a 16-byte pad against bank conflicts)
            uint32_t* ob = reinterpret_cast<uint32_t*>(lds[wv]);
#pragma unroll
            for (int g4 = 0; g4 < 4; ++g4)
                *reinterpret_cast<u4*>(&ob[36 * r + 8 * g4 + 4 * hf]) =
                    u4{(uint32_t)q[4 * g4], (uint32_t)q[4 * g4 + 1], (uint32_t)q[4 * g4 + 2], (uint32_t)q[4 * g4 + 3]};
            __builtin_amdgcn_wave_barrier();
            asm volatile("" ::: "memory");
            // one descriptor over the tile's m valid outputs: the stores of a partial tile that
            // fall past m are dropped by the range check, so every tile issues the same 4 stores
            pend_rd = mf_rsrc(y + t.ts, (uint32_t)m * 4u);
#pragma unroll
            for (int rho = 0; rho < 4; ++rho) {  // 1 KiB rows: outputs 256 rho + 4 lane .. + 3
                const int o = 256 * rho + 4 * lane;
                pend[rho] = *reinterpret_cast<const u4*>(&ob[36 * (o >> 5) + (o & 31)]);
            }
        } else {
            // bytes: block n at [48 n, 48 n + 32)
            uint8_t* ob = lds[wv];
#pragma unroll
            for (int g4 = 0; g4 < 4; ++g4) {
                uint32_t w;
                if constexpr (FAST) {  // clamped biased sums: the byte is (c >> frac), c in [0, 2^(frac+8))
                    w = (uint32_t)q[4 * g4] >> frac;
                    w |= ((uint32_t)q[4 * g4 + 1] >> frac) << 8;
                    w |= ((uint32_t)q[4 * g4 + 2] >> frac) << 16;
                    w |= ((uint32_t)q[4 * g4 + 3] >> frac) << 24;
                } else {
                    w = (uint32_t)stage_out32<STAGE>(q[4 * g4]) | ((uint32_t)stage_out32<STAGE>(q[4 * g4 + 1]) << 8) |
                        ((uint32_t)stage_out32<STAGE>(q[4 * g4 + 2]) << 16) |
                        ((uint32_t)stage_out32<STAGE>(q[4 * g4 + 3]) << 24);
                }
                *reinterpret_cast<uint32_t*>(&ob[48 * r + 8 * g4 + 4 * hf]) = w;
            }
            __builtin_amdgcn_wave_barrier();
            asm volatile("" ::: "memory");
            const int o = 16 * lane;
            pend[0] = *reinterpret_cast<const u4*>(&ob[48 * (o >> 5) + (o & 31)]);
            pend_rd = mf_rsrc(y + t.ts, (uint32_t)m);
        }
        __builtin_amdgcn_wave_barrier();  // the output reads are done before the next tile's staging
        asm volatile("" ::: "memory");
    };
    if (tile < nt32) {
        body(tile, true, rawA);
        tile += step;
        if constexpr (DEPTH > 1) {
            // two windows in flight: tiles alternate between the two register sets
            while (tile < nt32) {
                body(tile, false, rawB);
                tile += step;
                if (tile >= nt32) break;
                body(tile, false, rawA);
                tile += step;
            }
        } else {
            for (; tile < nt32; tile += step) body(tile, false, rawA);
        }
        flush();  // the last tile's outputs
    }
}

// ---------------------------------------------------------------------------------------
// Step form (round 3b; the default up to FIR_MFMA_LONG_FROM taps): the same Toeplitz product,
// but a wave's grid-stride unit is a STEP of TPS consecutive tiles of one row, whose window
// (TPS * 1024 + 32 KS - 32 samples) is loaded at once and staged as byte planes in the wave's
// LDS, the tiles' MFMAs reading it at offsets 1024 q.  Why: the tile kernel above keeps about
// 2.2 KiB of useful loads in flight per wave (one window) and its loop header drains the
// second window when two are prefetched (hipcc's wait merges the loop's entry edge, where no
// stores follow the loads, with the back edge: measured DEPTH 2 = no gain), so its int16 forms
// sat at the 147 us the same loop reaches as a pure copy (profiles/r03/long_taps_mfma_structure
// .txt).  Here each wave keeps TPS * 2 KiB (int16) in flight during the whole step's math, the
// window's halo is re-read once per step instead of once per tile, and the loop is shaped so
// the compiler's waits are exact: every path into the loop header has the same memory operations
// in flight (the entry edge issues the step's store count as dropped stores, descriptor size 0),
// every load and store is unconditional (ranges clipped by the descriptors), and the wait at the
// top of a step is vmcnt(stores of the previous step).
#ifndef FIR_MF2                      // 0: the tile kernel for every short filter (A/B)
#define FIR_MF2 1
#endif
#ifndef FIR_MF2_TPS                  // tiles per step
#define FIR_MF2_TPS 2
#endif
#ifndef FIR_MF2_MINB                 // waves per SIMD the register allocation must allow
#define FIR_MF2_MINB 4
#endif
#ifndef FIR_MF2_BLOCKS               // grid-stride blocks (4 waves each; 2048 = two resident rounds)
#define FIR_MF2_BLOCKS 2048
#endif
#ifndef FIR_MF2_OLDS                 // int32 outputs through LDS as 1 KiB rows (0: permlane32 pairs)
#define FIR_MF2_OLDS 1
#endif
#ifndef FIR_MF2_ACC3                 // int16: one accumulator for both cross products
#define FIR_MF2_ACC3 1
#endif
#ifndef FIR_MF2_LDAUX                // cache policy of the body loads: -1 = non-temporal for int16 input
#define FIR_MF2_LDAUX -1             // (i16 -> u8 150-155 -> 141-146 us), default for u8 input (whose
#endif                               // 256 MiB planes partly stay in the Infinity Cache between calls)
#ifndef FIR_MF2_TWIN                 // A/B twins: 1 = no MFMAs, 2 = no window loads, 3 = no stores
#define FIR_MF2_TWIN 0
#endif
constexpr int kMf2Tps = FIR_MF2_TPS;

// (a << S) + b (v_lshl_add_u32; pure VALU, no hazards)
template <int S>
__device__ __forceinline__ uint32_t mf_lshl_add(uint32_t a, uint32_t b) {
    uint32_t d;
    asm("v_lshl_add_u32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "n"(S), "v"(b));
    return d;
}
// clamp(a, 0, hi) for hi > 0 (v_med3_i32)
__device__ __forceinline__ uint32_t mf_med3_0(uint32_t a, int32_t hi) {
    uint32_t d;
    asm("v_med3_i32 %0, %1, 0, %2" : "=v"(d) : "v"(a), "s"(hi));
    return d;
}
// byte B of w replaced by (c >> f) (< 256), the other bytes kept: one SDWA shift
template <int B>
__device__ __forceinline__ uint32_t mf_shr_byte(uint32_t w, uint32_t c, int f) {
    static_assert(B >= 1 && B <= 3, "byte");
    if constexpr (B == 1)
        asm("v_lshrrev_b32_sdwa %0, %1, %2 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD"
            : "+v"(w) : "s"(f), "v"(c));
    else if constexpr (B == 2)
        asm("v_lshrrev_b32_sdwa %0, %1, %2 dst_sel:BYTE_2 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD"
            : "+v"(w) : "s"(f), "v"(c));
    else
        asm("v_lshrrev_b32_sdwa %0, %1, %2 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD"
            : "+v"(w) : "s"(f), "v"(c));
    return w;
}

template <typename InT, int STAGE, int KS, bool ACC32, bool FAST>
__global__ __launch_bounds__(kBlock, FIR_MF2_MINB) void fir1d_mfma_step_kernel(const InT* __restrict__ x,
                                                                typename OutTraits<STAGE>::T* __restrict__ y,
                                                                int64_t rowlen, uint32_t steps_per_row, uint32_t nsteps,
                                                                MfmaTaps taps, int P, uint32_t bias, int shl, int frac) {
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    typedef uint32_t u2 __attribute__((ext_vector_type(2)));
    typedef int i32x2 __attribute__((ext_vector_type(2)));
    constexpr bool I16 = sizeof(InT) == 2;
    constexpr int TPS = kMf2Tps;
    constexpr int HX = 32 * KS - 32;           // window samples past the step's TPS * 1024
    constexpr int NB = 2 * TPS;                // body loads per lane: 8 samples each, 512 per load
    constexpr int NL = NB + 1;                 // + one halo load (lanes 0 .. HX/8 - 1 distinct)
    constexpr int PL = TPS * kMfTile + HX;     // bytes per byte plane
    constexpr bool OLDS = STAGE == FIR_OUT_I32 && FIR_MF2_OLDS;
    constexpr int OB = OLDS ? 4608 : 0;        // int32 output image (36-dword rows)
    constexpr int WB = (I16 ? 2 * PL : PL) + OB;
    constexpr int NST = STAGE == FIR_OUT_I32 ? 4 * TPS : TPS;  // 16-byte stores per lane and step
    static_assert(HX / 8 >= 1 && HX / 8 <= kWave, "halo vectors");
    __shared__ __attribute__((aligned(16))) uint8_t lds[kMfWaves][WB];

    const int lane = threadIdx.x & (kWave - 1);
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int r = lane & 31, hf = lane >> 5;
    uint8_t* pl = lds[wv];             // xs (u8) or xls (int16) plane
    uint8_t* ph = lds[wv] + PL;        // xh plane (int16)
    uint32_t* ob = reinterpret_cast<uint32_t*>(lds[wv] + (I16 ? 2 * PL : PL));

    // tap fragments A[r][32 s + 16 hf + j], j = 0..15 (as fir1d_mfma_kernel)
    mf_i32x4 a_lo[KS], a_hi[KS];
#pragma unroll
    for (int s = 0; s < KS; ++s) {
        uint32_t lo[4] = {0u, 0u, 0u, 0u}, hi[4] = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int e = 31 - r + 32 * s + 16 * hf + j;
            lo[j / 4] |= (uint32_t)(uint8_t)taps.lo[e] << (8 * (j % 4));
            hi[j / 4] |= (uint32_t)(uint8_t)taps.hi[e] << (8 * (j % 4));
        }
        a_lo[s] = mf_i32x4{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3]};
        a_hi[s] = mf_i32x4{(int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
    }
    const int32_t sat_hi = FAST ? (int32_t)((256u << (frac & 31)) - 1u) : 0;

    const uint32_t stride = gridDim.x * kMfWaves;
    uint32_t st = blockIdx.x * kMfWaves + wv;
    if (st >= nsteps) return;  // wave-uniform: nothing issued yet

    // ---- a step's window: NB body vectors per lane + one halo vector, from a descriptor over
    // the row's part of [w0, w0 + PL); samples outside the row read as zeros
    uint32_t raw[NL][4];
    auto step_start = [&](uint32_t s, int64_t& rs, int64_t& re) __attribute__((always_inline)) -> int64_t {
        const uint32_t row = __builtin_amdgcn_readfirstlane(s / steps_per_row);
        const uint32_t k = __builtin_amdgcn_readfirstlane(s - row * steps_per_row);
        rs = (int64_t)row * rowlen;
        re = rs + rowlen;
        return rs + (int64_t)k * (TPS * kMfTile);
    };
    auto load_step = [&](uint32_t s) __attribute__((always_inline)) {
        int64_t rs, re;
        const int64_t w0 = step_start(s, rs, re) - P;
        const int64_t base = w0 > rs ? w0 : rs, end = re < w0 + PL ? re : w0 + PL;
        const __amdgpu_buffer_rsrc_t rd = mf_rsrc(x + base, (uint32_t)(end > base ? (end - base) * (int64_t)sizeof(InT) : 0));
#pragma unroll
        for (int it = 0; it < NL; ++it) {
            const int v = it < NB ? it * kWave + lane : NB * kWave + (lane & (HX / 8 - 1));
            const int64_t g = w0 + 8 * v;
            const uint32_t off = g >= base ? (uint32_t)((g - base) * (int64_t)sizeof(InT)) : kMfOff;
            constexpr int aux = FIR_MF2_LDAUX >= 0 ? FIR_MF2_LDAUX : (I16 ? kMfAuxNt : 0);
            if constexpr (FIR_MF2_TWIN == 2) {
                raw[it][0] = off, raw[it][1] = off + 1, raw[it][2] = off + 2, raw[it][3] = off + 3;
            } else if constexpr (I16) {
                const mf_i32x4 q = it < NB ? __builtin_amdgcn_raw_buffer_load_b128(rd, off, 0, aux)
                                           : __builtin_amdgcn_raw_buffer_load_b128(rd, off, 0, 0);
                raw[it][0] = q.x, raw[it][1] = q.y, raw[it][2] = q.z, raw[it][3] = q.w;
            } else {
                const i32x2 q = it < NB ? __builtin_amdgcn_raw_buffer_load_b64(rd, off, 0, aux)
                                        : __builtin_amdgcn_raw_buffer_load_b64(rd, off, 0, 0);
                raw[it][0] = q.x, raw[it][1] = q.y, raw[it][2] = 0u, raw[it][3] = 0u;
            }
        }
    };
    load_step(st);
    {
        // the entry edge issues the step's store count as dropped stores (descriptor size 0), so
        // both edges into the loop header have the same operations in flight and hipcc's wait
        // for the window there is exact (vmcnt(NST)) instead of a drain
        const __amdgpu_buffer_rsrc_t none = mf_rsrc(y, 0u);
#pragma unroll
        for (int k = 0; k < NST; ++k)
            __builtin_amdgcn_raw_buffer_store_b128(mf_i32x4{0, 0, 0, 0}, none, (uint32_t)(1024 * k + 16 * lane), 0,
                                                   kMfAuxNt);  // distinct offsets: not merged as redundant
    }

    for (;;) {
        int64_t rs, re;
        const int64_t ss = step_start(st, rs, re);
        // ---- the window as signed-byte planes: vector v at plane bytes [8 v, 8 v + 8)
#pragma unroll
        for (int it = 0; it < NL; ++it) {
            const int v = it < NB ? it * kWave + lane : NB * kWave + (lane & (HX / 8 - 1));
            const uint32_t* d = raw[it];
            if constexpr (I16) {
                *reinterpret_cast<u2*>(&ph[8 * v]) =
                    u2{__builtin_amdgcn_perm(d[1], d[0], 0x07050301u), __builtin_amdgcn_perm(d[3], d[2], 0x07050301u)};
                *reinterpret_cast<u2*>(&pl[8 * v]) = u2{__builtin_amdgcn_perm(d[1], d[0], 0x06040200u) ^ 0x80808080u,
                                                        __builtin_amdgcn_perm(d[3], d[2], 0x06040200u) ^ 0x80808080u};
            } else {
                *reinterpret_cast<u2*>(&pl[8 * v]) = u2{d[0] ^ 0x80808080u, d[1] ^ 0x80808080u};
            }
        }
        // ---- the next step's window goes out now, in flight during this step's math (past the
        // last step: this one again, so every path into the header has the same loads in flight)
        const uint32_t nx = st + stride;
        load_step(nx < nsteps ? nx : st);
        __builtin_amdgcn_wave_barrier();  // one wave's LDS ops complete in order
        asm volatile("" ::: "memory");

#pragma unroll
        for (int q = 0; q < TPS; ++q) {
            const int64_t ts = ss + (int64_t)q * kMfTile;
            // outputs of this tile (0: past the row; the twin 3 drops every store)
            const int m = FIR_MF2_TWIN == 3 ? 0 : (int)max((int64_t)0, min((int64_t)kMfTile, re - ts));
            mf_i32x16 acc_ll = {}, acc_mid = {}, acc_m2 = {}, acc_hh = {};
#pragma unroll
            for (int s = 0; s < KS; ++s) {
                const int i = q * kMfTile + 32 * r + 32 * s + 16 * hf;
                const mf_i32x4 b_l = *reinterpret_cast<const mf_i32x4*>(&pl[i]);
                if constexpr (FIR_MF2_TWIN == 1) {  // memory-only twin: keep the B reads, drop the MFMAs
                    acc_ll[s] += b_l.x ^ a_lo[s].y;
                    if constexpr (I16) acc_hh[s] += (*reinterpret_cast<const mf_i32x4*>(&ph[i])).z;
                    continue;
                }
                acc_ll = __builtin_amdgcn_mfma_i32_32x32x32_i8(a_lo[s], b_l, acc_ll, 0, 0, 0);
                acc_mid = __builtin_amdgcn_mfma_i32_32x32x32_i8(a_hi[s], b_l, acc_mid, 0, 0, 0);
                if constexpr (I16) {
                    const mf_i32x4 b_h = *reinterpret_cast<const mf_i32x4*>(&ph[i]);
                    acc_hh = __builtin_amdgcn_mfma_i32_32x32x32_i8(a_hi[s], b_h, acc_hh, 0, 0, 0);
                    if constexpr (FIR_MF2_ACC3)
                        acc_mid = __builtin_amdgcn_mfma_i32_32x32x32_i8(a_lo[s], b_h, acc_mid, 0, 0, 0);
                    else
                        acc_m2 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a_lo[s], b_h, acc_m2, 0, 0, 0);
                }
            }
            // combine (mod 2^32), wrap, round; register i is tile output 32 r + (i & 3) + 8 (i >> 2) + 4 hf
            // (the accumulators are read by compiler-visible code only: hipcc's hazard recognizer
            // does not pad an inline-asm read of an MFMA result, which then reads stale values)
            int32_t o[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                uint32_t a;
                if constexpr (I16) {
                    const uint32_t mid = FIR_MF2_ACC3 ? (uint32_t)acc_mid[i] : (uint32_t)(acc_mid[i] + acc_m2[i]);
                    // 3 VALU: (hh << 8) + mid and ll + bias by hipcc (which pads the MFMA reads), the
                    // outer (t << 8) + u as asm (hipcc would re-associate it into 2 shifts + add3)
                    a = mf_lshl_add<8>(((uint32_t)acc_hh[i] << 8) + mid, (uint32_t)acc_ll[i] + bias);
                } else {
                    a = (((uint32_t)acc_mid[i] << 8) + (uint32_t)acc_ll[i]) + bias;
                }
                if constexpr (FAST)
                    o[i] = STAGE == FIR_OUT_U8_SAT ? (int32_t)mf_med3_0(a, sat_hi) : (int32_t)a >> frac;
                else
                    o[i] = round_acc<ACC32>(a, shl, frac);
            }
            if constexpr (STAGE == FIR_OUT_U8_SAT) {
                // 4 outputs per dword g (bytes 32 r + 8 g + 4 hf ..); one permlane32 swap per pair of
                // dwords gives each lane 16 contiguous bytes: lanes 0-31 at 32 r, 32-63 at 32 r + 16
                uint32_t w[4];
#pragma unroll
                for (int g4 = 0; g4 < 4; ++g4) {
                    if constexpr (FAST)  // clamped sums c in [0, 2^(frac+8)): the byte is c >> frac
                        w[g4] = mf_shr_byte<3>(mf_shr_byte<2>(mf_shr_byte<1>((uint32_t)o[4 * g4] >> frac, (uint32_t)o[4 * g4 + 1], frac),
                                                              (uint32_t)o[4 * g4 + 2], frac),
                                               (uint32_t)o[4 * g4 + 3], frac);
                    else
                        w[g4] = (uint32_t)stage_out32<STAGE>(o[4 * g4]) | ((uint32_t)stage_out32<STAGE>(o[4 * g4 + 1]) << 8) |
                                ((uint32_t)stage_out32<STAGE>(o[4 * g4 + 2]) << 16) |
                                ((uint32_t)stage_out32<STAGE>(o[4 * g4 + 3]) << 24);
                }
                const auto s02 = __builtin_amdgcn_permlane32_swap(w[0], w[2], false, false);
                const auto s13 = __builtin_amdgcn_permlane32_swap(w[1], w[3], false, false);
                __builtin_amdgcn_raw_buffer_store_b128(mf_i32x4{(int)s02[0], (int)s02[1], (int)s13[0], (int)s13[1]},
                                                       mf_rsrc(y + ts, (uint32_t)m), (uint32_t)(32 * r + 16 * hf), 0, kMfAuxNt);
            } else if constexpr (OLDS) {
                // LDS image: block n at dwords [36 n, 36 n + 32), read back as 1 KiB rows
                __builtin_amdgcn_wave_barrier();
                asm volatile("" ::: "memory");
#pragma unroll
                for (int g4 = 0; g4 < 4; ++g4)
                    *reinterpret_cast<u4*>(&ob[36 * r + 8 * g4 + 4 * hf]) =
                        u4{(uint32_t)o[4 * g4], (uint32_t)o[4 * g4 + 1], (uint32_t)o[4 * g4 + 2], (uint32_t)o[4 * g4 + 3]};
                __builtin_amdgcn_wave_barrier();
                asm volatile("" ::: "memory");
                const __amdgpu_buffer_rsrc_t rd = mf_rsrc(y + ts, (uint32_t)m * 4u);
#pragma unroll
                for (int rho = 0; rho < 4; ++rho) {
                    const int oo = 256 * rho + 4 * lane;
                    __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const mf_i32x4*>(&ob[36 * (oo >> 5) + (oo & 31)]), rd,
                                                           (uint32_t)oo * 4u, 0, kMfAuxNt);
                }
            } else {
                // permlane32 pairs: lanes 0-31 hold outputs 32 r + 0..15, lanes 32-63 32 r + 16..31
                uint32_t g[4][4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const auto s02 = __builtin_amdgcn_permlane32_swap((uint32_t)o[k], (uint32_t)o[8 + k], false, false);
                    const auto s13 = __builtin_amdgcn_permlane32_swap((uint32_t)o[4 + k], (uint32_t)o[12 + k], false, false);
                    g[0][k] = s02[0], g[1][k] = s02[1], g[2][k] = s13[0], g[3][k] = s13[1];
                }
                const __amdgpu_buffer_rsrc_t rd = mf_rsrc(y + ts, (uint32_t)m * 4u);
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    __builtin_amdgcn_raw_buffer_store_b128(mf_i32x4{(int)g[j][0], (int)g[j][1], (int)g[j][2], (int)g[j][3]}, rd,
                                                           (uint32_t)(128 * r + 64 * hf + 16 * j), 0, kMfAuxNt);
            }
        }
        st = nx;
        if (st >= nsteps) break;
        __builtin_amdgcn_wave_barrier();  // the B reads of this step are done before the next staging
        asm volatile("" ::: "memory");
    }
    (void)ob;
}

// ---------------------------------------------------------------------------------------
// Filters longer than kMfMaxTaps (any length): the same Toeplitz product with K = 32 + L/2 + P
// split into chunks of kMlChunk k-steps.  Per tile and chunk the wave stages the chunk's window
// (992 + 32 * steps samples) as byte planes in its LDS, then runs the chunk's k-steps with the
// accumulators carried over: the tap fragments no longer fit VGPRs, so each k-step's A fragments
// come from a table in HBM (frag[s][plane][lane], 16 bytes per lane: one coalesced 1 KiB load per
// plane, the same for every tile, so L2-resident).
constexpr int kMlChunk = 16;                          // k-steps per staged window
constexpr int kMlWin = 32 * 31 + 32 * kMlChunk;       // window samples per chunk (1504)
constexpr int kMlNV = kMlWin / 8;                     // 8-sample vectors
constexpr int kMlNIT = (kMlNV + kWave - 1) / kWave;   // per lane
constexpr int kMlPlane = mf_pos(kMlWin);

template <typename InT, int STAGE, bool ACC32, bool FAST>
__global__ __launch_bounds__(kBlock) void fir1d_mfma_long_kernel(const InT* __restrict__ x,
                                                                 typename OutTraits<STAGE>::T* __restrict__ y,
                                                                 int64_t rowlen, int64_t tiles_per_row, int64_t ntiles,
                                                                 const mf_i32x4* __restrict__ frag, int KS, int P,
                                                                 uint32_t bias, int shl, int frac) {
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    typedef uint32_t u2 __attribute__((ext_vector_type(2)));
    constexpr bool I16 = sizeof(InT) == 2;
    constexpr int WBYTES = (I16 ? 2 * kMlPlane : kMlPlane) > 4608 ? (I16 ? 2 * kMlPlane : kMlPlane) : 4608;
    __shared__ __attribute__((aligned(16))) uint8_t lds[kMfWaves][WBYTES];

    const int lane = threadIdx.x & (kWave - 1);
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int r = lane & 31, hf = lane >> 5;
    uint8_t* pl = lds[wv];
    uint8_t* ph = lds[wv] + kMlPlane;
    const int32_t sat_hi = FAST ? (int32_t)((256u << (frac & 31)) - 1u) : 0;
    const uint32_t step = gridDim.x * kMfWaves, nt32 = (uint32_t)ntiles, tpr = (uint32_t)tiles_per_row;

    for (uint32_t tile = blockIdx.x * kMfWaves + wv; tile < nt32; tile += step) {
        const MfTile t = mf_tile(tile, rowlen, tpr);
        const int m = (int)min((int64_t)kMfTile, t.re - t.ts);
        mf_i32x16 acc_ll = {}, acc_mid = {}, acc_m2 = {}, acc_hh = {};
        for (int s0 = 0; s0 < KS; s0 += kMlChunk) {
            const int steps = min(kMlChunk, KS - s0);
            const int nv = (32 * 31 + 32 * steps) / 8;
            // ---- the chunk's window [w0, w0 + 8 nv) through a descriptor over this row's part of it
            const int64_t w0 = t.ts - P + 32 * (int64_t)s0, base = w0 > t.rs ? w0 : t.rs;
            const int64_t end = t.re < w0 + 8 * nv ? t.re : w0 + 8 * nv;
            const __amdgpu_buffer_rsrc_t rs = mf_rsrc(x + base, (uint32_t)(end > base ? (end - base) * (int64_t)sizeof(InT) : 0));
            uint32_t raw[kMlNIT][4];
#pragma unroll
            for (int it = 0; it < kMlNIT; ++it) {
                const int v = min(it * kWave + lane, nv - 1);
                const int64_t g = w0 + 8 * v;
                const uint32_t off = g >= base ? (uint32_t)((g - base) * (int64_t)sizeof(InT)) : kMfOff;
                if constexpr (I16) {
                    const mf_i32x4 q = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
                    raw[it][0] = q.x, raw[it][1] = q.y, raw[it][2] = q.z, raw[it][3] = q.w;
                } else {
                    typedef int i32x2 __attribute__((ext_vector_type(2)));
                    const i32x2 q = __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, 0);
                    raw[it][0] = q.x, raw[it][1] = q.y, raw[it][2] = 0u, raw[it][3] = 0u;
                }
            }
            __builtin_amdgcn_wave_barrier();  // the previous chunk's B reads are done
            asm volatile("" ::: "memory");
#pragma unroll
            for (int it = 0; it < kMlNIT; ++it) {
                const int v = it * kWave + lane;
                if (v < nv) {
                    const uint32_t* d = raw[it];
                    if constexpr (I16) {
                        *reinterpret_cast<u2*>(&ph[mf_pos(8 * v)]) =
                            u2{__builtin_amdgcn_perm(d[1], d[0], 0x07050301u), __builtin_amdgcn_perm(d[3], d[2], 0x07050301u)};
                        *reinterpret_cast<u2*>(&pl[mf_pos(8 * v)]) =
                            u2{__builtin_amdgcn_perm(d[1], d[0], 0x06040200u) ^ 0x80808080u,
                               __builtin_amdgcn_perm(d[3], d[2], 0x06040200u) ^ 0x80808080u};
                    } else {
                        *reinterpret_cast<u2*>(&pl[mf_pos(8 * v)]) = u2{d[0] ^ 0x80808080u, d[1] ^ 0x80808080u};
                    }
                }
            }
            __builtin_amdgcn_wave_barrier();
            asm volatile("" ::: "memory");
            // ---- the chunk's k-steps: A from the fragment table, B from the planes
            const mf_i32x4* fa = frag + (int64_t)s0 * 2 * kWave + lane;
            for (int s = 0; s < steps; ++s) {
                const mf_i32x4 a_lo = fa[(2 * s) * kWave], a_hi = fa[(2 * s + 1) * kWave];
                const int i = mf_pos(32 * r + 32 * s + 16 * hf);
                const mf_i32x4 b_l = *reinterpret_cast<const mf_i32x4*>(&pl[i]);
                acc_ll = __builtin_amdgcn_mfma_i32_32x32x32_i8(a_lo, b_l, acc_ll, 0, 0, 0);
                acc_mid = __builtin_amdgcn_mfma_i32_32x32x32_i8(a_hi, b_l, acc_mid, 0, 0, 0);
                if constexpr (I16) {
                    const mf_i32x4 b_h = *reinterpret_cast<const mf_i32x4*>(&ph[i]);
                    acc_m2 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a_lo, b_h, acc_m2, 0, 0, 0);
                    acc_hh = __builtin_amdgcn_mfma_i32_32x32x32_i8(a_hi, b_h, acc_hh, 0, 0, 0);
                }
            }
        }
        // ---- combine, wrap, round, stage; outputs through LDS as whole 1 KiB rows (as above)
        int32_t q[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            uint32_t a;
            if constexpr (I16)
                a = ((uint32_t)(acc_mid[i] + acc_m2[i]) << 8) + (uint32_t)acc_ll[i] + ((uint32_t)acc_hh[i] << 16) + bias;
            else
                a = ((uint32_t)acc_mid[i] << 8) + (uint32_t)acc_ll[i] + bias;
            if constexpr (FAST)
                q[i] = STAGE == FIR_OUT_U8_SAT ? min(max((int32_t)a, 0), sat_hi) : (int32_t)a >> frac;
            else
                q[i] = round_acc<ACC32>(a, shl, frac);
        }
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");
        if constexpr (STAGE == FIR_OUT_I32) {
            uint32_t* ob = reinterpret_cast<uint32_t*>(lds[wv]);
#pragma unroll
            for (int g4 = 0; g4 < 4; ++g4)
                *reinterpret_cast<u4*>(&ob[36 * r + 8 * g4 + 4 * hf]) =
                    u4{(uint32_t)q[4 * g4], (uint32_t)q[4 * g4 + 1], (uint32_t)q[4 * g4 + 2], (uint32_t)q[4 * g4 + 3]};
            __builtin_amdgcn_wave_barrier();
            asm volatile("" ::: "memory");
            const __amdgpu_buffer_rsrc_t rd = mf_rsrc(y + t.ts, (uint32_t)m * 4u);
#pragma unroll
            for (int rho = 0; rho < 4; ++rho) {
                const int o = 256 * rho + 4 * lane;
                __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const mf_i32x4*>(&ob[36 * (o >> 5) + (o & 31)]), rd,
                                                       (uint32_t)(256 * rho + 4 * lane) * 4u, 0, kMfAuxNt);
            }
        } else {
            uint8_t* ob = lds[wv];
#pragma unroll
            for (int g4 = 0; g4 < 4; ++g4) {
                uint32_t w;
                if constexpr (FAST) {
                    w = (uint32_t)q[4 * g4] >> frac;
                    w |= ((uint32_t)q[4 * g4 + 1] >> frac) << 8;
                    w |= ((uint32_t)q[4 * g4 + 2] >> frac) << 16;
                    w |= ((uint32_t)q[4 * g4 + 3] >> frac) << 24;
                } else {
                    w = (uint32_t)stage_out32<STAGE>(q[4 * g4]) | ((uint32_t)stage_out32<STAGE>(q[4 * g4 + 1]) << 8) |
                        ((uint32_t)stage_out32<STAGE>(q[4 * g4 + 2]) << 16) |
                        ((uint32_t)stage_out32<STAGE>(q[4 * g4 + 3]) << 24);
                }
                *reinterpret_cast<uint32_t*>(&ob[48 * r + 8 * g4 + 4 * hf]) = w;
            }
            __builtin_amdgcn_wave_barrier();
            asm volatile("" ::: "memory");
            const int o = 16 * lane;
            __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const mf_i32x4*>(&ob[48 * (o >> 5) + (o & 31)]),
                                                   mf_rsrc(y + t.ts, (uint32_t)m), (uint32_t)(16 * lane), 0, kMfAuxNt);
        }
        __builtin_amdgcn_wave_barrier();  // the output reads are done before the next tile's staging
        asm volatile("" ::: "memory");
    }
}

// frag[s][p][lane] = bytes j = 0..15 of plane p (0: hl, 1: hh) of the diagonal entries
// e = 31 - r + 32 s + 16 hf + j (lane = r + 32 hf), as MfmaTaps lays them out
// (keyed by the taps and the geometry: the table is built only on a cache miss)
static const mf_i32x4* mfma_frag_table(const int32_t* hq, int L, int P, int KS, std::string* err) {
    const int c = L / 2;
    TableHash h;
    h.add(hq, sizeof(int32_t) * (size_t)L);
    h.add_val(L), h.add_val(P), h.add_val(KS);
    const size_t bytes = (size_t)KS * 2 * kWave * 16;
    return (const mf_i32x4*)table_acquire(h, bytes, [&](void* dst) {
        int8_t* tab = (int8_t*)dst;
        for (int st = 0; st < KS; ++st)
            for (int lane = 0; lane < kWave; ++lane)
                for (int j = 0; j < 16; ++j) {
                    const int e = 31 - (lane & 31) + 32 * st + 16 * (lane >> 5) + j;
                    const int tap = 31 - e + c + P;
                    const int v = tap >= 0 && tap < L ? hq[tap] : 0;
                    const int lo = ((v + 128) & 255) - 128;
                    tab[(((size_t)st * 2 + 0) * kWave + lane) * 16 + j] = (int8_t)lo;
                    tab[(((size_t)st * 2 + 1) * kWave + lane) * 16 + j] = (int8_t)((v - lo) / 256);
                }
    }, err);
}

template <typename InT, int STAGE>
static hipError_t launch_mfma_long(const void* x, void* y, int64_t rl, int64_t tpr, int64_t ntiles, const int32_t* hq,
                                   int L, int P, int KS, uint32_t bias, bool fast, int frac, int acc_bits, hipStream_t s) {
    using OutT = typename OutTraits<STAGE>::T;
    std::string err;
    const mf_i32x4* fr = mfma_frag_table(hq, L, P, KS, &err);
    if (!fr) return hipErrorOutOfMemory;
    TableHold hold(fr, s);
    const int64_t want = (ntiles + kMfWaves - 1) / kMfWaves;
    const unsigned blocks = (unsigned)(want < FIR_MFMA_LONG_BLOCKS ? want : FIR_MFMA_LONG_BLOCKS);
    if (fast)
        hipLaunchKernelGGL((fir1d_mfma_long_kernel<InT, STAGE, true, true>), dim3(blocks), dim3(kBlock), 0, s,
                           (const InT*)x, (OutT*)y, rl, tpr, ntiles, fr, KS, P, bias, 0, frac);
    else if (acc_bits == 32)
        hipLaunchKernelGGL((fir1d_mfma_long_kernel<InT, STAGE, true, false>), dim3(blocks), dim3(kBlock), 0, s,
                           (const InT*)x, (OutT*)y, rl, tpr, ntiles, fr, KS, P, bias, 0, frac);
    else
        hipLaunchKernelGGL((fir1d_mfma_long_kernel<InT, STAGE, false, false>), dim3(blocks), dim3(kBlock), 0, s,
                           (const InT*)x, (OutT*)y, rl, tpr, ntiles, fr, KS, P, bias, 32 - acc_bits, frac);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// u8 filters past the step kernel's 3 k-steps (round 4; fir1d_mfma_long_kernel stays for int16).
// The long kernel above re-fetches every k-step's tap fragments from L2 for every tile: 2 KiB
// per k-step and tile, i.e. (4099 taps, 130 k-steps) 260 KiB of L2 reads per 1 KiB of samples,
// an L2-bound loop at 2.5-28 % of the HBM roofline.  Here a wave owns a RUN of
// kMrTps consecutive tiles (of any rows: each tile keeps its own window and row bounds) and
// walks the k-steps in chunks of kMrC: a chunk's tap fragments (kMrC x 2 x 16 B per lane, 128
// VGPRs) are loaded once and feed all the run's tiles, so fragment traffic drops kMrTps-fold,
// and when KS <= kMrC (up to ~450 taps) they are loaded once per wave for the whole grid-stride
// loop.  The run's accumulators (2 x 16 int32 per tile) stay in AGPRs across chunks; one wave per
// SIMD.  Windows (1024 + 32 kMrC - 32 samples per tile and chunk) arrive by LDS-DMA
// (buffer_load ... lds, the descriptor's range check zero-fills samples outside the tile's row),
// double-buffered: the next iteration's windows are in flight while this one's MFMAs run, with
// no VGPRs held.  The bytes land unsigned; the B fragment is XORed with 0x80 after its LDS read
// (xs = x - 128, as in every other kernel here).  The left halo P is rounded to 16 so a window
// vector never straddles a row start.
#ifndef FIR_MR_TPS                   // tiles per run
#define FIR_MR_TPS 2
#endif
#ifndef FIR_MR_C                     // k-steps per chunk
#define FIR_MR_C 16
#endif
#ifndef FIR_MR_WAVES                 // waves per SIMD the registers must allow (LDS: (DEPTH+1) TPS 2 KiB per wave)
#define FIR_MR_WAVES 2
#endif
#ifndef FIR_MR_DEPTH                 // iterations whose windows are in flight ahead of the one computed
#define FIR_MR_DEPTH 2
#endif
#ifndef FIR_MR_EXP                   // timing experiments (wrong results): 1 no MFMAs, 2 no window DMAs
#define FIR_MR_EXP 0
#endif
#ifndef FIR_MR_W4_NS                 // one-tile runs of up to this many k-steps: 4 waves per SIMD
#define FIR_MR_W4_NS 8                // (vs 6: 162 / 194 taps 140 / 136 us vs 149 / 139, profiles/r04/long_taps_w4ns_ab.txt)
#endif
#ifndef FIR_MR_BIASV                 // 1: bias folded into the first MFMA (below 4 waves per SIMD)
#define FIR_MR_BIASV 1
#endif
#ifndef FIR_MR_MTPS                  // tiles per run with several chunks (u8 stage)
#define FIR_MR_MTPS 4
#endif
#ifndef FIR_MR_ROLL                  // 1: next chunk's fragments loaded step by step behind the MFMAs
                                     // (A/B: 4099 taps 2091 vs 2020 us, profiles/r04/long_taps_run_v3_ab.txt)
#define FIR_MR_ROLL 0
#endif
#ifndef FIR_MR_MNS_MIN               // shortest chunk considered with 4-tile runs
#define FIR_MR_MNS_MIN 6
#endif
#ifndef FIR_MR_MDEPTH                // window iterations in flight with 4-tile runs (LDS: 2 WGs per CU)
#define FIR_MR_MDEPTH 1
#endif
#ifndef FIR_MR_CURSOR                // 1: incremental tile geometry for one-tile one-chunk runs
#define FIR_MR_CURSOR 1
#endif
#ifndef FIR_MR_DEPTH1                // window iterations in flight with one tile per run (u8 out; 12 waves
#define FIR_MR_DEPTH1 3               // per CU: (DEPTH1 + 1) x 2 KiB of LDS each)
#endif
#ifndef FIR_MR_U8_ONE                // u8 out: one chunk (fragments loaded once per wave) up to this many k-steps
#define FIR_MR_U8_ONE 32
#endif
#ifndef FIR_MR_T1_NS                 // one-chunk filters up to this many k-steps: one tile per run (A/B
#define FIR_MR_T1_NS 32               // vs 10, 2-tile runs past it: 290 / 322 / 450 taps 165 / 173 / 212 us
#endif                               // vs 196 / 189 / 221, profiles/r04/long_taps_t1ns_ab.txt)
#ifndef FIR_MR_BLOCKS                // grid-stride blocks (4 waves each): one resident round
#define FIR_MR_BLOCKS (256 * FIR_MR_WAVES)
#endif
#ifndef FIR_MR_XLDS_FROM             // chunk lengths whose windows are re-biased in LDS
#define FIR_MR_XLDS_FROM 8
#endif
#ifndef FIR_MR_BPD                   // k-steps whose B fragments are read ahead of the MFMAs
#define FIR_MR_BPD 3
#endif
constexpr int kMrTps = FIR_MR_TPS, kMrC = FIR_MR_C, kMrDepth = FIR_MR_DEPTH, kMrBpd = FIR_MR_BPD;
// f(integral_constant<I>) for I in [B, E), unrolled at compile time
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + 1, E>(f);
    }
}
constexpr int kMrTileLds = 2048;     // LDS bytes per tile window (128 vectors of 16 samples)

// NS: k-steps per chunk, a compile-time count (the fragment table is zero-padded to whole chunks;
// the launcher picks NS so the padding is at most one k-step below 9 and small above): the
// chunk's MFMAs are one straight line.  (A runtime count, as a skip per slot or a jump into the
// sequence, made the compiler copy every accumulator at each join: 600-800 v_mov per iteration,
// VALU-bound at 257 taps, profiles/r04/sq_run_kernel_257.csv.)  mode: 0 FAST (no wrap, no int32
// overflow), 1 acc_bits == 32, 2 acc_bits < 32 -- an epilogue branch, uniform per launch.
// TPS tiles per run: 2 (FIR_MR_TPS) at 2 waves per SIMD; 1 at 3 waves per SIMD (and windows one
// iteration deeper) for one-chunk filters up to 10 k-steps, whose registers fit a third wave
// (A/B at 66 / 128 / 257 taps: 109 / 119 / 151 us vs 127 / 131 / 170, profiles/r04/long_taps_run_v3_ab.txt)
// Several chunks: FIR_MR_MWAVES waves per SIMD.  FIR_MR_ADBL 1 loads the next chunk's fragments
// during this one's MFMAs into a second register set (A/B, profiles/r04/long_taps_run_v3_ab.txt:
// with chunks of 6-8 at 2 waves 4099 taps 2415 us, of up to 16 at 1 wave 3166, vs 2205 for one set
// loaded at the top of each iteration at 2 waves -- the per-iteration costs and the waves, not
// the fragment latency, bound this loop)
#ifndef FIR_MR_MWAVES
#define FIR_MR_MWAVES 2
#endif
#ifndef FIR_MR_ADBL
#define FIR_MR_ADBL 0
#endif
#ifndef FIR_MR_W3_NS                 // one-tile runs of up to this many k-steps: 3 waves per SIMD (2 past it)
#define FIR_MR_W3_NS 12
#endif
#ifndef FIR_MR_W2_NS                 // ... 2 waves up to this many (1 past it)
#define FIR_MR_W2_NS 24
#endif
constexpr int mr_waves_of(int stage, int tps, bool multi, int ns) {
    return multi ? FIR_MR_MWAVES
                 : tps == 1 ? (ns <= FIR_MR_W4_NS && stage == FIR_OUT_U8_SAT ? 4
                               : ns <= (stage == FIR_OUT_U8_SAT ? FIR_MR_W3_NS : 11) ? 3  // (int32 out: 12 spilled)
                               : ns <= FIR_MR_W2_NS ? 2 : 1)
                            : FIR_MR_WAVES;
}
template <int STAGE, int TPS_, bool MULTI, int NS>
constexpr int mr_waves() {
    return mr_waves_of(STAGE, TPS_, MULTI, NS);
}
template <int STAGE, int NS, bool MULTI, int TPS_>
__global__ __launch_bounds__(kBlock, (mr_waves<STAGE, TPS_, MULTI, NS>())) void fir1d_mfma_run_kernel(const uint8_t* __restrict__ x,
                                                                   typename OutTraits<STAGE>::T* __restrict__ y,
                                                                   int64_t rowlen, uint32_t tiles_per_row, uint32_t ntiles,
                                                                   const mf_i32x4* __restrict__ frag, int KS, int P,
                                                                   uint32_t bias, int mode, int shl, int frac) {
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    constexpr int TPS = TPS_, C = NS;
    constexpr bool OLDS = STAGE == FIR_OUT_I32;
    constexpr int kMrDepth = TPS == 1 ? (OLDS ? 3 : FIR_MR_DEPTH1) : TPS == 4 ? FIR_MR_MDEPTH : ::fir::kMrDepth;
    constexpr int WT = kMfTile + 32 * C - 32;  // window samples per tile and chunk
    constexpr int NVT = (WT + 15) / 16;         // 16-sample vectors per tile window
    static_assert(NVT > kWave && NVT <= 2 * kWave && 16 * 2 * kWave <= kMrTileLds, "two DMAs per tile window");
    constexpr int BUF = TPS * kMrTileLds;
    constexpr int NBUF = kMrDepth + 1;          // LDS window buffers per wave (a ring)
    constexpr int NDMA = 2 * TPS;               // DMA instructions per iteration
    constexpr int NST = TPS * (OLDS ? 4 : 1);   // store instructions per completed run
    // the x - 128 of the B operand: in LDS once per window (long chunks) or per fragment read
    constexpr bool XLDS = C >= FIR_MR_XLDS_FROM;
    __shared__ __attribute__((aligned(16))) uint8_t lds[kMfWaves][NBUF * BUF + (OLDS ? 4608 : 16)];

    const int lane = threadIdx.x & (kWave - 1);
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int r = lane & 31, hf = lane >> 5;
    uint32_t* ob = reinterpret_cast<uint32_t*>(lds[wv] + NBUF * BUF);
    const int32_t sat_hi = (int32_t)((256u << (frac & 31)) - 1u);  // (mode 0)
    const int nch = KS / C;  // KS: a multiple of C
    const uint32_t nruns = (ntiles + TPS - 1) / TPS;
    const uint32_t stride = gridDim.x * kMfWaves;
    uint32_t rn = blockIdx.x * kMfWaves + wv;
    if (rn >= nruns) return;  // wave-uniform: nothing issued yet

    // tap fragments: one set (one chunk: loaded once), or two (several chunks: the next iteration's
    // chunk loaded while this one's MFMAs run -- loaded at the top of each iteration instead, the
    // L2 latency of 2 C loads was exposed every iteration, 4099 taps 2087 us)
    constexpr bool ADBL = MULTI && FIR_MR_ADBL;
    mf_i32x4 a0_lo[C], a0_hi[C], a1_lo[ADBL ? C : 1], a1_hi[ADBL ? C : 1];
    auto load_a = [&](mf_i32x4 (&lo)[C], mf_i32x4 (&hi)[C], int c) __attribute__((always_inline)) {
        const mf_i32x4* f = frag + (int64_t)c * C * 2 * kWave + lane;
#pragma unroll
        for (int s = 0; s < C; ++s) lo[s] = f[(2 * s) * kWave], hi[s] = f[(2 * s + 1) * kWave];
    };
    // One tile per run and one chunk (the wave's tiles t, t + S, t + 2S, ...): the tile's row and
    // column advance by constant steps (one division at the start instead of one per tile and use,
    // ~40 of the loop's ~114 SALU per tile).  Past the last tile the cursor runs on; those tiles'
    // descriptors have size 0.
    constexpr bool CUR = TPS == 1 && !MULTI && FIR_MR_CURSOR;
    // the bias as the first MFMA's accumulator input (16 VGPRs) or one add per output
    // (23-24 k-steps at 2 waves per SIMD: no bias registers and 2 reads ahead, or they spill; at 1
    // wave both cost ~4 %: 800 / 930 taps 430 / 478 vs 414 / 461 us, profiles/r04/long_taps_one_chunk_ab.txt)
    constexpr bool TRIM = NS > 22 && mr_waves<STAGE, TPS_, MULTI, NS>() == 2;
    constexpr bool BIASV = FIR_MR_BIASV && mr_waves<STAGE, TPS_, MULTI, NS>() < 4 && !TRIM;
    constexpr int BPD = TPS == 4 ? 1 : TRIM ? 2 : mr_waves<STAGE, TPS_, MULTI, NS>() < 4 ? kMrBpd : 2;  // B reads ahead
    struct Cursor {
        uint32_t row, col;
        int64_t rs;
    };
    const uint32_t tpr = tiles_per_row, dr = stride / tpr, dc = stride - dr * tpr;
    const int64_t drs = (int64_t)dr * rowlen;
    auto cur_at = [&](uint32_t t) __attribute__((always_inline)) {
        Cursor k;
        k.row = __builtin_amdgcn_readfirstlane(t / tpr);
        k.col = __builtin_amdgcn_readfirstlane(t - k.row * tpr);
        k.rs = (int64_t)k.row * rowlen;
        return k;
    };
    auto cur_step = [&](Cursor& k) __attribute__((always_inline)) {
        k.col += dc, k.row += dr, k.rs += drs;
        if (k.col >= tpr) k.col -= tpr, ++k.row, k.rs += rowlen;
    };
    auto tile_of = [&](uint32_t t, const Cursor& k) __attribute__((always_inline)) {
        if constexpr (CUR) {
            MfTile tl;
            tl.rs = k.rs, tl.re = k.rs + rowlen, tl.ts = k.rs + (int64_t)k.col * kMfTile;
            return tl;
        } else {
            return mf_tile(t < ntiles ? t : ntiles - 1, rowlen, tiles_per_row);
        }
    };
    Cursor acur{}, rcur{};
    if constexpr (CUR) acur = cur_at(rn), rcur = acur;
    // the run's TPS tile windows of chunk c into LDS buffer `buf`: per tile two 1 KiB DMAs
    // (vectors lane and lane + 64; the second past the window's NVT vectors reads zeros)
    auto issue_win = [&](uint32_t run, int c, int buf) __attribute__((always_inline)) {
        if constexpr (FIR_MR_EXP == 2) return;
#pragma unroll
        for (int q = 0; q < TPS; ++q) {
            const uint32_t t = run < nruns ? run * TPS + q : ntiles;
            const MfTile tl = tile_of(t, acur);
            const int64_t w0 = tl.ts - P + 32 * (int64_t)C * c;
            const int64_t base = w0 > tl.rs ? w0 : tl.rs, end = tl.re < w0 + WT ? tl.re : w0 + WT;
            const __amdgpu_buffer_rsrc_t rd = mf_rsrc(x + base, (uint32_t)(end > base && t < ntiles ? end - base : 0));
            const uint32_t skip = (uint32_t)(base - w0);  // samples of the window before the row (multiple of 16)
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const uint32_t v16 = 16u * (uint32_t)(lane + kWave * i);
                const uint32_t off = v16 >= skip && (i == 0 || lane + kWave < NVT) ? v16 - skip : kMfOff;
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    rd, (__attribute__((address_space(3))) void*)(lds[wv] + buf * BUF + q * kMrTileLds + 1024 * i), 16, off,
                    0, 0, 0);
            }
        }
    };

    mf_i32x16 acc_ll[TPS], acc_mid[TPS];
#pragma unroll
    for (int q = 0; q < TPS; ++q) acc_ll[q] = mf_i32x16{}, acc_mid[q] = mf_i32x16{};
    mf_i32x16 biasv;
#pragma unroll
    for (int i = 0; i < 16; ++i) biasv[i] = (int)bias;
    if constexpr (!MULTI) load_a(a0_lo, a0_hi, 0);  // KS <= C: one chunk, fragments loaded once
    // iterations (run, chunk) in order; `ahead` is the one whose windows are issued next, kMrDepth
    // ahead of the one computed (past the last: runs past nruns, whose zero-size descriptors move
    // nothing -- every iteration issues the same NDMA operations, so the counted wait is exact)
    auto advance = [&](uint32_t& r, int& ch) __attribute__((always_inline)) {
        if (++ch == nch) ch = 0, r += stride;
    };
    int c = 0, buf = 0;
    uint32_t ar = rn;
    int ac = 0;
    auto advance_ahead = [&]() __attribute__((always_inline)) {
        advance(ar, ac);
        if constexpr (CUR) cur_step(acur);
    };
#pragma unroll
    for (int d = 0; d < kMrDepth; ++d) {
        issue_win(ar, ac, d);
        advance_ahead();
        if constexpr (!MULTI) {  // stand-ins for the stores of the iterations before the first (a
            const __amdgpu_buffer_rsrc_t none = mf_rsrc(y, 0u);  // zero-size range: nothing written),
#pragma unroll                                                   // so the counted wait below is exact
            for (int k = 0; k < NST; ++k) __builtin_amdgcn_raw_buffer_store_b32(0, none, 0, 0, 0);
        }
    }
    // ROLL (several chunks, one fragment set): each k-step's fragments for the NEXT iteration are
    // loaded right after that step's MFMAs issue, so they land during this iteration's remaining
    // MFMAs instead of being waited for at the top of the next one
    constexpr bool ROLL = MULTI && !ADBL && FIR_MR_ROLL;
    if constexpr (ADBL || ROLL) load_a(a0_lo, a0_hi, 0);  // behind the first windows (the first wait below)
    bool first = true, stored = false;
    // one iteration (run rn, chunk c) on fragments acur, loading anext for the next one; false at the end
    auto body = [&](mf_i32x4 (&a_lo)[C], mf_i32x4 (&a_hi)[C], mf_i32x4 (&an_lo)[C], mf_i32x4 (&an_hi)[C])
                    __attribute__((always_inline)) -> bool {
        uint32_t nr = rn;
        int nc = c;
        advance(nr, nc);
        if constexpr (ADBL) load_a(an_lo, an_hi, nc);  // (past the last run: a valid chunk, unused)
        else if constexpr (MULTI && !ROLL) load_a(a_lo, a_hi, c);  // issued before the next windows: its wait leaves them in flight
        issue_win(ar, ac, buf == 0 ? NBUF - 1 : buf - 1);  // the buffer computed last iteration
        advance_ahead();
        // this iteration's windows (and A) landed; the younger operations stay in flight.  vmcnt
        // also counts stores, in order with the loads.  One chunk: every iteration ends with its
        // NST stores, so kMrDepth iterations of DMAs + stores may stay outstanding (counting only
        // the DMAs drained the next iteration's windows too).  Several: A(i) was issued at the top
        // of the previous iteration, after this iteration's windows, so what may stay outstanding
        // is everything issued after A(i): the previous iteration's DMAs and stores (if it ended a
        // run) and this iteration's A(i + 1) and DMAs.
        if constexpr (MULTI && !ADBL) {
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kMrDepth * NDMA) : "memory");
        } else if constexpr (MULTI) {
            if (first)
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * C + NDMA) : "memory");
            else if (stored)
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * C + 2 * NDMA + NST) : "memory");
            else
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * C + 2 * NDMA) : "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kMrDepth * (NDMA + NST)) : "memory");
        }
        first = false;
        __builtin_amdgcn_wave_barrier();
        uint8_t* pl = lds[wv] + buf * BUF;
        if constexpr (XLDS) {  // xs = x - 128 once per window byte (each is read by ~C fragments)
#pragma unroll
            for (int q = 0; q < TPS; ++q)
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    mf_i32x4* v = reinterpret_cast<mf_i32x4*>(&pl[q * kMrTileLds + 1024 * i + 16 * lane]);
                    *v = *v ^ (int)0x80808080;
                }
            __builtin_amdgcn_wave_barrier();
            asm volatile("" ::: "memory");
        }
        // B fragments read kMrBpd k-steps ahead of their MFMAs (the sched barriers keep the reads
        // there: left to itself the scheduler put each read right before its use, exposing the LDS
        // latency every 2 MFMAs)
        mf_i32x4 bq[C][TPS];
        auto rd_b = [&](auto slc) __attribute__((always_inline)) {
            constexpr int sl = decltype(slc)::value;
#pragma unroll
            for (int q = 0; q < TPS; ++q)
                bq[sl][q] = *reinterpret_cast<const mf_i32x4*>(&pl[q * kMrTileLds + 32 * r + 32 * sl + 16 * hf]);
        };
        static_for<0, (BPD < C ? BPD : C)>([&](auto slc) { rd_b(slc); });
        static_for<0, C>([&](auto slc) {
            constexpr int sl = decltype(slc)::value;
            if constexpr (sl + BPD < C) rd_b(std::integral_constant<int, sl + BPD>{});
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (FIR_MR_EXP != 1) {  // (FIR_MR_EXP: timing experiments only)
#pragma unroll
                for (int q = 0; q < TPS; ++q) {
                    const mf_i32x4 b = XLDS ? bq[sl][q] : bq[sl][q] ^ (int)0x80808080;
                    if constexpr (!MULTI && sl == 0) {  // a run's first k-step: the bias, and zero
                        acc_ll[q] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a_lo[sl], b, BIASV ? biasv : mf_i32x16{}, 0, 0, 0);
                        acc_mid[q] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a_hi[sl], b, mf_i32x16{}, 0, 0, 0);
                    } else {
                        acc_ll[q] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a_lo[sl], b, acc_ll[q], 0, 0, 0);
                        acc_mid[q] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a_hi[sl], b, acc_mid[q], 0, 0, 0);
                    }
                }
            }
            if constexpr (ROLL) {  // step sl's fragments of the next iteration's chunk (nc)
                const mf_i32x4* fn = frag + (int64_t)nc * C * 2 * kWave + lane;
                a_lo[sl] = fn[(2 * sl) * kWave], a_hi[sl] = fn[(2 * sl + 1) * kWave];
            }
            __builtin_amdgcn_sched_barrier(0);
        });
        if (c == nch - 1) {  // the run's tiles are complete: combine, round, stage, store
#pragma unroll
            for (int q = 0; q < TPS; ++q) {
                const uint32_t t = rn * TPS + q;
                const MfTile tl = tile_of(t, rcur);
                const int m = t < ntiles ? (int)min((int64_t)kMfTile, tl.re - tl.ts) : 0;
                int32_t o[16];
                uint32_t a[16];
#pragma unroll
                for (int i = 0; i < 16; ++i)  // (one chunk: the bias started acc_ll)
                    a[i] = ((uint32_t)acc_mid[q][i] << 8) + (uint32_t)acc_ll[q][i] + (MULTI || !BIASV ? bias : 0u);
                if (mode == 0) {
#pragma unroll
                    for (int i = 0; i < 16; ++i)
                        o[i] = STAGE == FIR_OUT_U8_SAT ? (int32_t)mf_med3_0(a[i], sat_hi) : (int32_t)a[i] >> frac;
                } else if (mode == 1) {
#pragma unroll
                    for (int i = 0; i < 16; ++i) o[i] = round_acc<true>(a[i], 0, frac);
                } else {
#pragma unroll
                    for (int i = 0; i < 16; ++i) o[i] = round_acc<false>(a[i], shl, frac);
                }
                if constexpr (MULTI) acc_ll[q] = mf_i32x16{}, acc_mid[q] = mf_i32x16{};
                if constexpr (STAGE == FIR_OUT_U8_SAT) {
                    uint32_t w[4];
#pragma unroll
                    for (int g4 = 0; g4 < 4; ++g4) {
                        if (mode == 0)
                            w[g4] = mf_shr_byte<3>(mf_shr_byte<2>(mf_shr_byte<1>((uint32_t)o[4 * g4] >> frac, (uint32_t)o[4 * g4 + 1], frac),
                                                                  (uint32_t)o[4 * g4 + 2], frac),
                                                   (uint32_t)o[4 * g4 + 3], frac);
                        else
                            w[g4] = (uint32_t)stage_out32<STAGE>(o[4 * g4]) | ((uint32_t)stage_out32<STAGE>(o[4 * g4 + 1]) << 8) |
                                    ((uint32_t)stage_out32<STAGE>(o[4 * g4 + 2]) << 16) |
                                    ((uint32_t)stage_out32<STAGE>(o[4 * g4 + 3]) << 24);
                    }
                    const auto s02 = __builtin_amdgcn_permlane32_swap(w[0], w[2], false, false);
                    const auto s13 = __builtin_amdgcn_permlane32_swap(w[1], w[3], false, false);
                    __builtin_amdgcn_raw_buffer_store_b128(mf_i32x4{(int)s02[0], (int)s02[1], (int)s13[0], (int)s13[1]},
                                                           mf_rsrc(y + tl.ts, (uint32_t)m), (uint32_t)(32 * r + 16 * hf), 0,
                                                           kMfAuxNt);
                } else {
                    __builtin_amdgcn_wave_barrier();
                    asm volatile("" ::: "memory");
#pragma unroll
                    for (int g4 = 0; g4 < 4; ++g4)
                        *reinterpret_cast<u4*>(&ob[36 * r + 8 * g4 + 4 * hf]) =
                            u4{(uint32_t)o[4 * g4], (uint32_t)o[4 * g4 + 1], (uint32_t)o[4 * g4 + 2], (uint32_t)o[4 * g4 + 3]};
                    __builtin_amdgcn_wave_barrier();
                    asm volatile("" ::: "memory");
                    const __amdgpu_buffer_rsrc_t rd = mf_rsrc(y + tl.ts, (uint32_t)m * 4u);
#pragma unroll
                    for (int rho = 0; rho < 4; ++rho) {
                        const int oo = 256 * rho + 4 * lane;
                        __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const mf_i32x4*>(&ob[36 * (oo >> 5) + (oo & 31)]),
                                                               rd, (uint32_t)oo * 4u, 0, kMfAuxNt);
                    }
                }
            }
        }
        stored = c == nch - 1;
        if (nr >= nruns) return false;
        rn = nr, c = nc, buf = buf + 1 == NBUF ? 0 : buf + 1;
        if constexpr (CUR) cur_step(rcur);
        __builtin_amdgcn_wave_barrier();  // this iteration's B reads are done before its buffer is refilled
        asm volatile("" ::: "memory");
        return true;
    };
    if constexpr (ADBL) {
        for (;;) {  // the two fragment sets alternate (unrolled: registers are not indexable)
            if (!body(a0_lo, a0_hi, a1_lo, a1_hi)) break;
            if (!body(a1_lo, a1_hi, a0_lo, a0_hi)) break;
        }
    } else {
        while (body(a0_lo, a0_hi, a0_lo, a0_hi)) {}
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the DMAs past the end land before the wave exits
}

// k-steps per chunk for KS k-steps: one chunk of exactly KS (rounded up to an even count past 12)
// when KS <= kMrC; past it the chunk size among 8..kMrC (even) with the least zero padding, the
// larger on a tie (fewer iterations)
static int mfma_run_ns(int KS, int multi_max, int one_max) {
    if (KS <= 12) return KS < 4 ? 4 : KS;
    if (KS <= one_max) return (KS + 1) & ~1;
    int best = multi_max, pad = (KS + multi_max - 1) / multi_max * multi_max;
    for (int ns = multi_max - 2; ns >= (multi_max <= 8 ? FIR_MR_MNS_MIN : 8); ns -= 2) {
        const int p = (KS + ns - 1) / ns * ns;
        if (p < pad) best = ns, pad = p;
    }
    return best;
}

template <int STAGE>
static hipError_t launch_mfma_run(const void* x, void* y, int64_t rl, int64_t tpr, int64_t ntiles, const int32_t* hq,
                                  int L, int P, int KS, uint32_t bias, bool fast, int frac, int acc_bits, hipStream_t s) {
    using OutT = typename OutTraits<STAGE>::T;
    std::string err;
    // several chunks, u8 stage: runs of FIR_MR_MTPS tiles (4: each chunk's fragments, loaded once
    // per iteration from L2, feed 4 tiles, so their latency is paid per 4 tiles), chunks of <= 8
    // k-steps (the accumulators of 4 tiles and one fragment set fit two waves per SIMD)
    constexpr int MTPS = STAGE == FIR_OUT_U8_SAT ? FIR_MR_MTPS : kMrTps;
    const int ns = mfma_run_ns(KS, MTPS == 4 ? 8 : kMrC, STAGE == FIR_OUT_U8_SAT ? FIR_MR_U8_ONE : kMrC);
    const int ksp = (KS + ns - 1) / ns * ns;  // the table padded to whole chunks (zero fragments)
    const mf_i32x4* fr = mfma_frag_table(hq, L, P, ksp, &err);
    if (!fr) return hipErrorOutOfMemory;
    TableHold hold(fr, s);
    const bool multi = ksp > ns;
    const int tps = !multi && ns <= FIR_MR_T1_NS ? 1 : multi ? MTPS : kMrTps;
    const int64_t nruns = (ntiles + tps - 1) / tps;
    const int64_t want = (nruns + kMfWaves - 1) / kMfWaves;
    const int64_t cap = (int64_t)256 * mr_waves_of(STAGE, tps, multi, ns);
    const unsigned blocks = (unsigned)(want < cap ? want : cap);
    const uint32_t tp = (uint32_t)tpr, nt = (uint32_t)ntiles;
    const int mode = fast ? 0 : acc_bits == 32 ? 1 : 2;
    const int shl = mode == 2 ? 32 - acc_bits : 0;
    auto go = [&](auto nsc, auto mc) {
        constexpr int NS = decltype(nsc)::value;
        constexpr bool M = decltype(mc)::value;
        if constexpr (!M && NS <= FIR_MR_T1_NS)
            hipLaunchKernelGGL((fir1d_mfma_run_kernel<STAGE, NS, M, 1>), dim3(blocks), dim3(kBlock), 0, s,
                               (const uint8_t*)x, (OutT*)y, rl, tp, nt, fr, ksp, P, bias, mode, shl, frac);
        else if constexpr (M && MTPS == 4)
            hipLaunchKernelGGL((fir1d_mfma_run_kernel<STAGE, NS, M, 4>), dim3(blocks), dim3(kBlock), 0, s,
                               (const uint8_t*)x, (OutT*)y, rl, tp, nt, fr, ksp, P, bias, mode, shl, frac);
        else
            hipLaunchKernelGGL((fir1d_mfma_run_kernel<STAGE, NS, M, kMrTps>), dim3(blocks), dim3(kBlock), 0, s,
                               (const uint8_t*)x, (OutT*)y, rl, tp, nt, fr, ksp, P, bias, mode, shl, frac);
    };
    using std::integral_constant;
#define FIR_MR_NS(n)                                                                       \
    case n:                                                                                \
        if (multi) {                                                                       \
            if constexpr (MTPS == 4 ? (n == 6 || n == 8) : n >= 8 && n <= kMrC && n % 2 == 0)     \
                go(integral_constant<int, n>{}, std::true_type{});                         \
        } else {                                                                           \
            if constexpr (n <= (STAGE == FIR_OUT_U8_SAT ? FIR_MR_U8_ONE : kMrC))             \
                go(integral_constant<int, n>{}, std::false_type{});                        \
        }                                                                                  \
        break;
    switch (ns) {
        FIR_MR_NS(4) FIR_MR_NS(5) FIR_MR_NS(6) FIR_MR_NS(7) FIR_MR_NS(8) FIR_MR_NS(9) FIR_MR_NS(10) FIR_MR_NS(11) FIR_MR_NS(12)
        FIR_MR_NS(14) FIR_MR_NS(16) FIR_MR_NS(18) FIR_MR_NS(20) FIR_MR_NS(22) FIR_MR_NS(24) FIR_MR_NS(26)
        FIR_MR_NS(28) FIR_MR_NS(30) FIR_MR_NS(32)
        default: return hipErrorInvalidValue;
    }
#undef FIR_MR_NS
    return hipGetLastError();
}

template <typename InT, int STAGE, int KS>
static hipError_t launch_mfma_ks(const void* x, void* y, int64_t rowlen, int64_t tpr, int64_t ntiles, const MfmaTaps& t,
                                 const int32_t* hq, int L, int P, uint32_t bias, bool fast, int frac, int acc_bits,
                                 hipStream_t s) {
    using OutT = typename OutTraits<STAGE>::T;
    if constexpr (FIR_MF2) {
        const int64_t spr = (tpr + kMf2Tps - 1) / kMf2Tps, nsteps = ntiles / tpr * spr;
        const int64_t want2 = (nsteps + kMfWaves - 1) / kMfWaves;
        const unsigned b2 = (unsigned)(want2 < FIR_MF2_BLOCKS ? want2 : FIR_MF2_BLOCKS);
        const uint32_t sp = (uint32_t)spr, ns = (uint32_t)nsteps;
        if (fast)
            hipLaunchKernelGGL((fir1d_mfma_step_kernel<InT, STAGE, KS, true, true>), dim3(b2), dim3(kBlock), 0, s,
                               (const InT*)x, (OutT*)y, rowlen, sp, ns, t, P, bias, 0, frac);
        else if (acc_bits == 32)
            hipLaunchKernelGGL((fir1d_mfma_step_kernel<InT, STAGE, KS, true, false>), dim3(b2), dim3(kBlock), 0, s,
                               (const InT*)x, (OutT*)y, rowlen, sp, ns, t, P, bias, 0, frac);
        else
            hipLaunchKernelGGL((fir1d_mfma_step_kernel<InT, STAGE, KS, false, false>), dim3(b2), dim3(kBlock), 0, s,
                               (const InT*)x, (OutT*)y, rowlen, sp, ns, t, P, bias, 32 - acc_bits, frac);
        return hipGetLastError();
    }
    const int64_t want = (ntiles + kMfWaves - 1) / kMfWaves;
    unsigned blocks = (unsigned)(want < kMfMaxBlocks ? want : kMfMaxBlocks);
    const mf_i32x4* fr = nullptr;
    if constexpr (FIR_MFMA_TPW > 0) {
        std::string err;
        fr = mfma_frag_table(hq, L, P, KS, &err);
        if (!fr) return hipErrorOutOfMemory;
        const int64_t per_block = (int64_t)kMfWaves * FIR_MFMA_TPW;
        blocks = (unsigned)((ntiles + per_block - 1) / per_block);
    }
    if (fast)
        hipLaunchKernelGGL((fir1d_mfma_kernel<InT, STAGE, KS, true, true>), dim3(blocks), dim3(kBlock), 0, s, (const InT*)x,
                           (OutT*)y, rowlen, tpr, ntiles, t, fr, P, bias, 0, frac);
    else if (acc_bits == 32)
        hipLaunchKernelGGL((fir1d_mfma_kernel<InT, STAGE, KS, true, false>), dim3(blocks), dim3(kBlock), 0, s, (const InT*)x,
                           (OutT*)y, rowlen, tpr, ntiles, t, fr, P, bias, 0, frac);
    else
        hipLaunchKernelGGL((fir1d_mfma_kernel<InT, STAGE, KS, false, false>), dim3(blocks), dim3(kBlock), 0, s,
                           (const InT*)x, (OutT*)y, rowlen, tpr, ntiles, t, fr, P, bias, 32 - acc_bits, frac);
    if (fr) table_release(fr, s);  // (A/B variant's table) after the launch that reads it
    return hipGetLastError();
}

template <typename InT, int STAGE>
static hipError_t launch_mfma_t(const void* x, void* y, int64_t rows, int64_t rowlen, int64_t total, const int32_t* hq,
                                int L, int frac, int acc_bits, hipStream_t s) {
    const int c = L / 2, hl = L - 1 - c;
    const int P = (hl + 7) & ~7;
    const int K = 32 + c + P, KS = (K + 31) / 32;  // 2..3 up to kMfMaxTaps taps
    int64_t hsum = 0, habs = 0;
    for (int k = 0; k < L; ++k) hsum += hq[k], habs += hq[k] < 0 ? -(int64_t)hq[k] : hq[k];
    uint32_t bias = (uint32_t)(128 * hsum);  // mod 2^32
    // FAST: no sum can wrap acc_bits, nor overflow int32 once the rounding half is added
    const int64_t xmax = sizeof(InT) == 1 ? 255 : 32768;
    const bool fast = frac <= 22 && habs * xmax + ((int64_t)1 << (frac - 1)) < ((int64_t)1 << (acc_bits - 1));
    if (fast) bias += 1u << (frac - 1);
    const int64_t rl = rows > 1 ? rowlen : total;
    const int64_t tpr = (rl + kMfTile - 1) / kMfTile;
    const int64_t ntiles = (rows > 1 ? rows : 1) * tpr;
    if constexpr (sizeof(InT) == 1) {
        if (KS > 3 && FIR_MR) {  // u8 past the step kernel: the run kernel (halo rounded to 16)
            const int P16 = (hl + 15) & ~15, K16 = 32 + c + P16, KS16 = (K16 + 31) / 32;
            return launch_mfma_run<STAGE>(x, y, rl, tpr, ntiles, hq, L, P16, KS16, bias, fast, frac, acc_bits, s);
        }
    }
    if (KS > 3 || L > FIR_MFMA_LONG_FROM)
        return launch_mfma_long<InT, STAGE>(x, y, rl, tpr, ntiles, hq, L, P, KS, bias, fast, frac, acc_bits, s);
    MfmaTaps t;
    for (int e = 0; e < 128; ++e) {
        const int tap = 31 - e + c + P;
        const int v = tap >= 0 && tap < L ? hq[tap] : 0;
        const int lo = ((v + 128) & 255) - 128;  // balanced split: v = 256 hi + lo
        t.lo[e] = (int8_t)lo;
        t.hi[e] = (int8_t)((v - lo) / 256);
    }
    if (KS == 2) return launch_mfma_ks<InT, STAGE, 2>(x, y, rl, tpr, ntiles, t, hq, L, P, bias, fast, frac, acc_bits, s);
    return launch_mfma_ks<InT, STAGE, 3>(x, y, rl, tpr, ntiles, t, hq, L, P, bias, fast, frac, acc_bits, s);
}

bool mfma_path_ok(const void* x, const void* y, int in_dtype, int64_t rows, int64_t rowlen, int64_t total, int ch,
                  const int32_t* hq, int L, int frac, int acc_bits) {
    bool taps_ok = true;  // the high byte of the balanced split must be a signed byte
    for (int k = 0; k < L; ++k) taps_ok &= hq[k] >= -32768 && hq[k] <= 32639;
    // the tile index is a uint32 (one tile = 1024 outputs of one row)
    const int64_t ntiles = rows > 1 ? rows * ((rowlen + kMfTile - 1) / kMfTile) : (total + kMfTile - 1) / kMfTile;
    // filters up to FIR_MFMA_MAX_TAPS (fragment table KS x 2 KiB <= ~4 MiB); longer ones take the
    // generic kernel (a table near the 2^24-tap limit would be 512 MiB)
    return L >= 2 && L <= FIR_MFMA_MAX_TAPS && ch == 1 && taps_ok && acc_bits <= 32 && frac <= 31 &&
           (rows == 1 ? total : rowlen) % 8 == 0 &&  // row and tile edges on 8-sample vectors
           (uintptr_t)x % (in_dtype == FIR_IN_U8 ? 8 : 16) == 0 && (uintptr_t)y % 16 == 0 && total >= 8 &&
           total < ((int64_t)1 << 40) && ntiles < ((int64_t)1 << 32) - kMfMaxBlocks * kMfWaves;
}

hipError_t launch_fir1d_mfma(const void* x, int in_dtype, int64_t rows, int64_t rowlen, int64_t total,
                             const int32_t* hq, int L, int frac, int acc_bits, int stage, void* y, hipStream_t s) {
    if (in_dtype == FIR_IN_U8)
        return stage == FIR_OUT_U8_SAT ? launch_mfma_t<uint8_t, FIR_OUT_U8_SAT>(x, y, rows, rowlen, total, hq, L, frac, acc_bits, s)
                                       : launch_mfma_t<uint8_t, FIR_OUT_I32>(x, y, rows, rowlen, total, hq, L, frac, acc_bits, s);
    return stage == FIR_OUT_U8_SAT ? launch_mfma_t<int16_t, FIR_OUT_U8_SAT>(x, y, rows, rowlen, total, hq, L, frac, acc_bits, s)
                                   : launch_mfma_t<int16_t, FIR_OUT_I32>(x, y, rows, rowlen, total, hq, L, frac, acc_bits, s);
}

}  // namespace fir
