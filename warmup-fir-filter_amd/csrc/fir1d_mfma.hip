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
// Three kernels, by filter length: up to 3 k-steps (65 taps) the step kernel (tap fragments in
// VGPRs for the whole grid-stride loop, windows of 2 tiles loaded one step ahead and split into
// signed-byte planes on the way into wave-private LDS: u8 one XOR per 4 samples, int16 6 VALU
// per 8); past it, u8 input takes the run kernel (windows by LDS-DMA, fragments per chunk of
// k-steps shared by a run of tiles) and int16 the chunked kernel (fragments from an L2-resident
// table).  Each reads B fragments with one ds_read_b128 per plane and k-step.  Rows (images)
// whose length is a multiple of 8 are tiled row by row, samples of other rows zeroed while staging.
#include <string>
#include <type_traits>
#include <vector>

#include "fir_common.h"
#include "fir_launch.h"

namespace fir {

constexpr int kMfTile = 1024;        // outputs per wave tile (32 B columns x 32 A rows)
constexpr int kMfWaves = kBlock / kWave;
constexpr int kMfMaxTaps = 65536;    // longest filter on the matrix cores (fragment table <= 4 MiB)

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

// ---------------------------------------------------------------------------------------
// Step form (round 3b; every filter of up to 3 k-steps, i.e. 65 taps): the Toeplitz product
// above, a wave's grid-stride unit being a STEP of kMf2Tps consecutive tiles of one row, whose
// window (kMf2Tps * 1024 + 32 KS - 32 samples) is loaded at once and staged as byte planes in the
// wave's LDS, the tiles' MFMAs reading it at offsets 1024 q.  It replaced a one-tile-per-iteration
// kernel (removed in round 5, numbers in DESIGN.md §8) that kept about 2.2 KiB of loads in
// flight per wave and sat at the 147 us its loop reached as a pure copy (int16,
// profiles/r03/long_taps_mfma_structure.txt).  Here each wave keeps kMf2Tps * 2 KiB (int16) in
// flight during the whole step's math, the window's halo is re-read once per step instead of
// once per tile, and the loop is shaped so the compiler's waits are exact: every path into the
// loop header has the same memory operations in flight (the entry edge issues the step's store
// count as dropped stores, descriptor size 0), every load and store is unconditional (ranges
// clipped by the descriptors), and the wait at the top of a step is vmcnt(stores of the previous
// step).  int16 input: the two cross products share one accumulator, int32 outputs leave
// through LDS as whole 1 KiB rows, and the body loads are non-temporal (i16 -> u8 150-155 ->
// 141-146 us; u8 input keeps the default policy: its 256 MiB planes partly stay in the Infinity
// Cache between calls).
constexpr int kMf2Tps = 2;           // tiles per step
constexpr int kMf2Blocks = 2048;     // grid-stride blocks (4 waves each; two resident rounds)

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
__global__ __launch_bounds__(kBlock, 4) void fir1d_mfma_step_kernel(const InT* __restrict__ x,
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
    constexpr bool OLDS = STAGE == FIR_OUT_I32;
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

    // tap fragments A[r][32 s + 16 hf + j], j = 0..15 (entries of MfmaTaps by diagonal)
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
            constexpr int aux = I16 ? kMfAuxNt : 0;
            if constexpr (I16) {
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
            // outputs of this tile (0: past the row)
            const int m = (int)max((int64_t)0, min((int64_t)kMfTile, re - ts));
            mf_i32x16 acc_ll = {}, acc_mid = {}, acc_hh = {};
#pragma unroll
            for (int s = 0; s < KS; ++s) {
                const int i = q * kMfTile + 32 * r + 32 * s + 16 * hf;
                const mf_i32x4 b_l = *reinterpret_cast<const mf_i32x4*>(&pl[i]);
                acc_ll = __builtin_amdgcn_mfma_i32_32x32x32_i8(a_lo[s], b_l, acc_ll, 0, 0, 0);
                acc_mid = __builtin_amdgcn_mfma_i32_32x32x32_i8(a_hi[s], b_l, acc_mid, 0, 0, 0);
                if constexpr (I16) {
                    const mf_i32x4 b_h = *reinterpret_cast<const mf_i32x4*>(&ph[i]);
                    acc_hh = __builtin_amdgcn_mfma_i32_32x32x32_i8(a_hi[s], b_h, acc_hh, 0, 0, 0);
                    // two MFMAs (acc_hh) after acc_mid's first write this step: no back-to-back dependency
                    acc_mid = __builtin_amdgcn_mfma_i32_32x32x32_i8(a_lo[s], b_h, acc_mid, 0, 0, 0);
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
                    const uint32_t mid = (uint32_t)acc_mid[i];
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
// int16 filters past the step kernel's 3 k-steps: the same Toeplitz product with K = 32 + L/2 + P
// split into chunks of kMlChunk k-steps.  Per tile and chunk the wave stages the chunk's window
// (992 + 32 * steps samples) as byte planes in its LDS, then runs the chunk's k-steps with the
// accumulators carried over: the tap fragments no longer fit VGPRs, so each k-step's A fragments
// come from a table in HBM (frag[s][plane][lane], 16 bytes per lane: one coalesced 1 KiB load per
// plane, the same for every tile, so L2-resident).
constexpr int kMlChunk = 16;                          // k-steps per staged window
constexpr int kMlBlocks = 2048;                       // grid-stride blocks
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
    TableHash h(kTableMfmaFrag);
    h.add(hq, sizeof(int32_t) * (size_t)L);
    h.add_val(L), h.add_val(P), h.add_val(KS);
    const size_t bytes = (size_t)KS * 2 * kWave * 16;
    return (const mf_i32x4*)table_acquire(std::move(h), bytes, [&](void* dst) {
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
    const unsigned blocks = (unsigned)(want < kMlBlocks ? want : kMlBlocks);
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
// Shipped configuration (the A/B forms measured against it and removed in round 5 are listed in
// DESIGN.md §8, with their numbers):
constexpr int kMrTps = 2;            // tiles per run (one-chunk filters past kMrT1Ns k-steps)
constexpr int kMrC = 16;             // k-steps per chunk (int32 stage)
constexpr int kMrWaves = 2;          // waves per SIMD of 2-tile runs (LDS: (DEPTH+1) TPS 2 KiB per wave)
constexpr int kMrDepth = 2;          // iterations whose windows are in flight ahead of the one computed
constexpr int kMrW4Ns = 8;           // one-tile runs up to this many k-steps: 4 waves per SIMD (u8 out; vs 6:
                                     // 162 / 194 taps 140 / 136 us vs 149 / 139, profiles/r04/long_taps_w4ns_ab.txt)
constexpr int kMrMTps = 4;           // tiles per run with several chunks (u8 stage)
constexpr int kMrMNsMin = 6;         // shortest chunk considered with 4-tile runs
constexpr int kMrMDepth = 1;         // window iterations in flight with 4-tile runs (LDS: 2 WGs per CU)
constexpr int kMrDepth1 = 3;         // window iterations in flight with one tile per run (u8 out; 12 waves
                                     // per CU: (kMrDepth1 + 1) x 2 KiB of LDS each)
constexpr int kMrU8One = 32;         // u8 out: one chunk (fragments loaded once per wave) up to this many k-steps
constexpr int kMrT1Ns = 32;          // one-chunk filters up to this many k-steps: one tile per run (vs 10, 2-tile
                                     // runs past it: 290 / 322 / 450 taps 165 / 173 / 212 us vs 196 / 189 / 221,
                                     // profiles/r04/long_taps_t1ns_ab.txt)
constexpr int kMrXldsFrom = 8;       // chunk lengths whose windows are re-biased in LDS
constexpr int kMrBpd = 3;            // k-steps whose B fragments are read ahead of the MFMAs
constexpr int kMrMWaves = 2;         // waves per SIMD with several chunks
constexpr int kMrW3Ns = 12;          // one-tile runs of up to this many k-steps: 3 waves per SIMD (2 past it)
constexpr int kMrW2Ns = 24;          // ... 2 waves up to this many (1 past it)
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
// TPS tiles per run: 2 (kMrTps) at 2 waves per SIMD; 1 at 3 waves per SIMD (and windows one
// iteration deeper) for one-chunk filters up to 10 k-steps, whose registers fit a third wave
// (A/B at 66 / 128 / 257 taps: 109 / 119 / 151 us vs 127 / 131 / 170, profiles/r04/long_taps_run_v3_ab.txt)
// Several chunks: kMrMWaves waves per SIMD, one fragment set loaded at the top of each iteration.
constexpr int mr_waves_of(int stage, int tps, bool multi, int ns) {
    return multi ? kMrMWaves
                 : tps == 1 ? (ns <= kMrW4Ns && stage == FIR_OUT_U8_SAT ? 4
                               : ns <= (stage == FIR_OUT_U8_SAT ? kMrW3Ns : 11) ? 3  // (int32 out: 12 spilled)
                               : ns <= kMrW2Ns ? 2 : 1)
                            : kMrWaves;
}
template <int STAGE, int TPS_, bool MULTI, int NS>
constexpr int mr_waves() {
    return mr_waves_of(STAGE, TPS_, MULTI, NS);
}
// HN: the k-steps whose taps need the high byte plane.  -1: every k-step (both planes, one
// accumulator each).  0: none (every tap in [-128, 127]: a Q4.12 filter of small taps, e.g. a long
// smoothing window): low-plane MFMAs only, the even and odd k-steps in two accumulators (no
// back-to-back dependent MFMA).  2 / 4: the high plane for k-steps hs0 .. hs0 + HN - 1 only (a
// windowed filter's large centre taps), their B fragments read at that run-time offset, the low
// plane in two accumulators as for 0.  One chunk only (the launcher picks HN from the taps).
template <int STAGE, int NS, bool MULTI, int TPS_, int HN = -1>
__global__ __launch_bounds__(kBlock, (mr_waves<STAGE, TPS_, MULTI, NS>())) void fir1d_mfma_run_kernel(const uint8_t* __restrict__ x,
                                                                   typename OutTraits<STAGE>::T* __restrict__ y,
                                                                   int64_t rowlen, uint32_t tiles_per_row, uint32_t ntiles,
                                                                   const mf_i32x4* __restrict__ frag, int KS, int P,
                                                                   uint32_t bias, int mode, int shl, int frac, int hs0) {
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    constexpr int TPS = TPS_, C = NS;
    static_assert(HN < 0 || (!MULTI && HN <= NS), "high-plane k-step ranges: one chunk");
    constexpr bool OLDS = STAGE == FIR_OUT_I32;
    constexpr int kDepth = TPS == 1 ? (OLDS ? 3 : kMrDepth1) : TPS == 4 ? kMrMDepth : kMrDepth;
    constexpr int WT = kMfTile + 32 * C - 32;  // window samples per tile and chunk
    constexpr int NVT = (WT + 15) / 16;         // 16-sample vectors per tile window
    static_assert(NVT > kWave && NVT <= 2 * kWave && 16 * 2 * kWave <= kMrTileLds, "two DMAs per tile window");
    constexpr int BUF = TPS * kMrTileLds;
    constexpr int NBUF = kDepth + 1;            // LDS window buffers per wave (a ring)
    constexpr int NDMA = 2 * TPS;               // DMA instructions per iteration
    constexpr int NST = TPS * (OLDS ? 4 : 1);   // store instructions per completed run
    // the x - 128 of the B operand: in LDS once per window (long chunks) or per fragment read
    constexpr bool XLDS = C >= kMrXldsFrom;
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

    // tap fragments: one set (one chunk: loaded once per wave; several: the iteration's chunk,
    // loaded at the top of each iteration)
    constexpr int NH = HN < 0 ? C : HN > 0 ? HN : 1;  // high-plane fragment registers
    mf_i32x4 a0_lo[C], a0_hi[NH];
    auto load_a = [&](mf_i32x4 (&lo)[C], mf_i32x4 (&hi)[NH], int c) __attribute__((always_inline)) {
        const mf_i32x4* f = frag + (int64_t)c * C * 2 * kWave + lane;
        if constexpr (HN < 0) {
#pragma unroll
            for (int s = 0; s < C; ++s) lo[s] = f[(2 * s) * kWave], hi[s] = f[(2 * s + 1) * kWave];
        } else {
#pragma unroll
            for (int s = 0; s < C; ++s) lo[s] = f[(2 * s) * kWave];
#pragma unroll
            for (int j = 0; j < HN; ++j) hi[j] = f[(2 * (hs0 + j) + 1) * kWave];
        }
    };
    // One tile per run and one chunk (the wave's tiles t, t + S, t + 2S, ...): the tile's row and
    // column advance by constant steps (one division at the start instead of one per tile and use,
    // ~40 of the loop's ~114 SALU per tile).  Past the last tile the cursor runs on; those tiles'
    // descriptors have size 0.
    constexpr bool CUR = TPS == 1 && !MULTI;
    // the bias as the first MFMA's accumulator input (16 VGPRs) or one add per output
    // (23-24 k-steps at 2 waves per SIMD: no bias registers and 2 reads ahead, or they spill; at 1
    // wave both cost ~4 %: 800 / 930 taps 430 / 478 vs 414 / 461 us, profiles/r04/long_taps_one_chunk_ab.txt)
    constexpr bool TRIM = NS > 22 && mr_waves<STAGE, TPS_, MULTI, NS>() == 2;
    constexpr bool BIASV = mr_waves<STAGE, TPS_, MULTI, NS>() < 4 && !TRIM;
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

    // acc_ll: the low plane (HN >= 0: its even k-steps), acc_lo2 (HN >= 0): the odd k-steps' low
    // plane, acc_mid: the high plane
    mf_i32x16 acc_ll[TPS], acc_mid[TPS], acc_lo2[TPS];
#pragma unroll
    for (int q = 0; q < TPS; ++q) acc_ll[q] = mf_i32x16{}, acc_mid[q] = mf_i32x16{}, acc_lo2[q] = mf_i32x16{};
    mf_i32x16 biasv;
#pragma unroll
    for (int i = 0; i < 16; ++i) biasv[i] = (int)bias;
    if constexpr (!MULTI) load_a(a0_lo, a0_hi, 0);  // KS <= C: one chunk, fragments loaded once
    // iterations (run, chunk) in order; `ahead` is the one whose windows are issued next, kDepth
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
    for (int d = 0; d < kDepth; ++d) {
        issue_win(ar, ac, d);
        advance_ahead();
        if constexpr (!MULTI) {  // stand-ins for the stores of the iterations before the first (a
            const __amdgpu_buffer_rsrc_t none = mf_rsrc(y, 0u);  // zero-size range: nothing written),
#pragma unroll                                                   // so the counted wait below is exact
            for (int k = 0; k < NST; ++k) __builtin_amdgcn_raw_buffer_store_b32(0, none, 0, 0, 0);
        }
    }
    // one iteration (run rn, chunk c); false at the end
    auto body = [&](mf_i32x4 (&a_lo)[C], mf_i32x4 (&a_hi)[NH]) __attribute__((always_inline)) -> bool {
        uint32_t nr = rn;
        int nc = c;
        advance(nr, nc);
        if constexpr (MULTI) load_a(a_lo, a_hi, c);  // issued before the next windows: its wait leaves them in flight
        issue_win(ar, ac, buf == 0 ? NBUF - 1 : buf - 1);  // the buffer computed last iteration
        advance_ahead();
        // this iteration's windows (and A) landed; the younger operations stay in flight.  vmcnt
        // also counts stores, in order with the loads.  One chunk: every iteration ends with its
        // NST stores, so kDepth iterations of DMAs + stores may stay outstanding (counting only
        // the DMAs drained the next iteration's windows too).  Several: this iteration's A was
        // issued just above, before the next windows, so only those DMAs may stay outstanding.
        if constexpr (MULTI)
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kDepth * NDMA) : "memory");
        else
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kDepth * (NDMA + NST)) : "memory");
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
        // the high plane's B fragments (HN > 0: k-steps hs0 .., a run-time offset)
        mf_i32x4 bh[HN > 0 ? HN : 1][TPS];
        if constexpr (HN > 0) {
#pragma unroll
            for (int j = 0; j < HN; ++j)
#pragma unroll
                for (int q = 0; q < TPS; ++q) {
                    const mf_i32x4 v = *reinterpret_cast<const mf_i32x4*>(&pl[q * kMrTileLds + 32 * r + 32 * (hs0 + j) + 16 * hf]);
                    bh[j][q] = XLDS ? v : v ^ (int)0x80808080;
                }
        }
        static_for<0, (BPD < C ? BPD : C)>([&](auto slc) { rd_b(slc); });
        static_for<0, C>([&](auto slc) {
            constexpr int sl = decltype(slc)::value;
            if constexpr (sl + BPD < C) rd_b(std::integral_constant<int, sl + BPD>{});
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int q = 0; q < TPS; ++q) {
                const mf_i32x4 b = XLDS ? bq[sl][q] : bq[sl][q] ^ (int)0x80808080;
                if constexpr (HN >= 0) {  // low plane: even / odd k-steps in two accumulators
                    mf_i32x16& la = (sl & 1) ? acc_lo2[q] : acc_ll[q];
                    la = __builtin_amdgcn_mfma_i32_32x32x32_i8(a_lo[sl], b,
                                                                sl >= 2 ? la : sl == 0 && BIASV ? biasv : mf_i32x16{}, 0, 0, 0);
                    if constexpr (sl < HN)  // high plane of k-step hs0 + sl
                        acc_mid[q] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a_hi[sl], bh[sl][q], sl == 0 ? mf_i32x16{} : acc_mid[q],
                                                                           0, 0, 0);
                } else if constexpr (!MULTI && sl == 0) {  // a run's first k-step: the bias, and zero
                    acc_ll[q] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a_lo[sl], b, BIASV ? biasv : mf_i32x16{}, 0, 0, 0);
                    acc_mid[q] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a_hi[sl], b, mf_i32x16{}, 0, 0, 0);
                } else {
                    acc_ll[q] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a_lo[sl], b, acc_ll[q], 0, 0, 0);
                    acc_mid[q] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a_hi[sl], b, acc_mid[q], 0, 0, 0);
                }
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
                for (int i = 0; i < 16; ++i) {  // (one chunk: the bias started acc_ll)
                    const uint32_t lo = HN >= 0 ? (uint32_t)acc_ll[q][i] + (uint32_t)acc_lo2[q][i] : (uint32_t)acc_ll[q][i];
                    a[i] = (HN != 0 ? ((uint32_t)acc_mid[q][i] << 8) : 0u) + lo + (MULTI || !BIASV ? bias : 0u);
                }
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
        if (nr >= nruns) return false;
        rn = nr, c = nc, buf = buf + 1 == NBUF ? 0 : buf + 1;
        if constexpr (CUR) cur_step(rcur);
        __builtin_amdgcn_wave_barrier();  // this iteration's B reads are done before its buffer is refilled
        asm volatile("" ::: "memory");
        return true;
    };
    while (body(a0_lo, a0_hi)) {}
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the DMAs past the end land before the wave exits
}

// k-steps per chunk for KS k-steps: one chunk of exactly KS (rounded up to an even count past 12)
// when KS <= kMrC; past it the chunk size among 8..kMrC (even) with the least zero padding, the
// larger on a tie (fewer iterations)
static int mfma_run_ns(int KS, int multi_max, int one_max) {
    if (KS <= 12) return KS < 4 ? 4 : KS;
    if (KS <= one_max) return (KS + 1) & ~1;
    int best = multi_max, pad = (KS + multi_max - 1) / multi_max * multi_max;
    for (int ns = multi_max - 2; ns >= (multi_max <= 8 ? kMrMNsMin : 8); ns -= 2) {
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
    // several chunks, u8 stage: runs of kMrMTps tiles (4: each chunk's fragments, loaded once
    // per iteration from L2, feed 4 tiles, so their latency is paid per 4 tiles), chunks of <= 8
    // k-steps (the accumulators of 4 tiles and one fragment set fit two waves per SIMD)
    constexpr int MTPS = STAGE == FIR_OUT_U8_SAT ? kMrMTps : kMrTps;
    const int ns = mfma_run_ns(KS, MTPS == 4 ? 8 : kMrC, STAGE == FIR_OUT_U8_SAT ? kMrU8One : kMrC);
    const int ksp = (KS + ns - 1) / ns * ns;  // the table padded to whole chunks (zero fragments)
    const mf_i32x4* fr = mfma_frag_table(hq, L, P, ksp, &err);
    if (!fr) return hipErrorOutOfMemory;
    TableHold hold(fr, s);
    const bool multi = ksp > ns;
    const int tps = !multi && ns <= kMrT1Ns ? 1 : multi ? MTPS : kMrTps;
    const int64_t nruns = (ntiles + tps - 1) / tps;
    const int64_t want = (nruns + kMfWaves - 1) / kMfWaves;
    const int64_t cap = (int64_t)256 * mr_waves_of(STAGE, tps, multi, ns);
    const unsigned blocks = (unsigned)(want < cap ? want : cap);
    const uint32_t tp = (uint32_t)tpr, nt = (uint32_t)ntiles;
    const int mode = fast ? 0 : acc_bits == 32 ? 1 : 2;
    const int shl = mode == 2 ? 32 - acc_bits : 0;
    // one chunk, u8 stage: the k-steps whose taps need the high byte plane (a tap outside
    // [-128, 127]); k-step st multiplies taps c + P - 32 st - 31 .. c + P - 32 st + 31
    int hn = -1, hs0 = 0;
    if (!multi && tps == 1 && STAGE == FIR_OUT_U8_SAT) {
        const int c = L / 2;
        int smin = ksp, smax = -1;
        for (int t = 0; t < L; ++t) {
            if (hq[t] >= -128 && hq[t] <= 127) continue;
            const int lo_st = (c + P - t - 31 + 31) / 32, hi_st = (c + P - t + 31) / 32;  // ceil / floor
            for (int st = lo_st < 0 ? 0 : lo_st; st <= hi_st && st < ksp; ++st) smin = st < smin ? st : smin, smax = st > smax ? st : smax;
        }
        // a partial high plane pays a third accumulator (16 more registers and combine adds per
        // output): worth it only when it drops at least twice the k-steps it keeps (A/B at 66 / 128
        // / 257 / 450 / 900 taps, windowed sinc: 116 / 124 / 146 / 209 / 454 -> 138 / 137 / 149 / 191
        // / 338 us, profiles/r05/long_taps_hn_ab.txt)
        const int need = smax < 0 ? 0 : smax - smin + 1;
        hn = need == 0 ? 0 : need <= 2 ? 2 : need <= 4 ? 4 : -1;
        if (hn > 0 && ksp < 3 * hn) hn = -1;
        if (hn > 0) hs0 = smin < ksp - hn ? smin : ksp - hn;
    }
    auto go = [&](auto nsc, auto mc) {
        constexpr int NS = decltype(nsc)::value;
        constexpr bool M = decltype(mc)::value;
        if constexpr (!M && NS <= kMrT1Ns) {
            auto one = [&](auto hnc) {
                constexpr int H = decltype(hnc)::value;
                hipLaunchKernelGGL((fir1d_mfma_run_kernel<STAGE, NS, M, 1, H>), dim3(blocks), dim3(kBlock), 0, s,
                                   (const uint8_t*)x, (OutT*)y, rl, tp, nt, fr, ksp, P, bias, mode, shl, frac, hs0);
            };
            if constexpr (STAGE == FIR_OUT_U8_SAT) {
                if (hn == 0) return one(std::integral_constant<int, 0>{});
                if (hn == 2) return one(std::integral_constant<int, 2>{});
                if (hn == 4) return one(std::integral_constant<int, 4>{});
            }
            one(std::integral_constant<int, -1>{});
        } else if constexpr (M && MTPS == 4) {
            hipLaunchKernelGGL((fir1d_mfma_run_kernel<STAGE, NS, M, 4>), dim3(blocks), dim3(kBlock), 0, s,
                               (const uint8_t*)x, (OutT*)y, rl, tp, nt, fr, ksp, P, bias, mode, shl, frac, 0);
        } else {
            hipLaunchKernelGGL((fir1d_mfma_run_kernel<STAGE, NS, M, kMrTps>), dim3(blocks), dim3(kBlock), 0, s,
                               (const uint8_t*)x, (OutT*)y, rl, tp, nt, fr, ksp, P, bias, mode, shl, frac, 0);
        }
    };
    using std::integral_constant;
#define FIR_MR_NS(n)                                                                       \
    case n:                                                                                \
        if (multi) {                                                                       \
            if constexpr (MTPS == 4 ? (n == 6 || n == 8) : n >= 8 && n <= kMrC && n % 2 == 0)     \
                go(integral_constant<int, n>{}, std::true_type{});                         \
        } else {                                                                           \
            if constexpr (n <= (STAGE == FIR_OUT_U8_SAT ? kMrU8One : kMrC))                  \
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
                                 int P, uint32_t bias, bool fast, int frac, int acc_bits, hipStream_t s) {
    using OutT = typename OutTraits<STAGE>::T;
    const int64_t spr = (tpr + kMf2Tps - 1) / kMf2Tps, nsteps = ntiles / tpr * spr;
    const int64_t want = (nsteps + kMfWaves - 1) / kMfWaves;
    const unsigned blocks = (unsigned)(want < kMf2Blocks ? want : kMf2Blocks);
    const uint32_t sp = (uint32_t)spr, ns = (uint32_t)nsteps;
    if (fast)
        hipLaunchKernelGGL((fir1d_mfma_step_kernel<InT, STAGE, KS, true, true>), dim3(blocks), dim3(kBlock), 0, s,
                           (const InT*)x, (OutT*)y, rowlen, sp, ns, t, P, bias, 0, frac);
    else if (acc_bits == 32)
        hipLaunchKernelGGL((fir1d_mfma_step_kernel<InT, STAGE, KS, true, false>), dim3(blocks), dim3(kBlock), 0, s,
                           (const InT*)x, (OutT*)y, rowlen, sp, ns, t, P, bias, 0, frac);
    else
        hipLaunchKernelGGL((fir1d_mfma_step_kernel<InT, STAGE, KS, false, false>), dim3(blocks), dim3(kBlock), 0, s,
                           (const InT*)x, (OutT*)y, rowlen, sp, ns, t, P, bias, 32 - acc_bits, frac);
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
    if (KS > 3) {  // past the step kernel (66 taps and up): u8 the run kernel (halo rounded to 16), int16 the chunked one
        if constexpr (sizeof(InT) == 1) {
            const int P16 = (hl + 15) & ~15, K16 = 32 + c + P16, KS16 = (K16 + 31) / 32;
            return launch_mfma_run<STAGE>(x, y, rl, tpr, ntiles, hq, L, P16, KS16, bias, fast, frac, acc_bits, s);
        }
        return launch_mfma_long<InT, STAGE>(x, y, rl, tpr, ntiles, hq, L, P, KS, bias, fast, frac, acc_bits, s);
    }
    MfmaTaps t;
    for (int e = 0; e < 128; ++e) {
        const int tap = 31 - e + c + P;
        const int v = tap >= 0 && tap < L ? hq[tap] : 0;
        const int lo = ((v + 128) & 255) - 128;  // balanced split: v = 256 hi + lo
        t.lo[e] = (int8_t)lo;
        t.hi[e] = (int8_t)((v - lo) / 256);
    }
    if (KS == 2) return launch_mfma_ks<InT, STAGE, 2>(x, y, rl, tpr, ntiles, t, P, bias, fast, frac, acc_bits, s);
    return launch_mfma_ks<InT, STAGE, 3>(x, y, rl, tpr, ntiles, t, P, bias, fast, frac, acc_bits, s);
}

bool mfma_path_ok(const void* x, const void* y, int in_dtype, int64_t rows, int64_t rowlen, int64_t total, int ch,
                  const int32_t* hq, int L, int frac, int acc_bits) {
    bool taps_ok = true;  // the high byte of the balanced split must be a signed byte
    for (int k = 0; k < L; ++k) taps_ok &= hq[k] >= -32768 && hq[k] <= 32639;
    // the tile index is a uint32 (one tile = 1024 outputs of one row)
    const int64_t ntiles = rows > 1 ? rows * ((rowlen + kMfTile - 1) / kMfTile) : (total + kMfTile - 1) / kMfTile;
    // filters up to kMfMaxTaps (fragment table KS x 2 KiB <= ~4 MiB); longer ones take the
    // generic kernel (a table near the 2^24-tap limit would be 512 MiB)
    return L >= 2 && L <= kMfMaxTaps && ch == 1 && taps_ok && acc_bits <= 32 && frac <= 31 &&
           (rows == 1 ? total : rowlen) % 8 == 0 &&  // row and tile edges on 8-sample vectors
           (uintptr_t)x % (in_dtype == FIR_IN_U8 ? 8 : 16) == 0 && (uintptr_t)y % 16 == 0 && total >= 8 &&
           total < ((int64_t)1 << 40) && ntiles < ((int64_t)1 << 32) - kMf2Blocks * kMfWaves;
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
