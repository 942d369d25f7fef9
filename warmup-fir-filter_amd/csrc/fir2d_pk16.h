// fir2d_pk16.h — the separable packed-16 2-D kernel with strips of any height.
//
// Same arithmetic as fir2d_reg_kernel's PK16 form (fir2d_reg.h: rank-1 taps h = 2^s colq x rowq,
// both passes on v_pk_mad_u16 over pixel pairs, exact mod 2^16, the u8 stage taken from the
// provably 16-bit sum), but the strip loop is ROLLED in turns of U = lcm(R, PD + 1) input rows:
// the row ring (t % R) and the prefetch ring (t % (PD + 1)) are compile-time inside a turn, so a
// strip can be as tall as the launch wants without the code (and its register ring) growing.
// fir2d_reg_kernel unrolls its whole 32-row strip; taller strips spilled its ring to scratch
// (614-640 us per 4 frames, profiles/r02/ab2d_reg_pk_strip.txt), so 4 of every 36 input rows were
// re-read halo (PMC 1.064x) and the 2048-block grid ran 1.6 resident rounds.  Here the host sizes
// the strips so that the grid is ONE resident round (as fir2d_mfma.hip does).
//
// Rows are read through one buffer descriptor per frame: a row outside the frame, or past the
// strip's last input row, gets an offset outside the descriptor (its loads return zeros and issue
// no memory request), and an output row outside the frame or the strip likewise (the store is
// dropped): no branches around memory operations, so the compiler's wait counts stay exact.
#pragma once

#include "fir2d_reg.h"

namespace fir {

constexpr int p16_gcd(int a, int b) { return b ? p16_gcd(b, a % b) : a; }
constexpr int p16_lcm(int a, int b) { return a / p16_gcd(a, b) * b; }
constexpr uint32_t kP16Off = 0x80000000u;  // a buffer offset outside every descriptor

__device__ __forceinline__ __amdgpu_buffer_rsrc_t p16_rsrc(const void* p, uint32_t bytes) {
    const uint64_t a = (uint64_t)(uintptr_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    void* q = (void*)(uintptr_t)(((uint64_t)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(q, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

// MODE: kMode2dPk16 with kMode2dPkHi8 / kMode2dPkSigned as planned by plan_pk16 (u8 stage only).
template <int R, int C, int PD, int MODE, int MINW>
__global__ __launch_bounds__(kBlock, MINW) void fir2d_pk16_strip_kernel(const uint8_t* __restrict__ x,
                                                                        uint8_t* __restrict__ y, int64_t H,
                                                                        int64_t W, Taps2<R, C> taps, int S) {
    constexpr int VEC = 16, ND = 4, CC = C / 2;
    constexpr int HLE = C - 1 - CC, HRE = CC, TOP = R - 1 - R / 2;
    constexpr int RB = PD + 1;             // input-row ring
    constexpr int U = p16_lcm(R, RB);      // rows per unrolled turn
    static_assert(HLE <= 4 && HRE <= 4, "horizontal halo must fit in one dword");

    // XCD-major block order (dispatch is x fastest, then y, then z; blocks b, b + 8, ... share an
    // XCD): the blocks one XCD runs are consecutive strips, whose R - 1 shared rows then hit its L2
    int64_t bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
    {
        const int64_t gx = gridDim.x, gy = gridDim.y, nb = gx * gy * gridDim.z;
        const int64_t b = bx + gx * (by + gy * bz), q = nb / 8;
        const int64_t p = b < q * 8 ? (b % 8) * q + b / 8 : b;
        bx = p % gx;
        by = (p / gx) % gy;
        bz = p / (gx * gy);
    }
    // one descriptor per frame (H * W < 2^31, host-checked); 32-bit offsets row * W + column
    const __amdgpu_buffer_rsrc_t xs = p16_rsrc(x + bz * H * W, (uint32_t)(H * W));
    const __amdgpu_buffer_rsrc_t ys = p16_rsrc(y + bz * H * W, (uint32_t)(H * W));
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t col0 = (bx * kBlock + threadIdx.x) * VEC;
    const bool active = col0 < W;
    // halo dword: lane 0 the 4 pixels left of its vector, lane 63 the 4 right of it (others: none)
    const int64_t hraw = lane == 0 ? col0 - 4 : col0 + VEC;
    const bool hok = ((lane == 0 && HLE > 0) || (lane == kWave - 1 && HRE > 0)) && hraw >= 0 && hraw < W;
    const int r0 = (int)by * S;
    const int T = S + R - 1;  // input rows of this strip
    const int h32 = (int)H, w32 = (int)W;
    // Odd strips walk UP their rows: two neighbouring strips (consecutive blocks of one XCD, one
    // resident round) then read the R - 1 rows they share at the same moment — both at their
    // start or both at their end — so the second read is an L2 hit instead of an HBM re-read.
    // Step t reads row0 + dir * t; the column taps flip with the walk (the newest row of an
    // upward walk is the window's top row).
    const bool up = (by & 1) != 0;  // odd strips walk up (every strip down: 85.3 vs 78.8 us, r03/ab2d_pk16_rows.txt)
    const int row0 = up ? r0 + S - 1 + (R - 1 - TOP) : r0 - TOP, dir = up ? -1 : 1;
    const int orow0 = up ? r0 + S - 1 + (R - 1) : r0 - (R - 1);  // output row of step t: orow0 + dir * t
    uint32_t colb[R];
#pragma unroll
    for (int m = 0; m < R; ++m) colb[m] = up ? taps.colb[R - 1 - m] : taps.colb[m];

    uint32_t rows[RB][ND], hrows[RB];
    auto load_row = [&](int t, int slot) __attribute__((always_inline)) {
        const int row = row0 + dir * t;
        const bool ok = row >= 0 && row < h32 && t < T;  // wave-uniform
        const uint32_t rb = (uint32_t)row * (uint32_t)w32;
        typedef int i32x4 __attribute__((ext_vector_type(4)));
        const i32x4 q = __builtin_amdgcn_raw_buffer_load_b128(xs, ok && active ? rb + (uint32_t)col0 : kP16Off, 0, 0);
        rows[slot][0] = q.x, rows[slot][1] = q.y, rows[slot][2] = q.z, rows[slot][3] = q.w;
        hrows[slot] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(xs, ok && hok ? rb + (uint32_t)hraw : kP16Off, 0, 0);  // (non-temporal row loads: 105 us)
    };
    uint32_t rs2[R][VEC / 2] = {};  // row-sum pair ring
#pragma unroll
    for (int i = 0; i < PD; ++i) load_row(i, i);

    for (int t0 = 0; t0 < T; t0 += U) {
#pragma unroll
        for (int i = 0; i < U; ++i) {
            const int t = t0 + i;  // t0 % U == 0: every ring index below is a compile-time constant
            load_row(t + PD, (i + PD) % RB);
            const uint32_t* cur = rows[i % RB];
            const uint32_t hcur = hrows[i % RB];
            // byte stream [left-halo dword | own dwords | right-halo dword]; window pixel k is
            // stream byte k + (4 - HLE); P[k] = (w[k], w[k+1]) as 16-bit halves
            uint32_t sb[ND + 2];
            sb[0] = HLE > 0 ? from_prev_lane(hcur, cur[ND - 1]) : 0u;
#pragma unroll
            for (int k = 0; k < ND; ++k) sb[1 + k] = cur[k];
            sb[ND + 1] = HRE > 0 ? from_next_lane(hcur, cur[0]) : 0u;
            constexpr int NP = VEC + C - 1;
            uint32_t Pr[NP + 4 - HLE];
            PairBuilder<4 - HLE, NP>::run(sb, Pr);
            const uint32_t* P = Pr + (4 - HLE);
            uint32_t* r = rs2[i % R];
#pragma unroll
            for (int q = 0; q < VEC / 2; ++q) r[q] = pk_mul16(P[2 * q], taps.rowb[0]);
#pragma unroll
            for (int k = 1; k < C; ++k)
#pragma unroll
                for (int q = 0; q < VEC / 2; ++q) r[q] = pk_mad16(P[2 * q + k], taps.rowb[k], r[q]);
            // output row orow0 + dir * t = bias + sum_m colb[m] rs_{t-m}; computed for every t (the
            // first R - 1 steps' rows are dropped by the store offset, not by a branch)
            uint32_t pko[VEC / 2];
#pragma unroll
            for (int q = 0; q < VEC / 2; ++q) pko[q] = pk_mad16(r[q], colb[0], taps.pkbias);
#pragma unroll
            for (int m = 1; m < R; ++m)
#pragma unroll
                for (int q = 0; q < VEC / 2; ++q) pko[q] = pk_mad16(rs2[((i - m) % R + R) % R][q], colb[m], pko[q]);
            typedef int i32x4 __attribute__((ext_vector_type(4)));
            i32x4 val;
#pragma unroll
            for (int k = 0; k < ND; ++k) {
                uint32_t w;
                if constexpr ((MODE & kMode2dPkHi8) != 0) {
                    w = __builtin_amdgcn_perm(pko[2 * k + 1], pko[2 * k], 0x07050301u);
                } else {
                    constexpr bool SG = (MODE & kMode2dPkSigned) != 0;
                    const uint32_t lo = pk_stage_u8<SG>(pko[2 * k], taps.pkshift, taps.pkmax);
                    const uint32_t hi = pk_stage_u8<SG>(pko[2 * k + 1], taps.pkshift, taps.pkmax);
                    w = __builtin_amdgcn_perm(hi, lo, 0x06040200u);
                }
                val[k] = (int)w;
            }
            const int orow = orow0 + dir * t;
            const bool ook = t >= R - 1 && t < T && orow < h32 && active;
            __builtin_amdgcn_raw_buffer_store_b128(val, ys, ook ? (uint32_t)orow * (uint32_t)w32 + (uint32_t)col0 : kP16Off,
                                                   0, 2 /* non-temporal */);
        }
    }
}

}  // namespace fir
