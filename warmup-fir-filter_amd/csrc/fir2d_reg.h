// fir2d_reg.h — register/DPP 2-D FIR kernel template, shared by the library
// (fir2d.hip) and the A/B microbenchmark (tools/microbench/fir2d_micro.hip).
//
// y[i,j] = stage(round(wrap(sum_m sum_n hq[m][n] * x[i - m + R/2][j - n + C/2]))), zero padded.
//
// A lane owns VEC horizontally adjacent pixels (one VEC-byte load per input row); the
// horizontal (C-1)-pixel halo arrives from the neighbouring lanes by DPP wave shifts (lanes
// 0 / 63 load one dword of the neighbouring wave's pixels); the vertical (R-1)-row halo is a
// register ring of R partial output rows: each input row is loaded once per STRIP-row strip
// and scattered into the R output rows it feeds (input-stationary).  Strips overlap by R-1
// input rows (served from the Infinity Cache).  Input rows are loaded PD rows ahead of the
// one being consumed.
#pragma once

#include "fir_common.h"

namespace fir {

template <int R, int C>
struct Taps2 {
    int32_t h[R][C];
    // DOT2 form: pair p of row m = (h[m][C-1-2p], h[m][C-2-2p]) as two int16 (0 past the row)
    uint32_t p2[R][(C + 1) / 2];
    // SEP form (h[m][n] == col[m] * row[n] exactly): packed row taps, column taps
    uint32_t rowp[(C + 1) / 2];
    int32_t col[R];
    // SEP16 form: column taps packed in pairs (col[2p], col[2p+1]) for v_dot2 over row-sum pairs
    uint32_t colp[(R + 1) / 2];
    // PK16 form (h = 2^s * colq[m] * rowq[n]): every tap replicated into both 16-bit halves,
    // rowb[i] = rowq[C-1-i] (multiplies window pixel j+i of output j), colb[m] = colq[m];
    // pkbias = 2^(f-1-s) and pkshift = f-s in both halves, pkmax = 255 in both halves
    uint32_t rowb[C];
    uint32_t colb[R];
    uint32_t pkbias, pkshift, pkmax;
    // PK16 general form (any kernel, kMode2dDot2 | kMode2dPk16): pkh[m][i] = hq[m][C-1-i] / 2^s
    // replicated into both halves (multiplies window pixel j+i of output j)
    uint32_t pkh[R][C];
};

// 2-D kernel arithmetic: general 5x5 on v_mad_i32_i24 / packed v_dot2, or rank-1 separable
// (a horizontal dot2 pass per input row, then R column MACs on the row sums).
// MODE = arithmetic (low 2 bits) | kMode2dNoWrap: the host proved |acc| + 2^(f-1) can never
// reach the wrap limit, so every accumulator starts at the rounding bias 2^(f-1) and the
// epilogue is one arithmetic shift (exactly fir_1d_fixed_ref.py:110-120 when no wrap occurs).
// kMode2dSep16 (with kMode2dSep): the row sums fit int16 (255 * sum|row| <= 32767, host-checked),
// so two consecutive rows' sums pack into one dword and the column pass is (R+1)/2 v_dot2 per
// output pixel instead of R v_mad_i32_i24.
// kMode2dPk16 (with kMode2dSep, u8 stage): the host proved that the final sum
// V = 2^(f-1-s) + sum colq*rowq*x of every pixel lies in [0, 2^16) (unsigned) or, with
// kMode2dPkSigned, in [-2^15, 2^15).  Both passes then run on packed 16-bit v_pk_mad_u16 over
// pixel PAIRS, exact mod 2^16 (so intermediate row sums may wrap), and the u8 stage is
// (V >> (f-s)) clamped to [0, 255] = sat((2^s V_true + 2^(f-1)) >> f), the reference's value.
// kMode2dPkHi8: unsigned with f-s == 8, the output byte is V's high byte (one v_perm per 4 px).
// kMode2dPk16 with kMode2dDot2 (any kernel, not only rank-1): the same 16-bit argument over the
// full R x C taps, R*C v_pk_mad_u16 per pixel PAIR (12.5 per pixel for 5x5 instead of 15 v_dot2).
enum Fir2dMode : int {
    kMode2dMad = 0,
    kMode2dDot2 = 1,
    kMode2dSep = 2,
    kMode2dNoWrap = 4,
    kMode2dSep16 = 8,
    kMode2dPk16 = 16,
    kMode2dPkSigned = 32,
    kMode2dPkHi8 = 64,
};

template <int R, int C>
inline void pack_taps2(Taps2<R, C>& t) {
    for (int m = 0; m < R; ++m)
        for (int p = 0; p < (C + 1) / 2; ++p) {
            const int lo = t.h[m][C - 1 - 2 * p];
            const int hi = (C - 2 - 2 * p) >= 0 ? t.h[m][C - 2 - 2 * p] : 0;
            t.p2[m][p] = ((uint32_t)lo & 0xFFFFu) | ((uint32_t)hi << 16);
        }
}

// PK16 planning (host): given an exact factorisation h[m][n] == col[m] * row[n], move the
// largest power of two 2^s (s <= frac - 1) common to all taps into the shift, check that the
// final 16-bit sum V cannot leave [0, 2^16) (or [-2^15, 2^15) signed) for any u8 input, and
// fill the PK16 tap fields.  Returns the extra mode bits (kMode2dPk16 | ...) or 0 if unusable.
template <int R, int C>
inline int plan_pk16(Taps2<R, C>& t, const int32_t* col, const int32_t* row, int frac) {
    if (frac < 1 || frac > 22) return 0;
    auto tz = [](int64_t v) {
        int z = 0;
        while (v != 0 && (v & 1) == 0 && z < 40) v >>= 1, ++z;
        return v == 0 ? 40 : z;
    };
    int zc = 40, zr = 40;
    for (int m = 0; m < R; ++m) zc = zc < tz(col[m]) ? zc : tz(col[m]);
    for (int n = 0; n < C; ++n) zr = zr < tz(row[n]) ? zr : tz(row[n]);
    if (zc >= 40 || zr >= 40) return 0;  // an all-zero factor: leave it to the other paths
    int s = zc + zr < frac - 1 ? zc + zr : frac - 1;
    const int sc = s < zc ? s : zc, sr = s - sc;
    int64_t cq[R], rq[C], vmax = (int64_t)1 << (frac - 1 - s), vmin = vmax;
    for (int m = 0; m < R; ++m) cq[m] = (int64_t)col[m] >> sc;
    for (int n = 0; n < C; ++n) rq[n] = (int64_t)row[n] >> sr;
    for (int m = 0; m < R; ++m)
        for (int n = 0; n < C; ++n) {
            const int64_t p = cq[m] * rq[n];
            (p > 0 ? vmax : vmin) += 255 * p;
        }
    if (frac - s > 15) return 0;  // 16-bit shifts take the amount mod 16
    int mode;
    if (vmin >= 0 && vmax <= 65535)
        mode = kMode2dPk16 | (frac - s == 8 ? kMode2dPkHi8 : 0);
    else if (vmin >= -32768 && vmax <= 32767)
        mode = kMode2dPk16 | kMode2dPkSigned;
    else
        return 0;
    auto rep = [](int64_t v) { return ((uint32_t)v & 0xFFFFu) * 0x10001u; };
    for (int i = 0; i < C; ++i) t.rowb[i] = rep(rq[C - 1 - i]);
    for (int m = 0; m < R; ++m) t.colb[m] = rep(cq[m]);
    t.pkbias = rep((int64_t)1 << (frac - 1 - s));
    t.pkshift = rep(frac - s);
    t.pkmax = rep(255);
    return mode;
}

// PK16 planning for a general (not necessarily rank-1) kernel: the same power-of-two
// factoring and 16-bit range proof over all R*C taps.  Returns the extra mode bits or 0.
template <int R, int C>
inline int plan_pk16_gen(Taps2<R, C>& t, const int32_t* hq, int frac) {
    if (frac < 1 || frac > 22) return 0;
    int z = 40;
    for (int k = 0; k < R * C; ++k) {
        int64_t v = hq[k];
        int zk = 0;
        while (v != 0 && (v & 1) == 0 && zk < 40) v >>= 1, ++zk;
        if (v != 0 && zk < z) z = zk;
    }
    if (z >= 40) return 0;  // all-zero kernel: the other paths handle it
    const int s = z < frac - 1 ? z : frac - 1;
    if (frac - s > 15) return 0;  // 16-bit shifts take the amount mod 16
    int64_t vmax = (int64_t)1 << (frac - 1 - s), vmin = vmax;
    for (int k = 0; k < R * C; ++k) {
        const int64_t p = (int64_t)hq[k] >> s;
        (p > 0 ? vmax : vmin) += 255 * p;
    }
    int mode;
    if (vmin >= 0 && vmax <= 65535)
        mode = kMode2dPk16 | (frac - s == 8 ? kMode2dPkHi8 : 0);
    else if (vmin >= -32768 && vmax <= 32767)
        mode = kMode2dPk16 | kMode2dPkSigned;
    else
        return 0;
    auto rep = [](int64_t v) { return ((uint32_t)v & 0xFFFFu) * 0x10001u; };
    for (int m = 0; m < R; ++m)
        for (int i = 0; i < C; ++i) t.pkh[m][i] = rep((int64_t)hq[m * C + C - 1 - i] >> s);
    t.pkbias = rep((int64_t)1 << (frac - 1 - s));
    t.pkshift = rep(frac - s);
    t.pkmax = rep(255);
    return mode;
}

// Four clamped NOWRAP accumulators (each <= 256 * 2^frac - 1) -> four u8 in one dword: the
// shift of pixels 1..3 writes straight into its byte (SDWA dst_sel, other bytes preserved).
__device__ __forceinline__ uint32_t pack4_shifted(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, int frac) {
    uint32_t d = c0 >> frac;
    asm("v_lshrrev_b32_sdwa %0, %1, %2 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD"
        : "+v"(d) : "s"(frac), "v"(c1));
    asm("v_lshrrev_b32_sdwa %0, %1, %2 dst_sel:BYTE_2 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD"
        : "+v"(d) : "s"(frac), "v"(c2));
    asm("v_lshrrev_b32_sdwa %0, %1, %2 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD"
        : "+v"(d) : "s"(frac), "v"(c3));
    return d;
}

__device__ __forceinline__ uint32_t clamp_u8_acc(uint32_t acc, int32_t sat_hi) {
    uint32_t c;
    asm("v_med3_i32 %0, %1, 0, %2" : "=v"(c) : "v"(acc), "s"(sat_hi));
    return c;
}

// Branch-free row load: the address is always in bounds (the caller clamps it) and the
// value is zeroed by a select when the row/column is outside the frame, so the compiler can
// count outstanding loads exactly (a load inside a branch makes it wait for all of them).
template <int ND, bool NT = false>
__device__ __forceinline__ void load_row_px(const uint8_t* __restrict__ p, bool ok, uint32_t (&d)[ND]) {
    typedef uint32_t vN __attribute__((ext_vector_type(ND)));
    const vN* a = reinterpret_cast<const vN*>(p);
    const vN q = NT ? __builtin_nontemporal_load(a) : *a;
#pragma unroll
    for (int i = 0; i < ND; ++i) d[i] = ok ? q[i] : 0u;
}

// NTS: non-temporal output stores.  XCD: the (strip, column, frame) order is remapped so that
// the blocks one XCD runs are consecutive strips (their R-1 overlapping rows then hit that XCD's
// L2 instead of being fetched again through another XCD's).
template <int R, int C, int STAGE, int VEC, int STRIP, int MODE, int MINW = 1, int PD = 1, bool NTL = false,
          bool NTS = false, bool XCD = false>
__global__ __launch_bounds__(kBlock, MINW) void fir2d_reg_kernel(const uint8_t* __restrict__ x,
                                                           typename OutTraits<STAGE>::T* __restrict__ y, int64_t H,
                                                           int64_t W, Taps2<R, C> taps, int shl, int frac) {
    using OutT = typename OutTraits<STAGE>::T;
    int64_t bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
    if constexpr (XCD) {  // dispatch order is x fastest, then y, then z; blocks b, b+8, ... share an XCD
        const int64_t gx = gridDim.x, gy = gridDim.y, nb = gx * gy * gridDim.z;
        const int64_t b = bx + gx * (by + gy * bz), q = nb / 8;
        const int64_t p = b < q * 8 ? (b % 8) * q + b / 8 : b;
        bx = p % gx;
        by = (p / gx) % gy;
        bz = p / (gx * gy);
    }
    {  // gridDim.z frames of H x W stored back to back (one launch for a batch of frames)
        const int64_t fo = bz * H * W;
        x += fo;
        y += fo;
    }
    constexpr int ND = VEC / 4;  // dwords per lane per row
    constexpr int CC = C / 2;
    constexpr int HLE = C - 1 - CC, HRE = CC;  // horizontal halo
    constexpr int TOP = R - 1 - R / 2;         // input rows above an output row
    static_assert(HLE <= 4 && HRE <= 4, "horizontal halo must fit in one dword");
    constexpr int T = STRIP + R - 1;  // input rows per strip (the strip loop is fully unrolled)

    const int lane = threadIdx.x & (kWave - 1);
    const int64_t v = bx * kBlock + threadIdx.x;  // vector column index
    const int64_t col0 = v * VEC;
    const bool active = col0 < W;
    const int64_t colc = active ? col0 : W - VEC;  // in-bounds column for idle lanes
    const int64_t r0 = by * STRIP;
    // halo dword: lane 0 reads the 4 pixels left of its vector, lane 63 the 4 right of it;
    // every other lane re-reads its own first dword (same cache line, value unused)
    const int64_t hraw = lane == 0 ? col0 - 4 : (lane == kWave - 1 ? col0 + VEC : col0);
    const bool hlane = (lane == 0 && HLE > 0) || (lane == kWave - 1 && HRE > 0);
    const bool hin = hraw >= 0 && hraw < W;
    const int64_t hcol = hin ? hraw : colc;
    const bool hok = hlane && hin;

    constexpr bool NOWRAP = (MODE & kMode2dNoWrap) != 0;
    const int32_t sat_hi = (256 << frac) - 1;  // NOWRAP u8: clamp before the shift (frac <= 22)
    const uint32_t acc0 = NOWRAP ? (1u << (frac - 1)) : 0u;  // rounding bias folded into the init
    uint32_t acc0v;  // the same in a VGPR, for dot2_from
    asm("v_mov_b32 %0, %1" : "=v"(acc0v) : "s"(acc0));
    constexpr bool SEP16 = (MODE & 3) == kMode2dSep && (MODE & kMode2dSep16);
    uint32_t acc[R][VEC];
#pragma unroll
    for (int s = 0; s < R; ++s)
#pragma unroll
        for (int j = 0; j < VEC; ++j) acc[s][j] = acc0;
    uint32_t qr[R][VEC] = {}, rsprev[VEC] = {};  // SEP16: packed (rs_t, rs_t-1) ring and rs_t-1
    constexpr bool PK16 = (MODE & 3) == kMode2dSep && (MODE & kMode2dPk16);
    constexpr bool PKG = (MODE & 3) == kMode2dDot2 && (MODE & kMode2dPk16);  // general packed-16
    static_assert(!(PK16 || PKG) || STAGE == FIR_OUT_U8_SAT, "PK16 is a u8-stage form");
    uint32_t rs2[R][VEC / 2] = {}, pko[VEC / 2] = {};  // PK16: row-sum pair ring, output pairs
    uint32_t ag[R][VEC / 2] = {};                      // PKG: output-pair ring

    auto row_ptr = [&](int64_t row) { return x + (row < 0 ? 0 : (row >= H ? H - 1 : row)) * W; };
    // input rows of the strip: row t is loaded PD steps before it is consumed (the unrolled
    // array indices are compile-time, so only the PD + 1 live rows occupy registers)
    uint32_t rows[T][ND], hrows[T];
    auto load_row = [&](int t) {
        const int64_t row = r0 - TOP + t;
        const bool rok = row >= 0 && row < H;
        const uint8_t* rp = row_ptr(row);
        load_row_px<ND, NTL>(rp + colc, rok && active, rows[t]);
        const uint32_t hv = *reinterpret_cast<const uint32_t*>(rp + hcol);
        hrows[t] = (hok && rok) ? hv : 0u;
    };
#pragma unroll
    for (int t = 0; t < PD && t < T; ++t) load_row(t);

#pragma unroll
    for (int t = 0; t < T; ++t) {
        {
            const int s = t % R;
            if (t + PD < T) load_row(t + PD);  // compile-time after the unroll
            const uint32_t* cur = rows[t];
            const uint32_t hcur = hrows[t];
            if constexpr ((MODE & 3) != kMode2dMad) {
                // byte stream: [left-halo dword | own dwords | right-halo dword]; window pixel i
                // is stream byte i + (4 - HLE).  P[k] = (w[k], w[k+1]) as int16 halves.
                uint32_t sb[ND + 2];
                sb[0] = HLE > 0 ? from_prev_lane(hcur, cur[ND - 1]) : 0u;
#pragma unroll
                for (int i = 0; i < ND; ++i) sb[1 + i] = cur[i];
                sb[ND + 1] = HRE > 0 ? from_next_lane(hcur, cur[0]) : 0u;
                constexpr int NP = VEC + C - 1;  // pairs P[0 .. VEC+C-2]
                uint32_t Pr[NP + 4 - HLE];
                PairBuilder<4 - HLE, NP>::run(sb, Pr);
                const uint32_t* P = Pr + (4 - HLE);
                if constexpr (PKG) {  // input row t feeds R output rows, C pair MACs each
#pragma unroll
                    for (int m = 0; m < R; ++m) {
                        const int slot = (s + 1 + m) % R;
#pragma unroll
                        for (int q = 0; q < VEC / 2; ++q)  // m = R-1 opens the row from the bias
                            ag[slot][q] = pk_mad16(P[2 * q], taps.pkh[m][0], m == R - 1 ? taps.pkbias : ag[slot][q]);
#pragma unroll
                        for (int i = 1; i < C; ++i)
#pragma unroll
                            for (int q = 0; q < VEC / 2; ++q) ag[slot][q] = pk_mad16(P[2 * q + i], taps.pkh[m][i], ag[slot][q]);
                    }
                    // the completed row (m = 0) stays here, interleaved (see the PK16 pin below)
#pragma unroll
                    for (int q = 0; q < VEC / 2; ++q) asm volatile("" : "+v"(ag[(s + 1) % R][q]));
                } else if constexpr ((MODE & 3) == kMode2dDot2) {
#pragma unroll
                    for (int m = 0; m < R; ++m) {
                        const int slot = (s + 1 + m) % R;
#pragma unroll
                        for (int j = 0; j < VEC; ++j) {
                            // m = R-1 opens the row: its first MAC starts from the bias (acc0)
                            uint32_t a = m == R - 1 ? dot2_from(P[j], taps.p2[m][0], acc0v)
                                                    : dot2_acc(P[j], taps.p2[m][0], acc[slot][j]);
#pragma unroll
                            for (int p = 1; p < (C + 1) / 2; ++p) a = dot2_acc(P[j + 2 * p], taps.p2[m][p], a);
                            acc[slot][j] = a;
                        }
                    }
                } else if constexpr (PK16) {  // pixel pairs (j, j+1) on packed 16-bit MACs
                    // tap-outer loops: the VEC/2 independent chains interleave (a dependent
                    // v_pk_mad right after its producer costs an s_nop on gfx950)
                    uint32_t* r = rs2[t % R];
#pragma unroll
                    for (int q = 0; q < VEC / 2; ++q) r[q] = pk_mul16(P[2 * q], taps.rowb[0]);
#pragma unroll
                    for (int i = 1; i < C; ++i)
#pragma unroll
                        for (int q = 0; q < VEC / 2; ++q) r[q] = pk_mad16(P[2 * q + i], taps.rowb[i], r[q]);
                    if (t >= R - 1) {  // output t-(R-1) = bias + sum_m colq[m] rs_{t-m}
#pragma unroll
                        for (int q = 0; q < VEC / 2; ++q) pko[q] = pk_mad16(r[q], taps.colb[0], taps.pkbias);
#pragma unroll
                        for (int m = 1; m < R; ++m)
#pragma unroll
                            for (int q = 0; q < VEC / 2; ++q) pko[q] = pk_mad16(rs2[(t - m) % R][q], taps.colb[m], pko[q]);
                        // keep the column pass here, interleaved: sunk into the store's branch
                        // the compiler serialises its chains (an s_nop per dependent v_pk_mad)
#pragma unroll
                        for (int q = 0; q < VEC / 2; ++q) asm volatile("" : "+v"(pko[q]));
                    }
                } else if constexpr (SEP16) {  // int16 row sums packed with the previous row's
#pragma unroll
                    for (int j = 0; j < VEC; ++j) {
                        uint32_t r = dot2_from0(P[j], taps.rowp[0]);
#pragma unroll
                        for (int p = 1; p < (C + 1) / 2; ++p) r = dot2_acc(P[j + 2 * p], taps.rowp[p], r);
                        qr[t % R][j] = __builtin_amdgcn_perm(rsprev[j], r, 0x05040100u);  // (rs_t, rs_t-1)
                        rsprev[j] = r;
                    }
                    if (t >= R - 1) {  // output t-(R-1) = sum_m col[m] rs_{t-m}: (R+1)/2 dot2 per pixel
#pragma unroll
                        for (int j = 0; j < VEC; ++j) {
                            uint32_t a = dot2_from(qr[t % R][j], taps.colp[0], acc0v);
#pragma unroll
                            for (int p = 1; p < (R + 1) / 2; ++p) a = dot2_acc(qr[(t - 2 * p) % R][j], taps.colp[p], a);
                            acc[(s + 1) % R][j] = a;
                        }
                    }
                } else {  // separable: exact row sums (|r| < 2^23, host-checked), then the column taps
#pragma unroll
                    for (int j = 0; j < VEC; ++j) {
                        uint32_t r = dot2_from0(P[j], taps.rowp[0]);
#pragma unroll
                        for (int p = 1; p < (C + 1) / 2; ++p) r = dot2_acc(P[j + 2 * p], taps.rowp[p], r);
#pragma unroll
                        for (int m = 0; m < R; ++m) {
                            const int slot = (s + 1 + m) % R;
                            acc[slot][j] = mad_i24(r, taps.col[m], m == R - 1 ? acc0v : acc[slot][j]);
                        }
                    }
                }
            } else {
            int32_t w[HLE + VEC + HRE];
            if constexpr (HLE > 0) {
                const uint32_t p = from_prev_lane(hcur, cur[ND - 1]);
#pragma unroll
                for (int i = 0; i < HLE; ++i) w[i] = (int32_t)((p >> (8 * (4 - HLE + i))) & 0xFFu);
            }
#pragma unroll
            for (int j = 0; j < VEC; ++j) w[HLE + j] = (int32_t)((cur[j / 4] >> (8 * (j % 4))) & 0xFFu);
            if constexpr (HRE > 0) {
                const uint32_t nx = from_next_lane(hcur, cur[0]);
#pragma unroll
                for (int i = 0; i < HRE; ++i) w[HLE + VEC + i] = (int32_t)((nx >> (8 * i)) & 0xFFu);
            }
            // input row t feeds output rows o = t - (R-1) + m, ring slot (s + 1 + m) % R
#pragma unroll
            for (int m = 0; m < R; ++m) {
                const int slot = (s + 1 + m) % R;
#pragma unroll
                for (int j = 0; j < VEC; ++j) {
                    uint32_t a = m == R - 1 ? acc0 : acc[slot][j];
#pragma unroll
                    for (int n = 0; n < C; ++n) a += (uint32_t)__mul24(taps.h[m][n], w[HLE + j + CC - n]);
                    acc[slot][j] = a;
                }
            }
            }
            {  // output row o = t - (R-1) is complete in slot (s + 1) % R
                const int slot = (s + 1) % R;
                const int o = t - (R - 1);
                const int64_t orow = r0 + o;
                if (o >= 0 && active && orow < H) {
                    OutT* dst = y + orow * W + col0;
                    if constexpr (STAGE == FIR_OUT_U8_SAT) {
                        typedef uint32_t vN __attribute__((ext_vector_type(ND)));
                        vN val;
                        auto po = [&](int k) -> uint32_t {
                            if constexpr (PKG) return ag[slot][k];
                            else return pko[k];
                        };
#pragma unroll
                        for (int i = 0; i < ND; ++i) {
                            if constexpr (PK16 || PKG) {  // pairs (4i, 4i+1), (4i+2, 4i+3) -> 4 bytes
                                if constexpr ((MODE & kMode2dPkHi8) != 0) {
                                    val[i] = __builtin_amdgcn_perm(po(2 * i + 1), po(2 * i), 0x07050301u);
                                } else {
                                    constexpr bool SG = (MODE & kMode2dPkSigned) != 0;
                                    const uint32_t lo = pk_stage_u8<SG>(po(2 * i), taps.pkshift, taps.pkmax);
                                    const uint32_t hi = pk_stage_u8<SG>(po(2 * i + 1), taps.pkshift, taps.pkmax);
                                    val[i] = __builtin_amdgcn_perm(hi, lo, 0x06040200u);
                                }
                            } else if constexpr (NOWRAP) {
                                const uint32_t* a4 = &acc[slot][4 * i];
                                val[i] = pack4_shifted(clamp_u8_acc(a4[0], sat_hi), clamp_u8_acc(a4[1], sat_hi),
                                                       clamp_u8_acc(a4[2], sat_hi), clamp_u8_acc(a4[3], sat_hi), frac);
                            } else {
                                uint32_t o4 = 0;
#pragma unroll
                                for (int b = 0; b < 4; ++b)
                                    o4 |= sat_u8_pixel<NOWRAP>(acc[slot][4 * i + b], shl, frac, sat_hi) << (8 * b);
                                val[i] = o4;
                            }
                        }
                        if constexpr (NTS) __builtin_nontemporal_store(val, reinterpret_cast<vN*>(dst));
                        else *reinterpret_cast<vN*>(dst) = val;
                    } else {
                        typedef uint32_t v4 __attribute__((ext_vector_type(4)));
#pragma unroll
                        for (int i = 0; i < VEC / 4; ++i) {
                            v4 val;
#pragma unroll
                            for (int b = 0; b < 4; ++b) val[b] = (uint32_t)(NOWRAP ? (int32_t)acc[slot][4 * i + b] >> frac : round32(acc[slot][4 * i + b], shl, frac));
                            if constexpr (NTS) __builtin_nontemporal_store(val, reinterpret_cast<v4*>(dst) + i);
                            else reinterpret_cast<v4*>(dst)[i] = val;
                        }
                    }
                }
            }
        }
    }
}

template <int VEC, int STRIP>
inline dim3 fir2d_reg_grid(int64_t H, int64_t W, int64_t frames = 1) {
    const int64_t vecs = W / VEC;
    return dim3((unsigned)((vecs + kBlock - 1) / kBlock), (unsigned)((H + STRIP - 1) / STRIP), (unsigned)frames);
}

}  // namespace fir
