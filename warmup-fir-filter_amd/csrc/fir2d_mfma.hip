// fir2d_mfma.hip — the 2-D fixed-point FIR on the int8 matrix cores.
//
// y[i,j] = sat_u8(round(wrap(sum_m sum_n hq[m][n] * x[i - m + R/2][j - n + C/2]))), zero padded:
// the 2-D extension of fir_1d/model/python/fir_1d_fixed_ref.py:95-126 (reference root).
//
// Why MFMA: the v_pk_mad_u16 register kernel (fir2d_reg.h) needs R*C/2 VALU MACs per pixel for
// a kernel that is not rank-1 (12.5 per pixel for 5x5: 34 us per 8192^2 frame, 49 % of the HBM
// peak).  Each input row's contribution to an output row is a 1-D Toeplitz product, so a wave
// owning the output row segment y[i][j0 .. j0 + 1023] computes, with n = 32-pixel block and
// r = offset in the block,
//     Y[r][n] = sum_m ( A_m[r][k] B_rho[k][n]  (k < 32)  +  tail ),   rho = i - m + R/2,
//     A_m[r][k] = h[m][r + C/2 - k],   B_rho[k][n] = x[rho][j0 + 32 n + k],
// one v_mfma_i32_32x32x32_i8 per (input row, output row) over the block's own 32 pixels, plus ONE
// tail MFMA per output row for the <= 2 + 2 halo pixels of every block of all R input rows
// (k = 32 + 4 m'' + t: pixels 32n-2, 32n-1, 32n+32, 32n+33 of input row i - U + m'').
//
// The operands need no LDS: lane (n, h) of a B fragment holds bytes 16h..16h+15 of block n,
// which is exactly the 16-byte vector that lane loads when a wave loads a 1 KiB row segment
// with lane (n, h) at byte 32n + 16h (the addresses are permuted, the instruction is still one
// contiguous 1 KiB).  Input rows sit in a register ring (input-stationary: each row is loaded
// once per strip and feeds R output rows); the halo bytes of a block come from the neighbouring
// blocks' lanes by two ds_bpermute per row (the tile's outer halo from one edge-dword load).
// Exactness: u8 samples enter as signed bytes xs = x - 128 (x ^ 0x80; zero padding is x = 0
// like any other sample), taps h = 2^s h' with h' a signed byte (NP = 1) or a balanced byte pair
// h' = 256 hh + hl (NP = 2); sum h x = 2^s (sum h' xs + 128 sum h') exactly in int32 (mod 2^32:
// the reference's wrap bit for bit).  Outputs: the 16 accumulators of a lane are bytes
// 32n + 8g + 4h + 0..3; two v_permlane32_swap give every lane 16 contiguous output bytes, so each
// output row leaves as one 1 KiB store instruction (non-temporal).
#include <cstdlib>
#include <atomic>
#include <string>

#include "fir_common.h"
#include "fir_launch.h"

namespace fir {

constexpr int kM2Tile = 1024;   // output pixels per wave and row (32 blocks of 32)
constexpr int kM2MaxR = 7;
constexpr int kM2MaxC = 5;      // horizontal halo <= 2 pixels per side
constexpr int kM2MinWaves = 3;  // waves per SIMD the one-plane kernel's registers must allow
// Register-ring rows (R in use + 8 - R in flight).  With strips sized to one resident round an
// 8-row ring (8-row strip granularity: 3008 waves for 3072 slots at 8192^2 x 4) beats the 7-row
// ring (14-row granularity: 2688 waves): general 5x5 88.0 -> 87.4 us, two byte planes 109.0 ->
// 105.1 us per 4-frame launch; deeper rings are slower (16 rows: 110-165 us)
// (profiles/r02/ab2d_mfma_ring_*.txt).  The strip length is chosen at launch (m2_rows_per_strip).
template <int R>
struct M2Geom {
    static constexpr int RING = 8;
};

// Tap bytes by diagonal: tm[p][m][33 - d] = byte p of h'[m][C/2 + d] (0 outside the row), d = r - k
// of A_m[r][k] in [-33, 33]: the main k-steps use d in [-31, 31], the tail d = r + 2, r + 1,
// r - 32, r - 33 (pixels -2, -1, 32, 33 of a block).
struct Mfma2Taps {
    int8_t tm[2][kM2MaxR][72];
};

typedef int m2_i32x4 __attribute__((ext_vector_type(4)));
typedef int m2_i32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t m2_u4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t m2_rsrc(const void* p, uint32_t bytes) {
    const uint64_t a = (uint64_t)(uintptr_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    void* q = (void*)(uintptr_t)(((uint64_t)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(q, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}
constexpr int kM2AuxNt = 2;                // non-temporal cache policy (gfx950)
constexpr uint32_t kM2Off = 0x80000000u;   // a voffset outside every descriptor: loads 0, stores dropped

// R: tap rows; NP: tap byte planes (1 or 2); FAST: host-proven no wrap, f <= 16 and
// (255 sum|h| + 2^(f-1)) 2^(16-f) < 2^31, so bits 16..31 of (sum + 2^(f-1)) << (16 - f) are the
// rounded output as an int16, saturated to u8 by v_sat_pk_u8_i16.
template <int R, int NP, bool FAST, bool ACC32>
__global__ __launch_bounds__(kBlock, NP == 1 ? kM2MinWaves : 2) void fir2d_mfma_kernel(
    const uint8_t* __restrict__ x, uint8_t* __restrict__ y, int64_t H, int64_t W, uint32_t ncol, uint32_t nstrip,
    uint32_t nwaves, int rows_per_strip, Mfma2Taps taps, uint32_t bias, int sh, int shl, int frac) {
    constexpr int U = R - 1 - R / 2;  // input rows above an output row
    constexpr int D = R / 2;          // and below
    constexpr int kM2Ring = M2Geom<R>::RING;
    const int kM2Strip = rows_per_strip;  // a multiple of UN (host)
    constexpr int PD = kM2Ring - R;   // rows in flight ahead of the newest one in use
    static_assert(PD >= 1, "ring too small");
    static_assert(R >= 3, "the stage of row i - 1 is spread over the R + 1 >= 4 MFMAs of row i");

    const int lane = threadIdx.x & (kWave - 1);
    const int n = lane & 31, hf = lane >> 5;
    // blocks b, b + 8, ... run on one XCD: give each XCD a contiguous range of waves, so the
    // R - 1 rows two vertically adjacent strips share are fetched by the same L2
    uint32_t b = blockIdx.x;
    {
        const uint32_t nb = gridDim.x, q = nb / 8;
        b = b < q * 8 ? (b % 8) * q + b / 8 : b;
    }
    // wave-uniform (readfirstlane): strip, column and frame then live in SGPRs and the row
    // addressing below is scalar
    const uint32_t w = __builtin_amdgcn_readfirstlane(b * (kBlock / kWave) + (threadIdx.x >> 6));
    if (w >= nwaves) return;  // wave-uniform
    // column tiles fastest: the 4 waves of a block read 4 KiB contiguous of each row (strips fastest,
    // each wave a different DRAM page: 99 vs 87.3 us per 4 frames, profiles/r02/ab2d_mfma_colfast.txt)
    const uint32_t col = w % ncol, strip = (w / ncol) % nstrip, frame = w / (nstrip * ncol);
    const int64_t fo = (int64_t)frame * H * W;
    const uint8_t* xf = x + fo;
    uint8_t* yf = y + fo;
    const int64_t j0 = (int64_t)col * kM2Tile;
    const int64_t i0 = (int64_t)strip * kM2Strip;
    const uint32_t wb = (uint32_t)W;  // W < 2^31 (host-checked)
    // Walk direction: odd strips walk UP, so two vertically adjacent strips read the R - 1 rows
    // they share at the same moment (both at their start or both at their end) and the second
    // read hits L2 (fir2d_pk16.h measured it on the separable kernel).  Walk step q handles output
    // row orow0 + dir q; walk row s of the ring is input row wrow0 + dir s; the window position mm
    // (oldest first) multiplies tap row tap_row(mm).
    const bool up = (strip & 1) != 0;
    const int64_t dir = up ? -1 : 1;
    const int64_t orow0 = up ? i0 + kM2Strip - 1 : i0;
    const int64_t wrow0 = up ? i0 + kM2Strip - 1 + D : i0 - U;
    auto tap_row = [&](int mm) __attribute__((always_inline)) { return up ? mm : R - 1 - mm; };

    // ---- tap fragments by window position (am[p][mm] = tap row tap_row(mm)): A_m[r = n][k = 16 hf + j]
    // (main) and A_tail[r][32 + 16 hf + j]
    m2_i32x4 am[NP][R], at[NP];
#pragma unroll
    for (int p = 0; p < NP; ++p) {
#pragma unroll
        for (int m = 0; m < R; ++m) {
            uint32_t v[4] = {0u, 0u, 0u, 0u};
#pragma unroll
            for (int j = 0; j < 16; ++j) v[j / 4] |= (uint32_t)(uint8_t)taps.tm[p][tap_row(m)][33 - (n - 16 * hf - j)] << (8 * (j % 4));
            am[p][m] = m2_i32x4{(int)v[0], (int)v[1], (int)v[2], (int)v[3]};
        }
        uint32_t v[4] = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int mm = 4 * hf + j / 4, t = j % 4;  // tail window position m'', pixel
            const int kc = t == 0 ? -2 : (t == 1 ? -1 : 30 + t);
            const uint32_t tb = mm < R ? (uint32_t)(uint8_t)taps.tm[p][tap_row(mm < R ? mm : 0)][33 - (n - kc)] : 0u;
            v[j / 4] |= tb << (8 * (j % 4));
        }
        at[p] = m2_i32x4{(int)v[0], (int)v[1], (int)v[2], (int)v[3]};
    }

    // ---- the register ring: raw 16-byte vector and edge dword of each input row in flight
    m2_u4 ring[kM2Ring];
    uint32_t edge[kM2Ring], tl[kM2Ring];
    const uint32_t voff = (uint32_t)j0 + 32u * n + 16u * hf;
    // edge dword: lane 63 (never a left-halo source) the 4 pixels left of the tile, lane 0
    // (never a right-halo source) the 4 right of it
    const uint32_t eoff = lane == 63 ? (j0 >= 4 ? (uint32_t)j0 - 4u : kM2Off) : (lane == 0 ? (uint32_t)j0 + kM2Tile : kM2Off);
    // rows outside the frame: a descriptor of 0 bytes (every load of it returns 0)
    auto load_row = [&](int64_t rho, int slot) __attribute__((always_inline)) {
        const bool in = rho >= 0 && rho < H;
        const __amdgpu_buffer_rsrc_t rs = m2_rsrc(xf + (in ? rho : 0) * W, in ? wb : 0u);
        ring[slot] = __builtin_bit_cast(m2_u4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, 0, 0));
        edge[slot] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rs, eoff, 0, 0);
    };
    // signed bytes and the halo dword [x(32n-2), x(32n-1), x(32n+32), x(32n+33)] of block n
    const int srcl = 4 * (32 + ((n + 31) & 31)), srcr = 4 * ((n + 1) & 31);
    auto prep_row = [&](int slot) __attribute__((always_inline)) {
        m2_u4 v = ring[slot] ^ 0x80808080u;
        ring[slot] = v;
        const uint32_t e = edge[slot] ^ 0x80808080u;
        const uint32_t d3 = lane == 63 ? e : v.w, d0 = lane == 0 ? e : v.x;
        const uint32_t l = (uint32_t)__builtin_amdgcn_ds_bpermute(srcl, (int)d3);
        const uint32_t r = (uint32_t)__builtin_amdgcn_ds_bpermute(srcr, (int)d0);
        tl[slot] = __builtin_amdgcn_perm(r, l, 0x05040302u);  // l.b2, l.b3, r.b0, r.b1
    };

    // walk rows 0 .. RING - 2 into slots 0 .. RING - 2; slot(walk row s) = s % RING
#pragma unroll
    for (int s = 0; s < kM2Ring - 1; ++s) load_row(wrow0 + dir * s, s);
#pragma unroll
    for (int s = 0; s < R - 1; ++s) prep_row(s);

    const uint32_t hmask = hf ? 0xFFFFFFFFu : 0u;
    uint32_t shv;  // the shift in a VGPR (gfx9 VOP3: one SGPR operand per instruction)
    asm("v_mov_b32 %0, %1" : "=v"(shv) : "s"(sh));

    // ---- stage of one output row, 4 of its 16 outputs (group gi): register e of lane (n, hf) is
    // output pixel 32n + (e & 3) + 8 (e >> 2) + 4 hf; the byte ends up in bits 16..23
    auto stage4 = [&](const m2_i32x16& acc, const m2_i32x16& acch, int gi) __attribute__((always_inline)) {
        uint32_t c[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int e = 4 * gi + q;
            uint32_t a = (uint32_t)acc[e];
            if constexpr (NP == 2) a += (uint32_t)acch[e] << 8;
            if constexpr (FAST) {
                // (sum + 2^(f-1)) << (16 - f): the rounded output as an int16 in bits 16..31.
                // Plain C for the first use of the MFMA result (v_add_lshl_u32, the shift in a
                // VGPR): hipcc does not pad inline asm that reads an MFMA destination with the
                // wait states it needs (measured: wrong bytes 0, 1 of every block)
                c[q] = (a + bias) << shv;
            } else {
                c[q] = (uint32_t)min(max(round_acc<ACC32>((a + bias) << sh, shl, frac), 0), 255) << 16;
            }
        }
        if constexpr (FAST) {  // two int16 outputs per dword, saturated to u8 pairs by v_sat_pk_u8_i16
            uint32_t s01, s23;
            asm("v_sat_pk_u8_i16 %0, %1" : "=v"(s01) : "v"(__builtin_amdgcn_perm(c[1], c[0], 0x07060302u)));
            asm("v_sat_pk_u8_i16 %0, %1" : "=v"(s23) : "v"(__builtin_amdgcn_perm(c[3], c[2], 0x07060302u)));
            return s01 | (s23 << 16);
        } else {
            const uint32_t lo = __builtin_amdgcn_perm(c[1], c[0], 0x0C0C0602u);  // c0.b2, c1.b2
            const uint32_t hi = __builtin_amdgcn_perm(c[3], c[2], 0x06020C0Cu);  // c2.b2, c3.b2 in bytes 2, 3
            return lo | hi;
        }
    };
    // lane n: bytes 32n + 0..15, lane n + 32: bytes 32n + 16..31 (two v_permlane32_swap), then
    // through 1 KiB of wave-private LDS so that lane L stores bytes
    // 16L..16L+15: each 16-lane pass of the store then writes 256 contiguous bytes, whole lines,
    // instead of every other 16 bytes of 512.  One non-temporal store, dropped when the row is
    // outside the strip or the frame.
    __shared__ __attribute__((aligned(16))) uint8_t obuf[kBlock / kWave][kM2Tile];
    uint8_t* ob = obuf[threadIdx.x >> 6];
    const uint32_t soff = (uint32_t)j0 + 16u * lane;
    auto store_row = [&](const uint32_t* g, int64_t i, bool ok) __attribute__((always_inline)) {
        const auto s02 = __builtin_amdgcn_permlane32_swap(g[0], g[2], false, false);
        const auto s13 = __builtin_amdgcn_permlane32_swap(g[1], g[3], false, false);
        m2_u4 v = m2_u4{s02[0], s02[1], s13[0], s13[1]};
        *reinterpret_cast<m2_u4*>(ob + 32 * n + 16 * hf) = v;
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");
        v = *reinterpret_cast<const m2_u4*>(ob + 16 * lane);
        __builtin_amdgcn_wave_barrier();  // the read is done before the next row's write
        asm volatile("" ::: "memory");
        const bool in = ok && i < H;
        const __amdgpu_buffer_rsrc_t rs = m2_rsrc(yf + (in ? i : 0) * W, in ? wb : 0u);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(m2_i32x4, v), rs, soff, 0, kM2AuxNt);
    };

    // Software-pipelined by one row: iteration i issues the MFMAs of output row i into one
    // accumulator pair and, between them, stages row i - 1 out of the other, so the matrix
    // core and the VALU work at the same time inside a wave.
    m2_i32x16 acc[2] = {}, acch[2] = {};
    // unrolled over a whole number of ring turns with an even number of rows, so that both the
    // ring slot and the accumulator parity of every row are compile-time
    constexpr int UN = (kM2Ring & 1) ? 2 * kM2Ring : kM2Ring;
    static_assert(UN % 2 == 0, "rows per unrolled turn must be even (accumulator parity)");
    for (int64_t iq = 0; iq < kM2Strip; iq += UN) {
#pragma unroll
        for (int kk = 0; kk < UN; ++kk) {
            const int k = kk % kM2Ring;  // ring position
            const int64_t q = iq + kk;   // walk step: output row orow0 + dir q
            // keep each iteration's instructions in place: hipcc otherwise hoists a row's signed-
            // byte XOR up to its load, several iterations early, and waits for that load there
            __builtin_amdgcn_sched_barrier(0);
            prep_row((k + R - 1) % kM2Ring);                              // walk row q + R - 1 has arrived
            load_row(wrow0 + dir * (q + R - 1 + PD), (k + R - 1 + PD) % kM2Ring);  // slot of walk row q - 1

            m2_i32x16& a = acc[kk & 1];
            m2_i32x16& ah = acch[kk & 1];
            const m2_i32x16& pa = acc[(kk + 1) & 1];
            const m2_i32x16& pah = acch[(kk + 1) & 1];
            uint32_t g[4];
#pragma unroll
            for (int mm = 0; mm < R + 1; ++mm) {
                m2_i32x4 bv, av0, av1;
                if (mm < R) {  // walk row q + mm, tap row tap_row(mm)
                    bv = __builtin_bit_cast(m2_i32x4, ring[(k + mm) % kM2Ring]);
                    av0 = am[0][mm < R ? mm : 0];
                    if constexpr (NP == 2) av1 = am[1][mm < R ? mm : 0];
                } else {  // the tail: halo dwords of walk rows q + e (lanes h = 0), q + 4 + e (h = 1)
                    uint32_t tv[4];
#pragma unroll
                    for (int e = 0; e < 4; ++e) {  // a bit-select, not a select of array elements
                        // (hipcc turns that into a dynamically indexed array in LDS)
                        const uint32_t lo = tl[(k + e) % kM2Ring], hi = tl[(k + 4 + e) % kM2Ring];
                        tv[e] = (hi & hmask) | (lo & ~hmask);
                    }
                    bv = m2_i32x4{(int)tv[0], (int)tv[1], (int)tv[2], (int)tv[3]};
                    av0 = at[0];
                    if constexpr (NP == 2) av1 = at[1];
                }
                a = __builtin_amdgcn_mfma_i32_32x32x32_i8(av0, bv, mm ? a : m2_i32x16{}, 0, 0, 0);
                if constexpr (NP == 2) ah = __builtin_amdgcn_mfma_i32_32x32x32_i8(av1, bv, mm ? ah : m2_i32x16{}, 0, 0, 0);
                if (mm < 4) g[mm] = stage4(pa, pah, mm);  // row i - 1, between the MFMAs
            }
            store_row(g, orow0 + dir * (q - 1), q > 0);
        }
    }
    {  // the strip's last row
        constexpr int kl = UN - 1;  // the strip's last row: (strip - 1) % UN
        uint32_t g[4];
#pragma unroll
        for (int gi = 0; gi < 4; ++gi) g[gi] = stage4(acc[kl & 1], acch[kl & 1], gi);
        store_row(g, orow0 + dir * (kM2Strip - 1), true);
    }
}

// Output rows per wave: 32 for one tap plane (alternating walks, below); otherwise the strips are
// sized so that the launch is ONE round of resident waves (occupancy x CUs x 4), which removes the
// partial last round of fixed strips.
template <int R, int NP, bool FAST, bool ACC32>
static int m2_rows_per_strip(int64_t frames, int64_t ncol, int64_t H, hipStream_t s) {
    constexpr int UN = (M2Geom<R>::RING & 1) ? 2 * M2Geom<R>::RING : M2Geom<R>::RING;
    int64_t rows;
    if (NP == 1) {
        // one tap plane with alternating walks: short strips keep neighbours in step (their
        // shared rows then come from L2); 32 rows: the general 5x5 85.4 -> 81.2 us per 4
        // frames, while two planes stay faster with one round (108 vs 119;
        // profiles/r03/ab2d_mfma_alt_rows.txt)
        rows = 32;
    } else {
        // waves of this instantiation resident at once on the stream's device, cached per device
        // (a benign race: concurrent first calls compute the same value)
        constexpr int kMaxDev = 64;
        static std::atomic<int> resident_by_dev[kMaxDev];
        int dev = 0;
        if (hipStreamGetDevice(s, &dev) != hipSuccess && hipGetDevice(&dev) != hipSuccess) dev = 0;
        (void)hipGetLastError();
        int resident = dev >= 0 && dev < kMaxDev ? resident_by_dev[dev].load(std::memory_order_relaxed) : 0;
        if (!resident) {
            int cus = 0, nb = 0;
            if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
                hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fir2d_mfma_kernel<R, NP, FAST, ACC32>, kBlock, 0) !=
                    hipSuccess || cus <= 0 || nb <= 0) {
                (void)hipGetLastError();
                cus = 256, nb = 3;
            }
            resident = cus * nb * (kBlock / kWave);
            if (dev >= 0 && dev < kMaxDev) resident_by_dev[dev].store(resident, std::memory_order_relaxed);
        }
        const int64_t per = frames * ncol, strips = resident / per > 1 ? resident / per : 1;
        rows = (H + strips - 1) / strips;
    }
    rows = (rows + UN - 1) / UN * UN;
    const int64_t hmax = (H + UN - 1) / UN * UN;
    return (int)(rows < hmax ? rows : hmax);
}

template <int R, int NP, bool FAST, bool ACC32>
static hipError_t launch_m2v(const uint8_t* x, uint8_t* y, int64_t frames, int64_t H, int64_t W, const Mfma2Taps& t,
                             uint32_t bias, int sh, int acc_bits, int frac, hipStream_t s) {
    const int64_t ncol = (W + kM2Tile - 1) / kM2Tile;
    const int rows = m2_rows_per_strip<R, NP, FAST, ACC32>(frames, ncol, H, s);
    const int64_t nstrip = (H + rows - 1) / rows, nw = frames * ncol * nstrip;
    if (nw >= ((int64_t)1 << 31)) return hipErrorNotSupported;
    const unsigned blocks = (unsigned)((nw + (kBlock / kWave) - 1) / (kBlock / kWave));
    hipLaunchKernelGGL((fir2d_mfma_kernel<R, NP, FAST, ACC32>), dim3(blocks), dim3(kBlock), 0, s, x, y, H, W,
                       (uint32_t)ncol, (uint32_t)nstrip, (uint32_t)nw, rows, t, bias, sh, 32 - acc_bits, frac);
    return hipGetLastError();
}

template <int R, int NP>
static hipError_t launch_m2(const uint8_t* x, uint8_t* y, int64_t frames, int64_t H, int64_t W, const Mfma2Taps& t,
                            uint32_t bias, int sh, bool fast, int acc_bits, int frac, hipStream_t s) {
    if (fast) return launch_m2v<R, NP, true, true>(x, y, frames, H, W, t, bias, sh, acc_bits, frac, s);
    if (acc_bits == 32) return launch_m2v<R, NP, false, true>(x, y, frames, H, W, t, bias, sh, acc_bits, frac, s);
    return launch_m2v<R, NP, false, false>(x, y, frames, H, W, t, bias, sh, acc_bits, frac, s);
}

// Host plan: the power of two 2^s common to every tap moves into the final shift, the rest
// must be one signed byte (NP = 1) or a balanced byte pair (NP = 2).  Returns NP, 0 if unusable.
static int plan_mfma2(const int32_t* hq, int R, int C, int frac, int acc_bits, Mfma2Taps* t, uint32_t* bias, int* sh,
                      bool* fast) {
    if (R < 1 || R > kM2MaxR || C < 1 || C > kM2MaxC || frac < 1 || frac > 31 || acc_bits > 32) return 0;
    int s = 40;
    int64_t habs = 0, hsum = 0;
    for (int k = 0; k < R * C; ++k) {
        int64_t v = hq[k];
        habs += v < 0 ? -v : v;
        if (v == 0) continue;
        int z = 0;
        while ((v & 1) == 0) v >>= 1, ++z;
        s = s < z ? s : z;
    }
    if (s == 40) s = 0;  // all-zero kernel
    s = s < frac - 1 ? s : frac - 1;
    int np = 1;
    for (int k = 0; k < R * C; ++k) {
        const int64_t v = (int64_t)hq[k] >> s;
        if (v < -128 || v > 127) np = 2;
        if (v < -32768 || v > 32639) return 0;  // the high byte of the balanced split must be signed
    }
    *t = Mfma2Taps{};
    const int cc = C / 2;
    for (int p = 0; p < np; ++p)
        for (int m = 0; m < R; ++m)
            for (int idx = 0; idx < 72; ++idx) {
                const int d = 33 - idx, nn = cc + d;
                if (nn < 0 || nn >= C) continue;
                const int v = (int)((int64_t)hq[m * C + nn] >> s);
                const int lo = ((v + 128) & 255) - 128;
                t->tm[p][m][idx] = (int8_t)(np == 1 ? v : (p == 0 ? lo : (v - lo) / 256));
            }
    hsum = 0;
    for (int k = 0; k < R * C; ++k) hsum += (int64_t)hq[k] >> s;
    // no wrap: |sum| + 2^(f-1) below 2^(acc_bits-1); byte in bits 16..23 after << (16 - f + s)
    const bool nowrap = 255 * habs + ((int64_t)1 << (frac - 1)) < ((int64_t)1 << (acc_bits - 1));
    *fast = nowrap && frac <= 16 && ((255 * habs + ((int64_t)1 << (frac - 1))) << (16 - frac)) < ((int64_t)1 << 31);
    uint32_t b = (uint32_t)(128 * hsum);  // the x - 128 offset, mod 2^32
    if (*fast) {
        b += 1u << (frac - 1 - s);  // 2^(f-1) = 2^s 2^(f-1-s)
        *sh = s + 16 - frac;
    } else {
        *sh = s;
    }
    *bias = b;
    return np;
}

// The MFMA path applies to u8 -> sat-u8 frames with W % 16 == 0 (16-byte rows), 16-byte aligned
// buffers, R <= 7, C <= 5 and taps whose odd part fits a balanced byte pair.  Returns
// hipErrorNotSupported when the shape is not covered (the caller then takes the register path).
hipError_t launch_fir2d_mfma(const uint8_t* x, int64_t frames, int64_t H, int64_t W, const int32_t* hq, int R, int C,
                             int frac, int acc_bits, int stage, void* y, hipStream_t s) {
    if (stage != FIR_OUT_U8_SAT || W % 16 || W < 16 || W >= ((int64_t)1 << 31) || (uintptr_t)x % 16 ||
        (uintptr_t)y % 16 || frames < 1 || H < 1)
        return hipErrorNotSupported;
    Mfma2Taps t;
    uint32_t bias;
    int sh;
    bool fast;
    const int np = plan_mfma2(hq, R, C, frac, acc_bits, &t, &bias, &sh, &fast);
    if (!np) return hipErrorNotSupported;
    uint8_t* yy = (uint8_t*)y;
#define FIR2D_M2(r)                                                                                    \
    if (R == r)                                                                                        \
        return np == 1 ? launch_m2<r, 1>(x, yy, frames, H, W, t, bias, sh, fast, acc_bits, frac, s) \
                       : launch_m2<r, 2>(x, yy, frames, H, W, t, bias, sh, fast, acc_bits, frac, s);
    FIR2D_M2(3) FIR2D_M2(5)
#undef FIR2D_M2
    return hipErrorNotSupported;
}

}  // namespace fir
