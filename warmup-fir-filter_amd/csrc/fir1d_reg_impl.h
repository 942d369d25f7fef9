// fir1d_reg_impl.h — host launchers of fir1d_reg_kernel (the register/DPP hot kernel).
//
// The kernel has one instantiation per (sample type, stage, channels, filters, taps,
// variant); compiling them all in one translation unit took minutes, so
// fir1d_reg_inst.hip includes this file once per (InT, STAGE, CH, F) with -D macros (see
// the Makefile) and fir1d.hip only sees the declaration in fir1d_reg_launch.h.
#pragma once

#include "fir1d_reg.h"
#include "fir1d_reg_launch.h"

namespace fir {

// Hot-kernel shape chosen by the A/B microbenchmark (tools/microbench; profiles/r01/micro_*.txt;
// the chunk counts kRegU live in fir1d_reg_launch.h): one 64-vector chunk per wave
// (more chunks per wave or a persistent grid cost 3-15 %), int32 outputs staged through LDS
// into whole 1 KiB store instructions (272 -> 257 us), and those whole-row stores
// NON-TEMPORAL (257.9 -> 250.9 us, 80 % of HBM peak, micro_i16_nts.txt; non-temporal stores
// of the lane-strided layout had cost 25-45 %, non-temporal loads cost 4 %).
// One u8 filter: 4 chunks per wave (the per-wave edge loads and row arithmetic amortised over
// 4 KiB; 104.6 -> 94.0 us at 2^28, micro_u8_chunks.txt), non-temporal stores 94.7 -> 82.2 us
// (micro_u8_nts.txt).  A fused u8 bank: 1 chunk per wave with non-temporal stores (222.6 us vs
// 229.3 at 2 chunks with plain stores).
// Edge dwords (kEdgeDword): one wave-wide dword load for both tile edges instead of two
// lane-masked 16-byte loads: headline 246.6-250.6 -> 244.4-244.9 us, u8 bank 230.6 -> 224.3 us,
// one u8 filter unchanged (profiles/r02/micro_i16_edw.txt, micro_u8_edw.txt).
// A fused bank keeps the same flags: an XCD-major block order and a persistent grid measured
// slower or equal (profiles/r04/bank_ab.txt).
constexpr int kRegFlags = kCoal | kNtStore | kEdgeDword;
constexpr int kPersistBlocks = 2048;

template <typename InT>
static RowGeom make_geom(int64_t rows, int64_t total, int64_t rowlen, const void* hl, const void* hr) {
    RowGeom g;
    g.total = total;
    g.rowlen32 = (uint32_t)(rows > 1 ? rowlen : 0);
    g.multi_row = rows > 1;
    g.aligned = rows == 1 || rowlen % (4 * InTraits<InT>::kPerDword) == 0;
    g.halo_l = hl;
    g.halo_r = hr;
    return g;
}

// The kernel's tap record; false when the packed-16 plan the flags promise does not hold.
template <int L, int F, int FL>
static bool make_taps(TapsN<L, F>& t, const int32_t* hq, int frac) {
    for (int f = 0; f < F; ++f)
        for (int k = 0; k < L; ++k) t.h[f][k] = hq[f * L + k];
    pack_taps(t);
    plan_u8_noclamp(t, frac);
    if constexpr ((FL & kU8Pk16) != 0)
        if (!(plan_u8_pk16(t, frac) & kU8Pk16)) return false;  // caller checked
    return true;
}

template <typename InT, int STAGE, int L, int CH, int F, int FL>
static hipError_t launch_reg_flags(const void* x, void* y, int64_t rows, int64_t total, int64_t rowlen,
                                   const int32_t* hq, int frac, int acc_bits, hipStream_t stream, const void* hl,
                                   const void* hr) {
    using OutT = typename OutTraits<STAGE>::T;
    const RowGeom g = make_geom<InT>(rows, total, rowlen, hl, hr);
    TapsN<L, F> t;
    if (!make_taps<L, F, FL>(t, hq, frac)) return hipErrorInvalidValue;
    int64_t ntiles = 0, blocks = 0;
    reg_launch_geometry<InT, kRegU<InT, F>, FL>(total, kPersistBlocks, &ntiles, &blocks);
    // One int16 filter keeps the masked pair compiled in even where it cannot run: that code
    // layout is faster in every one of 12 interleaved pairs in one process (headline 244.98 vs
    // 246.02 us median, profiles/r06/ab_pairs_single_filter.txt).  u8 filters and banks drop it:
    // for one u8 filter the pairs tie (78.86 vs 79.01 us, 6 of 12 each way) and the kernel halves
    // (4321 -> 2037 instructions, 66 -> 62 VGPRs); a bank's VGPRs go 90 -> 39.
    constexpr int FM = F == 1 && sizeof(InT) == 2 ? kMasked : 0;
    if constexpr (F == 1) {
        if (hl != nullptr || hr != nullptr) {
            hipLaunchKernelGGL((fir1d_reg_kernel<InT, STAGE, L, CH, kRegU<InT, F>, FL | kHalo | FM, F>), dim3((unsigned)blocks),
                               dim3(kBlock), 0, stream, (const InT*)x, (OutT*)y, g, t, 32 - acc_bits, frac, ntiles);
            return hipGetLastError();
        }
    } else if (hl != nullptr || hr != nullptr) {
        return hipErrorInvalidValue;  // shards with halos are single-filter calls
    }
    if (!g.aligned) {  // rows straddle vectors: one signal with seams patched (u8 stage), else masked
        constexpr int FX = STAGE == FIR_OUT_U8_SAT && CH == 1 ? kRagged : kMasked;
        hipLaunchKernelGGL((fir1d_reg_kernel<InT, STAGE, L, CH, kRegU<InT, F>, FL | FX, F>), dim3((unsigned)blocks),
                           dim3(kBlock), 0, stream, (const InT*)x, (OutT*)y, g, t, 32 - acc_bits, frac, ntiles);
        return hipGetLastError();
    }
    hipLaunchKernelGGL((fir1d_reg_kernel<InT, STAGE, L, CH, kRegU<InT, F>, FL | FM, F>), dim3((unsigned)blocks), dim3(kBlock), 0,
                       stream, (const InT*)x, (OutT*)y, g, t, 32 - acc_bits, frac, ntiles);
    return hipGetLastError();
}

// One launch of up to kRegBatch images (u8 stage, one channel: rows that straddle vectors take
// the kRagged seam patch, whole-vector rows the plain form, decided per image in the kernel).
template <typename InT, int STAGE, int L, int CH, int F, int FL>
static hipError_t launch_reg_batch_flags(int n, const RegImage* im, const int32_t* hq, int frac, int acc_bits,
                                         hipStream_t stream) {
    if constexpr (STAGE != FIR_OUT_U8_SAT || CH != 1) {
        return hipErrorInvalidValue;
    } else {
        if (n < 1 || n > kRegBatch) return hipErrorInvalidValue;
        RegBatch b{};
        TapsN<L, F> t;
        if (!make_taps<L, F, FL>(t, hq, frac)) return hipErrorInvalidValue;
        int64_t tiles = 0;
        bool ragged = false;
        for (int i = 0; i < n; ++i) {
            const int64_t total = im[i].rows * im[i].rowlen;
            int64_t nt = 0, blocks = 0;
            reg_launch_geometry<InT, kRegU<InT, F>, FL>(total, kPersistBlocks, &nt, &blocks);
            b.x[i] = im[i].x;
            for (int f = 0; f < F; ++f) b.y[i][f] = im[i].y[f];
            b.g[i] = make_geom<InT>(im[i].rows, total, im[i].rowlen, nullptr, nullptr);
            ragged |= !b.g[i].aligned;
            b.tile0[i] = tiles;
            tiles += nt;
        }
        b.tile0[n] = tiles;
        b.n = n;
        const int64_t blocks = (tiles + kBlock / kWave - 1) / (kBlock / kWave);
        if (blocks == 0) return hipSuccess;
        if (ragged)  // an image whose rows straddle vectors: the deferred-store seam form (kDefer)
            hipLaunchKernelGGL((fir1d_reg_batch_kernel<InT, STAGE, L, CH, kRegU<InT, F>, FL | kRagged | kDefer, F>),
                               dim3((unsigned)blocks), dim3(kBlock), 0, stream, b, t, 32 - acc_bits, frac);
        else
            hipLaunchKernelGGL((fir1d_reg_batch_kernel<InT, STAGE, L, CH, kRegU<InT, F>, FL | kRagged, F>),
                               dim3((unsigned)blocks), dim3(kBlock), 0, stream, b, t, 32 - acc_bits, frac);
        return hipGetLastError();
    }
}

template <typename InT, int STAGE, int L, int CH, int F>
struct RegOne {  // one buffer (launch_reg_flags)
    const void *x;
    void* y;
    int64_t rows, total, rowlen;
    const int32_t* hq;
    int frac, acc_bits;
    hipStream_t s;
    const void *hl, *hr;
    template <int FL>
    hipError_t run() const {
        return launch_reg_flags<InT, STAGE, L, CH, F, FL>(x, y, rows, total, rowlen, hq, frac, acc_bits, s, hl, hr);
    }
};

template <typename InT, int STAGE, int L, int CH, int F>
struct RegMany {  // up to kRegBatch images (launch_reg_batch_flags)
    int n;
    const RegImage* im;
    const int32_t* hq;
    int frac, acc_bits;
    hipStream_t s;
    template <int FL>
    hipError_t run() const {
        return launch_reg_batch_flags<InT, STAGE, L, CH, F, FL>(n, im, hq, frac, acc_bits, s);
    }
};

// Picks the kernel variant: acc_bits == 32 drops the wrap shifts; int16 samples with int16
// taps (one channel) multiply on packed v_dot2_i32_i16; so do u8 samples (byte pairs) when
// no accumulator can wrap: 255 * sum|h| + 2^(f-1) < 2^(acc_bits-1) for every filter.
template <typename InT, int STAGE, int L, int CH, int F, typename Go>
static hipError_t launch_reg(const Go& go, const int32_t* hq, int frac, int acc_bits) {
    bool taps16 = true;
    for (int k = 0; k < F * L; ++k) taps16 &= hq[k] >= -32768 && hq[k] <= 32767;
    const bool acc32 = acc_bits == 32;
    if constexpr (sizeof(InT) == 1 && CH == 1) {
        bool nowrap = frac <= 22;
        for (int f = 0; f < F; ++f) {
            int64_t habs = 0;
            for (int k = 0; k < L; ++k) habs += hq[f * L + k] < 0 ? -(int64_t)hq[f * L + k] : hq[f * L + k];
            nowrap &= 255 * habs + ((int64_t)1 << (frac - 1)) < ((int64_t)1 << (acc_bits - 1));
        }
        if constexpr (F > 1 && STAGE == FIR_OUT_U8_SAT) {
            // a bank: filters whose 16-bit sum provably cannot overflow run on packed pairs
            TapsN<L, F> probe;
            for (int k = 0; k < F * L; ++k) probe.h[k / L][k % L] = hq[k];
            if (taps16 && nowrap && (plan_u8_pk16(probe, frac) & kU8Pk16))
                return go.template run<kRegFlags | kU8Dot2 | kU8Pk16>();
        }
        if (taps16 && nowrap)
            return go.template run<kRegFlags | kU8Dot2>();
    }
    if constexpr (sizeof(InT) == 2 && CH == 1) {
        if (taps16)
            return acc32 ? go.template run<kRegFlags | kDot2 | kAcc32>()
                         : go.template run<kRegFlags | kDot2>();
    }
    return acc32 ? go.template run<kRegFlags | kAcc32>()
                 : go.template run<kRegFlags>();
}

template <typename InT, int STAGE, int CH, int F>
hipError_t launch_reg_taps(int L, const void* x, void* y, int64_t rows, int64_t total, int64_t rowlen,
                           const int32_t* hq, int frac, int acc_bits, hipStream_t s, const void* hl, const void* hr) {
    switch (L) {
        case 1: return launch_reg<InT, STAGE, 1, CH, F>(RegOne<InT, STAGE, 1, CH, F>{x, y, rows, total, rowlen, hq, frac, acc_bits, s, hl, hr}, hq, frac, acc_bits);
        case 2: return launch_reg<InT, STAGE, 2, CH, F>(RegOne<InT, STAGE, 2, CH, F>{x, y, rows, total, rowlen, hq, frac, acc_bits, s, hl, hr}, hq, frac, acc_bits);
        case 3: return launch_reg<InT, STAGE, 3, CH, F>(RegOne<InT, STAGE, 3, CH, F>{x, y, rows, total, rowlen, hq, frac, acc_bits, s, hl, hr}, hq, frac, acc_bits);
        case 4: return launch_reg<InT, STAGE, 4, CH, F>(RegOne<InT, STAGE, 4, CH, F>{x, y, rows, total, rowlen, hq, frac, acc_bits, s, hl, hr}, hq, frac, acc_bits);
        case 5: return launch_reg<InT, STAGE, 5, CH, F>(RegOne<InT, STAGE, 5, CH, F>{x, y, rows, total, rowlen, hq, frac, acc_bits, s, hl, hr}, hq, frac, acc_bits);
        case 6: return launch_reg<InT, STAGE, 6, CH, F>(RegOne<InT, STAGE, 6, CH, F>{x, y, rows, total, rowlen, hq, frac, acc_bits, s, hl, hr}, hq, frac, acc_bits);
        case 7: return launch_reg<InT, STAGE, 7, CH, F>(RegOne<InT, STAGE, 7, CH, F>{x, y, rows, total, rowlen, hq, frac, acc_bits, s, hl, hr}, hq, frac, acc_bits);
        case 8: return launch_reg<InT, STAGE, 8, CH, F>(RegOne<InT, STAGE, 8, CH, F>{x, y, rows, total, rowlen, hq, frac, acc_bits, s, hl, hr}, hq, frac, acc_bits);
        case 9: return launch_reg<InT, STAGE, 9, CH, F>(RegOne<InT, STAGE, 9, CH, F>{x, y, rows, total, rowlen, hq, frac, acc_bits, s, hl, hr}, hq, frac, acc_bits);
        default: return hipErrorInvalidValue;
    }
}

template <typename InT, int STAGE, int CH, int F>
hipError_t launch_reg_batch_taps(int L, int n, const RegImage* im, const int32_t* hq, int frac, int acc_bits,
                                 hipStream_t s) {
    switch (L) {
#define FIR_BATCH_L(l) \
    case l: return launch_reg<InT, STAGE, l, CH, F>(RegMany<InT, STAGE, l, CH, F>{n, im, hq, frac, acc_bits, s}, hq, frac, acc_bits);
        FIR_BATCH_L(1) FIR_BATCH_L(2) FIR_BATCH_L(3) FIR_BATCH_L(4) FIR_BATCH_L(5)
        FIR_BATCH_L(6) FIR_BATCH_L(7) FIR_BATCH_L(8) FIR_BATCH_L(9)
#undef FIR_BATCH_L
        default: return hipErrorInvalidValue;
    }
}

}  // namespace fir
