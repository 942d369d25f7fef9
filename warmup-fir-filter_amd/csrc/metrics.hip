// metrics.hip — fixed-vs-ideal comparison metrics in one pass over HBM,
// bit for bit the reference's NumPy values.
//
// Restates fir_1d/sim/vector/gen_3tap_compare_report.py:67-112 (_compute_metrics): with
// d = fixed - ideal (float64), it needs max|d|, sum|d|, sum d^2, sum d, #(fixed == 0),
// #(fixed == 255) and #(ideal < 0 or ideal > 255).  The reference takes each from a separate
// NumPy reduction (seven passes over 9 bytes/sample); here one kernel reads each sample once.
// Counts and max|d| do not depend on the order of the reduction.  The three float64 sums do,
// and they follow NumPy's own order exactly (pinned against np.sum / np.mean of NumPy 2.2 on
// random arrays and image shapes: tests/test_metrics_order.py): a contiguous float64 array is
// summed in blocks of 8192 elements (the ufunc buffer), the block sums added in order to 0.0,
// each block by pairwise_sum: n < 8 a plain loop from 0.0; n <= 128 eight strided accumulators
// r[j] (element j, then += j + 8, j + 16, ...) combined as ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7))
// with the elements past the last multiple of 8 added in order; larger n split at
// n2 = floor(n/2) rounded down to a multiple of 8, sum = pw(left) + pw(right).
//
// A full 8192-sample block is a balanced tree of 64 leaves of 128 samples; its sums are
// reduced by one wave, the block sums then added in order by a dependent float64 chain (waves
// 0-2 of one workgroup: |d|, d^2, d; 2.7 ns per block).  Two forms:
//   16-byte aligned u8 (the pipeline's case): metrics_prep marks the words the next launch
//     publishes as unset and sums the ragged last block, then ONE launch of metrics_leaf_kernel: one lane per leaf (the leaf
//     combine in registers, the block tree by DPP row shifts and permlane swaps -- IEEE addition
//     is commutative, so a lane adding its partner's value matches either order), each block's
//     sums published to workgroup 0, which follows them (chain_follow) and finishes the call
//     (final_in_launch) inside the same launch.
//   any other dtype or alignment: the full blocks in parts of one launch each (8192 blocks, the
//     last 2048) of metrics_blocks (u8: 8 rounds of 8 leaves, transposed through the wave's LDS
//     so that lane (leaf, j) adds accumulator r[j]'s 16 terms in order) or metrics_blocks_any
//     (stride-8 loads, not a bandwidth path); the chain over part k-1 runs as an extra workgroup
//     of the launch streaming part k; metrics_ragged sums the ragged block by the general
//     recursion (leaves enumerated, summed one per thread, recombined in post-order), and
//     metrics_final adds the last part and reduces the counts and max.
#include <string>
#include <type_traits>

#include "fir_common.h"
#include "fir_launch.h"

namespace fir {

// Launch shapes (the forms measured against these and removed in round 5 are listed, with their
// numbers)
constexpr int kMetricBlocks = 512;  // workgroups per part launch at most (each wave streams 4 blocks
                                    // of an 8192-block part; 2^28: 453 -> 430 us vs 2048, 4096 slower)
constexpr int kPwBlock = 8192;   // NumPy's ufunc buffer (NPY_BUFSIZE elements)
constexpr int kPwLeaf = 128;     // pairwise_sum's PW_BLOCKSIZE
constexpr int kPwMaxLeaves = 128;  // leaves of a block shorter than 8192 (each >= 64 samples)

struct Cnt {
    double mx;
    unsigned long long lo, hi, clip;
};

// One sample: d = fixed - ideal, its |d|, d^2, d, and the max / counts.
struct Term {
    double a, q, d;
};
// F = uint32_t (u8 samples, integer compares) or double (any other fixed dtype converted as
// astype(np.float64) does; fixed == 0 / == 255 on the original values equal the same compares on
// the converted ones for every integer and float dtype: the conversion is exact near 0 and 255).
// max drops a NaN here (v_max_f64); metrics_final restores NumPy's NaN from sum|d| (below).
template <typename F>
__device__ __forceinline__ Term metrics_term(double id, F fx, double& mx, uint32_t& lo, uint32_t& hi,
                                             uint32_t& clip) {
    const double d = __dsub_rn((double)fx, id);
    const double ad = fabs(d);
    mx = fmax(mx, ad);
    lo += fx == (F)0;
    hi += fx == (F)255;
    clip += (id < 0.0) | (id > 255.0);
    return Term{ad, __dmul_rn(d, d), d};
}
// fixed sample -> the value metrics_term compares (u8: the integer; others: the float64 value)
template <typename FT>
__device__ __forceinline__ auto fixed_val(FT v) {
    if constexpr (std::is_same_v<FT, uint8_t>) return (uint32_t)v;
    else return (double)v;
}
__device__ __forceinline__ void tadd(Term& s, const Term& t) {
    s.a = __dadd_rn(s.a, t.a);
    s.q = __dadd_rn(s.q, t.q);
    s.d = __dadd_rn(s.d, t.d);
}
__device__ __forceinline__ Term tadd2(const Term& s, const Term& t) {
    return Term{__dadd_rn(s.a, t.a), __dadd_rn(s.q, t.q), __dadd_rn(s.d, t.d)};
}
// lane i receives lane i + D's value (only the tree's leader lanes, multiples of 2D, are used):
// DPP row_shl within 16-lane rows, v_permlane16/32_swap across rows (VALU, not the LDS unit
// that __shfl_xor's ds_bpermute uses)
template <int D>
__device__ __forceinline__ double dshift(double v) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    uint32_t lo = (uint32_t)b, hi = (uint32_t)(b >> 32);
    if constexpr (D < 16) {
        lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)lo, 0x100 + D, 0xF, 0xF, false);
        hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)hi, 0x100 + D, 0xF, 0xF, false);
    } else if constexpr (D == 16) {
        lo = __builtin_amdgcn_permlane16_swap(lo, lo, false, false)[1];
        hi = __builtin_amdgcn_permlane16_swap(hi, hi, false, false)[1];
    } else {
        lo = __builtin_amdgcn_permlane32_swap(lo, lo, false, false)[1];
        hi = __builtin_amdgcn_permlane32_swap(hi, hi, false, false)[1];
    }
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
template <int D>
__device__ __forceinline__ Term tshift(const Term& s) {
    return Term{dshift<D>(s.a), dshift<D>(s.q), dshift<D>(s.d)};
}

// pairwise_sum of one leaf (n <= 128) of samples [o, o + n), as NumPy's loop does it
template <typename FT>
__device__ Term pw_leaf(const double* ideal, const FT* fixed, int64_t o, int n, double& mx, uint32_t& lo,
                        uint32_t& hi, uint32_t& clip) {
    auto term = [&](int64_t i) { return metrics_term(ideal[i], fixed_val(fixed[i]), mx, lo, hi, clip); };
    if (n < 8) {
        Term res{0.0, 0.0, 0.0};
        for (int i = 0; i < n; ++i) tadd(res, term(o + i));
        return res;
    }
    Term r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = term(o + j);
    int i = 8;
    for (; i < n - (n % 8); i += 8) {
#pragma unroll
        for (int j = 0; j < 8; ++j) tadd(r[j], term(o + i + j));
    }
    Term res = tadd2(tadd2(tadd2(r[0], r[1]), tadd2(r[2], r[3])), tadd2(tadd2(r[4], r[5]), tadd2(r[6], r[7])));
    for (; i < n; ++i) tadd(res, term(o + i));
    return res;
}

// counts and max of a workgroup into *dst (wave shuffles, then the 4 wave results)
__device__ void block_counts(Cnt c, Cnt* dst) {
    __shared__ Cnt red[kBlock / kWave];
#pragma unroll
    for (int m = 1; m < kWave; m <<= 1) {
        c.mx = fmax(c.mx, __shfl_xor(c.mx, m));
        c.lo += __shfl_xor(c.lo, m);
        c.hi += __shfl_xor(c.hi, m);
        c.clip += __shfl_xor(c.clip, m);
    }
    if ((threadIdx.x & (kWave - 1)) == 0) red[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        Cnt a = red[0];
        for (int w = 1; w < kBlock / kWave; ++w)
            a.mx = fmax(a.mx, red[w].mx), a.lo += red[w].lo, a.hi += red[w].hi, a.clip += red[w].clip;
        *dst = a;
    }
}

// The running sums state[0..2] += block sums [lo, hi) of |d|, d^2, d, in order (from 0.0 when
// lo == 0).  Waves 0-2 take one array each: groups of kChainDepth x 64 block sums, loaded
// coalesced two groups ahead in chain_range (the loaded latency of one group, ~3 us beside a streaming
// launch, exceeds the 1.4 us its adds take), each staged in the wave's LDS and read back in order
// by every lane at the same address (a broadcast), so the dependent chain is one float64 add with
// a VGPR operand per 8192 samples (2.7 ns; fed by v_readlane instead: 8.7 ns,
// tools/microbench/chain_micro.hip).  `lds` holds 3 x kChainDepth x 64 doubles; no workgroup
// barrier inside.
constexpr int kChainDepth = 8;   // block sums per lane of a chain group (a group = 64 x this)
constexpr int kChainLds = 3 * kChainDepth * kWave * (int)sizeof(double);
constexpr int kChainGS = kChainDepth * kWave;  // block sums per group
// s += sh[0], sh[1], ..., sh[len - 1] in order (sh: a staged group in the wave's LDS)
__device__ __forceinline__ void add_group(double& s, const double* sh, int len) {
    constexpr int GS = kChainGS;
    int e = 0;
    if (len == GS) {  // a full group: 16-element batches, the next batch's reads in flight
        typedef double d2 __attribute__((ext_vector_type(2)));
        d2 va[8], vb[8];
        auto ld = [&](d2 (&v)[8], int e0) __attribute__((always_inline)) {
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = *reinterpret_cast<const d2*>(&sh[e0 + 2 * j]);
        };
        auto add = [&](const d2 (&v)[8]) __attribute__((always_inline)) {
#pragma unroll
            for (int j = 0; j < 8; ++j) s = __dadd_rn(__dadd_rn(s, v[j].x), v[j].y);
        };
        ld(va, 0);
#pragma unroll 1
        for (int e0 = 0; e0 < GS; e0 += 32) {  // (sched barriers: keep each batch's reads
            ld(vb, e0 + 16);                      // ahead of the previous batch's adds)
            __builtin_amdgcn_sched_barrier(0);
            add(va);
            ld(va, (e0 + 32) & (GS - 1));  // (the last one re-reads batch 0, unused)
            __builtin_amdgcn_sched_barrier(0);
            add(vb);
        }
        e = GS;
    }
    for (; e + 16 <= len; e += 16) {
        double v[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = sh[e + j];
#pragma unroll
        for (int j = 0; j < 16; ++j) s = __dadd_rn(s, v[j]);
    }
    for (; e < len; ++e) s = __dadd_rn(s, sh[e]);
}
__device__ __forceinline__ void chain_range(const double* __restrict__ bsum, int64_t nb, int64_t lo, int64_t hi, double* state,
                            uint8_t* lds, double* out = nullptr) {
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & (kWave - 1);
    if (wv >= 3) return;
    const double* src = bsum + (int64_t)wv * nb;
    double* sh = reinterpret_cast<double*>(lds) + wv * kChainDepth * kWave;
    double s = lo == 0 ? 0.0 : state[wv];
    constexpr int D = kChainDepth, NG = 2, GS = kChainGS;  // (deeper: no faster, more registers)
    auto fetch = [&](int64_t c0, double (&q)[D]) __attribute__((always_inline)) {
#pragma unroll
        for (int d = 0; d < D; ++d) q[d] = c0 + d * kWave + lane < hi ? src[c0 + d * kWave + lane] : 0.0;
    };
    double q[NG][D];
#pragma unroll
    for (int k = 0; k < NG; ++k) fetch(lo + (int64_t)k * GS, q[k]);
    for (int64_t g0 = lo; g0 < hi;) {
#pragma unroll
        for (int k = 0; k < NG; ++k) {  // group g0 is in q[k]
            if (g0 < hi) {
                __builtin_amdgcn_wave_barrier();  // the previous group's reads are done (one wave: in order)
#pragma unroll
                for (int d = 0; d < D; ++d) sh[d * kWave + lane] = q[k][d];
                __builtin_amdgcn_wave_barrier();
                fetch(g0 + (int64_t)NG * GS, q[k]);  // NG groups ahead, in flight during the adds
                add_group(s, sh, hi - g0 < GS ? (int)(hi - g0) : GS);
                g0 += GS;
            }
        }
    }
    if (lane == 0) {
        state[wv] = s;
        if (out) out[1 + wv] = s;
    }
}

// The chain inside the launch that produces the block sums (metrics_leaf_kernel).  Streaming wave
// w takes blocks w, w + nw, w + 2 nw, ... (nw waves); workgroup 0's waves 0-2 add the block sums
// of |d|, d^2 and d in order as they appear.  The hand-off is per location: every published word
// is its own "ready" flag.  The kernel ahead of the launch (metrics_prep) sets each block-sum and
// workgroup-count word to kUnset, a signalling-NaN pattern no sum can take (arithmetic results
// are quiet NaNs; a count never reaches 2^63); a producer stores each word once, by a relaxed
// agent-scope atomic store (write-through); a chain wave reads a group of kChainGS words by
// returning agent-scope atomics and takes it once none reads kUnset.  In the HIP memory model
// that needs no ordering between locations: an atomic read returns either the kUnset stored
// before the launch (kernel boundary) or the one value a producer stored, and per-location
// coherence makes the latter visible eventually -- so there is no progress word, no release
// fence and no acquire fence.  (An agent-scope release per published block -- buffer_wbl2 sc1 on
// gfx950 -- made the pass 4.6x slower, 1828 vs 395.5 us at 2^28, profiles/r05/metrics_release_ab.txt.)
// Blocks [nbf, nb) (the ragged block) were written by the earlier launch.  The chain's waves run
// at raised priority (a dependent float64 add per block, sharing a SIMD with streaming waves).  The
// waits share one deadline on the 100 MHz s_memrealtime clock, kChainTimeoutTicks after the
// chain starts (no correct run comes near it: the producers never wait, and a 288 GB call
// streams in ~50 ms); past it the sums are NaN and out[8] = 1.
constexpr uint64_t kChainTimeoutTicks = 1000000000ull;  // 10 s
constexpr uint64_t kUnset = 0x7FF0000000000001ull;      // a signalling NaN: "not published yet"
typedef __attribute__((address_space(1))) uint64_t gu64;
typedef __attribute__((address_space(1))) uint32_t gu32;
// A read of a word another XCD wrote in this launch (or the kernel before it) that no cache of the
// reading XCD can answer: a returning agent-scope atomic (performed past the XCD's L2).  Loads --
// plain, sc1, or behind an agent acquire -- are served by the reading XCD's L2, which can hold the
// line from an earlier call: in a graph replay the chain then saw the previous replay's words and
// sums (tests/test_gpu_graphs.py, all 9 full blocks of seed 1 in seed 2's sums).
// (The zero operand is opaque: with a literal 0 the compiler turns the idempotent RMW into a load.)
__device__ __forceinline__ uint32_t opaque_zero() {
    uint32_t z;
    asm volatile("v_mov_b32 %0, 0" : "=v"(z));
    return z;
}
__device__ __forceinline__ uint64_t coherent_read_bits(const void* p) {
    return __hip_atomic_fetch_or((gu64*)p, (uint64_t)opaque_zero(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double coherent_read(const double* p) {
    return __builtin_bit_cast(double, coherent_read_bits(p));
}
__device__ __forceinline__ void publish_bits(void* p, uint64_t v) {
    __hip_atomic_store((gu64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void chain_follow(const double* __restrict__ bsum, int64_t nb, int64_t nbf, double* state,
                                             uint8_t* lds) {
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & (kWave - 1);
    const double* src = bsum + (int64_t)wv * nb;
    double* sh = reinterpret_cast<double*>(lds) + wv * kChainDepth * kWave;
    constexpr int D = kChainDepth, GS = kChainGS;
    int* failed = reinterpret_cast<int*>(lds + kChainLds + 52);  // a chain wave gave up waiting
    uint64_t* deadline = reinterpret_cast<uint64_t*>(lds + kChainLds + 56);  // shared with final_in_launch
    if (threadIdx.x == 0) {
        *failed = 0;
        *deadline = __builtin_amdgcn_s_memrealtime() + kChainTimeoutTicks;
    }
    __syncthreads();  // (every wave of the workgroup: the words are set before anyone reads them)
    if (wv >= 3) return;
    const uint64_t dl = *deadline;
    __builtin_amdgcn_s_setprio(3);
    double s = 0.0;
    bool ok = true;
    for (int64_t g0 = 0; g0 < nbf; g0 += GS) {
        const int len = (int)(nbf - g0 < GS ? nbf - g0 : GS);
        uint64_t v[D];
        for (;;) {  // one wave-wide read of the group; again after a sleep until every word is published
            bool mine = true;
#pragma unroll
            for (int d = 0; d < D; ++d) {
                const int e = d * kWave + lane;
                v[d] = e < len ? coherent_read_bits(src + g0 + e) : 0ull;
                mine &= v[d] != kUnset;
            }
            if (__builtin_amdgcn_ballot_w64(!mine) == 0) break;
            if (__builtin_amdgcn_s_memrealtime() > dl) {
                ok = false;
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
        if (!ok) break;
        __builtin_amdgcn_wave_barrier();  // the previous group's reads are done
#pragma unroll
        for (int d = 0; d < D; ++d) sh[d * kWave + lane] = __builtin_bit_cast(double, v[d]);
        __builtin_amdgcn_wave_barrier();
        add_group(s, sh, len);
    }
    for (int64_t b = nbf; b < nb; ++b) s = __dadd_rn(s, coherent_read(src + b));
    if (lane == 0) {
        state[wv] = ok ? s : __builtin_nan("");
        reinterpret_cast<double*>(lds + kChainLds + 16)[wv] = ok ? s : __builtin_nan("");  // (for final_in_launch)
        if (!ok) __hip_atomic_store(failed, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    __builtin_amdgcn_s_setprio(0);
}

// A round's 64 lane sums (lane (leaf k, accumulator j)) -> lane 0: each leaf's
// ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)), then the round's 8 leaves pairwise.
__device__ __forceinline__ Term round_tree(Term t) {
    t = tadd2(t, tshift<1>(t));
    t = tadd2(t, tshift<2>(t));
    t = tadd2(t, tshift<4>(t));
    t = tadd2(t, tshift<8>(t));
    t = tadd2(t, tshift<16>(t));
    return tadd2(t, tshift<32>(t));
}
// Round rd's sum into the block's tree ((R0+R1)+(R2+R3))+((R4+R5)+(R6+R7)): st[0] R_even,
// st[1] pairs, st[2] quads, st[3] the block after round 7.
__device__ __forceinline__ void fold_round(Term (&st)[4], int rd, const Term& t) {
    if ((rd & 1) == 0) {
        st[0] = t;
    } else {
        const Term pr = tadd2(st[0], t);
        if ((rd & 2) == 0) {
            st[1] = pr;
        } else {
            const Term q = tadd2(st[1], pr);
            if ((rd & 4) == 0) st[2] = q;
            else st[3] = tadd2(st[2], q);
        }
    }
}

// One WAVE per full block (no workgroup barrier: waves stream independently), grid-stride over
// the blocks; a block = 8 rounds of 8 leaves (1024 samples, one balanced subtree each).  A round
// is loaded as contiguous 1 KiB rows (leaf i by load i: 16 bytes per lane) plus one 16-byte load
// of its fixed bytes, staged in the wave's LDS and read back transposed: lane (leaf k, j) takes
// the 16 terms of accumulator r[j] (samples 8 s + j) in order.  (Reading those stride-8 samples
// straight from HBM touches 16 half lines per load and ran at 3.3 TB/s.)
constexpr int kMetRow = 1024 + 64;                      // LDS bytes per leaf row (+64: conflict-free reads)
constexpr int kMetWaveLds = 8 * kMetRow + 1024;         // + the round's 1 KiB of fixed bytes
static_assert(kBlock / kWave * kMetWaveLds >= kChainLds, "the chain's staging shares the wave buffers");
// (u8 arrays not 16-byte aligned: the aligned ones take metrics_leaf_kernel)
__global__ __launch_bounds__(kBlock, 4) void metrics_blocks(const double* __restrict__ ideal,
                                                                         const uint8_t* __restrict__ fixed,
                                                                         double* __restrict__ bsum, int64_t nb,
                                                                         int64_t b_lo, int64_t b_hi, int64_t c_lo,
                                                                         int64_t c_hi, double* __restrict__ state,
                                                                         Cnt* __restrict__ parts) {
    typedef double d2 __attribute__((ext_vector_type(2)));
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    __shared__ __attribute__((aligned(16))) uint8_t smem[kBlock / kWave * kMetWaveLds];
    const bool chain = c_hi > c_lo;
    if (chain && blockIdx.x == 0) {  // dispatched first: the chain starts with the part
        chain_range(bsum, nb, c_lo, c_hi, state, smem);
        return;
    }
    const int wg = blockIdx.x - (chain ? 1 : 0);
    const int lane = threadIdx.x & (kWave - 1), wv = threadIdx.x >> 6;
    const int k = lane >> 3, j = lane & 7;  // leaf of the round, accumulator
    uint8_t* wl = smem + wv * kMetWaveLds;
    const int64_t nwaves = (int64_t)(gridDim.x - (chain ? 1 : 0)) * (kBlock / kWave);
    double mx = 0.0;
    uint32_t lo = 0, hi = 0, clip = 0;

    for (int64_t b = b_lo + (int64_t)wg * (kBlock / kWave) + wv; b < b_hi; b += nwaves) {
        Term st[4];  // pairwise stack of round sums: ((R0+R1)+(R2+R3))+((R4+R5)+(R6+R7))
#pragma unroll 1
        for (int rd = 0; rd < 8; ++rd) {
            const int64_t base = b * kPwBlock + rd * 1024;
            d2 v[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] = d2{ideal[base + 128 * i + 2 * lane], ideal[base + 128 * i + 2 * lane + 1]};
            uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
            for (int e = 0; e < 16; ++e) w[e / 4] |= (uint32_t)fixed[base + 16 * lane + e] << (8 * (e % 4));
            const u4 fx = u4{w[0], w[1], w[2], w[3]};
            __builtin_amdgcn_wave_barrier();  // the previous round's reads are done (one wave: in order)
#pragma unroll
            for (int i = 0; i < 8; ++i) *reinterpret_cast<d2*>(wl + i * kMetRow + 16 * lane) = v[i];
            // fixed bytes transposed to [leaf][accumulator j][step s]: lane (k', m) holds samples
            // 16 m .. 16 m + 15 of leaf k', i.e. steps 2m, 2m + 1 of every j (bytes j, j + 8)
            {
                const uint32_t fw[4] = {fx.x, fx.y, fx.z, fx.w};
                uint8_t* fdst = wl + 8 * kMetRow + 128 * (lane >> 3) + 2 * (lane & 7);
#pragma unroll
                for (int jj = 0; jj < 8; ++jj)
                    *reinterpret_cast<uint16_t*>(fdst + 16 * jj) =
                        (uint16_t)__builtin_amdgcn_perm(fw[2 + jj / 4], fw[jj / 4], (uint32_t)(jj % 4) | ((4u + jj % 4) << 8));
            }
            __builtin_amdgcn_wave_barrier();
            const uint8_t* row = wl + k * kMetRow + 8 * j;
            const u4 fr = *reinterpret_cast<const u4*>(wl + 8 * kMetRow + 128 * k + 16 * j);  // steps 0..15
            const uint32_t frw[4] = {fr.x, fr.y, fr.z, fr.w};
            Term r{0.0, 0.0, 0.0};
#pragma unroll
            for (int s = 0; s < 16; ++s) {
                double id = *reinterpret_cast<const double*>(row + 64 * s);
                uint32_t f = (frw[s / 4] >> (8 * (s % 4))) & 0xFFu;
                // opaque: one LDS read per term, as round 3 measured it (hipcc otherwise hoists all 16)
                asm volatile("" : "+v"(id), "+v"(f), "+v"(mx), "+v"(lo), "+v"(hi), "+v"(clip));
                const Term t = metrics_term(id, f, mx, lo, hi, clip);
                if (s == 0) r = t;
                else tadd(r, t);
            }
            fold_round(st, rd, round_tree(r));
        }
        const Term s = st[3];
        if (lane == 0) bsum[b] = s.a, bsum[nb + b] = s.q, bsum[2 * nb + b] = s.d;
    }
    block_counts(Cnt{mx, lo, hi, clip}, parts + wg);
}

// The block pass with one LANE per leaf (round 4): lane l owns leaf l (samples 128 l .. 128 l +
// 127) of the wave's block and keeps all 8 of its accumulators r[0..7] in registers, so the leaf
// combine ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) is 7 adds per 128 samples and only the block tree
// over the 64 leaves crosses lanes (6 DPP / permlane levels per 8192 samples) -- against one
// lane per accumulator above, whose 6-level tree ran every 1024 samples.  A round q (0..7) is the
// 16-sample band [16 q, 16 q + 16) of every leaf: loaded as 8 coalesced 1 KiB instructions (8
// lanes per leaf's 128-byte band row), staged in the wave's LDS as [leaf][16 doubles] rows of
// 144 bytes (conflict-free ds_read_b128 of a lane's own row), the next round's band loaded into
// registers while this one is reduced.  The block's 8 KiB of fixed bytes arrive with its first
// band (coalesced, staged as [leaf][128 bytes] rows).  Counts without per-sample VALU adds: zeros
// and 255s of four fixed bytes at once (byte tricks + v_bcnt), the ideal range test as two
// compares whose lane masks are counted on the SALU.
constexpr int kLfRow = 144;                       // LDS bytes per leaf row (128 + 16: conflict-free b128)
constexpr int kLfWaveLds = 2 * kWave * kLfRow;    // ideal band + the block's fixed bytes
static_assert(kBlock / kWave * kLfWaveLds >= kChainLds, "the chain's staging shares the wave buffers");
__device__ __forceinline__ __amdgpu_buffer_rsrc_t mt_rsrc(const void* p, uint32_t bytes) {
    const uint64_t a = (uint64_t)(uintptr_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    return __builtin_amdgcn_make_buffer_rsrc((void*)(uintptr_t)(((uint64_t)hi << 32) | lo), (short)0, (int)bytes, 0x00020000);
}
// block_counts for the publishing launch: the workgroup's counts, each word published once
// (kUnset until then; see chain_follow).
__device__ void block_counts_pub(Cnt c, Cnt* dst) {
    __shared__ Cnt red[kBlock / kWave];
#pragma unroll
    for (int m = 1; m < kWave; m <<= 1) {
        c.mx = fmax(c.mx, __shfl_xor(c.mx, m));
        c.lo += __shfl_xor(c.lo, m);
        c.hi += __shfl_xor(c.hi, m);
        c.clip += __shfl_xor(c.clip, m);
    }
    if ((threadIdx.x & (kWave - 1)) == 0) red[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        Cnt a = red[0];
        for (int w = 1; w < kBlock / kWave; ++w)
            a.mx = fmax(a.mx, red[w].mx), a.lo += red[w].lo, a.hi += red[w].hi, a.clip += red[w].clip;
        uint64_t* d = reinterpret_cast<uint64_t*>(dst);
        publish_bits(d + 0, __builtin_bit_cast(uint64_t, a.mx));
        publish_bits(d + 1, (uint64_t)a.lo);
        publish_bits(d + 2, (uint64_t)a.hi);
        publish_bits(d + 3, (uint64_t)a.clip);
    }
}

// metrics_final's work inside the publishing launch (its chain workgroup, after the chain): each
// thread reads its share of the nparts workgroup counts once every word is published (the same
// per-location hand-off as the block sums), then the reduction and the chain's sums go to
// out[0..8].  A wait past the chain's deadline writes NaN sums and out[8] = 1.
__device__ void final_in_launch(const Cnt* parts, int nparts, int64_t n, double* out, uint8_t* lds) {
    const int t = threadIdx.x;
    double* sums = reinterpret_cast<double*>(lds + kChainLds + 16);  // the chain's three sums
    int* flag = reinterpret_cast<int*>(lds + kChainLds + 48);
    Cnt* red = reinterpret_cast<Cnt*>(lds + kChainLds + 64);
    if (t == 0) *flag = 1;
    __syncthreads();  // the chain's sums and deadline are in LDS
    const uint64_t dl = *reinterpret_cast<const uint64_t*>(lds + kChainLds + 56);
    Cnt c{0.0, 0, 0, 0};
    bool mine = true;
    for (int i = t; i < nparts; i += kBlock) {
        const uint64_t* q = reinterpret_cast<const uint64_t*>(parts + i);
        uint64_t w[4];
        for (;;) {
            bool done = true;
#pragma unroll
            for (int k = 0; k < 4; ++k) w[k] = coherent_read_bits(q + k), done &= w[k] != kUnset;
            if (done) break;
            if (__builtin_amdgcn_s_memrealtime() > dl) {
                mine = false;
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
        if (!mine) break;
        c.mx = fmax(c.mx, __builtin_bit_cast(double, w[0]));
        c.lo += w[1], c.hi += w[2], c.clip += w[3];
    }
    if (!mine) __hip_atomic_store(flag, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    red[t] = c;
    __syncthreads();
    const bool ok = *flag != 0;
    const bool chain_ok = reinterpret_cast<const int*>(lds + kChainLds + 52)[0] == 0;
    for (int w = kBlock / 2; w > 0; w >>= 1) {
        if (t < w) {
            Cnt& a = red[t];
            const Cnt& b = red[t + w];
            a.mx = fmax(a.mx, b.mx), a.lo += b.lo, a.hi += b.hi, a.clip += b.clip;
        }
        __syncthreads();
    }
    if (t == 0) {
        const double nan = __builtin_nan("");
        const double s0 = ok ? sums[0] : nan;
        out[1] = s0, out[2] = ok ? sums[1] : nan, out[3] = ok ? sums[2] : nan;
        out[0] = s0 != s0 ? s0 : red[0].mx;  // NumPy's NaN max (metrics_final)
        out[4] = (double)red[0].lo, out[5] = (double)red[0].hi, out[6] = (double)red[0].clip;
        out[7] = (double)n, out[8] = ok && chain_ok ? 0.0 : 1.0;  // 1: a hand-off wait timed out
    }
}

// One launch over every full block [0, nbf) of a 16-byte aligned u8 call: the streaming workgroups
// publish each block's sums to workgroup 0, which follows them (chain_follow) and finishes the
// call (final_in_launch).
__global__ __launch_bounds__(kBlock, 2) void metrics_leaf_kernel(const double* __restrict__ ideal,
                                                                const uint8_t* __restrict__ fixed,
                                                                double* __restrict__ bsum, int64_t nb, int64_t nbf,
                                                                double* __restrict__ state, Cnt* __restrict__ parts,
                                                                const Cnt* parts_all, int nparts_all, int64_t n,
                                                                double* __restrict__ out) {
    typedef double d2 __attribute__((ext_vector_type(2)));
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    typedef int i4 __attribute__((ext_vector_type(4)));
    __shared__ __attribute__((aligned(16))) uint8_t smem[kBlock / kWave * kLfWaveLds];
    if (blockIdx.x == 0) {
        chain_follow(bsum, nb, nbf, state, smem);
        final_in_launch(parts_all, nparts_all, n, out, smem);
        return;
    }
    const int wg = blockIdx.x - 1;
    const int lane = threadIdx.x & (kWave - 1), wv = threadIdx.x >> 6;
    uint8_t* wl = smem + wv * kLfWaveLds;
    uint8_t* fl = wl + kWave * kLfRow;  // fixed rows
    const int64_t nwaves = (int64_t)(gridDim.x - 1) * (kBlock / kWave);
    const int64_t sw = (int64_t)wg * (kBlock / kWave) + wv;  // streaming wave index
    const int64_t b0 = sw;
    const int64_t nrounds = b0 < nbf ? ((nbf - 1 - b0) / nwaves + 1) * 8 : 0;
    double mx = 0.0;
    uint32_t nz_acc = 0, ff_acc = 0, ndw = 0;  // v_bcnt sums (28 + count per dword) and dwords seen
    uint64_t clip = 0;                          // wave-uniform (SALU)
    // band q of a block: load i, lane p -> leaf 8 i + p / 8, doubles 2 (p % 8) .. of its band row:
    // byte offset 1024 (8 i + p / 8) + 128 q + 16 (p % 8) from the block (soffset: the uniform part)
    const uint32_t voff = 1024u * (uint32_t)(lane >> 3) + 16u * (uint32_t)(lane & 7);
    const int lrow = lane >> 3, lcol = lane & 7;
    d2 nx[8];
    u4 fx[8];
    auto load_band = [&](int64_t t, bool with_fixed) __attribute__((always_inline)) {
        const int64_t blk = b0 + (t >> 3) * nwaves;
        const __amdgpu_buffer_rsrc_t ri = mt_rsrc(ideal + blk * kPwBlock, kPwBlock * 8);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const i4 v = __builtin_amdgcn_raw_buffer_load_b128(ri, voff, 8192 * i + 128 * (int)(t & 7), 2);
            nx[i] = __builtin_bit_cast(d2, v);
        }
        if (with_fixed) {
            const __amdgpu_buffer_rsrc_t rf = mt_rsrc(fixed + blk * kPwBlock, kPwBlock);
#pragma unroll
            for (int i = 0; i < 8; ++i) fx[i] = __builtin_bit_cast(u4, __builtin_amdgcn_raw_buffer_load_b128(rf, 16u * lane, 1024 * i, 0));
        }
    };
    if (nrounds) load_band(0, true);
    Term r[8];
    // one band of this lane's leaf: 16 terms into r[s % 8] (FIRST: the leaf's first band, whose
    // first 8 terms start the accumulators, as pairwise_sum's r[j] = a[j])
    auto band = [&](auto first, const double (&idv)[16], const uint32_t (&fw)[4]) __attribute__((always_inline)) {
        constexpr bool FIRST = decltype(first)::value;
        uint32_t clip_band = 0;  // <= 1024 per band: 32-bit SALU adds, one 64-bit add per band
#pragma unroll
        for (int s = 0; s < 16; ++s) {
            const double id = idv[s];
            const uint32_t f = (fw[s / 4] >> (8 * (s % 4))) & 0xFFu;
            const double d = __dsub_rn((double)f, id);
            const double ad = fabs(d);
            mx = fmax(mx, ad);
            // (id < 0) and (id > 255) exclude each other: two lane masks counted on the SALU
            clip_band += (uint32_t)__builtin_popcountll(__builtin_amdgcn_ballot_w64(id < 0.0)) +
                         (uint32_t)__builtin_popcountll(__builtin_amdgcn_ballot_w64(id > 255.0));
            const Term tt{ad, __dmul_rn(d, d), d};
            if (FIRST && s < 8) r[s] = tt;
            else tadd(r[s & 7], tt);
        }
        clip += clip_band;
    };
#pragma unroll 1
    for (int64_t t = 0; t < nrounds; ++t) {
        const int q = (int)(t & 7);
        __builtin_amdgcn_wave_barrier();  // the previous round's LDS reads are done
#pragma unroll
        for (int i = 0; i < 8; ++i) *reinterpret_cast<d2*>(wl + (8 * i + lrow) * kLfRow + 16 * lcol) = nx[i];
        if (q == 0) {
#pragma unroll
            for (int i = 0; i < 8; ++i) *reinterpret_cast<u4*>(fl + (8 * i + lrow) * kLfRow + 16 * lcol) = fx[i];
        }
        __builtin_amdgcn_wave_barrier();
        if (t + 1 < nrounds) load_band(t + 1, q == 7);  // the next band (+ the next block's fixed bytes)
        // this lane's leaf: 16 doubles and 16 fixed bytes of band q
        double idv[16];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const d2 v = *reinterpret_cast<const d2*>(wl + lane * kLfRow + 16 * k);
            idv[2 * k] = v.x, idv[2 * k + 1] = v.y;
        }
        const u4 fr = *reinterpret_cast<const u4*>(fl + lane * kLfRow + 16 * q);
        const uint32_t fw[4] = {fr.x, fr.y, fr.z, fr.w};
#pragma unroll
        for (int w = 0; w < 4; ++w) {  // zeros / 255s of 4 bytes: high bit of each byte = "nonzero" / "== 255"
            const uint32_t lo7 = fw[w] & 0x7F7F7F7Fu;
            nz_acc += (uint32_t)__builtin_popcount((lo7 + 0x7F7F7F7Fu) | fw[w] | 0x7F7F7F7Fu);
            ff_acc += (uint32_t)__builtin_popcount(((lo7 + 0x01010101u) & fw[w]) | 0x7F7F7F7Fu);
        }
        ndw += 4;
        if (q == 0)
            band(std::true_type{}, idv, fw);
        else
            band(std::false_type{}, idv, fw);
        if (q == 7) {  // the leaf is complete: its pairwise combine, then the block's tree over lanes
            Term lf = tadd2(tadd2(tadd2(r[0], r[1]), tadd2(r[2], r[3])), tadd2(tadd2(r[4], r[5]), tadd2(r[6], r[7])));
            lf = tadd2(lf, tshift<1>(lf));
            lf = tadd2(lf, tshift<2>(lf));
            lf = tadd2(lf, tshift<4>(lf));
            lf = tadd2(lf, tshift<8>(lf));
            lf = tadd2(lf, tshift<16>(lf));
            lf = tadd2(lf, tshift<32>(lf));
            if (lane == 0) {  // published: each word is its own ready flag (chain_follow)
                const int64_t b = b0 + (t >> 3) * nwaves;
                publish_bits(bsum + b, __builtin_bit_cast(uint64_t, lf.a));
                publish_bits(bsum + nb + b, __builtin_bit_cast(uint64_t, lf.q));
                publish_bits(bsum + 2 * nb + b, __builtin_bit_cast(uint64_t, lf.d));
            }
        }
    }
    const uint32_t lo = 4 * ndw - (nz_acc - 28 * ndw), hi = ff_acc - 28 * ndw;
    block_counts_pub(Cnt{mx, lo, hi, lane == 0 ? clip : 0ull}, parts + wg);
}

// Fixed arrays of any other dtype (int8..int64, uint16..uint64, float16/32/64: the reference's
// astype(np.float64) accepts them all): the same blocks, rounds, leaves and trees, each lane
// reading its accumulator's 16 samples (stride 8) straight from memory.  Not a bandwidth path.
template <typename FT>
__global__ __launch_bounds__(kBlock) void metrics_blocks_any(const double* __restrict__ ideal,
                                                             const FT* __restrict__ fixed, double* __restrict__ bsum,
                                                             int64_t nb, int64_t b_lo, int64_t b_hi, int64_t c_lo,
                                                             int64_t c_hi, double* __restrict__ state,
                                                             Cnt* __restrict__ parts) {
    __shared__ __attribute__((aligned(16))) uint8_t smem[kChainLds];
    const bool chain = c_hi > c_lo;
    if (chain && blockIdx.x == 0) {
        chain_range(bsum, nb, c_lo, c_hi, state, smem);
        return;
    }
    const int wg = blockIdx.x - (chain ? 1 : 0);
    const int lane = threadIdx.x & (kWave - 1), wv = threadIdx.x >> 6;
    const int k = lane >> 3, j = lane & 7;
    const int64_t nwaves = (int64_t)(gridDim.x - (chain ? 1 : 0)) * (kBlock / kWave);
    double mx = 0.0;
    uint32_t lo = 0, hi = 0, clip = 0;
    for (int64_t b = b_lo + (int64_t)wg * (kBlock / kWave) + wv; b < b_hi; b += nwaves) {
        Term st[4];
#pragma unroll 1
        for (int rd = 0; rd < 8; ++rd) {
            const int64_t o = b * kPwBlock + rd * 1024 + k * kPwLeaf + j;
            Term r{0.0, 0.0, 0.0};
#pragma unroll 4
            for (int s = 0; s < 16; ++s) {
                const Term t = metrics_term(ideal[o + 8 * s], fixed_val(fixed[o + 8 * s]), mx, lo, hi, clip);
                if (s == 0) r = t;
                else tadd(r, t);
            }
            fold_round(st, rd, round_tree(r));
        }
        if (lane == 0) bsum[b] = st[3].a, bsum[nb + b] = st[3].q, bsum[2 * nb + b] = st[3].d;
    }
    block_counts(Cnt{mx, lo, hi, clip}, parts + wg);
}

// The ragged last block [nbf * 8192, n) (0 < m < 8192 samples): NumPy's recursion over it, by one
// whole workgroup (leaves enumerated, summed one per thread, recombined in post-order).
template <typename FT>
__device__ void ragged_block(const double* __restrict__ ideal, const FT* __restrict__ fixed, int64_t n,
                             double* __restrict__ bsum, int64_t nb, Cnt* __restrict__ part) {
    __shared__ int leaf_off[kPwMaxLeaves], leaf_len[kPwMaxLeaves];
    __shared__ Term lsum[kPwMaxLeaves];
    __shared__ int nleaves;
    const int64_t nbf = n / kPwBlock;
    const int m = (int)(n - nbf * kPwBlock);
    double mx = 0.0;
    uint32_t lo = 0, hi = 0, clip = 0;
    {
        const int64_t o0 = nbf * kPwBlock;
        if (threadIdx.x == 0) {  // leaves in left-to-right order (a right part pushed before its left)
            int so[16], sl[16], sp = 1, cnt = 0;
            so[0] = 0, sl[0] = m;
            while (sp) {
                --sp;
                const int o = so[sp], len = sl[sp];
                if (len <= kPwLeaf) {
                    leaf_off[cnt] = o, leaf_len[cnt] = len, ++cnt;
                } else {
                    const int n2 = len / 2 - (len / 2) % 8;
                    so[sp] = o + n2, sl[sp] = len - n2, ++sp;
                    so[sp] = o, sl[sp] = n2, ++sp;
                }
            }
            nleaves = cnt;
        }
        __syncthreads();
        for (int l = threadIdx.x; l < nleaves; l += kBlock)
            lsum[l] = pw_leaf(ideal, fixed, o0 + leaf_off[l], leaf_len[l], mx, lo, hi, clip);
        __syncthreads();
        if (threadIdx.x == 0) {  // post-order: sum = pw(left) + pw(right)
            int fl[16], fst[16], fp = 1, vp = 0, li = 0;
            Term vs[16];
            fl[0] = m, fst[0] = 0;
            while (fp) {
                const int len = fl[fp - 1];
                if (len <= kPwLeaf) {
                    vs[vp++] = lsum[li++];
                    --fp;
                    continue;
                }
                const int n2 = len / 2 - (len / 2) % 8;
                if (fst[fp - 1] == 0) {
                    fst[fp - 1] = 1, fl[fp] = n2, fst[fp] = 0, ++fp;
                } else if (fst[fp - 1] == 1) {
                    fst[fp - 1] = 2, fl[fp] = len - n2, fst[fp] = 0, ++fp;
                } else {
                    const Term rr = vs[--vp], ll = vs[--vp];
                    vs[vp++] = tadd2(ll, rr);
                    --fp;
                }
            }
            bsum[nbf] = vs[0].a, bsum[nb + nbf] = vs[0].q, bsum[2 * nb + nbf] = vs[0].d;
        }
    }

    block_counts(Cnt{mx, lo, hi, clip}, part);
}

template <typename FT>
__global__ __launch_bounds__(kBlock) void metrics_ragged(const double* __restrict__ ideal, const FT* __restrict__ fixed,
                                                         int64_t n, double* __restrict__ bsum, int64_t nb,
                                                         Cnt* __restrict__ part) {
    ragged_block(ideal, fixed, n, bsum, nb, part);
}

// The kernel ahead of the publishing launch: every word that launch publishes (the block sums
// [0, nbf) of the three arrays and the streaming workgroups' nunset counts) set to kUnset,
// grid-stride -- a kernel, not a memset node: replayed in a graph behind other kernels, a
// captured hipMemsetAsync left the previous replay's words in place (tests/test_gpu_graphs.py) --
// and, by workgroup 0, the ragged block (if any), whose sums the chain adds last.
template <typename FT>
__global__ __launch_bounds__(kBlock) void metrics_prep(const double* __restrict__ ideal, const FT* __restrict__ fixed,
                                                       int64_t n, double* __restrict__ bsum, int64_t nb,
                                                       Cnt* __restrict__ ragged_part, Cnt* __restrict__ unset,
                                                       int nunset) {
    const int64_t nbf = n / kPwBlock, tid = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const int64_t nth = (int64_t)gridDim.x * kBlock;
    uint64_t* words = reinterpret_cast<uint64_t*>(bsum);
    for (int w = 0; w < 3; ++w)
        for (int64_t b = tid; b < nbf; b += nth) words[w * nb + b] = kUnset;
    uint64_t* cw = reinterpret_cast<uint64_t*>(unset);
    for (int64_t i = tid; i < 4 * (int64_t)nunset; i += nth) cw[i] = kUnset;
    if (blockIdx.x == 0 && n % kPwBlock) ragged_block(ideal, fixed, n, bsum, nb, ragged_part);
}

// out: [max_abs, sum_abs, sum_sq, sum_d, n_low, n_high, n_clip, n, 0]: the last part's chain
// (and the ragged block's sum, the last in order), the counts and max of every workgroup.
__global__ __launch_bounds__(kBlock) void metrics_final(const double* __restrict__ bsum, int64_t nb, int64_t c_lo,
                                                        double* __restrict__ state, const Cnt* __restrict__ parts,
                                                        int nparts, int64_t n, double* __restrict__ out) {
    __shared__ Cnt red[kBlock];
    __shared__ __attribute__((aligned(16))) uint8_t smem[kChainLds];
    const int t = threadIdx.x;
    Cnt c{0.0, 0, 0, 0};
    for (int i = t; i < nparts; i += kBlock) {
        const Cnt& q = parts[i];
        c.mx = fmax(c.mx, q.mx), c.lo += q.lo, c.hi += q.hi, c.clip += q.clip;
    }
    red[t] = c;
    if (c_lo < nb) chain_range(bsum, nb, c_lo, nb, state, smem, out);  // out[1..3]
    if (c_lo >= nb && t < 3) out[1 + t] = nb > 0 ? state[t] : 0.0;  // (no last part: n == 0)
    __syncthreads();
    for (int w = kBlock / 2; w > 0; w >>= 1) {
        if (t < w) {
            Cnt& a = red[t];
            const Cnt& q = red[t + w];
            a.mx = fmax(a.mx, q.mx), a.lo += q.lo, a.hi += q.hi, a.clip += q.clip;
        }
        __syncthreads();
    }
    __syncthreads();  // out[1] (the chain's sum|d|) is written
    if (t == 0) {
        // np.max propagates NaN; fmax dropped it.  sum|d| is NaN exactly when some |d| is (|d| >= 0:
        // no inf - inf), and its order is NumPy's, so NaN there = NaN in the reference's max.
        out[0] = out[1] != out[1] ? out[1] : red[0].mx;
        out[4] = (double)red[0].lo;
        out[5] = (double)red[0].hi;
        out[6] = (double)red[0].clip;
        out[7] = (double)n;
        out[8] = 0.0;
    }
}

static int64_t metrics_nblocks(int64_t n) { return (n + kPwBlock - 1) / kPwBlock; }

// Work buffer: Cnt per workgroup of every launch (+ the ragged block's), the 3 running sums, then
// the block sums [3][nb].
constexpr int64_t kTailPart = 2048;  // blocks of the last part (its chain is the exposed one)
constexpr int64_t kBodyPart = 8192;  // blocks of every earlier part
constexpr int kMaxParts = 16;
constexpr int64_t kCntSlots = (int64_t)kMaxParts * kMetricBlocks + 1;

// aligned u8 with full blocks: ONE launch (metrics_leaf_kernel) of this many streaming workgroups
constexpr int kMetricPBlocks = 256;
static_assert(kMetricPBlocks + 1 <= kCntSlots, "count slots");
constexpr int kMetricPrepBlocks = 64;  // workgroups of metrics_prep (grid-stride)

// Work buffer: Cnt per workgroup of every launch (+ the ragged block's), the 3 running sums, then
// the block sums [3][nb].
size_t metrics_work_bytes(int64_t n) {
    if (n < 0) n = 0;
    return sizeof(Cnt) * kCntSlots + 64 + 3 * sizeof(double) * (size_t)metrics_nblocks(n);
}

namespace {

template <typename FT>
int launch_metrics_t(const double* ideal, const FT* fixed, int64_t n, double* out, void* work, hipStream_t stream,
                     std::string* err) {
    const int64_t nb = metrics_nblocks(n), nbf = n / kPwBlock;
    Cnt* parts = (Cnt*)work;
    double* state = (double*)((char*)parts + sizeof(Cnt) * kCntSlots);
    double* bsum = state + 8;
    const bool vec = (uintptr_t)ideal % 16 == 0 && (uintptr_t)fixed % 16 == 0;
    if constexpr (std::is_same_v<FT, uint8_t>) {
        if (vec && nbf > 0) {  // one streaming launch
            // the published words set to kUnset and the ragged block (if any) summed first: the chain adds it last
            const int slot = nb > nbf ? 1 : 0;
            const int64_t want = (nbf + kBlock / kWave - 1) / (kBlock / kWave);
            const int g = (int)(want > kMetricPBlocks ? kMetricPBlocks : want);
            hipLaunchKernelGGL(metrics_prep<FT>, dim3(kMetricPrepBlocks), dim3(kBlock), 0, stream, ideal, fixed, n, bsum, nb,
                               parts, parts + slot, g);
            hipLaunchKernelGGL(metrics_leaf_kernel, dim3(g + 1), dim3(kBlock), 0, stream, ideal, fixed, bsum, nb, nbf,
                               state, parts + slot, (const Cnt*)parts, slot + g, n, out);
            const hipError_t e = hipGetLastError();
            if (e != hipSuccess) return *err = std::string("metrics launch failed: ") + hipGetErrorString(e), FIR_EHIP;
            return FIR_OK;
        }
    }
    // parts from the end: kTailPart blocks last, kBodyPart before it, the first part the rest; the
    // chain of a part (2.7 ns per block) hides under the next part's streaming (~14 ns per block),
    // only the last part's chain is exposed (A/B, profiles/r03/metrics_exact_ab.txt: equal parts
    // of 4096 blocks 472 us, sizes shrinking geometrically toward the end lost to the extra launches)
    int64_t bounds[kMaxParts + 1];
    int nparts = 0;
    {
        int64_t sizes[kMaxParts], left = nbf;
        while (left > 0) {
            const int64_t want = nparts == 0 ? kTailPart : kBodyPart;
            const int64_t take = nparts == kMaxParts - 1 || left <= want ? left : want;
            sizes[nparts++] = take;
            left -= take;
        }
        bounds[0] = 0;
        for (int q = 0; q < nparts; ++q) bounds[q + 1] = bounds[q] + sizes[nparts - 1 - q];
    }
    int slot = 0;
    int64_t prev_lo = 0, prev_hi = 0;  // the part whose chain runs in the next launch
    for (int k = 0; k < nparts; ++k) {
        const int64_t lo = bounds[k], hi = bounds[k + 1];
        const int64_t want = (hi - lo + kBlock / kWave - 1) / (kBlock / kWave);
        const int g = (int)(want > kMetricBlocks ? kMetricBlocks : want);
        const unsigned grid = (unsigned)g + (prev_hi > prev_lo ? 1u : 0u);
        if constexpr (std::is_same_v<FT, uint8_t>) {  // (not 16-byte aligned)
            hipLaunchKernelGGL(metrics_blocks, dim3(grid), dim3(kBlock), 0, stream, ideal, fixed, bsum, nb, lo, hi,
                               prev_lo, prev_hi, state, parts + slot);
        } else {
            hipLaunchKernelGGL(metrics_blocks_any<FT>, dim3(grid), dim3(kBlock), 0, stream, ideal, fixed, bsum, nb, lo,
                               hi, prev_lo, prev_hi, state, parts + slot);
        }
        slot += g;
        prev_lo = lo, prev_hi = hi;
    }
    if (nb > nbf) {  // the ragged last block (its sum is the last in order)
        hipLaunchKernelGGL(metrics_ragged<FT>, dim3(1), dim3(kBlock), 0, stream, ideal, fixed, n, bsum, nb, parts + slot);
        ++slot;
    }
    hipLaunchKernelGGL(metrics_final, dim3(1), dim3(kBlock), 0, stream, (const double*)bsum, nb, prev_lo, state,
                       (const Cnt*)parts, slot, n, out);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return *err = std::string("metrics launch failed: ") + hipGetErrorString(e), FIR_EHIP;
    return FIR_OK;
}

}  // namespace

int metrics_dtype_size(int dt) {
    switch (dt) {
        case FIR_DT_U8: case FIR_DT_I8: return 1;
        case FIR_DT_U16: case FIR_DT_I16: case FIR_DT_F16: return 2;
        case FIR_DT_U32: case FIR_DT_I32: case FIR_DT_F32: return 4;
        case FIR_DT_U64: case FIR_DT_I64: case FIR_DT_F64: return 8;
        default: return 0;
    }
}

int launch_metrics(const double* ideal, const void* fixed, int fixed_dtype, int64_t n, double* out, void* work,
                   hipStream_t stream, std::string* err) {
    if (n < 0) return *err = "n must be >= 0", FIR_EINVAL;
    if (!out || !work || (n > 0 && (!ideal || !fixed))) return *err = "null pointer argument", FIR_EINVAL;
    const int es = metrics_dtype_size(fixed_dtype);
    if (!es) return *err = "unknown fixed dtype", FIR_EINVAL;
    switch (fixed_dtype) {
        case FIR_DT_U8: return launch_metrics_t(ideal, (const uint8_t*)fixed, n, out, work, stream, err);
        case FIR_DT_I8: return launch_metrics_t(ideal, (const int8_t*)fixed, n, out, work, stream, err);
        case FIR_DT_U16: return launch_metrics_t(ideal, (const uint16_t*)fixed, n, out, work, stream, err);
        case FIR_DT_I16: return launch_metrics_t(ideal, (const int16_t*)fixed, n, out, work, stream, err);
        case FIR_DT_U32: return launch_metrics_t(ideal, (const uint32_t*)fixed, n, out, work, stream, err);
        case FIR_DT_I32: return launch_metrics_t(ideal, (const int32_t*)fixed, n, out, work, stream, err);
        case FIR_DT_U64: return launch_metrics_t(ideal, (const uint64_t*)fixed, n, out, work, stream, err);
        case FIR_DT_I64: return launch_metrics_t(ideal, (const int64_t*)fixed, n, out, work, stream, err);
        case FIR_DT_F16: return launch_metrics_t(ideal, (const _Float16*)fixed, n, out, work, stream, err);
        case FIR_DT_F32: return launch_metrics_t(ideal, (const float*)fixed, n, out, work, stream, err);
        default: return launch_metrics_t(ideal, (const double*)fixed, n, out, work, stream, err);
    }
}

}  // namespace fir
