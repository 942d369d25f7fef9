/*
 * oracle/fir_oracle.c — CPU oracle for the fixed-point FIR hot path.
 * TEST INFRASTRUCTURE ONLY: linked only by tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg (as the checker / reported CPU baseline), never by
 * the product library.
 *
 * Plain-C restatement of the reference arithmetic (paths relative to the
 * reference root), pinned by the tests/golden fixtures (vectors produced by the reference):
 *   MAC loop, same-mode, centre-aligned, zero padded
 *        fir_1d/model/python/fir_1d_fixed_ref.py:95-107
 *   wrap to acc_bits + sign extend          fir_1d_fixed_ref.py:94,110-115
 *   + 2^(f-1), arithmetic >> f              fir_1d_fixed_ref.py:118-120
 *   saturate to [0,255]                     fir_1d_fixed_ref.py:123-126
 *   row-wise application                    fir_1d/sim/vector/gen_fixed_output.py:34-60
 * plus the build-defined variants a6 (int16 -> int32, no clamp / no saturation),
 * a7 (interleaved complex channels, real taps) and a8 (2-D, centre-aligned);
 * see oracle/fir_oracle.py for their definitions.
 *
 * Index convention: y[n] = sum_k hq[k] * x[n - k + c], c = L/2.
 * Sums are accumulated mod 2^64 (uint64: exact for the wrap to acc_bits < 64, and the true
 * sum for acc_bits >= 64 while |sum| < 2^63, which the library checks).
 */
#include <stdint.h>
#include <stddef.h>
#ifdef _OPENMP
#include <omp.h>
#endif

enum { OR_IN_U8 = 0, OR_IN_I16 = 1 };
enum { OR_OUT_U8_SAT = 0, OR_OUT_I32 = 1 };

static inline int64_t wrap_round(int64_t acc, int frac_bits, int acc_bits) {
    if (acc_bits < 64) {
        const int s = 64 - acc_bits;
        acc = (int64_t)((uint64_t)acc << s) >> s; /* gcc: arithmetic >> on signed */
    }
    /* (v + 2^(f-1)) >> f on unbounded ints == (v >> f) + bit (f-1) of v; 0 for f >= 64, |v| < 2^63 */
    if (frac_bits >= 64) return 0;
    return (acc >> frac_bits) + ((acc >> (frac_bits - 1)) & 1);
}

static inline int64_t load_sample(const void* x, int in_dtype, int64_t i) {
    return in_dtype == OR_IN_U8 ? (int64_t)((const uint8_t*)x)[i] : (int64_t)((const int16_t*)x)[i];
}

static inline void store_out(void* y, int out_stage, int64_t i, int64_t q) {
    if (out_stage == OR_OUT_U8_SAT) {
        ((uint8_t*)y)[i] = (uint8_t)(q < 0 ? 0 : (q > 255 ? 255 : q));
    } else {
        ((int32_t*)y)[i] = (int32_t)q;
    }
}

/* Generic row-wise 1-D FIR.  Row r holds width*channels interleaved samples.
 * halo_left / halo_right (nullable, same dtype as x, only with rows == 1) supply the
 * (L-1-c)*channels samples before and c*channels samples after the row instead of zeros. */
int oracle_fir1d_rows(const void* x, int in_dtype, int64_t rows, int64_t width, int channels,
                      const int32_t* hq, int L, int frac_bits, int acc_bits, int out_stage,
                      const void* halo_left, const void* halo_right, void* y, int nthreads) {
    if (!x || !hq || !y || L < 1 || rows < 0 || width < 0 || channels < 1) return 1;
    if ((halo_left || halo_right) && rows != 1) return 1;
    const int c = L / 2;
    const int HL = L - 1 - c;
    const int64_t rowlen = width * channels;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
    /* fast path (acc_bits == 32): interior outputs in vectorisable uint32 wrap-around
     * arithmetic (exact mod 2^32, which is all the 32-bit wrap needs) */
    const int fast = (acc_bits == 32 && frac_bits >= 1 && frac_bits <= 31 && L <= 64);
    const int64_t nblk = (width + 4095) / 4096;
    /* one parallel loop over (row, 4096-output block) so narrow rows parallelise too */
#pragma omp parallel for schedule(static)
    for (int64_t t = 0; t < rows * nblk; ++t) {
        const int64_t r = t / nblk, blk = t % nblk;
        const int64_t base = r * rowlen;
        const int64_t lo = (int64_t)HL, hi = width - c; /* outputs with no padding */
        const int64_t n0 = blk * 4096;
        const int64_t n1 = n0 + 4096 < width ? n0 + 4096 : width;
        for (int64_t n = n0; n < n1; ++n) {
            if (fast && n >= lo && n < hi) {
                const int64_t run_end = hi < n1 ? hi : n1;
                const int64_t m0 = n * channels, m1 = run_end * channels;
                if (in_dtype == OR_IN_I16) {
                    const int16_t* xs = (const int16_t*)x + base;
                    for (int64_t m = m0; m < m1; ++m) {
                        uint32_t a = 0;
                        for (int k = 0; k < L; ++k)
                            a += (uint32_t)hq[k] * (uint32_t)(int32_t)xs[m + (int64_t)(c - k) * channels];
                        const int32_t s = (int32_t)a;
                        store_out(y, out_stage, base + m, (s >> frac_bits) + ((s >> (frac_bits - 1)) & 1));
                    }
                } else {
                    const uint8_t* xs = (const uint8_t*)x + base;
                    for (int64_t m = m0; m < m1; ++m) {
                        uint32_t a = 0;
                        for (int k = 0; k < L; ++k)
                            a += (uint32_t)hq[k] * (uint32_t)xs[m + (int64_t)(c - k) * channels];
                        const int32_t s = (int32_t)a;
                        store_out(y, out_stage, base + m, (s >> frac_bits) + ((s >> (frac_bits - 1)) & 1));
                    }
                }
                n = run_end - 1;
                continue;
            }
            for (int ch = 0; ch < channels; ++ch) {
                uint64_t acc = 0;
                for (int k = 0; k < L; ++k) {
                    const int64_t idx = n - k + c;
                    int64_t v = 0;
                    if (idx >= 0 && idx < width) {
                        v = load_sample(x, in_dtype, base + idx * channels + ch);
                    } else if (idx < 0 && halo_left) {
                        v = load_sample(halo_left, in_dtype, (HL + idx) * channels + ch);
                    } else if (idx >= width && halo_right) {
                        v = load_sample(halo_right, in_dtype, (idx - width) * channels + ch);
                    }
                    acc += (uint64_t)((int64_t)hq[k] * v);
                }
                store_out(y, out_stage, base + n * channels + ch, wrap_round(acc, frac_bits, acc_bits));
            }
        }
    }
    return 0;
}

/* 2-D FIR (a8): y[i,j] = stage(wrap(sum_m sum_n hq[m*C+n] * x[i-m+R/2][j-n+C/2])). */
int oracle_fir2d(const uint8_t* x, int64_t H, int64_t W, const int32_t* hq, int R, int C,
                 int frac_bits, int acc_bits, int out_stage, void* y, int nthreads) {
    if (!x || !hq || !y || R < 1 || C < 1 || H < 0 || W < 0) return 1;
    const int cr = R / 2, cc = C / 2;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < H; ++i) {
        for (int64_t j = 0; j < W; ++j) {
            uint64_t acc = 0;
            for (int m = 0; m < R; ++m) {
                const int64_t ii = i - m + cr;
                if (ii < 0 || ii >= H) continue;
                for (int n = 0; n < C; ++n) {
                    const int64_t jj = j - n + cc;
                    if (jj < 0 || jj >= W) continue;
                    acc += (uint64_t)((int64_t)hq[m * C + n] * (int64_t)x[ii * W + jj]);
                }
            }
            store_out(y, out_stage, i * W + j, wrap_round(acc, frac_bits, acc_bits));
        }
    }
    return 0;
}

/* Reference fir_1d_ideal per row (fir_1d/model/python/fir_1d_ref.py:43-65):
 * float64, k-order, products and sums rounded separately (built with -ffp-contract=off). */
int oracle_fir1d_ideal_rows(const uint8_t* x, int64_t rows, int64_t width, const double* h, int L,
                            double* y, int nthreads) {
    if (!x || !h || !y || L < 1) return 1;
    const int c = L / 2;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
#pragma omp parallel for schedule(static)
    for (int64_t r = 0; r < rows; ++r) {
        for (int64_t n = 0; n < width; ++n) {
            double acc = 0.0;
            for (int k = 0; k < L; ++k) {
                const int64_t idx = n - k + c;
                if (idx >= 0 && idx < width) {
                    volatile double t = h[k] * (double)x[r * width + idx];
                    acc = acc + t;
                }
            }
            y[r * width + n] = acc;
        }
    }
    return 0;
}
