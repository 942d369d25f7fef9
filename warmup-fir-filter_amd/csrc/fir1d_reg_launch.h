// fir1d_reg_launch.h — declaration of the register-kernel launcher (defined in
// fir1d_reg_impl.h, explicitly instantiated by fir1d_reg_inst.hip per configuration).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fir {

// Launch fir1d_reg_kernel for L taps (1..9) of F filters over rows x rowlen samples of
// InT with CH interleaved channels; picks the dot2 / acc32 / u8 no-wrap variant.
// halo_l / halo_r (rows == 1, total a multiple of reg_tile_samples): device samples around
// the row that replace its zero padding (RowGeom::halo_l / halo_r).
template <typename InT, int STAGE, int CH, int F>
hipError_t launch_reg_taps(int L, const void* x, void* y, int64_t rows, int64_t total, int64_t rowlen,
                           const int32_t* hq, int frac, int acc_bits, hipStream_t s, const void* halo_l = nullptr,
                           const void* halo_r = nullptr);

constexpr int kRegBatch = 8;  // images per batch launch

// One image of a batch: rows x rowlen samples at x (16-byte aligned, rowlen >= a vector + L - 1
// when rows > 1), output plane f (f < F <= 4) at y[f], any byte.
struct RegImage {
    const void* x;
    void* y[4];
    int64_t rows, rowlen;
};

// ONE launch over n <= kRegBatch (8) images, u8 stage, one channel (other configurations:
// hipErrorInvalidValue); picks the variant as launch_reg_taps does.
template <typename InT, int STAGE, int CH, int F>
hipError_t launch_reg_batch_taps(int L, int n, const RegImage* im, const int32_t* hq, int frac, int acc_bits,
                                 hipStream_t s);

// Chunks of 64 vectors per wave (the tile), by sample type and filter count (rationale and
// measurements: fir1d_reg_impl.h).
template <typename InT, int F>
constexpr int kRegU = sizeof(InT) == 1 && F == 1 ? 4 : 1;

// Samples per wave tile of the single-filter register kernel (64 lanes x U chunks x 16 bytes).
inline int64_t reg_tile_samples(bool u8) { return u8 ? 64 * kRegU<uint8_t, 1> * 16 : 64 * kRegU<int16_t, 1> * 8; }

}  // namespace fir
