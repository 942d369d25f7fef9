// fir1d_reg_launch.h — declaration of the register-kernel launcher (defined in
// fir1d_reg_impl.h, explicitly instantiated by fir1d_reg_inst.hip per configuration).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fir {

// Launch fir1d_reg_kernel for L taps (1..9) of F filters over rows x rowlen samples of
// InT with CH interleaved channels; picks the dot2 / acc32 / u8 no-wrap variant.
template <typename InT, int STAGE, int CH, int F>
hipError_t launch_reg_taps(int L, const void* x, void* y, int64_t rows, int64_t total, int64_t rowlen,
                           const int32_t* hq, int frac, int acc_bits, hipStream_t s);

}  // namespace fir
