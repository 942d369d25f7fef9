// fir1d_reg_inst.hip — one explicit instantiation of the register-kernel launcher per
// object file: the Makefile compiles this file once per (InT, STAGE, CH, F) configuration
// the dispatchers in fir1d.hip use, in parallel.
#include "fir1d_reg_impl.h"

namespace fir {
template hipError_t launch_reg_taps<FIR_INST_T, FIR_INST_STAGE, FIR_INST_CH, FIR_INST_F>(
    int L, const void* x, void* y, int64_t rows, int64_t total, int64_t rowlen, const int32_t* hq, int frac,
    int acc_bits, hipStream_t s, const void* halo_l, const void* halo_r);
template hipError_t launch_reg_batch_taps<FIR_INST_T, FIR_INST_STAGE, FIR_INST_CH, FIR_INST_F>(
    int L, int n, const RegImage* im, const int32_t* hq, int frac, int acc_bits, hipStream_t s);
}  // namespace fir
