// alu_micro.hip — VALU throughput of the integer ops the FIR kernels use (dev tool).
// Each kernel runs 8 independent accumulator chains x N iterations per lane on a full grid
// (many waves per SIMD); reports wave-instructions per SIMD-cycle at the measured clock.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(e)                                                                              \
    do {                                                                                   \
        hipError_t _e = (e);                                                               \
        if (_e != hipSuccess) {                                                            \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(_e));      \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

typedef short s2 __attribute__((ext_vector_type(2)));
constexpr int kIters = 4096;

template <int OP>
__global__ __launch_bounds__(256) void alu(uint32_t* out, uint32_t a0, uint32_t b0) {
    uint32_t acc[8];
    uint32_t a = a0 + threadIdx.x, b = b0 ^ blockIdx.x;
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = threadIdx.x * (i + 1);
    for (int it = 0; it < kIters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if constexpr (OP == 0) acc[i] = (uint32_t)__builtin_amdgcn_sdot2(__builtin_bit_cast(s2, a + i), __builtin_bit_cast(s2, b), (int)acc[i], false);
            if constexpr (OP == 1) acc[i] = (uint32_t)__mul24((int)acc[i], (int)b) + (a + i);
            if constexpr (OP == 2) acc[i] += a + i;
            if constexpr (OP == 3) acc[i] = __builtin_amdgcn_perm(acc[i], a + i, b);
            if constexpr (OP == 4) acc[i] = acc[i] * (a + i) + b;  // v_mad_u32_u24? / v_mul_lo
            if constexpr (OP == 5) acc[i] = (uint32_t)__builtin_amdgcn_udot4(acc[i], a + i, b, false);
        }
    }
    uint32_t r = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) r ^= acc[i];
    out[blockIdx.x * 256 + threadIdx.x] = r;
}

int main() {
    const int blocks = 256 * 16;  // 16 x 256-thread blocks per CU -> 16 waves/SIMD requested
    uint32_t* out;
    CK(hipMalloc(&out, blocks * 256 * 4));
    const char* names[] = {"v_dot2c_i32_i16", "v_mad_i32_i24", "v_add_u32", "v_perm_b32", "v_mul_lo_u32",
                           "v_dot4_u32_u8"};
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](int op) {
        switch (op) {
            case 0: hipLaunchKernelGGL(alu<0>, dim3(blocks), dim3(256), 0, 0, out, 1u, 3u); break;
            case 1: hipLaunchKernelGGL(alu<1>, dim3(blocks), dim3(256), 0, 0, out, 1u, 3u); break;
            case 2: hipLaunchKernelGGL(alu<2>, dim3(blocks), dim3(256), 0, 0, out, 1u, 3u); break;
            case 3: hipLaunchKernelGGL(alu<3>, dim3(blocks), dim3(256), 0, 0, out, 1u, 0x05040100u); break;
            case 4: hipLaunchKernelGGL(alu<4>, dim3(blocks), dim3(256), 0, 0, out, 1u, 3u); break;
            case 5: hipLaunchKernelGGL(alu<5>, dim3(blocks), dim3(256), 0, 0, out, 1u, 3u); break;
        }
    };
    for (int op = 0; op < 6; ++op) run(op);
    CK(hipDeviceSynchronize());
    const double wave_instr = (double)blocks * 4 * kIters * 8;  // per op kind
    printf("%-20s %10s %14s %s\n", "op", "ms", "wave-instr/us", "cycles/wave-instr/SIMD @2.4GHz");
    for (int op = 0; op < 6; ++op) {
        float best = 1e9;
        for (int r = 0; r < 5; ++r) {
            CK(hipEventRecord(e0));
            run(op);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = ms < best ? ms : best;
        }
        const double per_us = wave_instr / (best * 1e3);
        printf("%-20s %10.3f %14.1f %8.2f\n", names[op], best, per_us, 1024.0 * 2400.0 / per_us);
    }
    return 0;
}
