// mfma_i8_layout.hip — checks the lane map of v_mfma_i32_32x32x32_i8 on exact integers (dev tool).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));
// hypothesis: lane l (r = l&31, h = l>>5) holds A[r][16h + j], B[16h + j][r], j = 0..15 (byte j of the 16-byte operand)
__global__ void k(const signed char* A, const signed char* B, int* D) {
    const int l = threadIdx.x, r = l & 31, h = l >> 5;
    i32x4 a, b;
    signed char* pa = (signed char*)&a; signed char* pb = (signed char*)&b;
    for (int j = 0; j < 16; ++j) { pa[j] = A[r * 32 + 16 * h + j]; pb[j] = B[(16 * h + j) * 32 + r]; }
    i32x16 c = {};
    c = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c, 0, 0, 0);
    for (int i = 0; i < 16; ++i) { int row = (i & 3) + 8 * (i >> 2) + 4 * h; D[row * 32 + r] = c[i]; }
}
int main() {
    signed char hA[1024], hB[1024]; int hD[1024], ref[1024];
    srand(1);
    for (int i = 0; i < 1024; ++i) { hA[i] = (signed char)(rand() % 256 - 128); hB[i] = (signed char)(rand() % 256 - 128); }
    for (int i = 0; i < 32; ++i) for (int j = 0; j < 32; ++j) { int s = 0; for (int q = 0; q < 32; ++q) s += hA[i*32+q] * hB[q*32+j]; ref[i*32+j] = s; }
    signed char *dA, *dB; int* dD;
    hipMalloc(&dA, 1024); hipMalloc(&dB, 1024); hipMalloc(&dD, 4096);
    hipMemcpy(dA, hA, 1024, hipMemcpyHostToDevice); hipMemcpy(dB, hB, 1024, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dD);
    hipMemcpy(hD, dD, 4096, hipMemcpyDeviceToHost);
    int bad = 0; for (int i = 0; i < 1024; ++i) bad += hD[i] != ref[i];
    printf("i8 32x32x32 layout hypothesis: %d / 1024 mismatches (D[0]=%d ref %d)\n", bad, hD[0], ref[0]);
    return bad != 0;
}
