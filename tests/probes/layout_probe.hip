// Probe of the gfx950 operand/result layouts the attention kernel relies on.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef short i16x4_t __attribute__((ext_vector_type(4)));

__global__ void mfma32(const float* A, const float* B, float* C) {  // A[32][16], B[16][32]
    int l = threadIdx.x, r = l & 31, h = l >> 5;
    bf16x8_t a, b;
    for (int j = 0; j < 8; ++j) { a[j] = (__bf16)A[r * 16 + 8 * h + j]; b[j] = (__bf16)B[(8 * h + j) * 32 + r]; }
    f32x16_t c = {};
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
    for (int i = 0; i < 16; ++i) C[((i & 3) + 8 * (i >> 2) + 4 * h) * 32 + r] = c[i];
}
__global__ void tr(short* out) {
    __shared__ __attribute__((aligned(16))) short lds[8 * 64];
    for (int i = threadIdx.x; i < 8 * 64; i += 64) lds[i] = (short)i;   // row = i/64, col = i%64
    __syncthreads();
    int l = threadIdx.x, g = l >> 4, q = (l & 15) >> 2, p = l & 3;
    // group g reads rows g..g+3? use block rows 0..3, columns 16g .. 16g+15
    short* addr = lds + q * 64 + 16 * g + 4 * p;
    i16x4_t v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) i16x4_t*)addr);
    for (int e = 0; e < 4; ++e) out[l * 4 + e] = v[e];
}
int main() {
    float hA[512], hB[512], hC[1024], ref[1024];
    for (int r = 0; r < 32; ++r) for (int k = 0; k < 16; ++k) hA[r * 16 + k] = (float)((r + 2 * k) % 5 - 2);
    for (int k = 0; k < 16; ++k) for (int c = 0; c < 32; ++c) hB[k * 32 + c] = (float)((3 * k + c * c) % 7 - 3);
    for (int r = 0; r < 32; ++r) for (int c = 0; c < 32; ++c) { float s = 0; for (int k = 0; k < 16; ++k) s += hA[r*16+k]*hB[k*32+c]; ref[r*32+c] = s; }
    float *dA, *dB, *dC; short* dT;
    hipMalloc(&dA, 2048); hipMalloc(&dB, 2048); hipMalloc(&dC, 4096); hipMalloc(&dT, 512);
    hipMemcpy(dA, hA, 2048, hipMemcpyHostToDevice); hipMemcpy(dB, hB, 2048, hipMemcpyHostToDevice);
    mfma32<<<1, 64>>>(dA, dB, dC); hipMemcpy(hC, dC, 4096, hipMemcpyDeviceToHost);
    int bad = 0; for (int i = 0; i < 1024; ++i) bad += hC[i] != ref[i];
    printf("mfma32x32x16 layout: %d mismatches of 1024\n", bad);
    if (bad) { for (int r = 0; r < 4; ++r) { for (int c = 0; c < 8; ++c) printf("%5.0f/%-5.0f ", hC[r*32+c], ref[r*32+c]); printf("\n"); } }
    short hT[256];
    tr<<<1, 64>>>(dT); hipMemcpy(hT, dT, 512, hipMemcpyDeviceToHost);
    printf("ds_read_tr16_b64: lane -> 4 values (row*64+col)\n");
    for (int l = 0; l < 64; ++l) { printf("L%02d:", l); for (int e = 0; e < 4; ++e) printf(" %3d", hT[l*4+e]); printf(l % 4 == 3 ? "\n" : "  "); }
    return 0;
}
