// Probe: operand lane layout of v_mfma_scale_f32_32x32x64_f8f6f4 (fp8 e4m3, unit scales) on gfx950.
// Hypotheses for lane l (r = l&31, h = l>>5), byte j of the 32-byte operand:
//   H1: k = 32h + j            H2: k = (j<16) ? 16h + j : 32 + 16h + (j-16)
// A[r][k], B[k][c] are small integers (exact in e4m3); C compared with a CPU product.
#include <hip/hip_runtime.h>
#include <hip/hip_fp8.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

__global__ void k(const v8i* a, const v8i* b, float* c) {
    int l = threadIdx.x;
    v16f acc = {};
    acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a[l], b[l], acc, 0, 0, 0, 0x7f, 0, 0x7f);
    for (int i = 0; i < 16; ++i) {
        int row = (i & 3) + 8 * (i >> 2) + 4 * (l >> 5), col = l & 31;
        c[row * 32 + col] = acc[i];
    }
}

static unsigned char enc(float x) { __hip_fp8_e4m3 v(x); return *(unsigned char*)&v; }

int main() {
    float A[32][64], B[64][32], C[32][32];
    srand(1);
    for (int r = 0; r < 32; ++r) for (int kk = 0; kk < 64; ++kk) A[r][kk] = (float)(rand() % 5 - 2);
    for (int kk = 0; kk < 64; ++kk) for (int c = 0; c < 32; ++c) B[kk][c] = (float)(rand() % 7 - 3);
    for (int r = 0; r < 32; ++r) for (int c = 0; c < 32; ++c) {
        float s = 0; for (int kk = 0; kk < 64; ++kk) s += A[r][kk] * B[kk][c]; C[r][c] = s; }
    v8i *da, *db; float* dc;
    hipMalloc(&da, 64 * 32); hipMalloc(&db, 64 * 32); hipMalloc(&dc, 32 * 32 * 4);
    for (int hyp = 1; hyp <= 2; ++hyp) {
        unsigned char ha[64][32], hb[64][32];
        for (int l = 0; l < 64; ++l) {
            int r = l & 31, h = l >> 5;
            for (int j = 0; j < 32; ++j) {
                int kk = hyp == 1 ? 32 * h + j : (j < 16 ? 16 * h + j : 32 + 16 * h + (j - 16));
                ha[l][j] = enc(A[r][kk]);
                hb[l][j] = enc(B[kk][r]);
            }
        }
        hipMemcpy(da, ha, sizeof ha, hipMemcpyHostToDevice);
        hipMemcpy(db, hb, sizeof hb, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, da, db, dc);
        float out[32 * 32];
        hipMemcpy(out, dc, sizeof out, hipMemcpyDeviceToHost);
        float err = 0;
        for (int i = 0; i < 1024; ++i) err = fmaxf(err, fabsf(out[i] - C[i / 32][i % 32]));
        printf("H%d max |err| = %g\n", hyp, err);
    }
    return 0;
}
