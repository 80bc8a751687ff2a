// ds_read_b64_tr_b16 with arbitrary per-lane addresses: which lane's address feeds which result?
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
typedef short i16x4_t __attribute__((ext_vector_type(4)));
__global__ void tr(const int* addr_elems, short* out) {
    __shared__ __attribute__((aligned(16))) short lds[4096];
    for (int i = threadIdx.x; i < 4096; i += 64) lds[i] = (short)i;
    __syncthreads();
    int l = threadIdx.x;
    short* a = lds + addr_elems[l];
    i16x4_t v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) i16x4_t*)a);
    for (int e = 0; e < 4; ++e) out[l * 4 + e] = v[e];
}
int main() {
    int h_addr[64]; short h_out[256];
    srand(7);
    for (int l = 0; l < 64; ++l) h_addr[l] = (rand() % 1000) * 4;   // 8-byte aligned element offsets
    int* d_addr; short* d_out;
    (void)hipMalloc(&d_addr, sizeof(h_addr)); (void)hipMalloc(&d_out, sizeof(h_out));
    (void)hipMemcpy(d_addr, h_addr, sizeof(h_addr), hipMemcpyHostToDevice);
    tr<<<1, 64>>>(d_addr, d_out);
    (void)hipMemcpy(h_out, d_out, sizeof(h_out), hipMemcpyDeviceToHost);
    int bad = 0;
    for (int l = 0; l < 64; ++l) {
        int g = l >> 4, i = l & 15;
        for (int q = 0; q < 4; ++q) {
            int src_lane = 16 * g + 4 * q + (i >> 2);
            int expect = h_addr[src_lane] + (i & 3);
            if (h_out[l * 4 + q] != expect) bad++;
        }
    }
    printf("per-lane-address model (lane 4q+p supplies row q cols 4p..): %d mismatches of 256\n", bad);
    for (int l = 0; l < 8; ++l) { printf("L%d addr=%d got:", l, h_addr[l]); for (int e = 0; e < 4; ++e) printf(" %d", h_out[l*4+e]); printf("\n"); }
    for (int l = 0; l < 16; ++l) printf("addr[%d]=%d ", l, h_addr[l]);
    printf("\n");
    return 0;
}
