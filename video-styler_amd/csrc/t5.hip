// UMT5-XXL text encoder kernels (diffsynth/models/wan_video_text_encoder.py) for gfx950.  The
// encoder's GEMMs, RMS norms and the per-head QK^T / PV products reuse vs_gemm, vs_rmsnorm_rope
// and the batched-GEMM mode of vs_vae_conv; these kernels cover what is T5-specific:
//  * token embedding row gather;
//  * attention scores -> probabilities with the per-block relative-position bias, the padding mask
//    and the reference's bf16 rounding points (bf16 scores, bf16 bias add, fp32 softmax, bf16 P);
//  * the gated FFN product fc1(x) * GELU(gate(x)) with the GELU evaluated as the reference's chain
//    of bf16 tensor ops.
#include "common.h"

namespace {

__global__ __launch_bounds__(256) void embed_rows_kernel(const long long* __restrict__ ids,
                                                         const bf16_t* __restrict__ table, long long ld_table,
                                                         bf16_t* __restrict__ out, long long ld_out, int dim,
                                                         long long vocab) {
    const long long row = blockIdx.x;
    const long long id = ids[row];
    if (id < 0 || id >= vocab) return;          // validated on the host; never read out of range
    const u32x4_t* src = reinterpret_cast<const u32x4_t*>(table + id * ld_table);
    u32x4_t* dst = reinterpret_cast<u32x4_t*>(out + row * ld_out);
    for (int c = threadIdx.x; c < dim / 8; c += 256) dst[c] = src[c];
}

// One wave per score row (z = head, i = query).  s: fp32 scores [nz][L][ld_s]; p: bf16 [nz][L][ld_p]
// with columns L..ld_p-1 zeroed.  bias(i, j) = emb[bucket[i*L + j]][head0 + z] (bf16), replaced by
// the bf16 lowest value where keymask[j] == 0 (T5Attention.forward :69-83).
__global__ __launch_bounds__(256) void t5_bias_softmax_kernel(const float* __restrict__ s, long long zs_s,
                                                              long long ld_s, bf16_t* __restrict__ p, long long zs_p,
                                                              long long ld_p, const int* __restrict__ buckets,
                                                              const bf16_t* __restrict__ emb, int nheads, int head0,
                                                              const int* __restrict__ keymask, int L, int nz) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= nz * L) return;
    const int z = row / L, i = row % L;
    const float* sr = s + z * zs_s + (long long)i * ld_s;
    bf16_t* pr = p + z * zs_p + (long long)i * ld_p;
    const int* br = buckets + (long long)i * L;
    const float lowest = -3.3895313892515355e38f;   // torch.finfo(torch.bfloat16).min
    float mx = -INFINITY;
    for (int j = lane; j < L; j += 64) {
        const float bias = keymask[j] ? bf2f(emb[br[j] * nheads + head0 + z]) : lowest;
        mx = fmaxf(mx, rbf(rbf(sr[j]) + bias));
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    float sum = 0.f;
    for (int j = lane; j < L; j += 64) {
        const float bias = keymask[j] ? bf2f(emb[br[j] * nheads + head0 + z]) : lowest;
        sum += expf(rbf(rbf(sr[j]) + bias) - mx);
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) sum += __shfl_xor(sum, o);
    for (int j = lane; j < ld_p; j += 64) {
        float v = 0.f;
        if (j < L) {
            const float bias = keymask[j] ? bf2f(emb[br[j] * nheads + head0 + z]) : lowest;
            v = expf(rbf(rbf(sr[j]) + bias) - mx) / sum;
        }
        pr[j] = (bf16_t)f2bf(v);
    }
}

// out = bf16(a * gelu(g)), gelu = 0.5*x*(1 + tanh(sqrt(2/pi)*(x + 0.044715*x^3))) one bf16 op at a
// time (GELU.forward :15-19 on a bf16 tensor; T5FeedForward.forward :105-110).
__global__ __launch_bounds__(256) void t5_gelu_mul_kernel(const bf16_t* __restrict__ a, const bf16_t* __restrict__ g,
                                                          bf16_t* __restrict__ out, long long n) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float x = bf2f(g[i]);
    const float x3 = rbf(x * x * x);
    const float t1 = rbf(0.044715f * x3);
    const float t2 = rbf(x + t1);
    const float t3 = rbf(0.7978845608028654f * t2);
    const float t4 = rbf(tanhf(t3));
    const float t5 = rbf(1.0f + t4);
    const float t6 = rbf(0.5f * x);
    const float ge = rbf(t6 * t5);
    out[i] = (bf16_t)f2bf(bf2f(a[i]) * ge);
}

}  // namespace

extern "C" int vs_embed_rows(const long long* ids, const void* table, long long ld_table, long long vocab, void* out,
                             long long ld_out, long long rows, int dim, void* stream) {
    if (!ids || !table || !out || rows <= 0 || dim <= 0 || dim % 8 || ld_table % 8 || ld_out % 8 || vocab <= 0)
        return VS_E_INVALID;
    hipLaunchKernelGGL(embed_rows_kernel, dim3((unsigned)rows), dim3(256), 0, (hipStream_t)stream, ids,
                       (const bf16_t*)table, ld_table, (bf16_t*)out, ld_out, dim, vocab);
    VS_CHECK_LAUNCH();
    return VS_OK;
}

extern "C" int vs_t5_bias_softmax(const float* s, long long zs_s, long long ld_s, void* p, long long zs_p,
                                  long long ld_p, const int* buckets, const void* emb, int nheads, int head0,
                                  const int* keymask, int L, int nz, void* stream) {
    if (!s || !p || !buckets || !emb || !keymask || L <= 0 || nz <= 0 || ld_s < L || ld_p < L ||
        head0 < 0 || head0 + nz > nheads)
        return VS_E_INVALID;
    const long long rows = (long long)nz * L;
    hipLaunchKernelGGL(t5_bias_softmax_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, (hipStream_t)stream,
                       s, zs_s, ld_s, (bf16_t*)p, zs_p, ld_p, buckets, (const bf16_t*)emb, nheads, head0, keymask, L,
                       nz);
    VS_CHECK_LAUNCH();
    return VS_OK;
}

extern "C" int vs_t5_gelu_mul(const void* a, const void* g, void* out, long long n, void* stream) {
    if (!a || !g || !out || n <= 0) return VS_E_INVALID;
    hipLaunchKernelGGL(t5_gelu_mul_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       (const bf16_t*)a, (const bf16_t*)g, (bf16_t*)out, n);
    VS_CHECK_LAUNCH();
    return VS_OK;
}
