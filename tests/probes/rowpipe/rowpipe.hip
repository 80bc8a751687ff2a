// Probe (not product code): a persistent, software-pipelined LayerNorm+modulate -- each block walks
// rows blockIdx.x, += gridDim.x with the next row's x loads in flight during the current row's
// reductions, and the per-batch shift / scale rows held in registers -- against the library's one-
// block-per-row ln_modulate_kernel (same arithmetic: outputs must be bit-identical).
#include <hip/hip_runtime.h>
#include <stdint.h>
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

namespace {
constexpr int RT = 128, MC = 5;
__device__ __forceinline__ float bflo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bfhi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }
__device__ __forceinline__ uint32_t f2bf(float f) { return (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)f); }
__device__ __forceinline__ uint32_t pack2(float lo, float hi) { return f2bf(lo) | (f2bf(hi) << 16); }
__device__ __forceinline__ float rbf(float f) { return __uint_as_float(f2bf(f) << 16); }
__device__ __forceinline__ void unpack8(const u32x4_t& w, float* v) {
    for (int i = 0; i < 4; ++i) { v[2 * i] = bflo(w[i]); v[2 * i + 1] = bfhi(w[i]); }
}
__device__ __forceinline__ u32x4_t pack8(const float* v) {
    u32x4_t w;
    for (int i = 0; i < 4; ++i) w[i] = pack2(v[2 * i], v[2 * i + 1]);
    return w;
}
__device__ __forceinline__ float block_sum(float v, float* red) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    __syncthreads();
    if (lane == 0) red[w] = v;
    __syncthreads();
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < RT / 64; ++i) t += red[i];
    return t;
}

template <int WPS>
__global__ __launch_bounds__(RT, WPS) void ln_mod_pipe(const uint16_t* __restrict__ x, long long ldx,
                                                        uint16_t* __restrict__ out, long long ldo, int rows, int dim,
                                                        int rpb, const uint16_t* __restrict__ shift,
                                                        const uint16_t* __restrict__ scale, long long mbs, float eps) {
    __shared__ float red[RT / 64];
    const int nch = dim >> 3;
    long long row = blockIdx.x;
    u32x4_t cur[MC], nxt[MC], sh[MC], sc[MC];
    auto load = [&](long long r, u32x4_t* d) {
#pragma unroll
        for (int c = 0; c < MC; ++c) {
            const int ch = threadIdx.x + c * RT;
            if (ch < nch && r < rows) d[c] = *reinterpret_cast<const u32x4_t*>(x + r * ldx + ch * 8);
        }
    };
    long long mb = -1;
    load(row, cur);
    for (; row < rows; row += gridDim.x) {
        load(row + gridDim.x, nxt);
        float v[MC][8];
        float s = 0.f;
#pragma unroll
        for (int c = 0; c < MC; ++c) {
            const int ch = threadIdx.x + c * RT;
            if (ch < nch) {
                unpack8(cur[c], v[c]);
#pragma unroll
                for (int e = 0; e < 8; ++e) s += v[c][e];
            }
        }
        const long long bidx = row / rpb;
        if (bidx != mb) {
            mb = bidx;
#pragma unroll
            for (int c = 0; c < MC; ++c) {
                const int ch = threadIdx.x + c * RT;
                if (ch < nch) {
                    sh[c] = *reinterpret_cast<const u32x4_t*>(shift + bidx * mbs + ch * 8);
                    sc[c] = *reinterpret_cast<const u32x4_t*>(scale + bidx * mbs + ch * 8);
                }
            }
        }
        const float mean = block_sum(s, red) / dim;
        float q = 0.f;
#pragma unroll
        for (int c = 0; c < MC; ++c) {
            const int ch = threadIdx.x + c * RT;
            if (ch < nch)
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    const float d = v[c][e] - mean;
                    q += d * d;
                }
        }
        const float rstd = rsqrtf(block_sum(q, red) / dim + eps);
        uint16_t* orow = out + row * ldo;
#pragma unroll
        for (int c = 0; c < MC; ++c) {
            const int ch = threadIdx.x + c * RT;
            if (ch >= nch) continue;
            float y[8], shv[8], scv[8];
            unpack8(sh[c], shv);
            unpack8(sc[c], scv);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                y[e] = (v[c][e] - mean) * rstd;
                y[e] = rbf(rbf(rbf(y[e]) * rbf(1.f + scv[e])) + shv[e]);
            }
            *reinterpret_cast<u32x4_t*>(orow + ch * 8) = pack8(y);
        }
#pragma unroll
        for (int c = 0; c < MC; ++c) cur[c] = nxt[c];
    }
}
}  // namespace

extern "C" int rowpipe_ln(const void* x, long long ldx, void* out, long long ldo, int rows, int dim, int rpb,
                          const void* shift, const void* scale, long long mbs, float eps, int blocks, int wps,
                          void* stream) {
    if (dim > RT * MC * 8 || dim % 8) return 1;
    auto k = wps == 2 ? ln_mod_pipe<2> : wps == 4 ? ln_mod_pipe<4> : ln_mod_pipe<1>;
    hipLaunchKernelGGL(k, dim3(blocks), dim3(RT), 0, (hipStream_t)stream, (const uint16_t*)x, ldx,
                       (uint16_t*)out, ldo, rows, dim, rpb, (const uint16_t*)shift, (const uint16_t*)scale, mbs, eps);
    return hipGetLastError() == hipSuccess ? 0 : 2;
}
