// HBM-bound row/elementwise kernels of the Wan2.1 DiT path, gfx950.
// All loads/stores are 16-B vectorised (8 bf16 per lane); normalisations keep the row in
// registers between the reduction and the write (one HBM read + one write per element).
#include "common.h"

namespace {

#ifndef VS_RT
#define VS_RT 128
#define VS_MAXCH 5
#endif
// threads per row-kernel block / 8-element chunks per thread (dim <= RT * MAXCH * 8 = 5120; wider rows
// up to 8192 on an 8-chunk instantiation, ROW_MAX).  r5:
// 128 threads x 5 chunks instead of 256 x 3 -- LayerNorm+modulate at 59 280 x 5120 309-317 -> 279-289 us
// (the 256-thread rows split 640 chunks 3 / 2 unevenly); 320 and 640 threads were slower
// (profiles/r5/rowkernel_threads_ab_s41.log)
constexpr int RT = VS_RT;
constexpr int MAXCH = VS_MAXCH;

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

__device__ __forceinline__ void unpack8(const u32x4_t& w, float* v) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        v[2 * i] = bflo(w[i]);
        v[2 * i + 1] = bfhi(w[i]);
    }
}
__device__ __forceinline__ u32x4_t pack8(const float* v) {
    u32x4_t w;
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = pack2(v[2 * i], v[2 * i + 1]);
    return w;
}

__device__ __forceinline__ float block_max(float v, float* red) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    __syncthreads();
    if (lane == 0) red[w] = v;
    __syncthreads();
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < RT / 64; ++i) t = fmaxf(t, red[i]);
    return t;
}

// LayerNorm (fp32, eps) [affine] -> bf16, then optional modulate  (layers.py:89-91,
// wan_video_dit.py:64-65): out = bf16(bf16(n * bf16(1 + scale)) + shift).
// Q8 (r5, config 5): the row is not stored as bf16 but handed straight to fp8_linear's activation
// quantisation (layers.py:115-151, vs_quant_fp8_rows): per-row s = max(bf16(max|h| / 448), 1) and
// e4m3(h / (s + 1e-8)) of the bf16 values h the plain kernel would store -- bit-identical to the two
// passes, without the bf16 write and the quantisation's read (the row's consumer is an fp8 GEMM).
template <bool Q8, int MC = MAXCH>
__global__ __launch_bounds__(RT) void ln_modulate_kernel(
    const bf16_t* __restrict__ x, long long ldx, bf16_t* __restrict__ out, long long ldo, int dim,
    int rpb, const bf16_t* __restrict__ shift, const bf16_t* __restrict__ scale, long long mbs,
    const bf16_t* __restrict__ w, const bf16_t* __restrict__ bb, float eps, uint8_t* __restrict__ x8,
    long long ld8, float* __restrict__ qscale) {
    __shared__ float red[RT / 64];
    const long long row = blockIdx.x;
    const int nch = dim >> 3;
    const bf16_t* xr = x + row * ldx;
    float v[MC][8];
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < MC; ++c) {
        const int ch = threadIdx.x + c * RT;
        if (ch < nch) {
            unpack8(*reinterpret_cast<const u32x4_t*>(xr + ch * 8), v[c]);
#pragma unroll
            for (int e = 0; e < 8; ++e) s += v[c][e];
        }
    }
    const float mean = block_sum(s, red) / dim;
    float q = 0.f;
#pragma unroll
    for (int c = 0; c < MC; ++c) {
        const int ch = threadIdx.x + c * RT;
        if (ch < nch) {
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const float d = v[c][e] - mean;
                q += d * d;
            }
        }
    }
    const float rstd = rsqrtf(block_sum(q, red) / dim + eps);
    const long long bidx = row / rpb;
    bf16_t* orow = out + row * ldo;
#pragma unroll
    for (int c = 0; c < MC; ++c) {
        const int ch = threadIdx.x + c * RT;
        if (ch >= nch) continue;
        float y[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) y[e] = (v[c][e] - mean) * rstd;
        if (w) {
            float wv[8], bv[8];
            unpack8(*reinterpret_cast<const u32x4_t*>(w + ch * 8), wv);
            unpack8(*reinterpret_cast<const u32x4_t*>(bb + ch * 8), bv);
#pragma unroll
            for (int e = 0; e < 8; ++e) y[e] = y[e] * wv[e] + bv[e];
        }
        if (shift) {
            float sh[8], sc[8];
            unpack8(*reinterpret_cast<const u32x4_t*>(shift + bidx * mbs + ch * 8), sh);
            unpack8(*reinterpret_cast<const u32x4_t*>(scale + bidx * mbs + ch * 8), sc);
#pragma unroll
            for (int e = 0; e < 8; ++e) y[e] = rbf(rbf(rbf(y[e]) * rbf(1.f + sc[e])) + sh[e]);
        }
        if constexpr (Q8) {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[c][e] = rbf(y[e]);       // the bf16 row h, kept for the quantisation
        } else {
            *reinterpret_cast<u32x4_t*>(orow + ch * 8) = pack8(y);
        }
    }
    if constexpr (Q8) {
        float mx = 0.f;
#pragma unroll
        for (int c = 0; c < MC; ++c)
            if ((int)threadIdx.x + c * RT < nch)
#pragma unroll
                for (int e = 0; e < 8; ++e) mx = fmaxf(mx, fabsf(v[c][e]));
        mx = block_max(mx, red);
        const float s8 = fmaxf(rbf(mx / 448.0f), 1.0f);
        const float d = s8 + 1e-8f;
        if (threadIdx.x == 0) qscale[row] = s8;
        uint8_t* yr = x8 + row * ld8;
#pragma unroll
        for (int c = 0; c < MC; ++c) {
            const int ch = threadIdx.x + c * RT;
            if (ch >= nch) continue;
            u32x2_t o;
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                int t = __builtin_amdgcn_cvt_pk_fp8_f32(v[c][4 * e] / d, v[c][4 * e + 1] / d, 0, false);
                t = __builtin_amdgcn_cvt_pk_fp8_f32(v[c][4 * e + 2] / d, v[c][4 * e + 3] / d, t, true);
                o[e] = (uint32_t)t;
            }
            *reinterpret_cast<u32x2_t*>(yr + ch * 8) = o;
        }
    }
}

// Gated / plain residual add of a staged projection y (the hipBLASLt route's bf16(A W^T + bias))
// into x, then LayerNorm [+ affine] [+ modulate] of the updated row into out: the vs_gemm epilogue
// (VS_EPI_GATE_RES: x = bf16(x + bf16(gate*y)) [+ bf16(hint*s)]; VS_EPI_RES: x = bf16(x + bf16(alpha*y)))
// followed by ln_modulate_kernel's arithmetic on the stored bf16 row -- the same rounding points as
// the two separate passes, one read of x instead of two (wan_video_dit.py:225-228).
template <int MC = MAXCH>
__global__ __launch_bounds__(RT) void residual_ln_kernel(
    const bf16_t* __restrict__ y, long long ldy, bf16_t* __restrict__ x, long long ldx, bf16_t* __restrict__ out,
    long long ldo, int dim, int mode, const bf16_t* __restrict__ gate, long long gate_bstride, int rpb_gate,
    float alpha, const bf16_t* __restrict__ hint, long long ld_hint, float hint_scale, int rpb,
    const bf16_t* __restrict__ shift, const bf16_t* __restrict__ scale, long long mbs,
    const bf16_t* __restrict__ w, const bf16_t* __restrict__ bb, float eps) {
    __shared__ float red[RT / 64];
    const long long row = blockIdx.x;
    const int nch = dim >> 3;
    const bf16_t* yr = y + row * ldy;
    bf16_t* xr = x + row * ldx;
    const bf16_t* gr = gate ? gate + (row / rpb_gate) * gate_bstride : nullptr;
    float v[MC][8];
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < MC; ++c) {
        const int ch = threadIdx.x + c * RT;
        if (ch < nch) {
            float yv[8], xv[8];
            unpack8(*reinterpret_cast<const u32x4_t*>(yr + ch * 8), yv);
            unpack8(*reinterpret_cast<const u32x4_t*>(xr + ch * 8), xv);
            if (mode == VS_EPI_GATE_RES) {
                float gv[8];
                unpack8(*reinterpret_cast<const u32x4_t*>(gr + ch * 8), gv);
#pragma unroll
                for (int e = 0; e < 8; ++e) v[c][e] = rbf(xv[e] + rbf(gv[e] * yv[e]));
                if (hint) {
                    float hv[8];
                    unpack8(*reinterpret_cast<const u32x4_t*>(hint + row * ld_hint + ch * 8), hv);
#pragma unroll
                    for (int e = 0; e < 8; ++e) v[c][e] = v[c][e] + rbf(hv[e] * hint_scale);
                }
            } else {
#pragma unroll
                for (int e = 0; e < 8; ++e) v[c][e] = xv[e] + rbf(alpha * yv[e]);
            }
            const u32x4_t pk = pack8(v[c]);
            *reinterpret_cast<u32x4_t*>(xr + ch * 8) = pk;
            unpack8(pk, v[c]);                           // LayerNorm reads the stored bf16 row
#pragma unroll
            for (int e = 0; e < 8; ++e) s += v[c][e];
        }
    }
    const float mean = block_sum(s, red) / dim;
    float q = 0.f;
#pragma unroll
    for (int c = 0; c < MC; ++c) {
        const int ch = threadIdx.x + c * RT;
        if (ch < nch) {
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const float d = v[c][e] - mean;
                q += d * d;
            }
        }
    }
    const float rstd = rsqrtf(block_sum(q, red) / dim + eps);
    const long long bidx = row / rpb;
    bf16_t* orow = out + row * ldo;
#pragma unroll
    for (int c = 0; c < MC; ++c) {
        const int ch = threadIdx.x + c * RT;
        if (ch >= nch) continue;
        float o8[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) o8[e] = (v[c][e] - mean) * rstd;
        if (w) {
            float wv[8], bv[8];
            unpack8(*reinterpret_cast<const u32x4_t*>(w + ch * 8), wv);
            unpack8(*reinterpret_cast<const u32x4_t*>(bb + ch * 8), bv);
#pragma unroll
            for (int e = 0; e < 8; ++e) o8[e] = o8[e] * wv[e] + bv[e];
        }
        if (shift) {
            float sh[8], sc[8];
            unpack8(*reinterpret_cast<const u32x4_t*>(shift + bidx * mbs + ch * 8), sh);
            unpack8(*reinterpret_cast<const u32x4_t*>(scale + bidx * mbs + ch * 8), sc);
#pragma unroll
            for (int e = 0; e < 8; ++e) o8[e] = rbf(rbf(rbf(o8[e]) * rbf(1.f + sc[e])) + sh[e]);
        }
        *reinterpret_cast<u32x4_t*>(orow + ch * 8) = pack8(o8);
    }
}

// NR row sums at once: the same shuffle tree and slot order as block_sum, one barrier pair
template <int NR>
__device__ __forceinline__ void block_sum_n(float* v, float* red) {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
    for (int i = 0; i < NR; ++i)
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v[i] += __shfl_xor(v[i], o);
    __syncthreads();
    if (lane == 0)
#pragma unroll
        for (int i = 0; i < NR; ++i) red[i * (RT / 64) + w] = v[i];
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NR; ++i) {
        float t = 0.f;
#pragma unroll
        for (int k = 0; k < RT / 64; ++k) t += red[i * (RT / 64) + k];
        v[i] = t;
    }
}

// RMSNorm over the full row (wan_video_dit.py:106-111) + interleaved 3-D RoPE (:92-97).
// NR rows per block (VS_RMS_ROWS, default 1): their loads all issue before the one reduction.
// Measured at the 14B shape on q|k|v slices (tests/probes/rownorm_ab.py, profiles/r1/rownorm_ab_r1s.log):
// NR = 1 262 us, 2 270 us, 4 331 us -- more rows per block cost occupancy, not latency.  The
// LDS-gathered RoPE pairs took NR = 1 from 294 us (4 global 8-B gathers per 16-B chunk) to 262 us.
template <int NR, int MC = MAXCH>
__global__ __launch_bounds__(RT) void rmsnorm_rope_kernel(
    bf16_t* __restrict__ x, long long ldx, int rows, int dim, int hd, const bf16_t* __restrict__ w, float eps,
    const float2* __restrict__ rope, int gf, int gh, int gw, int rpb, int tok_off) {
    __shared__ float red[NR * (RT / 64)];
    __shared__ __attribute__((aligned(16))) float2 rc[NR][64];   // each row's 64 RoPE pairs (hd = 128)
    const long long row0 = (long long)blockIdx.x * NR;
    const int nr = (int)min((long long)NR, rows - row0);
    const int nch = dim >> 3;
    const int half = hd >> 1;
    const int tdim = half - 2 * (hd / 3 / 2);   // 22 temporal pairs for hd=128
    const int hdim = hd / 3 / 2;                 // 21
    if (rope && threadIdx.x < half) {
        // the row's (f, h, w) picks one table row per pair group: gathered once per row into LDS
        // (visible after the reduction's barriers) instead of 4 scattered 8-B loads per 16-B chunk
        const int j = threadIdx.x;
#pragma unroll
        for (int i = 0; i < NR; ++i) {
            if (i >= nr) break;
            const int t = (int)((row0 + i) % rpb) + tok_off;
            const int pos = j < tdim ? t / (gw * gh) : (j < tdim + hdim ? (t / gw) % gh : t % gw);
            rc[i][j] = rope[(long long)pos * half + j];
        }
    }
    float v[NR][MC][8];
    float s[NR];
#pragma unroll
    for (int i = 0; i < NR; ++i) {
        s[i] = 0.f;
        if (i >= nr) continue;
        const bf16_t* xr = x + (row0 + i) * ldx;
#pragma unroll
        for (int c = 0; c < MC; ++c) {
            const int ch = threadIdx.x + c * RT;
            if (ch < nch) unpack8(*reinterpret_cast<const u32x4_t*>(xr + ch * 8), v[i][c]);
        }
    }
#pragma unroll
    for (int i = 0; i < NR; ++i)
#pragma unroll
        for (int c = 0; c < MC; ++c) {
            const int ch = threadIdx.x + c * RT;
            if (i < nr && ch < nch)
#pragma unroll
                for (int e = 0; e < 8; ++e) s[i] += v[i][c][e] * v[i][c][e];
        }
    block_sum_n<NR>(s, red);
#pragma unroll
    for (int c = 0; c < MC; ++c) {
        const int ch = threadIdx.x + c * RT;
        if (ch >= nch) continue;
        float wv[8];
        unpack8(*reinterpret_cast<const u32x4_t*>(w + ch * 8), wv);
        const int pair0 = ((ch * 8) % hd) >> 1;
#pragma unroll
        for (int i = 0; i < NR; ++i) {
            if (i >= nr) break;
            const float r = rsqrtf(s[i] / dim + eps);
            float y[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) y[e] = rbf(rbf(v[i][c][e] * r) * wv[e]);
            if (rope) {
                const f32x4_t c01 = *reinterpret_cast<const f32x4_t*>(&rc[i][pair0]);
                const f32x4_t c23 = *reinterpret_cast<const f32x4_t*>(&rc[i][pair0 + 2]);
                const float2 css[4] = {{c01[0], c01[1]}, {c01[2], c01[3]}, {c23[0], c23[1]}, {c23[2], c23[3]}};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float2 cs = css[e];
                    const float a = y[2 * e], b = y[2 * e + 1];
                    y[2 * e] = a * cs.x - b * cs.y;
                    y[2 * e + 1] = a * cs.y + b * cs.x;
                }
            }
            *reinterpret_cast<u32x4_t*>(x + (row0 + i) * ldx + ch * 8) = pack8(y);
        }
    }
}

// Conv3d (1,2,2) im2col: one thread per (token, channel) writes 4 contiguous columns
__global__ void patchify_kernel(const bf16_t* __restrict__ lat, bf16_t* __restrict__ tok, int C,
                                int T, int H, int W, long long total) {
    const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (i >= total) return;
    const int h2 = H >> 1, w2 = W >> 1;
    const int c = (int)(i % C);
    const long long t = i / C;                 // global token (b, f, hh, ww)
    const int ww = (int)(t % w2);
    const int hh = (int)((t / w2) % h2);
    const int f = (int)((t / ((long long)w2 * h2)) % T);
    const long long b = t / ((long long)w2 * h2 * T);
    const bf16_t* src = lat + (((b * C + c) * T + f) * H + 2 * hh) * (long long)W + 2 * ww;
    const uint32_t top = *reinterpret_cast<const uint32_t*>(src);
    const uint32_t bot = *reinterpret_cast<const uint32_t*>(src + W);
    u32x2_t o;
    o[0] = top;
    o[1] = bot;
    *reinterpret_cast<u32x2_t*>(tok + t * (4LL * C) + 4 * c) = o;
}

// unpatchify: out[b][c][f][2hh+y][2ww+z] = tok[(b,f,hh,ww)][(2y+z)*C + c]
__global__ void unpatchify_kernel(const bf16_t* __restrict__ tok, bf16_t* __restrict__ lat, int C,
                                  int T, int H, int W, long long total) {
    const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (i >= total) return;
    const int h2 = H >> 1, w2 = W >> 1;
    const int ww = (int)(i % w2);
    const int hh = (int)((i / w2) % h2);
    const int f = (int)((i / ((long long)w2 * h2)) % T);
    const int c = (int)((i / ((long long)w2 * h2 * T)) % C);
    const long long b = i / ((long long)w2 * h2 * T * C);
    const long long t = ((b * T + f) * h2 + hh) * (long long)w2 + ww;
    const bf16_t* src = tok + t * (4LL * C) + c;
    bf16_t* dst = lat + (((b * C + c) * T + f) * H + 2 * hh) * (long long)W + 2 * ww;
    const uint32_t top = (uint32_t)src[0] | ((uint32_t)src[C] << 16);
    const uint32_t bot = (uint32_t)src[2 * C] | ((uint32_t)src[3 * C] << 16);
    *reinterpret_cast<uint32_t*>(dst) = top;
    *reinterpret_cast<uint32_t*>(dst + W) = bot;
}

__global__ void cfg_euler_kernel(const bf16_t* __restrict__ vp, const bf16_t* __restrict__ vn,
                                 bf16_t* __restrict__ x, long long n8, float g, float ds, int use_cfg,
                                 const float* __restrict__ ds_dev) {
    const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (i >= n8) return;
    if (ds_dev) ds = *ds_dev;
    float a[8], b[8], xv[8];
    unpack8(reinterpret_cast<const u32x4_t*>(vp)[i], a);
    unpack8(reinterpret_cast<const u32x4_t*>(x)[i], xv);
    if (use_cfg) unpack8(reinterpret_cast<const u32x4_t*>(vn)[i], b);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        float v = a[e];
        if (use_cfg) v = rbf(b[e] + rbf(g * rbf(a[e] - b[e])));
        xv[e] = xv[e] + rbf(v * ds);
    }
    reinterpret_cast<u32x4_t*>(x)[i] = pack8(xv);
}


// FlowUniPCMultistepScheduler tensor updates (denoising_enhancing/wan/utils/fm_solvers_unipc.py),
// fp32, each op rounded as the reference's separate fp32 tensor ops (no contraction):
//   mode 0 convert   : out = x - c[0]*mt                                       (:317-323)
//   mode 1 UniP o1   : out = c1*x - c2*m0                                       (:469,475)
//   mode 2 UniP o2   : out = (c1*x - c2*m0) - c3*(r0*((m1 - m0)/rk))            (:427,469-475)
//   mode 3 UniC o1   : out = (c1*x - c2*m0) - c3*(r1*(mt - m0))                 (:612-618)
//   mode 4 UniC o2   : out = (c1*x - c2*m0) - c3*(r0*((m1 - m0)/rk) + r1*(mt - m0))
// with c = {c1, c2, c3, r0, r1, rk}; m0 = newest stored x0 prediction, m1 = the one before, mt = the
// current model output (mode 0: raw velocity; modes 3/4: current x0 prediction).
__global__ void unipc_kernel(float* __restrict__ out, const float* __restrict__ x, const float* __restrict__ m0,
                             const float* __restrict__ m1, const float* __restrict__ mt, long long n, int mode,
                             float c1, float c2, float c3, float r0, float r1, float rk) {
    // the reference rounds after every op: hipcc's default -ffp-contract=fast would fuse
    // c*x - y into one v_fma_f32 (the __f*_rn helpers do not stop it: their inlined bodies carry
    // the contract flag), so the expressions are written here, under contract(off)
#pragma clang fp contract(off)
    const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (mode == 0) {
        out[i] = x[i] - c1 * mt[i];
        return;
    }
    const float base = c1 * x[i] - c2 * m0[i];
    float res;
    if (mode == 1) {
        out[i] = base;
        return;
    } else if (mode == 2) {
        res = r0 * ((m1[i] - m0[i]) / rk);
    } else if (mode == 3) {
        res = r1 * (mt[i] - m0[i]);
    } else {
        res = r0 * ((m1[i] - m0[i]) / rk) + r1 * (mt[i] - m0[i]);
    }
    out[i] = base - c3 * res;
}

__global__ void cast_kernel(const void* __restrict__ src, void* __restrict__ dst, long long n, int to_bf16) {
    const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (to_bf16)
        ((bf16_t*)dst)[i] = (bf16_t)f2bf(((const float*)src)[i]);
    else
        ((float*)dst)[i] = bf2f(((const bf16_t*)src)[i]);
}

__global__ void time_sinusoid_kernel(const bf16_t* __restrict__ t, bf16_t* __restrict__ out, int dim) {
    const int b = blockIdx.x;
    const int half = dim >> 1;
    const double pos = (double)bf2f(t[b]);
    for (int i = threadIdx.x; i < half; i += blockDim.x) {
        const double ang = pos * pow(10000.0, -(double)i / (double)half);
        out[(long long)b * dim + i] = (bf16_t)f2bf((float)cos(ang));
        out[(long long)b * dim + half + i] = (bf16_t)f2bf((float)sin(ang));
    }
}

__global__ void mod_add_kernel(const bf16_t* __restrict__ p, const bf16_t* __restrict__ tv,
                               bf16_t* __restrict__ out, int rows, int dim, long long tbs,
                               long long trs, long long total) {
    const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (i >= total) return;
    const int d = (int)(i % dim);
    const int r = (int)((i / dim) % rows);
    const long long b = i / ((long long)dim * rows);
    const float v = bf2f(p[(long long)r * dim + d]) + bf2f(tv[b * tbs + r * trs + d]);
    out[i] = (bf16_t)f2bf(v);
}

__global__ void axpy_kernel(bf16_t* __restrict__ x, const bf16_t* __restrict__ y, float s, long long n8) {
    const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (i >= n8) return;
    float a[8], b[8];
    unpack8(reinterpret_cast<const u32x4_t*>(x)[i], a);
    unpack8(reinterpret_cast<const u32x4_t*>(y)[i], b);
#pragma unroll
    for (int e = 0; e < 8; ++e) a[e] = a[e] + rbf(b[e] * s);
    reinterpret_cast<u32x4_t*>(x)[i] = pack8(a);
}


// Ulysses sequence-parallel row permutations (8 bf16 = 16 B per thread).  Canonical index
// (j, b, t, c): rank-chunk j, batch b, local token t, column c within a rank's head group.
//   packed: j*jstride + (b*Sl + t)*pld + c         (all_to_all_single chunk j; pld >= cpr)
//   local : (b*Sl + t)*ld + j*cpr + c             (token-sharded activations, all heads)
//   full  : (b*P*Sl + j*Sl + t)*cpr + c            (head-sharded, full sequence)
// mode 0 local->packed, 1 packed->local, 2 packed->full, 3 full->packed.
__global__ void ulysses_permute_kernel(const bf16_t* __restrict__ src, bf16_t* __restrict__ dst, int B,
                                       int Sl, int P, int cpr, long long ld, long long jstride, long long pld,
                                       int mode, long long total8) {
    const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (i >= total8) return;
    const int c8 = cpr >> 3;
    const int c = (int)(i % c8) * 8;
    long long r = i / c8;
    const int t = (int)(r % Sl);
    r /= Sl;
    const int b = (int)(r % B);
    const int j = (int)(r / B);
    const long long packed = j * jstride + ((long long)b * Sl + t) * pld + c;
    const long long local = ((long long)b * Sl + t) * ld + (long long)j * cpr + c;
    const long long full = ((long long)b * P * Sl + (long long)j * Sl + t) * cpr + c;
    long long so, d;
    switch (mode) {
        case 0: so = local; d = packed; break;
        case 1: so = packed; d = local; break;
        case 2: so = packed; d = full; break;
        default: so = full; d = packed; break;
    }
    *reinterpret_cast<u32x4_t*>(dst + d) = *reinterpret_cast<const u32x4_t*>(src + so);
}

bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }
// rows up to RT * MAXCH * 8 = 5120 (every Wan width) on the measured 5-chunk instantiation; wider
// rows, up to RT * MCW * 8 = 8192, on an 8-chunk one (r1-r4 accepted up to 6144)
constexpr int MCW = 8;
constexpr int ROW_MAX = RT * MCW * 8;
bool narrow(int dim) { return dim <= RT * MAXCH * 8; }
unsigned nblk(long long n, int t) { return (unsigned)((n + t - 1) / t); }

}  // namespace

extern "C" int vs_layernorm_modulate(const void* x, long long ldx, void* out, long long ldo,
                                     int rows, int dim, int rows_per_batch, const void* shift,
                                     const void* scale, long long mod_bstride, const void* weight,
                                     const void* bias, float eps, void* stream) {
    if (!x || !out || rows <= 0 || dim <= 0 || dim % 8 || dim > ROW_MAX) return VS_E_INVALID;
    if (ldx < dim || ldo < dim || (ldx & 7) || (ldo & 7) || !al16(x) || !al16(out)) return VS_E_INVALID;
    if ((shift == nullptr) != (scale == nullptr)) return VS_E_INVALID;
    if ((weight == nullptr) != (bias == nullptr)) return VS_E_INVALID;
    if (shift && (!al16(shift) || !al16(scale) || (mod_bstride & 7))) return VS_E_INVALID;
    if (weight && (!al16(weight) || !al16(bias))) return VS_E_INVALID;
    if (rows_per_batch <= 0) rows_per_batch = rows;
    hipLaunchKernelGGL((narrow(dim) ? ln_modulate_kernel<false> : ln_modulate_kernel<false, MCW>), dim3(rows), dim3(RT), 0,
                       (hipStream_t)stream,
                       (const bf16_t*)x, ldx, (bf16_t*)out, ldo, dim, rows_per_batch,
                       (const bf16_t*)shift, (const bf16_t*)scale, mod_bstride,
                       (const bf16_t*)weight, (const bf16_t*)bias, eps, nullptr, 0LL, nullptr);
    VS_CHECK_LAUNCH();
    return VS_OK;
}

extern "C" int vs_layernorm_modulate_fp8(const void* x, long long ldx, void* x8, long long ld8, float* qscale,
                                         int rows, int dim, int rows_per_batch, const void* shift,
                                         const void* scale, long long mod_bstride, const void* weight,
                                         const void* bias, float eps, void* stream) {
    if (!x || !x8 || !qscale || rows <= 0 || dim <= 0 || dim % 8 || dim > ROW_MAX) return VS_E_INVALID;
    if (ldx < dim || ld8 < dim || (ldx & 7) || (ld8 & 7) || !al16(x) || (reinterpret_cast<uintptr_t>(x8) & 7))
        return VS_E_INVALID;
    if ((shift == nullptr) != (scale == nullptr)) return VS_E_INVALID;
    if ((weight == nullptr) != (bias == nullptr)) return VS_E_INVALID;
    if (shift && (!al16(shift) || !al16(scale) || (mod_bstride & 7))) return VS_E_INVALID;
    if (weight && (!al16(weight) || !al16(bias))) return VS_E_INVALID;
    if (rows_per_batch <= 0) rows_per_batch = rows;
    hipLaunchKernelGGL((narrow(dim) ? ln_modulate_kernel<true> : ln_modulate_kernel<true, MCW>), dim3(rows), dim3(RT), 0,
                       (hipStream_t)stream,
                       (const bf16_t*)x, ldx, nullptr, 0LL, dim, rows_per_batch,
                       (const bf16_t*)shift, (const bf16_t*)scale, mod_bstride,
                       (const bf16_t*)weight, (const bf16_t*)bias, eps, (uint8_t*)x8, ld8, qscale);
    VS_CHECK_LAUNCH();
    return VS_OK;
}

extern "C" int vs_residual_layernorm(const void* y, long long ldy, void* x, long long ldx, void* out, long long ldo,
                                     int rows, int dim, int epilogue, const vs_epilogue* epi, int rows_per_batch,
                                     const void* shift, const void* scale, long long mod_bstride,
                                     const void* weight, const void* bias, float eps, void* stream) {
    if (!y || !x || !out || !epi || rows <= 0 || dim <= 0 || dim % 8 || dim > ROW_MAX) return VS_E_INVALID;
    if (epilogue != VS_EPI_GATE_RES && epilogue != VS_EPI_RES) return VS_E_INVALID;
    if (ldy < dim || ldx < dim || ldo < dim || ((ldy | ldx | ldo) & 7) || !al16(y) || !al16(x) || !al16(out))
        return VS_E_INVALID;
    if (epilogue == VS_EPI_GATE_RES) {
        if (!epi->gate || !al16(epi->gate) || (epi->gate_bstride & 7)) return VS_E_INVALID;
        if (epi->hint && (!al16(epi->hint) || (epi->ld_hint & 7) || epi->ld_hint < dim)) return VS_E_INVALID;
    }
    if ((shift == nullptr) != (scale == nullptr) || (weight == nullptr) != (bias == nullptr)) return VS_E_INVALID;
    if (shift && (!al16(shift) || !al16(scale) || (mod_bstride & 7))) return VS_E_INVALID;
    if (weight && (!al16(weight) || !al16(bias))) return VS_E_INVALID;
    const int rpb_gate = epi->rows_per_batch > 0 ? epi->rows_per_batch : rows;
    if (rows_per_batch <= 0) rows_per_batch = rows;
    const bool gated = epilogue == VS_EPI_GATE_RES;
    hipLaunchKernelGGL((narrow(dim) ? residual_ln_kernel<> : residual_ln_kernel<MCW>), dim3(rows), dim3(RT), 0,
                       (hipStream_t)stream, (const bf16_t*)y, ldy,
                       (bf16_t*)x, ldx, (bf16_t*)out, ldo, dim, epilogue,
                       gated ? (const bf16_t*)epi->gate : nullptr, epi->gate_bstride, rpb_gate, epi->alpha,
                       gated ? (const bf16_t*)epi->hint : nullptr, epi->ld_hint, epi->hint_scale, rows_per_batch,
                       (const bf16_t*)shift, (const bf16_t*)scale, mod_bstride, (const bf16_t*)weight,
                       (const bf16_t*)bias, eps);
    VS_CHECK_LAUNCH();
    return VS_OK;
}

extern "C" int vs_rmsnorm_rope(void* x, long long ldx, int rows, int dim, int head_dim,
                               const void* weight, float eps, const void* rope, int rope_len,
                               int gf, int gh, int gw, int rows_per_batch, int token_offset,
                               void* stream) {
    if (!x || !weight || rows <= 0 || dim <= 0 || dim % 8 || dim > ROW_MAX) return VS_E_INVALID;
    if (ldx < dim || (ldx & 7) || !al16(x) || !al16(weight)) return VS_E_INVALID;
    if (rope) {
        if (head_dim != 128 || dim % head_dim) return VS_E_UNSUPPORTED;
        if (gf <= 0 || gh <= 0 || gw <= 0 || gf > rope_len || gh > rope_len || gw > rope_len)
            return VS_E_INVALID;
        if (rows_per_batch <= 0 || token_offset < 0 ||
            (long long)token_offset + rows_per_batch > (long long)gf * gh * gw)
            return VS_E_INVALID;
    }
    if (rows_per_batch <= 0) rows_per_batch = rows;
#ifndef VS_RMS_ROWS
#define VS_RMS_ROWS 1
#endif
    constexpr int NR = VS_RMS_ROWS;
    hipLaunchKernelGGL((narrow(dim) ? rmsnorm_rope_kernel<NR> : rmsnorm_rope_kernel<NR, MCW>),
                       dim3((unsigned)((rows + NR - 1) / NR)), dim3(RT), 0,
                       (hipStream_t)stream, (bf16_t*)x, ldx, rows, dim, head_dim, (const bf16_t*)weight, eps,
                       (const float2*)rope, gf, gh, gw, rows_per_batch, token_offset);
    VS_CHECK_LAUNCH();
    return VS_OK;
}

extern "C" int vs_patchify(const void* lat, void* tokens, int batch, int channels, int frames,
                           int height, int width, void* stream) {
    if (!lat || !tokens || batch <= 0 || channels <= 0 || frames <= 0 || height <= 0 || width <= 0)
        return VS_E_INVALID;
    if (height % 2 || width % 2 || (reinterpret_cast<uintptr_t>(lat) & 3) || (reinterpret_cast<uintptr_t>(tokens) & 7))
        return VS_E_INVALID;
    const long long total = (long long)batch * frames * (height / 2) * (width / 2) * channels;
    hipLaunchKernelGGL(patchify_kernel, dim3(nblk(total, 256)), dim3(256), 0, (hipStream_t)stream,
                       (const bf16_t*)lat, (bf16_t*)tokens, channels, frames, height, width, total);
    VS_CHECK_LAUNCH();
    return VS_OK;
}

extern "C" int vs_unpatchify(const void* tokens, void* lat, int batch, int channels, int frames,
                             int height, int width, void* stream) {
    if (!lat || !tokens || batch <= 0 || channels <= 0 || frames <= 0 || height <= 0 || width <= 0)
        return VS_E_INVALID;
    if (height % 2 || width % 2 || (reinterpret_cast<uintptr_t>(lat) & 3)) return VS_E_INVALID;
    const long long total = (long long)batch * channels * frames * (height / 2) * (width / 2);
    hipLaunchKernelGGL(unpatchify_kernel, dim3(nblk(total, 256)), dim3(256), 0, (hipStream_t)stream,
                       (const bf16_t*)tokens, (bf16_t*)lat, channels, frames, height, width, total);
    VS_CHECK_LAUNCH();
    return VS_OK;
}

extern "C" int vs_cfg_euler(const void* v_pos, const void* v_neg, void* x, long long n,
                            float cfg_scale, float dsigma, int use_cfg, void* stream) {
    if (!v_pos || !x || n <= 0 || n % 8 || (use_cfg && !v_neg)) return VS_E_INVALID;
    if (!al16(v_pos) || !al16(x) || (use_cfg && !al16(v_neg))) return VS_E_INVALID;
    const long long n8 = n / 8;
    hipLaunchKernelGGL(cfg_euler_kernel, dim3(nblk(n8, 256)), dim3(256), 0, (hipStream_t)stream,
                       (const bf16_t*)v_pos, (const bf16_t*)v_neg, (bf16_t*)x, n8, cfg_scale,
                       dsigma, use_cfg, (const float*)nullptr);
    VS_CHECK_LAUNCH();
    return VS_OK;
}

extern "C" int vs_cfg_euler_dev(const void* v_pos, const void* v_neg, void* x, long long n, float cfg_scale,
                                const float* dsigma, int use_cfg, void* stream) {
    if (!v_pos || !x || !dsigma || n <= 0 || n % 8 || (use_cfg && !v_neg)) return VS_E_INVALID;
    if (!al16(v_pos) || !al16(x) || (use_cfg && !al16(v_neg))) return VS_E_INVALID;
    const long long n8 = n / 8;
    hipLaunchKernelGGL(cfg_euler_kernel, dim3(nblk(n8, 256)), dim3(256), 0, (hipStream_t)stream,
                       (const bf16_t*)v_pos, (const bf16_t*)v_neg, (bf16_t*)x, n8, cfg_scale,
                       0.0f, use_cfg, dsigma);
    VS_CHECK_LAUNCH();
    return VS_OK;
}

extern "C" int vs_time_sinusoid(const void* t, void* out, int batch, int dim, void* stream) {
    if (!t || !out || batch <= 0 || dim <= 0 || dim % 2) return VS_E_INVALID;
    hipLaunchKernelGGL(time_sinusoid_kernel, dim3(batch), dim3(128), 0, (hipStream_t)stream,
                       (const bf16_t*)t, (bf16_t*)out, dim);
    VS_CHECK_LAUNCH();
    return VS_OK;
}

extern "C" int vs_mod_add(const void* param, const void* tv, void* out, int batch, int rows,
                          int dim, long long tv_bstride, long long tv_rstride, void* stream) {
    if (!param || !tv || !out || batch <= 0 || rows <= 0 || dim <= 0) return VS_E_INVALID;
    const long long total = (long long)batch * rows * dim;
    hipLaunchKernelGGL(mod_add_kernel, dim3(nblk(total, 256)), dim3(256), 0, (hipStream_t)stream,
                       (const bf16_t*)param, (const bf16_t*)tv, (bf16_t*)out, rows, dim,
                       tv_bstride, tv_rstride, total);
    VS_CHECK_LAUNCH();
    return VS_OK;
}

extern "C" int vs_axpy(void* x, const void* y, float scale, long long n, void* stream) {
    if (!x || !y || n <= 0 || n % 8 || !al16(x) || !al16(y)) return VS_E_INVALID;
    const long long n8 = n / 8;
    hipLaunchKernelGGL(axpy_kernel, dim3(nblk(n8, 256)), dim3(256), 0, (hipStream_t)stream,
                       (bf16_t*)x, (const bf16_t*)y, scale, n8);
    VS_CHECK_LAUNCH();
    return VS_OK;
}


extern "C" int vs_ulysses_permute_rows(const void* src, void* dst, int batch, int s_local, int world,
                                       int cols_per_rank, long long ld_local, long long jstride,
                                       long long packed_ld, int mode, void* stream) {
    if (!src || !dst || batch <= 0 || s_local <= 0 || world <= 0 || cols_per_rank <= 0) return VS_E_INVALID;
    if (cols_per_rank % 8 || (ld_local & 7) || (jstride & 7) || (packed_ld & 7) || mode < 0 || mode > 3)
        return VS_E_INVALID;
    if ((mode <= 1) && ld_local < (long long)world * cols_per_rank) return VS_E_INVALID;
    if (packed_ld < cols_per_rank) return VS_E_INVALID;
    if (jstride < ((long long)batch * s_local - 1) * packed_ld + cols_per_rank) return VS_E_INVALID;
    if (!al16(src) || !al16(dst)) return VS_E_INVALID;
    const long long total8 = (long long)world * batch * s_local * (cols_per_rank / 8);
    hipLaunchKernelGGL(ulysses_permute_kernel, dim3(nblk(total8, 256)), dim3(256), 0, (hipStream_t)stream,
                       (const bf16_t*)src, (bf16_t*)dst, batch, s_local, world, cols_per_rank, ld_local,
                       jstride, packed_ld, mode, total8);
    VS_CHECK_LAUNCH();
    return VS_OK;
}

extern "C" int vs_ulysses_permute(const void* src, void* dst, int batch, int s_local, int world,
                                  int cols_per_rank, long long ld_local, long long jstride, int mode,
                                  void* stream) {
    return vs_ulysses_permute_rows(src, dst, batch, s_local, world, cols_per_rank, ld_local, jstride,
                                   cols_per_rank, mode, stream);
}

extern "C" const char* vs_strerror(int code) {
    switch (code) {
        case VS_OK: return "VS_OK";
        case VS_E_INVALID: return "VS_E_INVALID: invalid shape, stride, alignment or pointer";
        case VS_E_LAUNCH: return "VS_E_LAUNCH: kernel launch failed";
        case VS_E_UNSUPPORTED: return "VS_E_UNSUPPORTED: configuration not implemented";
        case VS_E_COMM: return "VS_E_COMM: RCCL unavailable or failed (vs_sp_last_error)";
        default: return "unknown vstyler error";
    }
}

extern "C" int vs_abi_version(void) { return 2; }

extern "C" int vs_unipc_update(float* out, const float* x, const float* m0, const float* m1, const float* mt,
                               long long n, int mode, const float* coef, void* stream) {
    if (!out || !coef || n <= 0 || mode < 0 || mode > 4 || !x) return VS_E_INVALID;
    if ((mode >= 1 && !m0) || ((mode == 2 || mode == 4) && !m1) || ((mode == 0 || mode >= 3) && !mt))
        return VS_E_INVALID;
    hipLaunchKernelGGL(unipc_kernel, dim3(nblk(n, 256)), dim3(256), 0, (hipStream_t)stream, out, x, m0, m1, mt, n,
                       mode, coef[0], coef[1], coef[2], coef[3], coef[4], coef[5]);
    VS_CHECK_LAUNCH();
    return VS_OK;
}

extern "C" int vs_cast(const void* src, void* dst, long long n, int to_bf16, void* stream) {
    if (!src || !dst || n <= 0) return VS_E_INVALID;
    hipLaunchKernelGGL(cast_kernel, dim3(nblk(n, 256)), dim3(256), 0, (hipStream_t)stream, src, dst, n, to_bf16);
    VS_CHECK_LAUNCH();
    return VS_OK;
}
