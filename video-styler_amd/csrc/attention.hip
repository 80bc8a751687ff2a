// Flash attention forward for Wan2.1 DiT (head_dim 128, non-causal, no mask), gfx950.
//
// Replaces flash_attention()/AttentionModule (reference diffsynth/models/wan_video_dit.py:28-61,
// 114-121): self-attention over S = T'*(H/16)*(W/16) latent tokens and cross-attention over the
// 512 T5 context tokens.
//
// Structure (one workgroup = 8 waves = 256 query rows of one (batch, head)):
//  * each wave owns 32 query rows; its Q slice (32 x 128 bf16) lives in 32 VGPRs for the whole
//    key sweep, in the B-operand layout of v_mfma_f32_32x32x16_bf16;
//  * K/V tiles of 64 keys (2 x 16 KB) are register-staged global->LDS, double-buffered: the
//    global loads of tile i+1 are issued before the MFMAs of tile i and written to LDS after
//    them (issue-early / write-late), one barrier per tile;
//  * S^T = K Q^T (swapped product): every lane holds 32 scores of ONE query row, so the online
//    softmax row max needs a single lane^32 exchange and the row sum stays lane-partial;
//  * O^T = V^T P: the S^T accumulator is directly the B operand of the PV MFMA (no LDS round
//    trip for P), V^T fragments come from LDS with ds_read_b64_tr_b16 (hardware transpose), and
//    the O accumulator of a lane also belongs to its own query row, so the rescale is lane-local;
//  * K/V LDS image: 256-B rows with the 16-B chunk XOR swizzle that keeps both the ds_read_b128
//    row reads (K) and the transposed reads (V) bank-conflict free;
//  * workgroup ids are remapped so each XCD works through contiguous (batch, head) ranges: the
//    K/V of one head is streamed by the 32 CUs of one XCD together and served from its L2.
#include "common.h"

namespace {

constexpr int HD = 128;          // head dim
constexpr int BQ = 256;          // query rows per workgroup
constexpr int BKV = 64;          // keys per tile
constexpr int NTHR = 512;
constexpr int TILE = BKV * HD * 2;  // 16 KB per K (or V) tile

__device__ __forceinline__ int lds_off(int row, int ch) {
    return row * 256 + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}

__global__ __launch_bounds__(NTHR) void attn_fwd_d128(
    const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K, const bf16_t* __restrict__ V,
    bf16_t* __restrict__ O, int Sq, int Skv, int H, long long ldq, long long ldk, long long ldv,
    long long ldo, long long bsq, long long bsk, long long bsv, long long bso, float c, int nqb) {
    extern __shared__ __attribute__((aligned(16))) char smem[];

    const int g = xcd_remap(blockIdx.x, gridDim.x);
    const int qb = g % nqb;
    const int bh = g / nqb;
    const int h = bh % H, b = bh / H;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int r = lane & 31, hh = lane >> 5;
    const int q0 = qb * BQ + wave * 32;

    const bf16_t* Qb = Q + (long long)b * bsq + h * HD;
    const bf16_t* Kb = K + (long long)b * bsk + h * HD;
    const bf16_t* Vb = V + (long long)b * bsv + h * HD;

    // Q slice as the B operand of S^T = K Q^T: lane (r, hh) holds Q[q0+r][16s + 8hh .. +7].
    bf16x8_t qf[8];
    {
        const int qrow = min(q0 + r, Sq - 1);
        const bf16_t* qp = Qb + (long long)qrow * ldq + 8 * hh;
#pragma unroll
        for (int s = 0; s < 8; ++s) qf[s] = *reinterpret_cast<const bf16x8_t*>(qp + 16 * s);
    }

    f32x16_t o[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i) o[dt][i] = 0.f;
    float m = -1e30f, l = 0.f;

    // register staging: thread owns chunks tid and tid+512 (row = ci>>4, 16-B chunk = ci&15)
    u32x4_t kst[2], vst[2];
    auto load_tile = [&](int kv0) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int ci = tid + NTHR * j, row = ci >> 4, ch = ci & 15;
            const long long kr = min(kv0 + row, Skv - 1);
            kst[j] = *reinterpret_cast<const u32x4_t*>(Kb + kr * ldk + ch * 8);
            vst[j] = *reinterpret_cast<const u32x4_t*>(Vb + kr * ldv + ch * 8);
        }
    };
    auto store_tile = [&](int buf) {
        char* kb = smem + buf * 2 * TILE;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int ci = tid + NTHR * j, row = ci >> 4, ch = ci & 15;
            *reinterpret_cast<u32x4_t*>(kb + lds_off(row, ch)) = kst[j];
            *reinterpret_cast<u32x4_t*>(kb + TILE + lds_off(row, ch)) = vst[j];
        }
    };

    // per-lane constants of the transposed V read (ds_read_b64_tr_b16): group g4 of 16 lanes,
    // lane 4*q4+p4 of the group addresses row q4 / columns 4*p4.. of a 4 x 16 block.
    const int g4 = lane >> 4, q4 = (lane & 15) >> 2, p4 = lane & 3;
    const int vrow = 4 * (g4 >> 1) + q4;
    const int vch = 2 * (g4 & 1) + (p4 >> 1);
    const int vbyte = 8 * (p4 & 1);

    auto compute = [&](int buf, int kv0, bool mask) {
        const char* kb = smem + buf * 2 * TILE;
        const char* vb = kb + TILE;
        f32x16_t s[2];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
#pragma unroll
            for (int i = 0; i < 16; ++i) s[t][i] = 0.f;
            const int row = 32 * t + r;
#pragma unroll
            for (int ss = 0; ss < 8; ++ss) {
                const bf16x8_t kf = *reinterpret_cast<const bf16x8_t*>(kb + lds_off(row, 2 * ss + hh));
                s[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[ss], s[t], 0, 0, 0);
            }
        }
        if (mask) {
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const int key = kv0 + 32 * t + (i & 3) + 8 * (i >> 2) + 4 * hh;
                    if (key >= Skv) s[t][i] = -INFINITY;
                }
        }
        // online softmax (scores scaled into the exp2 domain by c = scale*log2(e))
        float mx = s[0][0];
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int i = 0; i < 16; ++i) mx = fmaxf(mx, s[t][i]);
        mx = fmaxf(mx, __shfl_xor(mx, 32));
        const float mnew = fmaxf(m, mx * c);
        const float alpha = __builtin_amdgcn_exp2f(m - mnew);
        m = mnew;
        float rs = 0.f;
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const float p = __builtin_amdgcn_exp2f(fmaf(s[t][i], c, -mnew));
                s[t][i] = p;
                rs += p;
            }
        l = l * alpha + rs;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
            for (int i = 0; i < 16; ++i) o[dt][i] *= alpha;

        // O^T += V^T P over 4 k-steps of 16 keys
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            const int t = ks >> 1, u = ks & 1;
            bf16x8_t pf;
#pragma unroll
            for (int j = 0; j < 8; ++j) pf[j] = (__bf16)s[t][8 * u + j];
            const int row0 = 16 * ks + vrow;
#pragma unroll
            for (int dt = 0; dt < 4; ++dt) {
                const int ch = 4 * dt + vch;
                const i16x4_t v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                    (LDS_AS i16x4_t*)(vb + lds_off(row0, ch) + vbyte));
                const i16x4_t v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                    (LDS_AS i16x4_t*)(vb + lds_off(row0 + 8, ch) + vbyte));
                const bf16x8_t vf = __builtin_shufflevector(__builtin_bit_cast(bf16x4_t, v0),
                                                            __builtin_bit_cast(bf16x4_t, v1), 0, 1, 2, 3,
                                                            4, 5, 6, 7);
                o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf, o[dt], 0, 0, 0);
            }
        }
    };

    const int nkv = (Skv + BKV - 1) / BKV;
    load_tile(0);
    store_tile(0);
    __syncthreads();
    for (int it = 0; it < nkv; ++it) {
        const bool has_next = it + 1 < nkv;
        if (has_next) load_tile((it + 1) * BKV);
        compute(it & 1, it * BKV, (it + 1) * BKV > Skv);
        if (has_next) store_tile((it + 1) & 1);
        __syncthreads();
    }

    const float lt = l + __shfl_xor(l, 32);
    const float inv = 1.f / lt;
    if (q0 + r < Sq) {
        bf16_t* op = O + (long long)b * bso + (long long)(q0 + r) * ldo + h * HD;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
            for (int gi = 0; gi < 4; ++gi) {
                const int d = 32 * dt + 8 * gi + 4 * hh;
                u32x2_t w;
                w[0] = pack2(o[dt][4 * gi] * inv, o[dt][4 * gi + 1] * inv);
                w[1] = pack2(o[dt][4 * gi + 2] * inv, o[dt][4 * gi + 3] * inv);
                *reinterpret_cast<u32x2_t*>(op + d) = w;
            }
    }
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace

extern "C" int vs_attn_fwd(const void* q, const void* k, const void* v, void* o, int batch, int sq,
                           int skv, int heads, int head_dim, long long ldq, long long ldk,
                           long long ldv, long long ldo, long long bsq, long long bsk,
                           long long bsv, long long bso, float scale, void* stream) {
    if (!q || !k || !v || !o || batch <= 0 || sq <= 0 || skv <= 0 || heads <= 0) return VS_E_INVALID;
    if (head_dim != HD) return VS_E_UNSUPPORTED;
    if (ldq < (long long)heads * HD || ldk < (long long)heads * HD || ldv < (long long)heads * HD ||
        ldo < (long long)heads * HD)
        return VS_E_INVALID;
    if ((ldq | ldk | ldv | ldo | bsq | bsk | bsv | bso) & 7) return VS_E_INVALID;
    if (!aligned16(q) || !aligned16(k) || !aligned16(v) || !aligned16(o)) return VS_E_INVALID;
    const int nqb = (sq + BQ - 1) / BQ;
    const long long nwg = (long long)nqb * heads * batch;
    if (nwg > 0x7fffffff) return VS_E_INVALID;
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)attn_fwd_d128, hipFuncAttributeMaxDynamicSharedMemorySize,
                            4 * TILE);
        attr_set = true;
    }
    const float c = scale * 1.4426950408889634f;
    hipLaunchKernelGGL(attn_fwd_d128, dim3((unsigned)nwg), dim3(NTHR), 4 * TILE,
                       (hipStream_t)stream, (const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v,
                       (bf16_t*)o, sq, skv, heads, ldq, ldk, ldv, ldo, bsq, bsk, bsv, bso, c, nqb);
    VS_CHECK_LAUNCH();
    return VS_OK;
}
