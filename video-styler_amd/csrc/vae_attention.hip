// Flash attention for the causal VAE's AttentionBlock (diffsynth/models/wan_video_vae.py:304-342):
// per frame, ONE head over the frame's h*w pixels with head width d = C (384 in Wan2.1's middle
// blocks), F.scaled_dot_product_attention(q, k, v) with the default 1/sqrt(C) scale (:331).
//
// r1-r6 ran this as an fp32-score GEMM + softmax + a P.V GEMM through the conv kernel (scores of
// rows x rows fp32 round-tripped through HBM, plus a V transpose pass); this kernel keeps the
// scores on chip.  Structure (gfx950, v_mfma_f32_32x32x16_bf16, wave64):
//  * one workgroup = 4 waves = 128 query rows of one frame; each wave owns 32 rows, its Q slice
//    (32 x C bf16) in registers in the B-operand layout for the whole key sweep;
//  * K / V tiles of 32 keys are staged by LDS-DMA (global_load_lds_dwordx4, no staging registers)
//    into a 2-slot ring: tile t+1's pieces are issued at the top of tile t, one wait + barrier per
//    tile.  A DMA piece lands lane-linear (lane i at byte 16 i of a 1-KB piece), so the layouts are
//    chosen by permuting the source chunks: K chunk c of row r at r * C/8 + (c ^ (r & 15)) (the
//    ds_read_b128 row fragments conflict-free), V chunk c at r * C/8 + (c ^ 4 (r & 3)) (the four rows
//    of a ds_read_b64_tr_b16 half-wave on disjoint banks); C % 128 == 0 keeps both XORs in range;
//  * S^T = K Q^T: a lane holds 16 scores of ONE query row (keys 8g + 4h + e), and the O^T = V^T P
//    accumulator of a lane belongs to the same row (cdna_hip_programming.md, "an accumulator tile as
//    the next MFMA's operand": P goes from the S^T registers straight into the B operand; V^T
//    fragments by the transposed LDS read);
//  * exact two-pass softmax over one flattened tile sequence: pass 1 sweeps K for each row's max
//    and sum (exp2 domain, scale log2(e)/sqrt(C) on the fp32 scores; lane-local, the two lane
//    halves merged once), pass 2 recomputes S^T and accumulates O^T += V^T P with
//    P = bf16(exp2(s - m) / l) -- the softmax rounded to bf16 before P.V as the r1-r6 GEMM route
//    did, and no O rescale at all: the accumulator is touched only by MFMAs and stays in AGPRs
//    (an online-softmax rescale made the compiler copy the 192 accumulator registers AGPR -> VGPR
//    every tile and spill at C = 384).  Pass 1 is a third of the MFMA work.
// Keys >= rows read the last row (in range) and are masked to -inf; query rows >= rows are not stored.
#include "common.h"

#include <mutex>

namespace {

constexpr int FA_THR = 256, FA_BQ = 128, FA_BK = 32;

template <int NCB>
struct FaGeom {
    static constexpr int C = 32 * NCB;            // head width
    static constexpr int CH = C / 8;              // 16-B chunks per row
    static constexpr int KT = FA_BK * 2 * C;      // one K (or V) tile, unpadded
    static constexpr int SLOT = 2 * KT;
    static constexpr int LDS = 2 * SLOT;
    static constexpr int NP = KT / 1024 / 4;      // 1-KB DMA pieces per wave per operand
    static_assert(C % 128 == 0 && KT % 4096 == 0, "C must be a multiple of 128");
    static_assert(LDS <= 160 * 1024, "LDS");
};

__device__ __forceinline__ f32x16_t fa_mfma(bf16x8_t a, bf16x8_t b, f32x16_t c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

template <int NCB>
__global__ __launch_bounds__(FA_THR, 1) void vae_attn_kernel(const bf16_t* __restrict__ qkv, long long qkv_zs,
                                                             long long ld, bf16_t* __restrict__ out,
                                                             long long o_zs, long long ldo, int rows,
                                                             float sc) {
    using G = FaGeom<NCB>;
    constexpr int C = G::C;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int h = lane >> 5, col = lane & 31;
    // XCD-aware order: each XCD takes a contiguous range of (frame, query block) ids, so the query
    // blocks of one frame stream its K / V tiles together through one L2
    const int nqb = gridDim.x, wg = xcd_remap(blockIdx.x + nqb * blockIdx.y, nqb * gridDim.y);
    const int z = wg / nqb;
    const bf16_t* base = qkv + z * qkv_zs;
    const int qr = (wg % nqb) * FA_BQ + wave * 32 + col;          // this lane's query row

    // Q^T fragments (B operand): k-step s covers d = 16s .. 16s+15, lane half h its 8 at 16s + 8h
    bf16x8_t qf[2 * NCB];
    {
        const bf16_t* qrow = base + (long long)min(qr, rows - 1) * ld + 8 * h;
#pragma unroll
        for (int s = 0; s < 2 * NCB; ++s) {
            u32x4_t v = *reinterpret_cast<const u32x4_t*>(qrow + 16 * s);
            if (qr >= rows) v = u32x4_t{0u, 0u, 0u, 0u};
            qf[s] = __builtin_bit_cast(bf16x8_t, v);
        }
    }

    // LDS-DMA of one K / V tile into `slot`: piece P of an operand = LDS bytes 1024 P ..; lane i's
    // 16 B land at position 64 P + i = row r, physical chunk c' -> it fetches logical chunk c' ^ f(r)
    auto load_tile = [&](int key0, int slot, bool with_v) {
        char* sb = smem + slot * G::SLOT;
#pragma unroll
        for (int j = 0; j < G::NP; ++j) {
            const int piece = wave * G::NP + j, pos = 64 * piece + lane;
            const int r = pos / G::CH, cp = pos % G::CH;
            const bf16_t* src = base + (long long)min(key0 + r, rows - 1) * ld + C;
            __builtin_amdgcn_global_load_lds((const GLB_AS void*)(src + 8 * (cp ^ (r & 15))),
                                             (LDS_AS void*)(sb + 1024 * piece), 16, 0, 0);
            if (with_v)
                __builtin_amdgcn_global_load_lds((const GLB_AS void*)(src + C + 8 * (cp ^ (4 * (r & 3)))),
                                                 (LDS_AS void*)(sb + G::KT + 1024 * piece), 16, 0, 0);
        }
    };

    const unsigned smem_base = (unsigned)(uintptr_t)smem;
    // K fragment (A operand of S^T = K Q^T): key row `col`, logical chunk c = 2 ks + h at c ^ (col & 15):
    // 8 lane offsets (ks & 7), the 256-B step of ks >> 3 an immediate
    unsigned koff[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) koff[j] = col * 2 * C + 16 * ((2 * j + h) ^ (col & 15));
    // V^T fragment (A operand of O^T = V^T P): ds_read_b64_tr_b16, 16-lane group g4 reads rows
    // (keys) 16 kk + 4 (g4 >> 1) + q4 (+ 8) at columns 16 (g4 & 1) + 4 p4 of column block b; element j
    // of lane half h = key 16 kk + 8 (j >> 2) + 4h + (j & 3), the order of P's registers.  Rows
    // r & 3 = q4 in both reads: logical chunk 4b + 2 (g4 & 1) + (p4 >> 1) sits at 4 (b ^ q4) + ...:
    // 4 lane offsets (b & 3), the rest immediates
    const int g4 = lane >> 4, q4 = (lane & 15) >> 2, p4 = lane & 3;
    unsigned voff[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
        voff[j] = G::KT + (4 * (g4 >> 1) + q4) * 2 * C + 16 * (4 * (j ^ q4) + 2 * (g4 & 1) + (p4 >> 1)) + 8 * (p4 & 1);

    f32x16_t o[NCB];
#pragma unroll
    for (int b = 0; b < NCB; ++b)
#pragma unroll
        for (int i = 0; i < 16; ++i) o[b][i] = 0.f;
    float m = -INFINITY, l = 0.f;

    // S^T[key][q] = sum_d K[key][d] Q[q][d] of the tile in slot base sb, scaled to the exp2 domain,
    // keys >= rows at -inf; the K fragment reads KD steps ahead
    auto scores = [&](unsigned sb, int key0) {
        constexpr int KD = 4;
        unsigned kb[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            kb[j] = sb + koff[j];
            asm volatile("" : "+v"(kb[j]));   // one add per lane offset and tile, steps as immediates
        }
        auto kread = [&](int ks) {
            return *reinterpret_cast<const LDS_AS bf16x8_t*>((const LDS_AS char*)(uintptr_t)(kb[ks & 7] + 256 * (ks >> 3)));
        };
        f32x16_t s;
#pragma unroll
        for (int i = 0; i < 16; ++i) s[i] = 0.f;
        bf16x8_t kf[2 * NCB];
#pragma unroll
        for (int ks = 0; ks < KD; ++ks) kf[ks] = kread(ks);
#pragma unroll
        for (int ks = 0; ks < 2 * NCB; ++ks) {
            if (ks + KD < 2 * NCB) kf[ks + KD] = kread(ks + KD);
            __builtin_amdgcn_sched_barrier(0);
            s = fa_mfma(kf[ks], qf[ks], s);
        }
        __builtin_amdgcn_sched_barrier(0);
        const bool tail = key0 + FA_BK > rows;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            s[i] *= sc;
            if (tail && key0 + 8 * (i >> 2) + 4 * h + (i & 3) >= rows) s[i] = -INFINITY;
        }
        return s;
    };

    const int nt = (rows + FA_BK - 1) / FA_BK;
    // one tile sequence u = 0 .. 2 nt - 1 (pass u / nt over key tile u % nt) in slot u & 1, each tile's
    // DMA issued at the top of the one before; two loops, so that the accumulator is carried (and
    // touched) only by the MFMAs of the second
    load_tile(0, 0, false);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int t = 0; t < nt; ++t) {
        // pass 1: this lane's running max and sum over its keys
        if (t + 1 < nt) load_tile((t + 1) * FA_BK, (t + 1) & 1, false);
        else load_tile(0, nt & 1, true);
        const f32x16_t s = scores(smem_base + (t & 1) * G::SLOT, t * FA_BK);
        float mx = m;
#pragma unroll
        for (int i = 0; i < 16; ++i) mx = fmaxf(mx, s[i]);
        // reference point: mx, or 0 while every key this lane has seen is masked (no -inf - -inf)
        const float mr = mx == -INFINITY ? 0.f : mx;
        float ps = 0.f;
#pragma unroll
        for (int i = 0; i < 16; ++i) ps += __builtin_amdgcn_exp2f(s[i] - mr);
        l = l * __builtin_amdgcn_exp2f(m - mr) + ps;      // m = -inf before this lane's first key: 0
        m = mx;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    {
        // merge the two lane halves of each row; l becomes 1 / (row sum)
        const float m2 = __shfl_xor(m, 32), l2 = __shfl_xor(l, 32);
        const float mt = fmaxf(m, m2);
        l = 1.0f / (l * __builtin_amdgcn_exp2f(m - mt) + l2 * __builtin_amdgcn_exp2f(m2 - mt));
        m = mt;
    }
    for (int t = 0; t < nt; ++t) {
        // pass 2: P = bf16(softmax) as the B operand of O^T += V^T P
        const int u = nt + t;
        if (t + 1 < nt) load_tile((t + 1) * FA_BK, (u + 1) & 1, true);
        const unsigned sb = smem_base + (u & 1) * G::SLOT;
        const f32x16_t s = scores(sb, t * FA_BK);
        bf16x8_t pf[2];
#pragma unroll
        for (int i = 0; i < 16; ++i) pf[i >> 3][i & 7] = (__bf16)(__builtin_amdgcn_exp2f(s[i] - m) * l);
        // step j = (column block b = j / 2 of 32 d, k-step kk = j % 2 of 16 keys), its V^T fragment
        // read VD steps ahead
        constexpr int VD = 2;
        unsigned vb[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            vb[j] = sb + voff[j];
            asm volatile("" : "+v"(vb[j]));
        }
        auto vread = [&](int j) {
            const int b = j >> 1, kk = j & 1;
            const unsigned a0 = vb[b & 3] + 256 * (b >> 2) + kk * 16 * 2 * C;
            const i16x4_t v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS i16x4_t*)(uintptr_t)a0);
            const i16x4_t v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS i16x4_t*)(uintptr_t)(a0 + 8 * 2 * C));
            return __builtin_shufflevector(__builtin_bit_cast(bf16x4_t, v0), __builtin_bit_cast(bf16x4_t, v1), 0, 1,
                                           2, 3, 4, 5, 6, 7);
        };
        bf16x8_t vf[2 * NCB];
#pragma unroll
        for (int j = 0; j < VD; ++j) vf[j] = vread(j);
#pragma unroll
        for (int j = 0; j < 2 * NCB; ++j) {
            if (j + VD < 2 * NCB) vf[j + VD] = vread(j + VD);
            __builtin_amdgcn_sched_barrier(0);
            o[j >> 1] = fa_mfma(vf[j], pf[j & 1], o[j >> 1]);
        }
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }

    // O[q][d] = O^T: lane `col`'s row, d = 32b + 8g + 4h + e -> 8-byte stores
    if (qr < rows) {
        bf16_t* orow = out + z * o_zs + (long long)qr * ldo + 4 * h;
#pragma unroll
        for (int b = 0; b < NCB; ++b)
#pragma unroll
            for (int g = 0; g < 4; ++g)
                *reinterpret_cast<u32x2_t*>(orow + 32 * b + 8 * g) =
                    u32x2_t{pack2(o[b][4 * g], o[b][4 * g + 1]), pack2(o[b][4 * g + 2], o[b][4 * g + 3])};
    }
}

template <int NCB>
int launch_vae_attn(const void* qkv, long long qkv_zs, long long ld, void* out, long long o_zs, long long ldo,
                    int nz, int rows, hipStream_t st) {
    using G = FaGeom<NCB>;
    auto kern = vae_attn_kernel<NCB>;
    static std::once_flag attr;      // (per instantiation; the launch path may run on several host threads)
    std::call_once(attr, [&] {
        (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS);
    });
    const float sc = 1.4426950408889634f / sqrtf((float)G::C);
    dim3 grid((unsigned)((rows + FA_BQ - 1) / FA_BQ), (unsigned)nz);
    hipLaunchKernelGGL(kern, grid, dim3(FA_THR), G::LDS, st, (const bf16_t*)qkv, qkv_zs, ld, (bf16_t*)out, o_zs,
                       ldo, rows, sc);
    VS_CHECK_LAUNCH();
    return VS_OK;
}

}  // namespace

extern "C" int vs_vae_attention(const void* qkv, long long qkv_zs, long long ld_qkv, void* out, long long o_zs,
                                long long ld_o, int nz, int rows, int c, void* stream) {
    if (!qkv || !out || nz <= 0 || rows <= 0 || c <= 0 || c % 128 || c > 384 || ld_qkv < 3LL * c || ld_o < c ||
        ld_qkv % 8 || ld_o % 4 || qkv_zs < (long long)rows * ld_qkv || o_zs < (long long)rows * ld_o)
        return VS_E_INVALID;
    if ((uintptr_t)qkv & 15 || (uintptr_t)out & 7) return VS_E_INVALID;
    hipStream_t st = (hipStream_t)stream;
    switch (c / 32) {
        case 4: return launch_vae_attn<4>(qkv, qkv_zs, ld_qkv, out, o_zs, ld_o, nz, rows, st);
        case 8: return launch_vae_attn<8>(qkv, qkv_zs, ld_qkv, out, o_zs, ld_o, nz, rows, st);
        case 12: return launch_vae_attn<12>(qkv, qkv_zs, ld_qkv, out, o_zs, ld_o, nz, rows, st);
        default: return VS_E_INVALID;
    }
}
