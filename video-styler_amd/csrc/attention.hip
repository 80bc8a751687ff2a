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
constexpr int KROW = 272;        // LDS row pitch of the K tile (256 B + 16): row reads conflict-free
constexpr int VROW = 320;        // LDS row pitch of the V tile (256 B + 64): transposed reads conflict-free
constexpr int KT = BKV * KROW;   // 17408
constexpr int VT = BKV * VROW;   // 20480
constexpr int LDS_BYTES = 2 * (KT + VT);   // K ring 2 x 17408 + V ring 2 x 20480
constexpr float RESCALE_THR = 8.0f;   // lazy rescale (exp2 domain): skip while the max grows <= 2^8

typedef int i32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, unsigned bytes) {
    // raw buffer descriptor; out-of-range loads return 0 (rows past Skv, masked anyway)
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, bytes, 0x00020000);
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
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
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

    // buffer descriptors over this (batch, head)'s K/V rows; per-lane byte offset constant, the
    // tile's row offset goes to the scalar soffset
    const unsigned kbytes = (unsigned)min((long long)(Skv - 1) * ldk * 2 + HD * 2, 0xffffffffLL);
    const unsigned vbytes = (unsigned)min((long long)(Skv - 1) * ldv * 2 + HD * 2, 0xffffffffLL);
    const __amdgpu_buffer_rsrc_t krs = make_rsrc(Kb, kbytes), vrs = make_rsrc(Vb, vbytes);
    const int srow = tid >> 4, sch = tid & 15;            // chunk tid -> row srow (and srow+32)
    const unsigned kvo0 = (unsigned)(srow * ldk * 2 + sch * 16), kvo1 = kvo0 + (unsigned)(32 * ldk * 2);
    const unsigned vvo0 = (unsigned)(srow * ldv * 2 + sch * 16), vvo1 = vvo0 + (unsigned)(32 * ldv * 2);
    const int kw = srow * KROW + sch * 16, vw = srow * VROW + sch * 16;

    // K ring (2 slots) runs one tile ahead of the V ring (2 slots): iteration i reads K(i+1)
    // (for the next S^T) and V(i) (for this tile's PV), and stages K(i+2), V(i+1).
    i32x4_t kst[2], vst[2];
    auto load_k = [&](int kv0) {
        const int ks = kv0 * (int)ldk * 2;
        kst[0] = __builtin_amdgcn_raw_buffer_load_b128(krs, kvo0, ks, 0);
        kst[1] = __builtin_amdgcn_raw_buffer_load_b128(krs, kvo1, ks, 0);
    };
    auto load_v = [&](int kv0) {
        const int vs = kv0 * (int)ldv * 2;
        vst[0] = __builtin_amdgcn_raw_buffer_load_b128(vrs, vvo0, vs, 0);
        vst[1] = __builtin_amdgcn_raw_buffer_load_b128(vrs, vvo1, vs, 0);
    };
    auto store_k = [&](int slot) {
        char* base = smem + slot * KT;
        *reinterpret_cast<i32x4_t*>(base + kw) = kst[0];
        *reinterpret_cast<i32x4_t*>(base + kw + 32 * KROW) = kst[1];
    };
    auto store_v = [&](int slot) {
        char* base = smem + 2 * KT + slot * VT;
        *reinterpret_cast<i32x4_t*>(base + vw) = vst[0];
        *reinterpret_cast<i32x4_t*>(base + vw + 32 * VROW) = vst[1];
    };

    // per-lane LDS read bases (everything else is an immediate offset)
    const int krd = r * KROW + 16 * hh;                   // + t*32*KROW + 32*ss
    const int g4 = lane >> 4, q4 = (lane & 15) >> 2, p4 = lane & 3;
    const int vrd = (4 * (g4 >> 1) + q4) * VROW + 32 * (g4 & 1) + 8 * p4;   // + ks*16*VROW + 64*dt (+8 rows)

    // S^T for keys 0-31 (t=0) and 32-63 (t=1) as two interleaved accumulation chains; K fragments
    // are read two d-steps ahead of their MFMAs so LDS latency hides under the chain.
    auto qk = [&](int slot, f32x16_t* s) {
        const char* base = smem + slot * KT + krd;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            s[0][i] = 0.f;
            s[1][i] = 0.f;
        }
        bf16x8_t ka = *reinterpret_cast<const bf16x8_t*>(base);
        bf16x8_t kb = *reinterpret_cast<const bf16x8_t*>(base + 32 * KROW);
#pragma unroll
        for (int ss = 0; ss < 8; ++ss) {
            bf16x8_t na, nb;
            if (ss + 1 < 8) {
                na = *reinterpret_cast<const bf16x8_t*>(base + 32 * (ss + 1));
                nb = *reinterpret_cast<const bf16x8_t*>(base + 32 * KROW + 32 * (ss + 1));
            }
            // keep the next fragments' LDS reads issued ahead of this step's MFMAs
            __builtin_amdgcn_sched_barrier(0);
            s[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ka, qf[ss], s[0], 0, 0, 0);
            s[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kb, qf[ss], s[1], 0, 0, 0);
            if (ss + 1 < 8) {
                ka = na;
                kb = nb;
            }
        }
    };
    // online softmax in the exp2 domain (c = scale*log2 e) with a lazy rescale: the reference max
    // m only moves when some row's max exceeds it by more than RESCALE_THR, so P <= 2^THR.
    // Runs after the previous tile's PV has been issued and before this tile's PV (T13 order).
    auto softmax = [&](f32x16_t* s, int kv0, bool mask) {
        if (mask) {
            asm volatile("");     // keep this a real (uniform) branch: never if-convert into every tile
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const int key = kv0 + 32 * t + (i & 3) + 8 * (i >> 2) + 4 * hh;
                    if (key >= Skv) s[t][i] = -INFINITY;
                }
        }
        float mx = s[0][0];
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int i = 0; i < 16; ++i) mx = fmaxf(mx, s[t][i]);
        mx = fmaxf(mx, __shfl_xor(mx, 32)) * c;
        if (__any(mx > m + RESCALE_THR)) {
            const float mnew = fmaxf(m, mx);
            const float alpha = __builtin_amdgcn_exp2f(m - mnew);
            m = mnew;
            l *= alpha;
#pragma unroll
            for (int dt = 0; dt < 4; ++dt)
#pragma unroll
                for (int i = 0; i < 16; ++i) o[dt][i] *= alpha;
        }
        float rs = 0.f;
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const float p = __builtin_amdgcn_exp2f(fmaf(s[t][i], c, -m));
                s[t][i] = p;
                rs += p;
            }
        l += rs;
    };
    // O^T += V^T P over 4 k-steps of 16 keys
    auto pv = [&](int slot, const f32x16_t* s) {
        const char* base = smem + 2 * KT + slot * VT;
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            const int t = ks >> 1, u = ks & 1;
            bf16x8_t pf;
#pragma unroll
            for (int j = 0; j < 8; ++j) pf[j] = (__bf16)s[t][8 * u + j];
#pragma unroll
            for (int dt = 0; dt < 4; ++dt) {
                const char* a0 = base + vrd + ks * 16 * VROW + 64 * dt;
                const i16x4_t v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS i16x4_t*)(a0));
                const i16x4_t v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS i16x4_t*)(a0 + 8 * VROW));
                const bf16x8_t vf = __builtin_shufflevector(__builtin_bit_cast(bf16x4_t, v0),
                                                            __builtin_bit_cast(bf16x4_t, v1), 0, 1, 2, 3,
                                                            4, 5, 6, 7);
                o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf, o[dt], 0, 0, 0);
            }
        }
    };

    const int nkv = (Skv + BKV - 1) / BKV;
    // prologue: K(0), K(1), V(0) in LDS; S(0) computed by every wave; K(2) in flight to registers
    load_k(0);
    load_v(0);
    store_k(0);
    store_v(0);
    if (nkv > 1) {
        load_k(BKV);
        store_k(1);
    }
    __syncthreads();
    f32x16_t sa[2], sb[2];
    qk(0, sa);
    if (nkv > 2) load_k(2 * BKV);
    __syncthreads();      // every wave has read K slot 0 before it is restaged with K(2)

    // Staggered two-phase loop.  Per tile i every wave runs
    //   A_i: [load V(i+1)] QK(i+1) (MFMA) + softmax(i) (VALU) ; store K(i+2) -> K slot i&1
    //   B_i: [load K(i+3)] PV(i) (MFMA)                      ; store V(i+1) -> V slot (i+1)&1
    // with a barrier after each phase.  Waves 4-7 pass one extra barrier first, so on every SIMD
    // one wave's softmax overlaps its partner's MFMAs.  Ring hazards (phase index of group 0 /
    // group 1 = 2i / 2i+1 for A_i, 2i+1 / 2i+2 for B_i): K(i+2) is written in phases 2i..2i+1
    // after its slot's last read (qk(i), phases 2i-2..2i-1) and before its first read (qk(i+2),
    // phases 2i+2..2i+3); V(i+1) is written in 2i+1..2i+2, after pv(i-1) (2i-1..2i) and before
    // pv(i+1) (2i+3..2i+4).
    auto phase_bar = [&]() {
        __builtin_amdgcn_sched_barrier(0);
        __syncthreads();
        __builtin_amdgcn_sched_barrier(0);
    };
    const int grp = wave >> 2;
    // static priority for the younger half (waves 4-7): it loses VALU arbitration to the older
    // half on every segment otherwise (CDNA guide T5 static form; readfirstlane keeps it scalar)
#ifdef VS_ATTN_YOUNG_PRIO  // measured -1.2 % on MI355X (1067 vs 1080 TF/s): off
    if (__builtin_amdgcn_readfirstlane(threadIdx.x) >= 256) __builtin_amdgcn_s_setprio(1);
#endif
    if (grp == 1) phase_bar();
    auto body = [&](int it, f32x16_t* cur, f32x16_t* nxt) {
        const bool has1 = it + 1 < nkv, has2 = it + 2 < nkv, has3 = it + 3 < nkv;
        // ---- phase A
        if (has1) load_v((it + 1) * BKV);
        if (has1) qk((it + 1) & 1, nxt);
        softmax(cur, it * BKV, (it + 1) * BKV > Skv);
        if (has2) store_k(it & 1);
        phase_bar();
        // ---- phase B
        if (has3) load_k((it + 3) * BKV);
        pv(it & 1, cur);
        if (has1) store_v((it + 1) & 1);
        phase_bar();
    };
    int it = 0;
    for (; it + 1 < nkv; it += 2) {
        body(it, sa, sb);
        body(it + 1, sb, sa);
    }
    if (it < nkv) body(it, sa, sb);
    if (grp == 0) phase_bar();

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
    // buffer addressing: one (batch, head) K/V slab and a tile's row offset must fit 32 bits
    if ((long long)skv * ldk * 2 >= (1LL << 31) || (long long)skv * ldv * 2 >= (1LL << 31)) return VS_E_UNSUPPORTED;
    const int nqb = (sq + BQ - 1) / BQ;
    const long long nwg = (long long)nqb * heads * batch;
    if (nwg > 0x7fffffff) return VS_E_INVALID;
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)attn_fwd_d128, hipFuncAttributeMaxDynamicSharedMemorySize,
                            LDS_BYTES);
        attr_set = true;
    }
    const float c = scale * 1.4426950408889634f;
    hipLaunchKernelGGL(attn_fwd_d128, dim3((unsigned)nwg), dim3(NTHR), LDS_BYTES,
                       (hipStream_t)stream, (const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v,
                       (bf16_t*)o, sq, skv, heads, ldq, ldk, ldv, ldo, bsq, bsk, bsv, bso, c, nqb);
    VS_CHECK_LAUNCH();
    return VS_OK;
}
