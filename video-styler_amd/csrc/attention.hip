// Flash attention forward for Wan2.1 DiT (head_dim 128, non-causal, no mask), gfx950.
//
// Replaces flash_attention()/AttentionModule (reference diffsynth/models/wan_video_dit.py:28-61,
// 114-121): self-attention over S = T'*(H/16)*(W/16) latent tokens and cross-attention over the
// 512 T5 context tokens.
//
// Structure (one workgroup = 8 waves = 256 query rows of one (batch, head)):
//  * each wave owns 32 query rows; its Q slice (32 x 128 bf16, pre-scaled by log2(e)/sqrt(d))
//    lives in 32 VGPRs for the whole key sweep, in the B-operand layout of v_mfma_f32_32x32x16_bf16;
//  * K/V tiles of 64 keys are register-staged global->LDS through 2-slot rings (buffer loads
//    issued two phases before their LDS writes), rows padded to 272 / 320 B so the K row reads
//    (ds_read_b128) and the V transposed reads (ds_read_b64_tr_b16) are bank-conflict free;
//  * S^T = K Q^T (swapped product): every lane holds 32 scores of ONE query row;
//    O^T = V^T P with P packed to bf16 in registers as the B operand; the O accumulator of a
//    lane belongs to its own query row, so every rescale is lane-local;
//  * two phases per tile with the two wave halves one barrier apart (kernel comment below);
//  * workgroup ids are remapped so each XCD works through contiguous (batch, head) ranges: the
//    K/V of one head is streamed by the 32 CUs of one XCD together and served from its L2;
//  * persistent grid (one workgroup per CU, several items each, r2): the K/V pipeline runs on
//    across item boundaries as one flattened tile sequence, the next item's Q is prefetched into
//    LDS (prescaled) during the current item's first 8 tiles, and the finished item's O is stored
//    inside the phase that completes it -- no per-item prologue or drain (worth most on the
//    cross-attention, whose 512 keys are only 8 tiles per item).
#include "common.h"
#include "attention.h"
#include <algorithm>
#include <set>

namespace {
using namespace vs_attn;

constexpr int NTHR = 512;
constexpr int KROW = 272;        // LDS row pitch of the K tile (256 B + 16): row reads conflict-free
constexpr int VROW = 320;        // LDS row pitch of the V tile (256 B + 64): transposed reads conflict-free
constexpr int KT = BKV * KROW;   // 17408
constexpr int VT = BKV * VROW;   // 20480
constexpr int LDS_BYTES = 2 * (KT + VT);   // K ring 2 x 17408 + V ring 2 x 20480
constexpr int PERSIST_MIN_TILES = 8;



// ---------------------------------------------------------------------------------------------
// Two phases per 64-key tile, the two wave halves one barrier apart, one S tile live:
//   B_{i-1}: [store K(i+1) -> slot (i+1)&1; load V(i)]   S = K(i) Q^T (16 MFMA) || exps of S's keys 0-31
//   A_i:     [store V(i) -> slot i&1; load K(i+2)]   O^T += V(i-1)^T P(i-1) (16 MFMA)
//            || pack keys 0-31, softmax of keys 32-63 -> P(i)
// (the LDS stores open the phase: +1 % over storing at its end, profiles/r1/attention_ab_r1l.log)
// (the split puts half of the exps and row sums into the QK phase's empty VALU slots: +2.3 % on
// the 14B shape, profiles/r1/attention_ab_r1l.log), and the softmax is a max-free fast path:
// p = exp2(c*s - m) against the current reference max m, packed to bf16, and a lane's tile
// partial sum rs (both halves) checked once per tile.  Every p <= rs,
// so rs <= SUM_THR (= 2^8) guarantees P <= 2^8 -- the bound of v1's lazy rescale (CDNA guide T13).
// When any lane of the wave exceeds it (only when a row's max has grown), the exact path runs
// after the tile's PV(i-1) MFMAs: row max, m' = max(m, max), O (which already holds
// P(i-1)V(i-1) at the old scale) and l scaled by exp2(m - m'), P(i) recomputed (the keys 0-31 half
// from log2 of its in-place exps, or from K in global memory if one overflowed or underflowed).
// An item starts from m = 0 and keeps it through its first tile unless a lane's partial sum is
// above SUM_THR or below SUM_MIN (r2; r1 always took the exact path there): exp2(S) of any row
// whose max score is above -60 (exp2 domain) is a normal float, and p's relative precision does
// not depend on the reference max, so the first tile needs no max pass on typical scores -- an
// eighth of the tiles of a 512-key cross-attention item.
// Ring hazards (group 0 runs B_{i-1} at phase 2i and A_i at 2i+1, group 1 one phase later):
// K(i+1) is written at 2i / 2i+1 into the slot K(i-1) was read from at 2i-2 / 2i-1 and first read
// at 2i+2; V(i) is written at 2i+1 / 2i+2 into the slot V(i-2) was read from at 2i-1 / 2i and first
// read at 2i+3.  Per-tile VALU ~460 issue cycles (the previous structure, with a max pass, a
// shuffle and a two-deep S ring: ~850).  Epilogue: permlane32_swap pairs -> 16-B stores (T21).
constexpr float SUM_THR = 256.0f;
constexpr float SUM_MIN = 0x1p-60f;
// ---------------------------------------------------------------------------------------------
// Optimistic softmax (NC, r2, M16 only; the default when the caller bound an item-flag workspace):
// no reference max at all -- p = exp2(c*qk) -- and no per-tile check, the row sums l on the matrix
// pipe as the O^T rows of a ones block of V^T (4 extra MFMAs per tile instead of 32 fp32 adds and
// the tile's check per lane: -24 % of the loop's VALU issue, +3.5...6 % self-attention throughput,
// profiles/r2/attn_nc_ab.log).  Exact while no p overflows or underflows; an item whose final row
// sum leaves [NC_LMIN, NC_LMAX] (a row max above 64 or below -64 in the exp2 domain) is flagged
// and recomputed by the checked kernel (the redo launch), so the result is either the optimistic
// one -- which sums the P actually multiplied with V -- or bit for bit the checked one.  With
// l <= 2^64 the fp32 O accumulators stay finite for |v| < 2^64.

// v_mfma_f32_32x32x16_bf16.  VS_ATTN_DIAG_MFMA16 (timing diagnostic only, wrong results): the same
// FLOPs as two v_mfma_f32_16x16x32_bf16 on the same operands, to measure the clock / issue effect
// of the smaller MFMA shape on this loop (MI355X_MICROARCH 'DVFS give-back' item 7)
__device__ __forceinline__ f32x16_t mfma32(bf16x8_t a, bf16x8_t b, f32x16_t c, int half = 0) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// v_mfma_f32_16x16x32_bf16 on the 4-value group g of a 16-value accumulator block (the M16 layout
// keeps the M32 register shapes: s[2], o[4] as f32x16, four 16x16 tiles each).  On random data the
// chip holds a higher clock on this shape than on 32x32x16 at equal cycles per FLOP
// (MI355X_MICROARCH 'DVFS give-back' item 7).
__device__ __forceinline__ f32x4_t grp4(const f32x16_t& c, int g) {
    return f32x4_t{c[4 * g], c[4 * g + 1], c[4 * g + 2], c[4 * g + 3]};
}
// c with group g replaced by a*b + acc
__device__ __forceinline__ f32x16_t mfma16g(bf16x8_t a, bf16x8_t b, f32x16_t c, int g, f32x4_t acc) {
    const f32x4_t t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
    c[4 * g] = t[0];
    c[4 * g + 1] = t[1];
    c[4 * g + 2] = t[2];
    c[4 * g + 3] = t[3];
    return c;
}

// scheduling fences inside the QK / PV step sequences (VS_ATTN_SB_FREE_QK / _PV: A/B builds that let
// the machine scheduler move instructions across k-steps)
#define ATTN_SB_QK() __builtin_amdgcn_sched_barrier(0)
#define ATTN_SB_PV() __builtin_amdgcn_sched_barrier(0)

#define ATTN_STAMP(slot) do {} while (0)


template <bool REBASE, bool M16, int MODE>
__global__ __launch_bounds__(NTHR) void attn_fwd_d128(const AttnArgs args) {
    // Persistent items: an item switch stores O and loads the next Q directly (one stall per item)
    // while the K/V pipeline runs on across the boundary (r2 measured the alternative -- the next
    // Q prefetched and O drained inside the first 8 tiles through range-gated loads / stores -- 6 %
    // slower on the 14B self-attention: the per-tile descriptor arithmetic costs more than the
    // stall; profiles/r2/attn_pf_ab.log).
    extern __shared__ __attribute__((aligned(16))) char smem[];
    // NC: optimistic softmax (comment at NC_LMIN); M16 only
    // REDO: the checked kernel over the items the NC launch listed (grid-strided over the list)
    constexpr bool NC = M16 && MODE == MODE_NC, REDO = MODE == MODE_REDO;
    // LDS images: M32 pads the rows (K 272 B, V 320 B); M16 (v_mfma_f32_16x16x32_bf16, see mfma16
    // below) stores K rows unpadded with the 16-B chunk XOR-swizzled by (row & 15) and pads V rows
    // to 288 B, so both of its read patterns are bank-conflict free
    constexpr int KRW = M16 ? 256 : KROW, VRW = M16 ? 288 : VROW;
    constexpr int KTS = BKV * KRW, VTS = BKV * VRW;
    // the argument block itself (the kernel's only argument, at the start of the kernarg segment):
    // volatile scalar loads of it are not hoisted out of the tile loop
    typedef const volatile AttnArgs __attribute__((address_space(4))) ColdArgs;
    ColdArgs* cold = (ColdArgs*)__builtin_amdgcn_kernarg_segment_ptr();
    const int Sq = args.Sq, Skv_all = args.Skv, nmain = args.nmain, npers = args.npers;
    const int nsplit = args.nsplit, piece_tiles = args.piece_tiles;
    const long long ldq = args.ldq, ldk = args.ldk, ldv = args.ldv, ldo = args.ldo;
    const float c = args.c;
    float* const part = args.part;

    int piece = -1, kv_begin = 0, Skv = Skv_all;
    int g0, gstride, n_items;
    const int* rlist = nullptr;
    if constexpr (REDO) {
        // block b takes list entries b, b + grid, ...; the last block to have read the count
        // resets count and done, every block clears the flags of its items
        int* const ws = args.flags;
        const int cnt = *reinterpret_cast<volatile int*>(ws);
        const int R = gridDim.x;
        g0 = blockIdx.x;
        gstride = R;
        n_items = cnt > g0 ? (cnt - g0 + R - 1) / R : 0;
        rlist = ws + 2 + args.nc_cap;
        __syncthreads();
        if (threadIdx.x == 0) {
            for (int j = 0; j < n_items; ++j) ws[2 + rlist[g0 + j * R]] = 0;
            if (atomicAdd(ws + 1, 1) == R - 1) {
                ws[0] = 0;
                ws[1] = 0;
            }
        }
    } else if ((int)blockIdx.x < npers) {
        const int x = blockIdx.x & 7, lb = blockIdx.x >> 3;
        const int qx = nmain >> 3, rx = nmain & 7, qbk = npers >> 3, rbk = npers & 7;
        const int cs = x < rx ? x * (qx + 1) : rx * (qx + 1) + (x - rx) * qx;
        const int csz = qx + (x < rx ? 1 : 0);
        gstride = qbk + (x < rbk ? 1 : 0);
        g0 = cs + lb;
        n_items = lb < csz ? (csz - lb + gstride - 1) / gstride : 0;
    } else {
        const int t = blockIdx.x - npers;
        g0 = nmain + t / nsplit;
        gstride = 0;
        n_items = 1;
        piece = t % nsplit;
        kv_begin = piece * piece_tiles * BKV;
        Skv = min(Skv_all - kv_begin, piece_tiles * BKV);
    }
    if (n_items == 0) return;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 31, hh = lane >> 5;

    // per-item offsets (b, h from the item id): element offsets of the item's Q / K / V / O head
    // column block, and the item's first query row (the wave's rows start 32 * wave further)
    auto item_bh = [&](int j, int& qrow0) {
        const int nqb = cold->nqb;
        const int g = REDO ? rlist[g0 + j * gstride] : g0 + j * gstride;
        const int qb = g % nqb, bh = g / nqb;
        qrow0 = qb * BQ;
        return bh;
    };
    auto q_base = [&](int bh) {
        const int H = cold->H;
        return cold->Q + (long long)(bh / H) * cold->bsq + (bh % H) * HD;
    };
    auto k_base = [&](int bh) {
        const int H = cold->H;
        return cold->K + (long long)(bh / H) * cold->bsk + (long long)kv_begin * ldk + (bh % H) * HD;
    };
    auto v_base = [&](int bh) {
        const int H = cold->H;
        return cold->V + (long long)(bh / H) * cold->bsv + (long long)kv_begin * ldv + (bh % H) * HD;
    };
    auto o_base = [&](int bh) {
        const int H = cold->H;
        return cold->O + (long long)(bh / H) * cold->bso + (bh % H) * HD;
    };
    const int g = g0;               // the first item (the split-tail piece's only one)
    int q0;
    int bh_cur = item_bh(0, q0);
    q0 += wave * 32;
    const bf16_t* Kb = k_base(bh_cur);   // K of the item whose tiles QK reads (exact-path recompute)

    // buffer descriptors over this (batch, head)'s K/V rows: per-lane byte offset constant, the
    // tile's row offset in soffset.  REBASE (a slab beyond 2^31 bytes, e.g. 1280x720x121 with the
    // fused q|k|v row layout: 111600 rows x 30 KB): the descriptor is rebuilt per tile on a 64-bit
    // base (1.6 % slower, so only when needed).  Rows past Skv read as 0 (masked anyway).  K loads
    // run two tiles ahead of QK, V loads one: across an item boundary each loader keeps the
    // descriptor of the item it loads from.
    const int srow = tid >> 4, sch = tid & 15;
    const unsigned kvo0 = (unsigned)(srow * ldk * 2 + sch * 16), kvo1 = kvo0 + (unsigned)(32 * ldk * 2);
    const unsigned vvo0 = (unsigned)(srow * ldv * 2 + sch * 16), vvo1 = vvo0 + (unsigned)(32 * ldv * 2);
    const int kw = srow * KRW + (M16 ? (sch ^ (srow & 15)) : sch) * 16, vw = srow * VRW + sch * 16;

    i32x4_t kst[2], vst[2];
    const int ldk32 = (int)ldk, ldv32 = (int)ldv;   // host: 64 * ld * 2 < 2^31
    auto slab_rsrc = [&](const bf16_t* base, int ld) {
        return make_rsrc(base, REBASE ? 0u : (unsigned)((Skv - 1) * ld * 2 + HD * 2));
    };
    const bf16_t* Kload = Kb;       // base of the K loader's item, and its descriptor
    const bf16_t* Vload = v_base(bh_cur);
    __amdgpu_buffer_rsrc_t krs = slab_rsrc(Kload, ldk32);
    __amdgpu_buffer_rsrc_t vrs = slab_rsrc(Vload, ldv32);
    auto tile_rsrc = [&](const bf16_t* base, int ld, int kv0) {
        const int rows = min(BKV, Skv - kv0);
        return make_rsrc(base + (long long)kv0 * ld, (unsigned)((rows - 1) * ld * 2 + HD * 2));
    };
    auto load_k = [&](int kv0) {
        if constexpr (REBASE) {
            const __amdgpu_buffer_rsrc_t rs = tile_rsrc(Kload, ldk32, kv0);
            kst[0] = __builtin_amdgcn_raw_buffer_load_b128(rs, kvo0, 0, 0);
            kst[1] = __builtin_amdgcn_raw_buffer_load_b128(rs, kvo1, 0, 0);
        } else {
            const int ks = kv0 * ldk32 * 2;
            kst[0] = __builtin_amdgcn_raw_buffer_load_b128(krs, kvo0, ks, 0);
            kst[1] = __builtin_amdgcn_raw_buffer_load_b128(krs, kvo1, ks, 0);
        }
    };
    auto load_v = [&](int kv0) {
        if constexpr (REBASE) {
            const __amdgpu_buffer_rsrc_t rs = tile_rsrc(Vload, ldv32, kv0);
            vst[0] = __builtin_amdgcn_raw_buffer_load_b128(rs, vvo0, 0, 0);
            vst[1] = __builtin_amdgcn_raw_buffer_load_b128(rs, vvo1, 0, 0);
        } else {
            const int vs = kv0 * ldv32 * 2;
            vst[0] = __builtin_amdgcn_raw_buffer_load_b128(vrs, vvo0, vs, 0);
            vst[1] = __builtin_amdgcn_raw_buffer_load_b128(vrs, vvo1, vs, 0);
        }
    };
    auto store_k = [&](int slot) {
        char* base = smem + slot * KTS;
        *reinterpret_cast<i32x4_t*>(base + kw) = kst[0];
        *reinterpret_cast<i32x4_t*>(base + kw + 32 * KRW) = kst[1];   // ((srow + 32) & 15 == srow & 15)
    };
    auto store_v = [&](int slot) {
        char* base = smem + 2 * KTS + slot * VTS;
        *reinterpret_cast<i32x4_t*>(base + vw) = vst[0];
        *reinterpret_cast<i32x4_t*>(base + vw + 32 * VRW) = vst[1];
    };

    const int nkv = (Skv + BKV - 1) / BKV;
    const int Ttot = n_items * nkv;           // the flattened tile sequence of all this block's items
    // K loader cursor: item kj, tile ki of the next K tile to load (two tiles ahead of QK)
    int kj = 0, ki = 0;
    auto k_next = [&]() {
        if (++ki == nkv) {
            ki = 0;
            if (++kj < n_items) {
                int unused;
                Kload = k_base(item_bh(kj, unused));
                krs = slab_rsrc(Kload, ldk32);
            }
        }
    };
    // prologue: K(0) staged and in LDS, K(1) in flight, Q fragments (B operand of S^T = K Q^T)
    load_k(0);
    k_next();
    // Q fragments, the B operand of S^T = K Q^T, pre-scaled by c = log2(e)/sqrt(d) (one bf16
    // rounding): S^T then lands in the exp2 domain and the softmax needs no multiply.
    //   M32: qf[s] = row q0 + r, columns 16s + 8hh .. +7;
    //   M16: qf[4qb + ks] = row q0 + 16qb + (lane & 15), columns 32ks + 8(lane >> 4) .. +7.
    // qoff(c): element offset of chunk c (the same mapping, relative to the wave's first row)
    const int lr = lane & 15, lg = lane >> 4;
    auto qoff = [&](int cidx) -> long long {
        if constexpr (M16)
            return (long long)(16 * (cidx >> 2) + lr) * ldq + 32 * (cidx & 3) + 8 * lg;
        else
            return (long long)r * ldq + 16 * cidx + 8 * hh;
    };
    bf16x8_t qf[8];
    // the item's Q rows from global memory (rows past Sq read row Sq - 1; their outputs are dropped)
    auto load_q = [&](const bf16_t* qb0, int q0v) __attribute__((always_inline)) {
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            const int qrow = q0v + (M16 ? 16 * (s >> 2) + lr : r);
            const long long off = qoff(s) + (qrow < Sq ? (long long)q0v * ldq
                                                      : (long long)(Sq - 1 - (qrow - q0v)) * ldq);
            const bf16x8_t raw = *reinterpret_cast<const bf16x8_t*>(qb0 + off);
#pragma unroll
            for (int j = 0; j < 8; ++j) qf[s][j] = (__bf16)((float)raw[j] * c);
        }
    };
    load_q(q_base(bh_cur), q0);
    store_k(0);
    if (Ttot > 1) {
        load_k(ki * BKV);
        k_next();
    }
    int q0_nxt = 0;                 // the next item: its Q rows and (b, h)
    int bh_nxt = n_items > 1 ? item_bh(1, q0_nxt) : 0;
    const bf16_t* qb_nxt = q_base(bh_nxt);
    q0_nxt += wave * 32;
    bf16_t* ob_cur = o_base(bh_cur);
    bf16_t* ob_prev = ob_cur;
    int q0_prev = q0;

    f32x16_t o[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i) o[dt][i] = 0.f;
    // Per-lane softmax state, per query row the lane holds: M32 one row (q0 + r; index 0), M16 two
    // (q0 + 16qb + (lane & 15), qb = 0, 1).  mq: the row's reference max (exp2 domain).  The QK
    // accumulators start at -m (negm, rewritten only by the exact path), so S^T = c*QK^T - m and
    // p = exp2(S).  m starts at 0; the exact path (on the first tile only when its sums leave
    // [SUM_MIN, SUM_THR]) moves it to a row max.  lq: the lane's partial row sums.
    float mq[2] = {0.f, 0.f}, lq[2] = {0.f, 0.f};
    // NC: the row sums of the bf16 P as O^T rows of a ones block of V^T (4 extra MFMAs per tile);
    // lane (lr, lg) holds row 16qb + lr's sum in every element of lsum[qb]
    f32x4_t lsum[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    bf16x8_t ones;
#pragma unroll
    for (int j = 0; j < 8; ++j) ones[j] = (__bf16)1.0f;
    f32x16_t negm;
#pragma unroll
    for (int i = 0; i < 16; ++i) negm[i] = 0.f;

    // Element layouts (M32 | M16):
    //   s[t][i]   S^T of keys 32t + (i&3) + 8(i>>2) + 4hh, row r | keys 32t + 16(i>>3) + 4lg + (i&3),
    //             row 16((i>>2)&1) + lr  (group (i>>2) = 2 kbl + qb of 4 values)
    //   pk[k]     P, the PV B operand: keys 16k .. 16k+15 of row r | keys 32(k&1) + {4lg .. 4lg+3,
    //             16+4lg .. 16+4lg+3} of row 16(k>>1) + lr (the V^T reads use the same key order)
    //   o[dt][i]  O^T of columns 32dt + (i&3) + 8(i>>2) + 4hh, row r | columns 16(2dt + (i>>3)) +
    //             4lg + (i&3), row 16((i>>2)&1) + lr
    const int krd = M16 ? 0 : r * KROW + 16 * hh;
    const int g4 = lane >> 4, q4 = (lane & 15) >> 2, p4 = lane & 3;
    const int vrd = M16 ? (4 * g4 + q4) * VRW + 8 * p4 : (4 * (g4 >> 1) + q4) * VROW + 32 * (g4 & 1) + 8 * p4;

    f32x16_t s[2];        // S^T of the current tile (layout above)
    u32x4_t pk[4];        // P as the PV B operands (bf16 pairs)
    // row-sum partials: rs0/rs1 of the s[1] half (PV phase), rsA/rsB of the s[0] half (QK phase);
    // M32: all four belong to the lane's one row; M16: rs0/rsA to row qb 0, rs1/rsB to qb 1
    float rs0, rs1;
    float rsA = 0.f, rsB = 0.f;
    auto row_tot = [&](int qb) { return M16 ? (qb ? rsB + rs1 : rsA + rs0) : rsA + rsB + rs0 + rs1; };
    auto p_chunk = [&](int ss) __attribute__((always_inline)) {   // elements 4ss..4ss+3 (flat 16t + i)
        const int t = ss >> 2, i0 = 4 * (ss & 3);
        const float p0 = __builtin_amdgcn_exp2f(s[t][i0]);
        const float p1 = __builtin_amdgcn_exp2f(s[t][i0 + 1]);
        const float p2 = __builtin_amdgcn_exp2f(s[t][i0 + 2]);
        const float p3 = __builtin_amdgcn_exp2f(s[t][i0 + 3]);
        const bf16x2_t w0 = {(__bf16)p0, (__bf16)p1}, w1 = {(__bf16)p2, (__bf16)p3};
        if constexpr (M16) {
            const int grp = ss & 3, kbl = grp >> 1, qb = grp & 1;
            if constexpr (!NC) (qb ? rs1 : rs0) += (p0 + p1) + (p2 + p3);
            pk[2 * qb + t][2 * kbl] = __builtin_bit_cast(unsigned, w0);
            pk[2 * qb + t][2 * kbl + 1] = __builtin_bit_cast(unsigned, w1);
        } else {
            rs0 += p0 + p1;
            rs1 += p2 + p3;
            const int ks = 2 * t + (i0 >> 3), j = (i0 & 7) >> 1;
            pk[ks][j] = __builtin_bit_cast(unsigned, w0);
            pk[ks][j + 1] = __builtin_bit_cast(unsigned, w1);
        }
    };
    // the s[0] half's exponentials (computed in place in the QK phase) packed into pk
    auto p_pack = [&](int ss) __attribute__((always_inline)) {
        const int i0 = 4 * ss;
        const bf16x2_t w0 = {(__bf16)s[0][i0], (__bf16)s[0][i0 + 1]};
        const bf16x2_t w1 = {(__bf16)s[0][i0 + 2], (__bf16)s[0][i0 + 3]};
        if constexpr (M16) {
            const int kbl = ss >> 1, qb = ss & 1;
            pk[2 * qb][2 * kbl] = __builtin_bit_cast(unsigned, w0);
            pk[2 * qb][2 * kbl + 1] = __builtin_bit_cast(unsigned, w1);
        } else {
            const int ks = i0 >> 3, j = (i0 & 7) >> 1;
            pk[ks][j] = __builtin_bit_cast(unsigned, w0);
            pk[ks][j + 1] = __builtin_bit_cast(unsigned, w1);
        }
    };
    auto mask_half = [&](int t, int kv0) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int key = M16 ? kv0 + 32 * t + 16 * (i >> 3) + 4 * lg + (i & 3)
                                : kv0 + 32 * t + (i & 3) + 8 * (i >> 2) + 4 * hh;
            if (key >= Skv) s[t][i] = -INFINITY;
        }
    };
    // S^T = K Q^T: the s[0] chain (keys 0-31, 8 d-steps) first, then the s[1] chain with the s[0]
    // half's softmax exps in place, two per MFMA gap, and their sum rsA (the QK phase's VALU slots
    // are otherwise empty; the PV phase keeps only the s[1] half).  K fragments are read
    // VS_ATTN_KDEPTH MFMAs ahead (default 4): with one step of look-ahead the QK burst stalls on
    // LDS latency and holds the SIMD's matrix pipe for ~2x its 16 MFMAs while the partner wave's
    // PV+softmax phase starves (measured with -DVS_ATTN_STAMPS).
#ifndef VS_ATTN_KDEPTH
#define VS_ATTN_KDEPTH 4
#endif
    auto qk16 = [&](int slot, int kv0) __attribute__((always_inline)) {
        // M16: 16 steps j = 8t + 2ks + kbl, each one K fragment (keys 16(2t + kbl) + lr, columns
        // 32ks + 8lg, from the swizzled image) feeding the two MFMAs of rows qb = 0, 1 into group
        // 2kbl + qb of s[t]; the s[0] half's exps, one per MFMA gap, in the s[1] half's steps
        const char* base = smem + slot * KTS;
#ifndef VS_ATTN_KDEPTH16
#define VS_ATTN_KDEPTH16 4
#endif
        constexpr int DEP = VS_ATTN_KDEPTH16;
        const bool last = kv0 + BKV > Skv;
        bf16x8_t kf[16];
        auto kaddr = [&](int j) {
            const int t = j >> 3, ks = (j >> 1) & 3, kbl = j & 1;
            return base + (16 * (2 * t + kbl) + lr) * KRW + (((4 * ks + lg) ^ lr) << 4);
        };
#pragma unroll
        for (int j = 0; j < DEP; ++j) kf[j] = *reinterpret_cast<const bf16x8_t*>(kaddr(j));
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            if (j + DEP < 16) kf[j + DEP] = *reinterpret_cast<const bf16x8_t*>(kaddr(j + DEP));
            if (j == 8 && last) mask_half(0, kv0);
            ATTN_SB_QK();
            const int t = j >> 3, ks = (j >> 1) & 3, kbl = j & 1;
#pragma unroll
            for (int qb = 0; qb < 2; ++qb) {
                const int g = 2 * kbl + qb;
                s[t] = mfma16g(kf[j], qf[4 * qb + ks], s[t], g, grp4(ks == 0 ? negm : s[t], g));
            }
            if (t == 1 && NC) {
                const int e = 2 * (j - 8);
                s[0][e] = __builtin_amdgcn_exp2f(s[0][e]);
                s[0][e + 1] = __builtin_amdgcn_exp2f(s[0][e + 1]);
                asm volatile("" : "+v"(s[0][e]), "+v"(s[0][e + 1]));
            } else if (t == 1) {
                const int e = 2 * (j - 8);
                s[0][e] = __builtin_amdgcn_exp2f(s[0][e]);
                s[0][e + 1] = __builtin_amdgcn_exp2f(s[0][e + 1]);
                const float pp = s[0][e] + s[0][e + 1];
                if ((e >> 2) & 1) {
                    rsB = (e & 3) == 0 && e < 8 ? pp : rsB + pp;
                    asm volatile("" : "+v"(rsB));
                } else {
                    rsA = e == 0 ? pp : rsA + pp;
                    asm volatile("" : "+v"(rsA));
                }
            }
        }
        __builtin_amdgcn_sched_barrier(0);
    };
    auto qk = [&](int slot, int kv0) __attribute__((always_inline)) {
        if constexpr (M16) {
            qk16(slot, kv0);
            return;
        }
        const char* base = smem + slot * KTS + krd;
        constexpr int DEP = VS_ATTN_KDEPTH;
        const bool last = kv0 + BKV > Skv;
        bf16x8_t kf[16];
        auto kaddr = [&](int j) { return base + (j >= 8 ? 32 * KROW : 0) + 32 * (j & 7); };
#pragma unroll
        for (int j = 0; j < DEP; ++j) kf[j] = *reinterpret_cast<const bf16x8_t*>(kaddr(j));
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            if (j + DEP < 16) kf[j + DEP] = *reinterpret_cast<const bf16x8_t*>(kaddr(j + DEP));
            if (j == 8 && last) mask_half(0, kv0);
            __builtin_amdgcn_sched_barrier(0);
            if (j < 8) {
                s[0] = mfma32(kf[j], qf[j], j == 0 ? negm : s[0], j & 1);
            } else {
                s[1] = mfma32(kf[j], qf[j - 8], j == 8 ? negm : s[1], j & 1);
                const int e = 2 * (j - 8);
                s[0][e] = __builtin_amdgcn_exp2f(s[0][e]);
                s[0][e + 1] = __builtin_amdgcn_exp2f(s[0][e + 1]);
                const float pp = s[0][e] + s[0][e + 1];
                rsA = j == 8 ? pp : rsA + pp;
                // pure VALU floats freely in the IR (past the phase barrier into its uses): tie
                // each pair to its MFMA gap
                asm volatile("" : "+v"(rsA));
            }
        }
        __builtin_amdgcn_sched_barrier(0);
    };
    // PV(prev) with the fast softmax of the current tile interleaved: the 4 MFMAs of k-step ks read
    // pk[ks] before the two chunks that overwrite it with P(i)
    // V^T fragments of k-step ks (4 B operands, one per 32-column block dt of O^T)
    auto read_vt = [&](const char* base, int ks, bf16x8_t* vf) {
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
            // M32: k-step ks (keys 16ks..), column block dt of 32; M16: step ks = 2c + h (key chunk
            // c of 32, column blocks db = 4h + dt of 16), rows 32c + 4lg + q4 and +16
            const char* a0 = M16 ? base + vrd + (ks >> 1) * 32 * VRW + 32 * (4 * (ks & 1) + dt)
                                 : base + vrd + ks * 16 * VROW + 64 * dt;
            const i16x4_t v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS i16x4_t*)(a0));
            const i16x4_t v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS i16x4_t*)(a0 + (M16 ? 16 : 8) * VRW));
            vf[dt] = __builtin_shufflevector(__builtin_bit_cast(bf16x4_t, v0), __builtin_bit_cast(bf16x4_t, v1),
                                             0, 1, 2, 3, 4, 5, 6, 7);
        }
    };
    // the MFMAs of PV step ks with V^T fragments vf: M32 4 (column blocks dt, P keys 16ks..);
    // M16 8 (column blocks db = 4(ks&1) + dt, rows qb, P key chunk c = ks >> 1)
    auto pv_step = [&](int ks, const bf16x8_t* vf) __attribute__((always_inline)) {
        if constexpr (M16) {
            const int cc = ks >> 1;
#pragma unroll
            for (int dt = 0; dt < 4; ++dt) {
                const int db = 4 * (ks & 1) + dt, ot = db >> 1;
#pragma unroll
                for (int qb = 0; qb < 2; ++qb) {
                    const int g = 2 * (db & 1) + qb;
                    o[ot] = mfma16g(vf[dt], __builtin_bit_cast(bf16x8_t, pk[2 * qb + cc]), o[ot], g, grp4(o[ot], g));
                }
            }
            if constexpr (NC) {
                if ((ks & 1) == 0) {
#pragma unroll
                    for (int qb = 0; qb < 2; ++qb)
                        lsum[qb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                            ones, __builtin_bit_cast(bf16x8_t, pk[2 * qb + cc]), lsum[qb], 0, 0, 0);
                }
            }
        } else {
#pragma unroll
            for (int dt = 0; dt < 4; ++dt)
                o[dt] = mfma32(vf[dt], __builtin_bit_cast(bf16x8_t, pk[ks]), o[dt], ks & 1);
        }
    };
    // PV(prev) with the fast softmax of the current tile interleaved; V^T fragments one step ahead.
    // M32: the 4 MFMAs of k-step ks read pk[ks] before the two chunks that overwrite it with P(i).
    // M16: the steps run key chunk 1 first (steps ks = 2, 3), then chunk 0 (ks = 0, 1): once chunk
    // 1's MFMAs are issued, the s[1] half's softmax (exps, sums, packs into the chunk-1 operands)
    // runs beside chunk 0's; the s[0] half (exponentiated in the QK phase) is packed at the end.
    auto pv_softmax = [&](int slot, bool with_pv) __attribute__((always_inline)) {
        const char* base = smem + 2 * KTS + slot * VTS;
        rs0 = 0.f;
        rs1 = 0.f;
        bf16x8_t va[4], vb[4];
        constexpr int order[4] = {M16 ? 2 : 0, M16 ? 3 : 1, M16 ? 0 : 2, M16 ? 1 : 3};
        if (with_pv) read_vt(base, order[0], va);
#pragma unroll
        for (int st = 0; st < 4; ++st) {
            const int ks = order[st];
            bf16x8_t* cur = (st & 1) ? vb : va;
            bf16x8_t* nxt = (st & 1) ? va : vb;
            if (with_pv) {
                if (st + 1 < 4) read_vt(base, order[st + 1], nxt);
                ATTN_SB_PV();
                pv_step(ks, cur);
            }
            if constexpr (M16) {
                if (st >= 2) {          // chunk 1's operands are free: the s[1] half, 2 groups a step
                    p_chunk(4 + 2 * (st - 2));
                    p_chunk(5 + 2 * (st - 2));
                    if constexpr (!NC) asm volatile("" : "+v"(rs0), "+v"(rs1));
                    asm volatile("" :: "v"(pk[1]), "v"(pk[3]));
                }
                if (st == 3) {          // chunk 0's operands are free once the last MFMAs issue
#pragma unroll
                    for (int ss = 0; ss < 4; ++ss) p_pack(ss);
                    asm volatile("" :: "v"(pk[0]), "v"(pk[2]));
                }
            } else {
                if (ks < 2) {               // keys 0-31: exponentiated in the QK phase, pack only
                    p_pack(2 * ks);
                    p_pack(2 * ks + 1);
                } else {                    // keys 32-63
                    p_chunk(2 * ks);
                    p_chunk(2 * ks + 1);
                    // tie the chunk's sums here so its exps land in this k-step's MFMA region
                    asm volatile("" : "+v"(rs0), "+v"(rs1));
                }
                // use P(i)'s packed k-step here: otherwise LLVM sinks every pack below the exact-path
                // branch and keeps the fp32 p values live through the PV phase
                asm volatile("" :: "v"(pk[ks]));
            }
            ATTN_SB_PV();
            if (with_pv) ATTN_STAMP(3 + st);
        }
    };
    // (the same step order as pv_softmax: O's fp32 sums then do not depend on where an item ends)
    auto pv_last = [&](int slot) {
        const char* base = smem + 2 * KTS + slot * VTS;
        constexpr int order[4] = {M16 ? 2 : 0, M16 ? 3 : 1, M16 ? 0 : 2, M16 ? 1 : 3};
#pragma unroll
        for (int st = 0; st < 4; ++st) {
            bf16x8_t vf[4];
            read_vt(base, order[st], vf);
            pv_step(order[st], vf);
        }
    };
    auto exact = [&](bool first) {
        // row max (S = c*qk - m, so the row's scaled max is max(S) + m): M32 over the lane's 32
        // values and its partner lane (xor 32); M16 per row qb over the lane's 16 values and the
        // 4 lanes holding that row (xor 16, xor 32)
        float mx[2];
#pragma unroll
        for (int qb = 0; qb < (M16 ? 2 : 1); ++qb) {
            float v = -INFINITY;
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int i = 0; i < 16; ++i)
                    if (!M16 || ((i >> 2) & 1) == qb) v = fmaxf(v, s[t][i]);
            if constexpr (M16) v = fmaxf(v, __shfl_xor(v, 16));
            mx[qb] = fmaxf(v, __shfl_xor(v, 32)) + mq[qb];
        }
        float delta[2], alpha[2];
#pragma unroll
        for (int qb = 0; qb < (M16 ? 2 : 1); ++qb) {
            const float mnew = first ? mx[qb] : fmaxf(mq[qb], mx[qb]);
            delta[qb] = mq[qb] - mnew;                   // <= 0 after the first tile
            // first tile: O and l are still 0 and delta is unbounded (exp2 may be inf): scale by 0
            alpha[qb] = first ? 0.f : __builtin_amdgcn_exp2f(delta[qb]);
            lq[qb] *= alpha[qb];
            mq[qb] = mnew;
        }
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
            for (int i = 0; i < 16; ++i) o[dt][i] *= alpha[M16 ? (i >> 2) & 1 : 0];
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int i = 0; i < 16; ++i) s[t][i] += delta[M16 ? (i >> 2) & 1 : 0];
#pragma unroll
        for (int i = 0; i < 16; ++i) negm[i] = -mq[M16 ? (i >> 2) & 1 : 0];
        rs0 = 0.f;
        rs1 = 0.f;
#pragma unroll
        for (int ss = 0; ss < 8; ++ss) p_chunk(ss);
    };
    // exact path of the split softmax: s[0] holds p0 = exp2(S0); restore S0 = log2(p0), or, when a
    // p0 overflowed (a row max grown by >= 128 in the exp2 domain), recompute S0 from K in global
    // memory (the K(i) LDS slot may already hold K(i+2) for the other wave half)
    auto exact_split = [&](bool first, int kv0, bool low) __attribute__((always_inline)) {
        // recompute S0 when an exp2 overflowed, or (first tile, a lane's sum below SUM_MIN) when
        // an in-place exp2 may have underflowed with the row's max also far below m = 0
        if (__any(!(rsA + rsB < INFINITY) || low)) {
            if constexpr (M16) {
#pragma unroll
                for (int kbl = 0; kbl < 2; ++kbl) {
                    const int krow = min(kv0 + 16 * kbl + lr, Skv - 1);
                    const bf16_t* kp = Kb + (long long)krow * ldk + 8 * lg;
#pragma unroll
                    for (int ks = 0; ks < 4; ++ks) {
                        const bf16x8_t kf = *reinterpret_cast<const bf16x8_t*>(kp + 32 * ks);
#pragma unroll
                        for (int qb = 0; qb < 2; ++qb) {
                            const int g = 2 * kbl + qb;
                            s[0] = mfma16g(kf, qf[4 * qb + ks], s[0], g, grp4(ks == 0 ? negm : s[0], g));
                        }
                    }
                }
            } else {
                const int krow = min(kv0 + r, Skv - 1);
                const bf16_t* kp = Kb + (long long)krow * ldk + 8 * hh;
#pragma unroll
                for (int ss = 0; ss < 8; ++ss) {
                    const bf16x8_t kf = *reinterpret_cast<const bf16x8_t*>(kp + 16 * ss);
                    s[0] = mfma32(kf, qf[ss], ss == 0 ? negm : s[0], ss & 1);
                }
            }
            if (kv0 + BKV > Skv) mask_half(0, kv0);
        } else {
#pragma unroll
            for (int i = 0; i < 16; ++i) s[0][i] = __builtin_amdgcn_logf(s[0][i]);
        }
        exact(first);
        rsA = 0.f;
        rsB = 0.f;
    };

    // phase barrier: this wave's LDS stores done (lgkmcnt), then s_barrier.  Written out rather than
    // __syncthreads(), whose workgroup fence also waits for every LDS-DMA in flight (vmcnt(0)) --
    // that would drain the next item's Q prefetch and this phase's K/V loads at every barrier
    auto phase_bar = [&]() {
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
    };
    __syncthreads();
    const int grp = wave >> 2;
    if (grp == 1) phase_bar();
    // the normalised bf16 output of a finished item in 8 chunks of 16 B per lane, emit(c, w) storing
    // or staging chunk c; one column block dt at a time (8 live registers).  Each lane's chunk c
    // lands at element ooff(c) of the wave's 32-row block (rows relative to its first row q0):
    //   M32: lane (r, hh) holds columns 32dt + 8gi + 4hh .. +3 of row r; pairs of groups (gi, gi+1)
    //        through one permlane32_swap per dword give chunk c = 2dt + gp = columns 16c + 8hh .. +7;
    //   M16: lane (lr, lg) holds columns 16db + 4lg .. +3 of rows 16qb + lr; column blocks
    //        (2dt, 2dt+1) through one permlane16_swap per dword give chunk c = 2dt + qb = columns
    //        16(2dt + (lg&1)) + 8(lg>>1) .. +7 of row 16qb + lr.
    // NC: flag item gi for the redo launch when one of the wave's row sums left [NC_LMIN, NC_LMAX]
    // (NaN included); every wave of the item may store the same 1
    auto nc_flag = [&](int gi) __attribute__((always_inline)) {
        if constexpr (NC) {
            const float l0 = lsum[0][0], l1 = lsum[1][0];
            const bool ok = l0 >= NC_LMIN && l0 <= NC_LMAX && l1 >= NC_LMIN && l1 <= NC_LMAX;
            if (__any(!ok) && lane == 0) nc_list_item(cold->flags, cold->nc_cap, gi);
        }
    };
    auto row_l = [&](int qb) {
        if constexpr (NC) return lsum[qb][0];
        float t = lq[qb];
        if constexpr (M16) t += __shfl_xor(t, 16);
        return t + __shfl_xor(t, 32);
    };
    auto ooff = [&](int cidx) -> long long {
        if constexpr (M16)
            return (long long)(16 * (cidx & 1) + lr) * ldo + 32 * (cidx >> 1) + 16 * (lg & 1) + 8 * (lg >> 1);
        else
            return (long long)r * ldo + 16 * cidx + 8 * hh;
    };
    auto out_row_ok = [&](int qrow0, int cidx) { return qrow0 + (M16 ? 16 * (cidx & 1) + lr : r) < Sq; };
    auto out_chunks = [&](auto emit) __attribute__((always_inline)) {
        const float inv0 = 1.f / row_l(0);
        const float inv1 = M16 ? 1.f / row_l(1) : inv0;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
            for (int gp = 0; gp < 2; ++gp) {
                if constexpr (M16) {
                    // gp = qb: groups (db = 2dt, qb) = o[dt][4qb..] and (2dt+1, qb) = o[dt][8+4qb..]
                    const float inv = gp ? inv1 : inv0;
                    const int a = 4 * gp, b = 8 + 4 * gp;
                    const unsigned x0 = pack2(o[dt][a] * inv, o[dt][a + 1] * inv);
                    const unsigned x1 = pack2(o[dt][a + 2] * inv, o[dt][a + 3] * inv);
                    const unsigned y0 = pack2(o[dt][b] * inv, o[dt][b + 1] * inv);
                    const unsigned y1 = pack2(o[dt][b + 2] * inv, o[dt][b + 3] * inv);
                    const auto s0 = __builtin_amdgcn_permlane16_swap(x0, y0, false, false);
                    const auto s1 = __builtin_amdgcn_permlane16_swap(x1, y1, false, false);
                    emit(2 * dt + gp, u32x4_t{s0[0], s1[0], s0[1], s1[1]});
                } else {
                    const int gi = 2 * gp;
                    const unsigned ax = pack2(o[dt][4 * gi] * inv0, o[dt][4 * gi + 1] * inv0);
                    const unsigned ay = pack2(o[dt][4 * gi + 2] * inv0, o[dt][4 * gi + 3] * inv0);
                    const unsigned bx = pack2(o[dt][4 * gi + 4] * inv0, o[dt][4 * gi + 5] * inv0);
                    const unsigned by = pack2(o[dt][4 * gi + 6] * inv0, o[dt][4 * gi + 7] * inv0);
                    const auto sx = __builtin_amdgcn_permlane32_swap(ax, bx, false, false);
                    const auto sy = __builtin_amdgcn_permlane32_swap(ay, by, false, false);
                    emit(2 * dt + gp, u32x4_t{sx[0], sy[0], sx[1], sy[1]});
                }
            }
    };

    // One tile T of the flattened sequence (tile ti of item tj): B_{T-1} (QK(T) + the s[0] half's
    // exps), A_T (PV(T-1) + the s[1] half).  Tile 0 (no PV) is peeled out of the loop: with one
    // loop body shape the kernel stays spill-free (a loop with the T == 0 cases inside spilled at
    // 256 VGPRs).  A later item's first tile starts from m = 0, O = 0, l = 0 exactly as tile 0
    // does, so every item's arithmetic is that of a one-item block (bit-identical results).
    // Persistent-mode traffic: chunk ti (0..7) of the NEXT item's Q rows is loaded in tile ti's B
    // phase and written prescaled to LDS slot ti in its A phase; the previous item's O, finished by
    // PV(T-1) in A_T of the new item's tile 0, is staged in LDS slots 8, 1..7 there and drained one
    // 16-B chunk per lane in the A phase of tiles 0..7 (each slot before that tile's Q chunk
    // overwrites it).  The Q load and the O store are issued in EVERY tile, through buffer
    // descriptors whose range is 0 when the tile has nothing to move (the load returns 0, the store
    // is dropped): with them conditional, the compiler's vmcnt waits -- merged over both paths --
    // waited for them at the next V-tile wait (measured: +20 % on the cross-attention).  Needs
    // nkv >= PERSIST_MIN_TILES (host).
    int ti = 0, tj = 0;
    auto tile = [&](int T, auto first_c) __attribute__((always_inline)) {
        constexpr bool first0 = decltype(first_c)::value;
        const bool first = first0 || ti == 0;
        const int kv0 = ti * BKV;
        ATTN_STAMP(0);
        // each phase opens with the LDS store of the tile staged one phase earlier (its slot's last
        // reader finished before the barrier that opened this phase), then the next global loads
        if (T + 1 < Ttot) store_k((T + 1) & 1);      // K(T+1), loaded at the start of A_{T-1}
        load_v(kv0);
        qk(T & 1, kv0);
        ATTN_STAMP(1);
        phase_bar();
        ATTN_STAMP(2);
        store_v(T & 1);                              // V(T), loaded at the start of B_{T-1}
        // K(T+2); issued unconditionally (past the end it re-reads an in-range tile that is never
        // stored) so the vmcnt waits of the phase do not depend on a branch
        load_k(ki * BKV);
        if (T + 2 < Ttot) k_next();
        if (kv0 + BKV > Skv) {
            asm volatile("");
            mask_half(1, kv0);
        }
        pv_softmax((T - 1) & 1, !first0);
        if (!first0 && ti == 0) {
            nc_flag(g0 + (tj - 1) * gstride);      // the finished item's row sums
            bf16_t* op = ob_prev + (long long)q0_prev * ldo;
            out_chunks([&](int cidx, u32x4_t w) __attribute__((always_inline)) {
                if (out_row_ok(q0_prev, cidx)) *reinterpret_cast<u32x4_t*>(op + ooff(cidx)) = w;
            });
            // the new item starts from O = 0, l = 0
            lq[0] = 0.f;
            lq[1] = 0.f;
            lsum[0] = f32x4_t{0.f, 0.f, 0.f, 0.f};
            lsum[1] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int dt = 0; dt < 4; ++dt)
#pragma unroll
                for (int i = 0; i < 16; ++i) o[dt][i] = 0.f;
        }
        if constexpr (!NC) {
            const float rt0 = row_tot(0), rt1 = M16 ? row_tot(1) : rt0;
            const bool low = first && !(fminf(rt0, rt1) >= SUM_MIN);
            if (__any(fmaxf(rt0, rt1) > SUM_THR || low)) exact_split(first, kv0, low);
        }
        if constexpr (!NC) {
            lq[0] += row_tot(0);
            if constexpr (M16) lq[1] += row_tot(1);
        }
        if (++ti == nkv && ++tj < n_items) {
            // switch to the next item: its prescaled Q from the LDS slots, m = 0 (as in a fresh
            // block); the V loader and the exact-path recompute follow the QK item, the K loader
            // is already on it
            ti = 0;
            load_q(qb_nxt, q0_nxt);
#pragma unroll
            for (int i = 0; i < 16; ++i) negm[i] = 0.f;
            mq[0] = 0.f;
            mq[1] = 0.f;
            ob_prev = ob_cur;
            q0_prev = q0;
            bh_cur = bh_nxt;
            q0 = q0_nxt;
            ob_cur = o_base(bh_cur);
            Kb = k_base(bh_cur);
            Vload = v_base(bh_cur);
            vrs = slab_rsrc(Vload, ldv32);
            if (tj + 1 < n_items) {
                bh_nxt = item_bh(tj + 1, q0_nxt);
                q0_nxt += wave * 32;
                qb_nxt = q_base(bh_nxt);
            }
        }
        ATTN_STAMP(7);
        phase_bar();
    };
    tile(0, std::true_type{});
    for (int T = 1; T < Ttot; ++T) tile(T, std::false_type{});
    // ---- B_{Ttot-1}: the last tile's PV.  Group 0 first waits for group 1's half of V(Ttot-1)
    // (stored in group 1's A_{Ttot-1}, one phase later): the extra barrier that balances the count
    if (grp == 0) phase_bar();
    pv_last((Ttot - 1) & 1);

    if (piece >= 0) {
        // split-tail piece: O unnormalised (fp32, natural column order) + the row's (m, l)
        float* pp = part + ((long long)(g - nmain) * nsplit + piece) * BQ * PROW + wave * 32 * PROW;
        if constexpr (M16) {
#pragma unroll
            for (int qb = 0; qb < 2; ++qb) {
                float* pr = pp + (16 * qb + lr) * PROW;
#pragma unroll
                for (int dt = 0; dt < 4; ++dt)
#pragma unroll
                    for (int dbl = 0; dbl < 2; ++dbl) {
                        const int gg = 4 * (2 * dbl + qb);
                        *reinterpret_cast<f32x4_t*>(pr + 16 * (2 * dt + dbl) + 4 * lg) =
                            f32x4_t{o[dt][gg], o[dt][gg + 1], o[dt][gg + 2], o[dt][gg + 3]};
                    }
                const float lt = row_l(qb);
                if (lg == 0) *reinterpret_cast<f32x2_t*>(pr + HD) = f32x2_t{mq[qb], lt};
            }
        } else {
            const float lt = row_l(0);
            float* pr = pp + r * PROW;
#pragma unroll
            for (int dt = 0; dt < 4; ++dt)
#pragma unroll
                for (int gi = 0; gi < 4; ++gi)
                    *reinterpret_cast<f32x4_t*>(pr + 32 * dt + 8 * gi + 4 * hh) =
                        f32x4_t{o[dt][4 * gi], o[dt][4 * gi + 1], o[dt][4 * gi + 2], o[dt][4 * gi + 3]};
            if (hh == 0) *reinterpret_cast<f32x2_t*>(pr + HD) = f32x2_t{mq[0], lt};
        }
        return;
    }
    {
        nc_flag(g0 + (n_items - 1) * gstride);     // (tj ran past the last item)
        bf16_t* op = ob_cur + (long long)q0 * ldo;
        out_chunks([&](int cidx, u32x4_t w) __attribute__((always_inline)) {
            if (out_row_ok(q0, cidx)) *reinterpret_cast<u32x4_t*>(op + ooff(cidx)) = w;
        });
    }
}

// Split-tail combine: one thread per (item, row, 4 columns).  A row's pieces j hold O_j and l_j
// against their own reference max m_j (exp2 domain): O = sum_j 2^(m_j - M) O_j / sum_j 2^(m_j - M) l_j.
__global__ __launch_bounds__(256) void attn_combine(const float* __restrict__ part, bf16_t* __restrict__ O,
                                                    int ntail, int nmain, int nsplit, int Sq, int H, int nqb,
                                                    long long ldo, long long bso, int* __restrict__ flags,
                                                    int nc_cap, float lmin) {
    const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
    const int c4 = (int)(idx & 31);
    const long long rowid = idx >> 5;              // item * BQ + row
    if (rowid >= (long long)ntail * BQ) return;
    const int it = (int)(rowid / BQ), row = (int)(rowid % BQ);
    const int g = nmain + it;
    const int qb = g % nqb, bh = g / nqb, h = bh % H, b = bh / H;
    const int q = qb * BQ + row;
    if (q >= Sq) return;
    const float* base = part + (long long)it * nsplit * BQ * PROW + (long long)row * PROW;
    float M = -INFINITY;
    for (int j = 0; j < nsplit; ++j) M = fmaxf(M, base[(long long)j * BQ * PROW + HD]);
    f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
    float lsum = 0.f;
    for (int j = 0; j < nsplit; ++j) {
        const float* pj = base + (long long)j * BQ * PROW;
        const float w = __builtin_amdgcn_exp2f(pj[HD] - M);
        lsum += w * pj[HD + 1];
        acc += w * *reinterpret_cast<const f32x4_t*>(pj + 4 * c4);
    }
    // NC pieces (all m_j = 0): a row sum outside [NC_LMIN, NC_LMAX] sends the item to the redo launch
    if (flags && !(lsum >= lmin && lsum <= NC_LMAX)) nc_list_item(flags, nc_cap, g);
    const float inv = 1.f / lsum;
    bf16_t* op = O + (long long)b * bso + (long long)q * ldo + h * HD + 4 * c4;
    const unsigned lo = pack2(acc[0] * inv, acc[1] * inv), hi = pack2(acc[2] * inv, acc[3] * inv);
    *reinterpret_cast<uint2*>(op) = make_uint2(lo, hi);
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// Split tail.  One workgroup fills a CU (2 waves per SIMD), so a grid of n items runs in
// ceil(n / CUs) rounds and the last, partial round leaves CUs idle (the 14B 832x480x73 self-
// attention: 9280 items = 36.25 rounds on 256 CUs; under Ulysses SP=8 1160 = 4.53).  The last
// n % CUs items instead run as nsplit key ranges each, chosen to minimise the tail's length in
// item units (ceil(tail * nsplit / CUs) / nsplit), then one combine launch.  Partials live in a
// caller-bound per-(device, stream) workspace (vs_split_workspace_bind; without one the grid runs
// unsplit).
constexpr int MAX_PIECES = 1024;
struct SplitPlan { int nmain = 0, ntail = 0, nsplit = 1, piece_tiles = 0; };

SplitPlan plan_split(long long nwg, int nkv, int cus) {
    SplitPlan p;
    p.nmain = (int)nwg;
    if (cus <= 0 || nkv < 32) return p;
    const int tail = (int)(nwg % cus);
    if (tail == 0 || nwg < cus) return p;
    double best = 1.0;
    int bf = 1;
    for (int f = 2; f <= 16 && tail * f <= MAX_PIECES && nkv / f >= 16; ++f) {
        const double cost = (double)((tail * f + cus - 1) / cus) / f + 0.01 * f;   // + per-piece overhead
        if (cost < best - 0.05) { best = cost; bf = f; }
    }
    if (bf == 1) return p;
    p.ntail = tail;
    p.nmain = (int)(nwg - tail);
    p.piece_tiles = (nkv + bf - 1) / bf;
    p.nsplit = (nkv + p.piece_tiles - 1) / p.piece_tiles;
    return p;
}


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
    // buffer addressing: a 64-row tile's span must fit the 32-bit per-lane offset
    if ((long long)BKV * ldk * 2 >= (1LL << 31) || (long long)BKV * ldv * 2 >= (1LL << 31)) return VS_E_UNSUPPORTED;
    const int nqb = (sq + BQ - 1) / BQ;
    const long long nwg = (long long)nqb * heads * batch;
    if (nwg > 0x7fffffff) return VS_E_INVALID;
    // MFMA shape of the QK / PV products (VS_OPT_ATTN_MFMA 16 | 32)
    const bool m16 = vs_opt(VS_OPT_ATTN_MFMA) == 16;
    const float c = scale * 1.4426950408889634f;
    const bool rebase = (long long)skv * ldk * 2 >= (1LL << 31) || (long long)skv * ldv * 2 >= (1LL << 31);
    const int nkv = (skv + BKV - 1) / BKV;
    const int cus = vs_cus_for_split(!vs_opt(VS_OPT_ATTN_SPLIT));
    SplitPlan sp = plan_split(nwg, nkv, cus);
    float* part = nullptr;
    if (sp.ntail) {
        part = vs_split_workspace(0, (size_t)sp.ntail * sp.nsplit * BQ * PROW * sizeof(float), (hipStream_t)stream);
        if (!part) sp = SplitPlan{(int)nwg, 0, 1, 0};
    }
    // persistent grid: one block per CU runs the whole items when there is more than one round of
    // them and an item has at least PERSIST_MIN_TILES key tiles (VS_OPT_ATTN_PERSIST 0: one block
    // per item, the r1 grid)
    const int ncu = vs_cus_for_split(false);
    const bool no_persist = !vs_opt(VS_OPT_ATTN_PERSIST);
    // (the Q prefetch and the O drain address a wave's rows through 32-bit buffer ranges)
    const bool span_ok = (long long)sq * ldq * 2 < (1LL << 32) && (long long)sq * ldo * 2 < (1LL << 32);
    const int npers =
        (!no_persist && span_ok && ncu > 0 && nkv >= PERSIST_MIN_TILES && sp.nmain > ncu) ? ncu : sp.nmain;
    // optimistic softmax (NC, comment at NC_LMIN): M16 only, needs the caller's item-flag workspace
    // (kind 4, zero-filled) and an O that does not overlap Q / K / V (the redo launch re-reads
    // them); VS_OPT_ATTN_NC 0 keeps the checked kernel
    int* flags = nullptr;
    int nc_cap = 0;
    if (m16 && vs_opt(VS_OPT_ATTN_NC)) {
        auto span = [&](const void* p, long long bs, long long ld, int rows) {
            const char* b = (const char*)p;
            return std::make_pair(b, b + 2 * ((long long)(batch - 1) * bs + (long long)(rows - 1) * ld + heads * HD));
        };
        const auto so = span(o, bso, ldo, sq);
        bool overlap = false;
        for (const auto& s : {span(q, bsq, ldq, sq), span(k, bsk, ldk, skv), span(v, bsv, ldv, skv)})
            overlap = overlap || (so.first < s.second && s.first < so.second);
        int dev = 0;
        long long bytes = 0;
        int* ws = (!overlap && hipGetDevice(&dev) == hipSuccess)
                      ? (int*)vs_bound_workspace(4, dev, (hipStream_t)stream, &bytes) : nullptr;
        const long long cap = bytes / 4 > 2 ? (bytes / 4 - 2) / 2 : 0;
        if (ws && cap >= nwg) {
            flags = ws;
            nc_cap = (int)std::min(cap, (long long)0x7fffffff);
        }
    }
    const int lds = LDS_BYTES;
    const long long grid = (long long)npers + (long long)sp.ntail * sp.nsplit;
    AttnArgs args{(const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, (bf16_t*)o, bsq, bsk, bsv, bso,
                  ldq, ldk, ldv, ldo, part, flags, c, sq, skv, heads, nqb, sp.nmain, npers, sp.nsplit,
                  sp.piece_tiles, nc_cap, nullptr};
    auto pick = [&](int mode) -> void (*)(AttnArgs) {
        constexpr int C = MODE_CHK, N = MODE_NC, R = MODE_REDO;
        if (mode == R) return rebase ? attn_fwd_d128<true, true, R> : attn_fwd_d128<false, true, R>;
        if (mode == N) return rebase ? attn_fwd_d128<true, true, N> : attn_fwd_d128<false, true, N>;
        return m16 ? (rebase ? attn_fwd_d128<true, true, C> : attn_fwd_d128<false, true, C>)
                   : (rebase ? attn_fwd_d128<true, false, C> : attn_fwd_d128<false, false, C>);
    };
    auto launch = [&](void (*kern)(AttnArgs), long long nblk, const AttnArgs& a) {
        static std::mutex mu;
        static std::set<const void*> attr_done;
        {
            std::lock_guard<std::mutex> lock(mu);
            if (attr_done.insert((const void*)kern).second)
                (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        }
        hipLaunchKernelGGL(kern, dim3((unsigned)nblk), dim3(NTHR), lds, (hipStream_t)stream, a);
        return hipGetLastError() == hipSuccess;
    };
    // the NC pass: attn_fwd_w4 (4 waves x 64 rows); VS_OPT_ATTN_IMPL 8 / 4 force the 8-wave / 4-wave kernel.
    // r5: the 512-key cross-attention (8 tiles per item) too -- 0.682 vs 0.746 ms at the 14B shape,
    // same box (profiles/r5/attn_skv_prefetch_ab_s10.log: both kernels pay ~7 us per item switch,
    // the 4-wave one less per tile); items under 4 tiles stay on the 8-wave kernel
    const int impl = vs_opt(VS_OPT_ATTN_IMPL);
    const bool w4 = flags && (impl ? impl == 4 : nkv >= 4);
    // attn_fwd_w4's persistent blocks take their items from XCD queues (kind-5 workspace, words from
    // VS_Q_ATTN) when there is more than one item per block (VS_OPT_QUEUE 0: static lists)
    if (w4 && npers < sp.nmain && nkv >= 4 && vs_opt(VS_OPT_QUEUE)) {
        unsigned* qw = (unsigned*)vs_split_workspace(5, 4096, (hipStream_t)stream);
        if (qw) args.queue = qw + VS_Q_ATTN;
    }
    if (w4) {
        if (attn_w4_launch(args, rebase, (unsigned)grid, (hipStream_t)stream) != hipSuccess) return VS_E_LAUNCH;
    } else if (!launch(pick(flags ? MODE_NC : MODE_CHK), grid, args)) {
        return VS_E_LAUNCH;
    }
    if (sp.ntail) {
        const long long threads = (long long)sp.ntail * BQ * 32;
        hipLaunchKernelGGL(attn_combine, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                           part, (bf16_t*)o, sp.ntail, sp.nmain, sp.nsplit, sq, heads, nqb, ldo, bso, flags, nc_cap,
                           w4 ? W4_LMIN : NC_LMIN);
        VS_CHECK_LAUNCH();
    }
    if (flags) {
        // redo: the checked kernel over the listed items, one block per CU walking the list (with
        // none listed every block returns at once); leaves the workspace's count and flags zero
        AttnArgs r = args;
        r.queue = nullptr;
        r.part = nullptr;
        r.nsplit = 1;
        r.piece_tiles = 0;
        const long long rgrid = std::min<long long>(nwg, ncu > 0 ? ncu : 256);
        r.nmain = r.npers = (int)rgrid;
        if (!launch(pick(MODE_REDO), rgrid, r)) return VS_E_LAUNCH;
    }
    return VS_OK;
}

extern "C" int vs_attn_split_plan(int batch, int sq, int skv, int heads, int cus, int* out) {
    if (!out || batch <= 0 || sq <= 0 || skv <= 0 || heads <= 0 || cus < 0) return VS_E_INVALID;
    const long long nwg = (long long)((sq + BQ - 1) / BQ) * heads * batch;
    const SplitPlan p = plan_split(nwg, (skv + BKV - 1) / BKV, cus);
    out[0] = p.nmain;
    out[1] = p.ntail;
    out[2] = p.nsplit;
    out[3] = p.piece_tiles;
    return VS_OK;
}

extern "C" long long vs_split_workspace_bytes(int kind) {
    if (kind == 0) return (long long)MAX_PIECES * BQ * PROW * (long long)sizeof(float);
    if (kind == 1) return vs_gemm_split_workspace_bytes_impl();
    if (kind == 2 || kind == 3) return 0;       // not used (no vendor-library route in this build)
    if (kind == 4) return 1LL << 20;            // attention item flags (int per item; zero-filled)
    if (kind == 5) return 4096;                 // GEMM tile-queue words (zero-filled; gemm.hip W4Sched)
    return -1;
}

// vs_set_option / vs_get_option (include/vstyler.h): the path-selection table of common.h
extern "C" int vs_set_option(int id, int value) {
    if (id < 0 || id >= VS_OPT_COUNT) return -VS_E_INVALID;
    bool ok = false;
    switch (id) {
        case VS_OPT_GEMM_TILE: ok = value == 0 || value == 128 || value == 256; break;
        case VS_OPT_GEMM_KERNEL: ok = value == 4 || value == 8; break;
        case VS_OPT_ATTN_IMPL: ok = value == 0 || value == 4 || value == 8; break;
        case VS_OPT_ATTN_MFMA: ok = value == 16 || value == 32; break;
        case VS_OPT_VAE_PXB: ok = value == 1 || value == 2; break;
        case VS_OPT_VAE_PRE: ok = value >= 1 && value <= 3; break;
        case VS_OPT_PIECE_QUEUE: ok = value >= 0 && value <= 2; break;
        default: ok = value == 0 || value == 1; break;           // the on / off options
    }
    if (!ok) return -VS_E_INVALID;
    const int old = g_vs_opt[id];
    g_vs_opt[id] = value;
    return old;
}
extern "C" int vs_get_option(int id) { return (id < 0 || id >= VS_OPT_COUNT) ? -VS_E_INVALID : g_vs_opt[id]; }

extern "C" int vs_split_workspace_bind(int kind, void* ptr, long long bytes, void* stream) {
    if (kind < 0 || kind > 5 || bytes < 0 || (ptr && ((uintptr_t)ptr & 15))) return VS_E_INVALID;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return VS_E_LAUNCH;
    std::mutex* mu;
    auto& reg = vs_ws_registry(mu);
    std::lock_guard<std::mutex> lock(*mu);
    if (!ptr) reg.erase({kind, dev, (hipStream_t)stream});
    else reg[{kind, dev, (hipStream_t)stream}] = VsWs{(float*)ptr, bytes};
    return VS_OK;
}
