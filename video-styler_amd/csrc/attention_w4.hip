// attn_fwd_w4: the 4-wave x 64-row flash-attention forward (NC pass), gfx950: a hand-pipelined
// four-phase loop body (described below).  Built with its own flags (Makefile W4FLAGS, for
// code-generation A/Bs).
#include <cstdlib>
#include <mutex>
#include <set>
#include <type_traits>

#include "attention.h"

namespace vs_attn {
namespace {

// ---------------------------------------------------------------------------------------------
// attn_fwd_w4 (r3): one wave per SIMD, 64 query rows per wave.  A workgroup is 4 waves = the same
// 256-row item of one (batch, head) as attn_fwd_d128, so the item list, the persistent grid, the
// split-tail pieces, the combine and the NC redo launch are shared with it.  What changes is the
// per-wave tile: every K / V^T fragment read from LDS feeds TWO 32-row MFMA blocks, which halves
// the LDS read traffic per FLOP of the 8-wave kernel (8 waves x 32 rows all re-reading the same
// fragments: SQ_WAIT_INST_LDS 15.6 %, profiles/r2/pmc_attn_ilp), and the matrix pipe of a SIMD is
// fed by one instruction stream with the softmax interleaved into its MFMA gaps (MI355X_MICROARCH
// 'one wave per SIMD': <= 5 single-issue fillers per v_mfma_f32_32x32x16_bf16 gap hide).
//
// Per 64-key tile T and wave (v_mfma_f32_32x32x16_bf16, the swapped products of the M32 layout):
//   QK(T):   S^T[kb][rb] = K(T)[32kb..] Q[32rb..]^T        16 K fragments -> 32 MFMAs
//   softmax: p = exp2(S) (Q pre-scaled by log2(e)/sqrt(d); optimistic, no reference max -- the NC
//            rule of attn_fwd_d128), row sums in fp32, P packed to bf16 as the PV B operands
//   PV(T-1): O^T[rb][dt] += V(T-1)^T[32dt..] P(T-1)[rb]     16 V^T fragments (32 tr reads) -> 32 MFMAs
// O^T (8 x 16 fp32 per lane) and the Q fragments live in AGPRs (512-register wave); the schedule
// that interleaves the softmax with the MFMAs is described at the loop body below.
//
// LDS: 4 slots x (K 16 KB | V 16 KB), filled by LDS-DMA (buffer_load ... lds, 1 KB = 4 rows per
// wave-instruction, 8 per wave per tile) two tiles ahead; unpadded 256-B rows with the 16-B chunk
// swizzled on the SOURCE address: K chunk c of row R at c ^ (R & 15) (conflict-free 32-row
// ds_read_b128), V at c ^ 4 (R & 3) (the 4 rows x 64 B of a ds_read_b64_tr_b16 half-wave in 4
// distinct bank quarters).  One s_barrier per tile; each wave retires its own DMA of a tile with a
// counted vmcnt before the barrier that makes the tile visible (the barrier placement and the slot
// reuse rule of each body are given with it).  The DMA is issued from inline asm (see dma16).
//
// Key masking without a branch: rows past Skv are outside the buffer range and load as 0, so a
// padded key scores exactly 0, contributes P = exp2(0) = 1 against a zero V row (O unchanged) and
// exactly 1 to every row sum; the item's (nkv * 64 - Skv) padded keys are subtracted from l at the
// end.  That subtraction cancels when the true l is tiny, so an item with a row sum below
// W4_LMIN (2^-4, a row whose scores all lie below -4 in the exp2 domain) goes to the redo launch
// with the overflow / underflow cases of the NC rule.
constexpr int W4_THR = 256;
constexpr int W4_TILE = BKV * HD * 2;      // 16 KB: one K or V tile
constexpr int W4_SLOT = 2 * W4_TILE;
constexpr int W4_LDS = 4 * W4_SLOT;        // 128 KB
constexpr int W4_QSLOT = W4_LDS;           // the next item's id (LDS word, the item hand-off)
constexpr int W4_LDS_BASE = W4_LDS + 16;
#ifdef VS_W4_STAMPS
// diagnostic build: s_memtime at the phase boundaries of the pipelined loop (iterations 8..39 of
// block 0, every wave): 0 start of A, 1 end of A, 2 end of B, 3 end of C, 4 after the barrier, 5 end
// of D, 6 after D step 3; kept in an LDS tail, copied out at the end (tests/probes/w4_stamps.py)
__device__ unsigned long long g_w4_stamps[4][32][7];
// and per item of block 0 (the first 16, every wave): 0 before its first tile, 1 after it, 2 after
// the paired tile loop, 3 after the next item's Q loads, 4 after the drain, 5 after the O store; 6-8
// inside the next-Q step: its start, the in-flight DMA drained, the Q loaded and converted
// (tests/probes/w4_stamps.py W4S_SKV=512: the item switch of the 8-tile cross-attention)
constexpr int W4_SWN = 9;
__device__ unsigned long long g_w4_sw[4][16][W4_SWN];
constexpr int W4_STAMP_OFF = W4_LDS_BASE;
constexpr int W4_SW_OFF = W4_STAMP_OFF + 4 * 32 * 7 * 8;
constexpr int W4_LDS_ALLOC = W4_SW_OFF + 4 * 16 * W4_SWN * 8;
#else
constexpr int W4_LDS_ALLOC = W4_LDS_BASE;
#endif

// Items of the persistent blocks (r5): XCD x owns the contiguous chunk [cs, cs + csz) of the item
// list and gs persistent blocks (block b: XCD b % 8, slot b / 8 < gs).  A block takes its items from
// the XCD's queue (positions cs + t, head word q[x]), then from other XCDs' queues (probed in ring
// order) -- or, without a queue, walks the static list cs + slot + j gs (r1-r4), where a block whose
// CU is held by another kernel (RCCL under the Ulysses overlap) delays its whole list: +24-38 % on
// the self-attention with 8-32 CUs held for half its time (profiles/r5/cu_hold_s4.log).  The first
// item costs one atomic round trip; after that wave 0 takes the id of the item after next at an
// item switch (its atomic under the next item's Q loads), hands it to the other waves through an
// LDS word read in the next item's first tile, and the K/V DMA cursor moves to it when it leaves
// that item, hundreds of tiles later.  The last persistent block to finish zeroes the queue words.
struct AttnChunks {
    int nmain, npers;
    __device__ __forceinline__ void of(int x, int& cs, int& csz, int& gs) const {
        const int qx = nmain >> 3, rx = nmain & 7, qb = npers >> 3, rb = npers & 7;
        cs = x < rx ? x * (qx + 1) : rx * (qx + 1) + (x - rx) * qx;
        csz = qx + (x < rx ? 1 : 0);
        gs = qb + (x < rb ? 1 : 0);
    }
    // the item after `nxt` (wave 0, all lanes; t0 = lane 0's returned own-queue head): -1 if none
    __device__ __forceinline__ int take(unsigned* q, unsigned t0, int nxt, int lane) const {
        const int x = blockIdx.x & 7;
        int cs, csz, gs;
        of(x, cs, csz, gs);
        if (!q) return nxt + gs < cs + csz ? nxt + gs : -1;
        const unsigned t = vs_queue_value<0>(t0);
        if ((int)t < csz) return cs + (int)t;
        for (int it = 0; it < 16; ++it) {          // other XCDs' queues, first live one in ring order
            int vcs, vcsz, vgs;
            of((x + 1 + lane) & 7, vcs, vcsz, vgs);
            unsigned h = 0x7fffffff;
            if (lane < 7) h = __hip_atomic_load(q + ((x + 1 + lane) & 7) * VS_Q_LINE, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
            const unsigned long long live = __ballot(lane < 7 && (int)h < vcsz);
            if (!live) return -1;
            const int v = (x + 1 + (int)__builtin_ctzll(live)) & 7;
            unsigned tv = 0;
            if (lane == 0) tv = vs_queue_add(q + v * VS_Q_LINE);
            tv = (unsigned)__builtin_amdgcn_readfirstlane((int)tv);
            of(v, vcs, vcsz, vgs);
            if ((int)tv < vcsz) return vcs + (int)tv;
        }
        return -1;
    }
};

template <bool REBASE>
__global__ __launch_bounds__(W4_THR, 1) void attn_fwd_w4(const AttnArgs args) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    typedef const volatile AttnArgs __attribute__((address_space(4))) ColdArgs;
    ColdArgs* cold = (ColdArgs*)__builtin_amdgcn_kernarg_segment_ptr();
    const int Sq = args.Sq, Skv_all = args.Skv, nmain = args.nmain, npers = args.npers;
    const int nsplit = args.nsplit, piece_tiles = args.piece_tiles;
    const long long ldq = args.ldq, ldk = args.ldk, ldv = args.ldv, ldo = args.ldo;
    const float c = args.c;

    // items: the persistent blocks' XCD chunks and queues (AttnChunks), the blocks after npers run
    // the split-tail pieces (one item each)
    int piece = -1, kv_begin = 0, Skv = Skv_all;
    int cur;                                       // the item being computed
    const bool pers = (int)blockIdx.x < npers;
    const AttnChunks chunks{nmain, npers};
    const int tid = threadIdx.x, lane = tid & 63;
    if (pers) {
        int cs, csz, gs;
        chunks.of(blockIdx.x & 7, cs, csz, gs);
        cur = (int)(blockIdx.x >> 3) < csz ? cs + (int)(blockIdx.x >> 3) : -1;
    } else {
        const int t = blockIdx.x - npers;
        cur = nmain + t / nsplit;
        piece = t % nsplit;
        kv_begin = piece * piece_tiles * BKV;
        Skv = min(Skv_all - kv_begin, piece_tiles * BKV);
    }
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    if (pers && args.queue) {                      // the first item from the queues too
        volatile LDS_AS int* qs = (volatile LDS_AS int*)(uintptr_t)((unsigned)(uintptr_t)smem + W4_QSLOT);
        if (wave == 0) {
            const unsigned t0 = vs_queue_issue(args.queue + (blockIdx.x & 7) * VS_Q_LINE);
            const int id = chunks.take(args.queue, t0, -1, lane);
            if (lane == 0) *qs = id;
        }
        __syncthreads();
        cur = __builtin_amdgcn_readfirstlane(*qs);
    }
    if (cur < 0) {                                 // (a persistent block with no item: counted out)
        if (pers && args.queue && tid == 0) vs_queue_done(args.queue, 9, npers);
        return;
    }
    const int r = lane & 31, hh = lane >> 5;

    auto item_bh = [&](int g, int& qrow0) {
        const int nqb = cold->nqb;
        qrow0 = (g % nqb) * BQ;
        return g / nqb;
    };
    auto q_base = [&](int bh) { const int H = cold->H; return cold->Q + (long long)(bh / H) * cold->bsq + (bh % H) * HD; };
    auto k_base = [&](int bh) {
        const int H = cold->H;
        return cold->K + (long long)(bh / H) * cold->bsk + (long long)kv_begin * ldk + (bh % H) * HD;
    };
    auto v_base = [&](int bh) {
        const int H = cold->H;
        return cold->V + (long long)(bh / H) * cold->bsv + (long long)kv_begin * ldv + (bh % H) * HD;
    };
    auto o_base = [&](int bh) { const int H = cold->H; return cold->O + (long long)(bh / H) * cold->bso + (bh % H) * HD; };

    const int nkv = (Skv + BKV - 1) / BKV;
    const float npad = (float)(nkv * BKV - Skv);

    // ---- LDS-DMA loader: tile T of the flattened sequence into slot T & 3, two tiles ahead of QK.
    // Wave w fills rows 16w .. 16w+15 of both tiles, 4 rows per instruction; lane L lands in chunk
    // L & 15 of row 16w + 4i + (L >> 4) and fetches the logical chunk the swizzle puts there.
    const int ldk32 = (int)ldk, ldv32 = (int)ldv;       // host: 64 * ld * 2 < 2^31
    unsigned kvo[4], vvo[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int R = 16 * wave + 4 * i + (lane >> 4), p = lane & 15;
        kvo[i] = (unsigned)(R * ldk32 * 2 + ((p ^ (R & 15)) << 4));
        vvo[i] = (unsigned)(R * ldv32 * 2 + ((p ^ ((R & 3) << 2)) << 4));
    }
    // The DMA is issued from inline asm: the compiler, which sees an LDS-DMA as a write to all of
    // LDS, would otherwise put vmcnt(0) before the first fragment read of every iteration and drain
    // the two-tile lead.  Ordering is the protocol above (counted vmcnt + s_barrier); the compiler's
    // own vmcnt waits (Q loads) only grow more conservative with the uncounted DMA.
    auto rsrc4 = [&](const bf16_t* base, unsigned bytes) {
        const unsigned long long a = (unsigned long long)(uintptr_t)base;
        return i32x4_t{(int)(unsigned)a, (int)((unsigned)(a >> 32) & 0xffffu), (int)bytes, 0x00020000};
    };
    auto slab_rsrc = [&](const bf16_t* base, int ld) {
        return rsrc4(base, REBASE ? 0u : (unsigned)((Skv - 1) * ld * 2 + HD * 2));
    };
    auto dma16 = [](unsigned lds, unsigned voff, i32x4_t rs, int soff) __attribute__((always_inline)) {
        asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
                     :: "s"(lds), "v"(voff), "s"(rs), "s"(soff) : "m0");
    };
    int li = 0;
    int dnext = -1;                 // the item the DMA cursor moves to after the current one (-1: none)
    int qrow_unused;
    const bf16_t* Kl = k_base(item_bh(cur, qrow_unused));
    const bf16_t* Vl = v_base(item_bh(cur, qrow_unused));
    i32x4_t krs = slab_rsrc(Kl, ldk32), vrs = slab_rsrc(Vl, ldv32);
    const unsigned lds0 = (unsigned)(uintptr_t)smem + wave * 16 * 256;
    // stage(T) = stage_piece(T, 0..7) (K rows, then V rows, 4 rows per piece) + stage_next()
    struct StageCtx { unsigned kdst, vdst; i32x4_t kr, vr; int ks, vs; } sc;
    auto stage_begin = [&](int T) __attribute__((always_inline)) {
        sc.kdst = lds0 + (T & 3) * W4_SLOT;
        sc.vdst = sc.kdst + W4_TILE;
        const int kv0 = li * BKV;
        sc.kr = krs;
        sc.vr = vrs;
        sc.ks = kv0 * ldk32 * 2;
        sc.vs = kv0 * ldv32 * 2;
        if constexpr (REBASE) {
            const int rows = min(BKV, Skv - kv0);
            sc.kr = rsrc4(Kl + (long long)kv0 * ldk, (unsigned)((rows - 1) * ldk32 * 2 + HD * 2));
            sc.vr = rsrc4(Vl + (long long)kv0 * ldv, (unsigned)((rows - 1) * ldv32 * 2 + HD * 2));
            sc.ks = 0;
            sc.vs = 0;
        }
    };
    auto stage_piece = [&](int i) __attribute__((always_inline)) {
        if (i < 4)
            dma16(sc.kdst + i * 1024, kvo[i], sc.kr, sc.ks);
        else
            dma16(sc.vdst + (i - 4) * 1024, vvo[i - 4], sc.vr, sc.vs);
    };
    // phase D's pieces (r4): M0 is written once before the barrier and stepped between the two PV
    // MFMAs of the previous step, so a piece is the load alone (no s_mov + hazard s_nop per piece;
    // the step declares no "m0" clobber -- the hazard recognizer would pad it after every MFMA --
    // and nothing else in this kernel reads M0)
    auto piece_go = [&](int i) __attribute__((always_inline)) {
        if (i < 4)
            asm volatile("buffer_load_dwordx4 %0, %1, %2 offen lds" :: "v"(kvo[i]), "s"(sc.kr), "s"(sc.ks) : "memory");
        else
            asm volatile("buffer_load_dwordx4 %0, %1, %2 offen lds" :: "v"(vvo[i - 4]), "s"(sc.vr), "s"(sc.vs) : "memory");
    };
    auto m0_step = [&](int i) __attribute__((always_inline)) {      // M0: piece i - 1 -> piece i
        if (i == 4) asm volatile("s_add_u32 m0, m0, %0" :: "i"(W4_TILE - 3 * 1024) : "memory");
        else asm volatile("s_add_u32 m0, m0, 0x400" ::: "memory");
    };
    auto stage_next = [&]() __attribute__((always_inline)) {
        if (++li == nkv) {
            li = 0;
            if (dnext >= 0) {
                const int bh = item_bh(dnext, qrow_unused);
                Kl = k_base(bh);
                Vl = v_base(bh);
                krs = slab_rsrc(Kl, ldk32);
                vrs = slab_rsrc(Vl, ldv32);
                dnext = -1;
            }
        }
    };
    auto stage = [&](int T) __attribute__((always_inline)) {
        stage_begin(T);
#pragma unroll
        for (int i = 0; i < 8; ++i) stage_piece(i);
        stage_next();
    };

    // ---- Q fragments (B operand of S^T = K Q^T), pre-scaled by c: qf[rb][j] = row q0 + 32rb + r,
    // columns 16j + 8hh .. +7 (rows past Sq read row Sq - 1; their outputs are dropped)
    bf16x8_t qf[2][8];
    auto load_q = [&](const bf16_t* qb0, int q0v) __attribute__((always_inline)) {
        bf16x8_t raw[2][8];
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) {
            const int qrow = min(q0v + 32 * rb + r, Sq - 1);
            const bf16_t* src = qb0 + (long long)qrow * ldq + 8 * hh;
#pragma unroll
            for (int j = 0; j < 8; ++j) raw[rb][j] = *reinterpret_cast<const bf16x8_t*>(src + 16 * j);
        }
#pragma unroll
        for (int rb = 0; rb < 2; ++rb)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
#pragma unroll
                for (int e = 0; e < 8; ++e) qf[rb][j][e] = (__bf16)((float)raw[rb][j][e] * c);
                asm volatile("" : "+a"(qf[rb][j]));    // the B operands live in AGPRs
            }
    };

    // ---- fragment addresses (bytes from the slot base).  K (kb, j): row 32kb + r, chunk
    // (2j + hh) ^ (r & 15).  V^T (ks, dt): the M32 transposed-read pattern of attn_fwd_d128 (rows
    // 16ks + 4(g4 >> 1) + q4 and +8, bytes 64dt + 32(g4 & 1) + 8p4) through the V swizzle, which
    // turns the 64-B block dt into dt ^ q4 (rows = q4 mod 4)
    int koff[8], voff[4];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        koff[j] = r * 256 + (((2 * j + hh) ^ (r & 15)) << 4);
        asm volatile("" : "+v"(koff[j]));
    }
    {
        const int g4 = lane >> 4, q4 = (lane & 15) >> 2, p4 = lane & 3;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
            voff[dt] = W4_TILE + (4 * (g4 >> 1) + q4) * 256 + ((dt ^ q4) << 6) + 32 * (g4 & 1) + 8 * p4;
            asm volatile("" : "+v"(voff[dt]));
        }
    }
    const unsigned smem_base = (unsigned)(uintptr_t)smem;
    auto lds16 = [&](unsigned addr) {
        return *reinterpret_cast<const LDS_AS bf16x8_t*>((const LDS_AS char*)(uintptr_t)addr);
    };
    auto tr8 = [&](unsigned addr) {
        return __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS i16x4_t*)(uintptr_t)addr);
    };

    f32x16_t o[2][4];
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
            for (int i = 0; i < 16; ++i) o[rb][dt][i] = 0.f;
    float lsum[2] = {0.f, 0.f};
    auto row_sum = [&](int rb) { return lsum[rb] + __shfl_xor(lsum[rb], 32); };
    f32x16_t zero;
#pragma unroll
    for (int i = 0; i < 16; ++i) zero[i] = 0.f;


    // ---- items run one after the other (the K/V DMA pipeline runs on across item boundaries);
    // within an item the tile loop is unrolled by two over the two P buffers, and its body --
    // barrier, QK(T) + softmax, PV(T - 1), the DMA of tile T + 2 -- has no branch before the DMA
    // cursor's item switch at its end, so the scheduler sees QK, softmax and PV as one region
    // finished item: row sums (both lane halves, padded keys removed), NC flag, normalised store
    // or (split-tail piece) the fp32 partial with m = 0
    auto finish = [&](bf16_t* ob, int qrow0, int gi) __attribute__((always_inline)) {
        float lt[2];
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) lt[rb] = row_sum(rb) - npad;
        if (piece >= 0) {
            float* pp = args.part + ((long long)(gi - nmain) * nsplit + piece) * BQ * PROW + wave * 64 * PROW;
#pragma unroll
            for (int rb = 0; rb < 2; ++rb) {
                float* pr = pp + (32 * rb + r) * PROW;
#pragma unroll
                for (int dt = 0; dt < 4; ++dt)
#pragma unroll
                    for (int gi4 = 0; gi4 < 4; ++gi4)
                        *reinterpret_cast<f32x4_t*>(pr + 32 * dt + 8 * gi4 + 4 * hh) =
                            f32x4_t{o[rb][dt][4 * gi4], o[rb][dt][4 * gi4 + 1], o[rb][dt][4 * gi4 + 2],
                                    o[rb][dt][4 * gi4 + 3]};
                if (hh == 0) *reinterpret_cast<f32x2_t*>(pr + HD) = f32x2_t{0.f, lt[rb]};
            }
            return;
        }
        const bool ok = lt[0] >= W4_LMIN && lt[0] <= NC_LMAX && lt[1] >= W4_LMIN && lt[1] <= NC_LMAX;
        if (__any(!ok) && lane == 0) nc_list_item(cold->flags, cold->nc_cap, gi);
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) {
            const float inv = 1.f / lt[rb];
            const int row = qrow0 + 32 * rb + r;
            bf16_t* op = ob + (long long)row * ldo + 8 * hh;
#pragma unroll
            for (int dt = 0; dt < 4; ++dt)
#pragma unroll
                for (int gp = 0; gp < 2; ++gp) {
                    // lane (r, hh) holds columns 32dt + 8gi + 4hh .. +3; one permlane32_swap per
                    // dword pairs groups (2gp, 2gp+1) into columns 16(2dt + gp) + 8hh .. +7
                    const int gi = 2 * gp;
                    const unsigned ax = pack2(o[rb][dt][4 * gi] * inv, o[rb][dt][4 * gi + 1] * inv);
                    const unsigned ay = pack2(o[rb][dt][4 * gi + 2] * inv, o[rb][dt][4 * gi + 3] * inv);
                    const unsigned bx = pack2(o[rb][dt][4 * gi + 4] * inv, o[rb][dt][4 * gi + 5] * inv);
                    const unsigned by = pack2(o[rb][dt][4 * gi + 6] * inv, o[rb][dt][4 * gi + 7] * inv);
                    const auto sx = __builtin_amdgcn_permlane32_swap(ax, bx, false, false);
                    const auto sy = __builtin_amdgcn_permlane32_swap(ay, by, false, false);
                    if (row < Sq)
                        *reinterpret_cast<u32x4_t*>(op + 16 * (2 * dt + gp)) = u32x4_t{sx[0], sy[0], sx[1], sy[1]};
                }
        }
    };

    // ---- hand-pipelined schedule (PIPE): each iteration is four phases of 16 MFMAs, every
    // phase a sequence of 8 fenced steps (2 MFMAs of the two row blocks + fillers), so the
    // program order is the issue order and the softmax VALU sits in the MFMA gaps:
    //   A  QK(T) kb0              | exp/sum/pack of S(T-1) kb1 rb0 -> P(T-1) ks2,3 | K(T) kb1 reads
    //   B  QK(T) kb1              | S(T-1) kb1 rb1                                  | V(T-1) ks0,1 reads
    //   C  PV(T-1) ks0,1          | S(T) kb0 rb0 + rb1 -> P(T) ks0,1                 | V(T-1) ks2,3 reads
    //   [lgkmcnt(0), vmcnt(8), s_barrier B(T+1)]
    //   D  PV(T-1) ks2,3          | DMA of tile T+3, one piece per step             | K(T+1) kb0 reads
    // (D carries no exps: VALU right after a barrier release stalls the segment's head --
    // MI355X_MICROARCH 'start-of-segment VALU penalty'; moving S(T) kb0 rb1 from D into C was
    // +1.2 % self-attention in three interleaved same-box pairs, profiles/r3/w4_c2_ab_r3v.log)
    // Barrier B(T+1) sits between C and D: it retires tile T+1 (so D can read K(T+1) for the
    // next A) and proves every wave has read V(T-1) (the slot tile T+3 is staged into, with its
    // K(T-1), read in iteration T-1).  Tile X is staged right after B(X-2); the wait is always
    // vmcnt(8) (tiles X, X+1 outstanding).  An item's first tile runs the phases without PV
    // and without the previous tile's softmax; after its last tile a drain finishes S kb1 and
    // runs PV(last) (no barrier), while the next item's Q loads.
    bf16x8_t kf0[8], kf1[8], vfa[8], vfb[8];
    f32x16_t s0[2], s1a[2], s1b[2];
    u32x4_t p0a[2][2], p0b[2][2], p1[2][2];
    auto fence = [] { __builtin_amdgcn_sched_barrier(0); };
#ifdef VS_W4_STAMPS
    unsigned long long stv[7] = {0, 0, 0, 0, 0, 0, 0};
    int st_it = -1;                      // index of the stamped iteration (-1: not stamped)
    auto stamp = [&](int k) __attribute__((always_inline)) {
        if (st_it >= 0) asm volatile("s_memtime %0" : "=s"(stv[k]));
    };
    // after a lgkmcnt(0): iteration st's stamps 0-3, and 4-5 of the one before
    auto stamp_store = [&](int st, int lo, int hi) __attribute__((always_inline)) {
        if (st >= 0 && lane == 0)
            for (int k = lo; k < hi; ++k)
                *reinterpret_cast<volatile LDS_AS unsigned long long*>(
                    (LDS_AS char*)(uintptr_t)(smem_base + W4_STAMP_OFF + 8 * ((wave * 32 + st) * 7 + k))) = stv[k];
    };
    unsigned long long swv[W4_SWN] = {};
    int sw_i = 0;                        // item index of block 0 (stamped while < 16)
    auto swst = [&](int k) __attribute__((always_inline)) {
        // (waited at once: the value must not be copied before it lands)
        if (blockIdx.x == 0 && sw_i < 16) asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(swv[k]) :: "memory");
    };
    auto sw_store = [&]() __attribute__((always_inline)) {
        if (blockIdx.x == 0 && sw_i < 16) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (lane == 0)
                for (int k = 0; k < W4_SWN; ++k)
                    *reinterpret_cast<volatile LDS_AS unsigned long long*>(
                        (LDS_AS char*)(uintptr_t)(smem_base + W4_SW_OFF + 8 * ((wave * 16 + sw_i) * W4_SWN + k))) = swv[k];
        }
        ++sw_i;
    };
#else
    auto stamp = [](int) {};
    auto swst = [](int) {};
    auto sw_store = [] {};
#endif
    // K fragment addresses: the slot's base + the lane's swizzled offset, made opaque once per tile
    // (in phase D, for its kb0 reads and the next phase A's kb1 reads), so the kb displacement
    // folds into the ds instruction's offset field -- with the slot base added in an SGPR, every
    // read cost its own v_add_u32.  -3.4 % self-attention time (profiles/r5/attn_ldsbase_kv_ab_s24.log:
    // the same for V bases too cost 4 more live VGPRs and measured no better than K alone)
    unsigned kbs[8], vbs[4];
    auto kbase = [&](int T) __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            kbs[j] = smem_base + (T & 3) * W4_SLOT + koff[j];
            asm volatile("" : "+v"(kbs[j]));
        }
    };
    auto vbase = [&](int T) __attribute__((always_inline)) {
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) vbs[dt] = smem_base + (T & 3) * W4_SLOT + voff[dt];
    };
    auto rdK = [&](bf16x8_t& d, int kb, int j) __attribute__((always_inline)) {
        d = lds16(kbs[j] + kb * 32 * 256);
    };
    auto rdV = [&](bf16x8_t& d, int ks, int dt) __attribute__((always_inline)) {
        const unsigned a0 = vbs[dt] + ks * 16 * 256;
        const i16x4_t v0 = tr8(a0), v1 = tr8(a0 + 8 * 256);
        d = __builtin_shufflevector(__builtin_bit_cast(bf16x4_t, v0), __builtin_bit_cast(bf16x4_t, v1), 0, 1, 2,
                                    3, 4, 5, 6, 7);
    };
    // QK MFMAs in inline asm: S is written straight to VGPRs (the builtin's result lands in AGPRs
    // next to O and then costs a v_accvgpr_read per value before the exps), the Q operand is read
    // from AGPRs.  Hazards the compiler cannot see inside asm are covered by the schedule: an S
    // block's first VALU read comes >= 16 MFMAs after its chain's last MFMA (XDL write -> VALU
    // read needs ~18 wait states); the chain itself accumulates in place (srcC == vdst, the
    // same opcode: forwarded); the K operand's lgkmcnt wait is inserted by the compiler (it
    // tracks the asm's register uses).
    auto mfV = [&](const bf16x8_t& vf, const u32x4_t (&pkv)[2][2], int ksl, int dt) __attribute__((always_inline)) {
#pragma unroll
        for (int rb = 0; rb < 2; ++rb)
        {
            o[rb][dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, __builtin_bit_cast(bf16x8_t, pkv[rb][ksl]),
                                                                 o[rb][dt], 0, 0, 0);
            asm volatile("" : "+a"(o[rb][dt]));
        }
    };
    auto mfV1 = [&](const bf16x8_t& vf, const u32x4_t (&pkv)[2][2], int ksl, int dt, int rb) __attribute__((always_inline)) {
        o[rb][dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, __builtin_bit_cast(bf16x8_t, pkv[rb][ksl]), o[rb][dt], 0, 0, 0);
        asm volatile("" : "+a"(o[rb][dt]));
    };
    // softmax of elements e, e+1 of one 16-value S block of row block rb: P pair -> dword
    // (e >> 1) & 3 of k-step (e >> 3) of pkd, the two p into rb's row sum.  The two v_add_f32
    // stay: packed (v_pk_add_f32 on a pair) or one v_dot2c_f32_bf16 of the packed P with (1, 1)
    // issue fewer VALU ops but stall beside the MFMAs -- +6 % and +11 % self-attention time
    // (profiles/r5/attn_pksum_ldsbase_ab_s23.log, attn_dot2_rowsum_ab_s25.log)
    auto smp = [&](const f32x16_t& sv, int e, u32x4_t (&pkd)[2], int rb) __attribute__((always_inline)) {
        const float pa = __builtin_amdgcn_exp2f(sv[e]), pb = __builtin_amdgcn_exp2f(sv[e + 1]);
        lsum[rb] += pa + pb;
        const bf16x2_t w = {(__bf16)pa, (__bf16)pb};
        unsigned wu = __builtin_bit_cast(unsigned, w);
        // pure VALU floats freely in the IR: tie it to this step
        asm volatile("" : "+v"(lsum[rb]), "+v"(wu));
        pkd[e >> 3][(e >> 1) & 3] = wu;
    };
    // the same softmax step in two halves for the split-gap placement: the two exps (8 issue
    // cycles each) in one MFMA gap, the row-sum adds and the pack in the next
    auto smp_e = [&](const f32x16_t& sv, int e, float& pa, float& pb) __attribute__((always_inline)) {
        pa = __builtin_amdgcn_exp2f(sv[e]);
        pb = __builtin_amdgcn_exp2f(sv[e + 1]);
        asm volatile("" : "+v"(pa), "+v"(pb));
    };
    auto smp_f = [&](float pa, float pb, int e, u32x4_t (&pkd)[2], int rb) __attribute__((always_inline)) {
        lsum[rb] += pa + pb;
        const bf16x2_t w = {(__bf16)pa, (__bf16)pb};
        unsigned wu = __builtin_bit_cast(unsigned, w);
        asm volatile("" : "+v"(lsum[rb]), "+v"(wu));
        pkd[e >> 3][(e >> 1) & 3] = wu;
    };
    auto mfK1 = [&](const bf16x8_t& kf, int j, f32x16_t (&sv)[2], int rb) __attribute__((always_inline)) {
        if (j == 0)
            asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=v"(sv[rb]) : "v"(kf), "a"(qf[rb][j]));
        else
            asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(sv[rb]) : "v"(kf), "a"(qf[rb][j]));
    };
    // B(T+1); the DMA of tile T+3 is issued one piece per step of phase D
    auto sync = [&](int T, auto first_c) __attribute__((always_inline)) {
        fence();
        stamp(3);
        if constexpr (!decltype(first_c)::value)     // phase D's first piece destination (piece_go)
            asm volatile("s_mov_b32 m0, %0" :: "s"(lds0 + ((T + 3) & 3) * W4_SLOT) : "m0");
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
        fence();
        stamp(4);
#ifdef VS_W4_STAMPS
        stamp_store(st_it, 0, 4);
#endif
        stage_begin(T + 3);
    };
    int nxt = -1, qv = 0;           // the next item (from the LDS word, read in an item's first tile)
    // one iteration on tile T; FIRST: the item's first tile (no PV, no previous softmax)
    auto iteration = [&](int T, f32x16_t (&s1c)[2], const f32x16_t (&s1p)[2], u32x4_t (&p0c)[2][2],
                         const u32x4_t (&p0p)[2][2], auto first_c) __attribute__((always_inline)) {
        constexpr bool FIRST = decltype(first_c)::value;
#ifdef VS_W4_STAMPS
        if (st_it >= 0) {                // stamps 4, 5 of the previous stamped iteration
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            stamp_store(st_it, 4, 7);
        }
        st_it = (blockIdx.x == 0 && !FIRST && T >= 8 && T < 40) ? T - 8 : -1;
#endif
        stamp(0);
        // A/B with the step's fillers split over its two MFMA gaps (program order pinned):
        // [read, MFMA rb0] [exp, exp] [MFMA rb1] [add, add, pack]
#pragma unroll
        for (int j = 0; j < 8; ++j) {                                   // A
            float pa = 0.f, pb = 0.f;
            rdK(kf1[j], 1, j);
            mfK1(kf0[j], j, s0, 0);
            fence();
            if (!FIRST) smp_e(s1p[0], 2 * j, pa, pb);
            fence();
            mfK1(kf0[j], j, s0, 1);
            fence();
            if (!FIRST) smp_f(pa, pb, 2 * j, p1[0], 0);
            fence();
        }
        stamp(1);
        if (!FIRST) vbase(T - 1);
#pragma unroll
        for (int j = 0; j < 8; ++j) {                                   // B
            float pa = 0.f, pb = 0.f;
            if (!FIRST) rdV(vfa[j], j >> 2, j & 3);
            mfK1(kf1[j], j, s1c, 0);
            fence();
            if (!FIRST) smp_e(s1p[1], 2 * j, pa, pb);
            fence();
            mfK1(kf1[j], j, s1c, 1);
            fence();
            if (!FIRST) smp_f(pa, pb, 2 * j, p1[1], 1);
            fence();
        }
        stamp(2);
#pragma unroll
        for (int i = 0; i < 8; ++i) {                                   // C
            if (!FIRST) {
                // V ks2,3 fragments in the first half of C: the lgkmcnt(0) before the barrier
                // then finds them landed
                if (i < 4) {
                    rdV(vfb[2 * i], 2 + (i >> 1), (2 * i) & 3);
                    rdV(vfb[2 * i + 1], 2 + (i >> 1), (2 * i + 1) & 3);
                }
                mfV(vfa[i], p0p, i >> 2, i & 3);
            }
            smp(s0[0], 2 * i, p0c[0], 0);
            smp(s0[1], 2 * i, p0c[1], 1);
            fence();
        }
        sync(T, first_c);
        kbase(T + 1);
#pragma unroll
        for (int i = 0; i < 8; ++i) {                                   // D
            if (FIRST) stage_piece(i);
            else piece_go(i);
            if (FIRST && i == 0)            // the item after this one (written by wave 0 before B(T+1))
                qv = *(volatile LDS_AS int*)(uintptr_t)(smem_base + W4_QSLOT);
            rdK(kf0[i], 0, i);
            if (!FIRST) {
                mfV1(vfb[i], p1, i >> 2, i & 3, 0);
                fence();
                if (i < 7) m0_step(i + 1);
                fence();
                mfV1(vfb[i], p1, i >> 2, i & 3, 1);
            }
            fence();
#ifdef VS_W4_STAMPS
            if (i == 3) stamp(6);
#endif
        }
        stamp(5);
        if constexpr (FIRST) {
            nxt = __builtin_amdgcn_readfirstlane(qv);
            dnext = nxt;
        }
        stage_next();
    };
    // after the item's last tile TL: S(TL) kb1 -> P ks2,3, PV(TL)
    auto drain = [&](int TL, const f32x16_t (&s1l)[2], const u32x4_t (&p0l)[2][2]) __attribute__((always_inline)) {
        vbase(TL);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            rdV(vfa[j], j >> 2, j & 3);
            smp(s1l[0], 2 * j, p1[0], 0);
            fence();
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            rdV(vfb[j], 2 + (j >> 2), j & 3);
            smp(s1l[1], 2 * j, p1[1], 1);
            fence();
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) mfV(vfa[i], p0l, i >> 2, i & 3);
#pragma unroll
        for (int i = 0; i < 8; ++i) mfV(vfb[i], p1, i >> 2, i & 3);
    };
    // prologue: tiles 0, 1 staged, B(0), tile 2 staged, K(0) kb0 fragments, the first Q
    stage(0);
    stage(1);
    fence();
    asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
    fence();
    stage(2);
    kbase(0);
#pragma unroll
    for (int i = 0; i < 8; ++i) rdK(kf0[i], 0, i);
    int T = 0, q0 = 0;
    int bh = item_bh(cur, q0);
    q0 += 64 * wave;
    // wave 0 takes the item after `after` (AttnChunks): the queue atomic goes out before the next Q's
    // loads, which retire it (they complete in issue order), and its id into the LDS word
    unsigned* const qw = pers ? args.queue : nullptr;
    auto next_q = [&](int after) __attribute__((always_inline)) {
        unsigned t0 = 0;
#ifdef VS_W4_STAMPS
        // (diagnostic split of the next-Q cost: 6 -> 7 the in-flight K/V DMA drained, 7 -> 8 the Q loads)
        swst(6);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        swst(7);
#endif
        if (qw && wave == 0) t0 = vs_queue_issue(qw + (blockIdx.x & 7) * VS_Q_LINE);
        load_q(q_base(bh), q0);
#ifdef VS_W4_STAMPS
        swst(8);
#endif
        if (wave == 0) {
            const int id = pers ? chunks.take(qw, t0, after, lane) : -1;
            if (lane == 0) *(volatile LDS_AS int*)(uintptr_t)(smem_base + W4_QSLOT) = id;
        }
    };
    next_q(cur);
    for (;;) {
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) {
            lsum[rb] = 0.f;
#pragma unroll
            for (int dt = 0; dt < 4; ++dt)
#pragma unroll
                for (int i = 0; i < 16; ++i) o[rb][dt][i] = 0.f;
        }
        swst(0);
        iteration(T, s1a, s1b, p0a, p0b, std::true_type{});
        swst(1);
        ++T;
        int t = 1;
        for (; t + 1 < nkv; t += 2) {
            iteration(T, s1b, s1a, p0b, p0a, std::false_type{});
            ++T;
            iteration(T, s1a, s1b, p0a, p0b, std::false_type{});
            ++T;
        }
        swst(2);
        const int bh_done = bh, q0_done = q0;
        if (nxt >= 0) {                  // the next item's Q (its QK starts after the drain)
            bh = item_bh(nxt, q0);
            q0 += 64 * wave;
        }
        if (t < nkv) {
            iteration(T, s1b, s1a, p0b, p0a, std::false_type{});
            ++T;
            swst(3);
            drain(T - 1, s1b, p0b);
        } else {
            swst(3);
            drain(T - 1, s1a, p0a);
        }
        swst(4);
        finish(o_base(bh_done), q0_done, cur);
        // the next item's Q after the O store (r5): its loads wait at once anyway (the scaling
        // pass), and loaded before the drain the new Q was live beside the old O through the drain
        // and the store -- the register allocator spilled part of it (scratch reloads whose vmcnt
        // waits drained the K/V DMA, profiles/r5/w4_lasttile_s16.log)
        if (nxt >= 0) next_q(nxt);
        swst(5);
        sw_store();
        if (nxt < 0) break;
        cur = nxt;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (qw && tid == 0) vs_queue_done(qw, 9, npers);
#ifdef VS_W4_STAMPS
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    stamp_store(st_it, 4, 7);
    __syncthreads();
    if (blockIdx.x == 0)
        for (int i = lane; i < 32 * 7; i += 64)
            (&g_w4_stamps[wave][0][0])[i] = *reinterpret_cast<volatile unsigned long long*>(smem + W4_STAMP_OFF + 8 * (wave * 32 * 7 + i));
    if (blockIdx.x == 0)
        for (int i = lane; i < 16 * W4_SWN; i += 64)
            (&g_w4_sw[wave][0][0])[i] = *reinterpret_cast<volatile unsigned long long*>(smem + W4_SW_OFF + 8 * (wave * 16 * W4_SWN + i));
#endif
}

}  // namespace

hipError_t attn_w4_launch(const AttnArgs& args, bool rebase, unsigned grid, hipStream_t stream) {
    void (*kern)(AttnArgs) = rebase ? attn_fwd_w4<true> : attn_fwd_w4<false>;
    static std::mutex mu;
    static std::set<const void*> done;
    {
        std::lock_guard<std::mutex> lock(mu);
        if (done.insert((const void*)kern).second)
            (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, W4_LDS_ALLOC);
    }
    hipLaunchKernelGGL(kern, dim3(grid), dim3(W4_THR), W4_LDS_ALLOC, stream, args);
    return hipGetLastError();
}

}  // namespace vs_attn

#ifdef VS_W4_STAMPS
extern "C" int vs_debug_w4_switch(unsigned long long* host_out) {
    return hipMemcpyFromSymbol(host_out, HIP_SYMBOL(vs_attn::g_w4_sw), sizeof(vs_attn::g_w4_sw)) == hipSuccess ? 0 : 2;
}
extern "C" int vs_debug_w4_stamps(unsigned long long* host_out) {
    return hipMemcpyFromSymbol(host_out, HIP_SYMBOL(vs_attn::g_w4_stamps), sizeof(vs_attn::g_w4_stamps)) == hipSuccess ? 0 : 2;
}
#endif
