// bf16 MFMA GEMM with fused epilogues, gfx950:  C = epi(A . W^T [+ A2 . W2^T]).
//
// Replaces every nn.Linear of the DiT / VACE hot path (reference diffsynth/models/wan_video_dit.py
// :131-134, 157-160, 209-210, 259, 308-319; wan_video_vace.py:10-11) as executed through
// AutoWrappedLinear.forward (diffsynth/vram_management/layers.py:173-188), with the elementwise
// op that follows each linear in the reference fused into the epilogue: GELU-tanh (ffn.0),
// SiLU (time MLP), GateModule x + g*y (o-proj, ffn.2; wan_video_dit.py:193-194), residual add
// (cross-attn, VACE before_proj), VACE hint add (wan_video_new.py:1450), LoRA merge
// (lora/__init__.py:40-43) and the un-merged LoRA term (layers.py:180-182) as a second K phase.
//
// Kernels sharing the epilogue:
//  * gemm_bf16_tn_8p (K >= 4096 and >= 240 tiles of 256x256): the staggered 8-phase schedule (see
//    its header) -- the un-merged LoRA second phase and VS_OPT_GEMM_KERNEL 8;
//  * gemm_fp8_tn_8p: the fp8 (config 5) variant of the same skeleton;
//  * gemm_bf16_tn (everything else): the structure described below.
// Structure: 128x128x64 tile, 4 waves (2x2, 64x64 each), v_mfma_f32_16x16x32_bf16 computing the
// transposed tile (W rows as the A operand) so every lane owns 4 consecutive output columns;
// both operands are K-contiguous ([rows][K]) and staged by global_load_lds_dwordx4 (LDS-DMA,
// no VGPR round trip) into a 2-stage LDS ring whose 128-B rows carry a 16-B-chunk XOR swizzle
// (chunk ^ (row & 7)) applied on the global SOURCE address, which makes the fragment
// ds_read_b128 conflict free; grouped (8 m-tiles) + XCD-aware tile order for L2 reuse.
#include "common.h"
#include <stdlib.h>
#include <utility>
#include <type_traits>

namespace {

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int NTHR = 256;
constexpr int STAGE_BYTES = (BM + BN) * BK * 2;  // 32 KB

struct Epi {
    const bf16_t* bias;
    const bf16_t* res;
    long long ld_res;
    const bf16_t* gate;
    long long gate_bstride;
    const bf16_t* hint;
    long long ld_hint;
    float hint_scale;
    float alpha;
    int rows_per_batch;
    int mode;
    int gm;           // M-tiles per raster group of the 256x256 tile order (VS_GEMM_GM)
};

__device__ __forceinline__ int g_off(int row, int ch) { return row * 128 + 16 * (ch ^ (row & 7)); }

template <int W>
__device__ __forceinline__ void loadw(const bf16_t* p, float* v) {
    if constexpr (W == 4) {
        const u32x2_t w = *reinterpret_cast<const u32x2_t*>(p);
#pragma unroll
        for (int i = 0; i < 2; ++i) { v[2 * i] = bflo(w[i]); v[2 * i + 1] = bfhi(w[i]); }
    } else {
        const u32x4_t w = *reinterpret_cast<const u32x4_t*>(p);
#pragma unroll
        for (int i = 0; i < 4; ++i) { v[2 * i] = bflo(w[i]); v[2 * i + 1] = bfhi(w[i]); }
    }
}

// the op that follows each linear, on W consecutive columns of row m: y = bf16(acc + bias), then
// GELU / SiLU / gate-residual [+ hint] / residual with the reference's bf16 rounding points
template <int W>
__device__ __forceinline__ void epilogue_store_w(const float* a, int m, int n, bf16_t* C, long long ldc,
                                                 const Epi& ep) {
    const int bidx = m / ep.rows_per_batch;
    float bv[W] = {};
    if (ep.bias) loadw<W>(ep.bias + n, bv);
    float y[W];
#pragma unroll
    for (int e = 0; e < W; ++e) y[e] = rbf(a[e] + bv[e]);
    if (ep.mode == VS_EPI_GELU) {
#pragma unroll
        for (int e = 0; e < W; ++e) y[e] = gelu_tanh_f(y[e]);
    } else if (ep.mode == VS_EPI_SILU) {
#pragma unroll
        for (int e = 0; e < W; ++e) y[e] = silu_f(y[e]);
    } else if (ep.mode == VS_EPI_GATE_RES) {
        float rv[W], gv[W];
        loadw<W>(ep.res + (long long)m * ep.ld_res + n, rv);
        loadw<W>(ep.gate + (long long)bidx * ep.gate_bstride + n, gv);
#pragma unroll
        for (int e = 0; e < W; ++e) y[e] = rbf(rv[e] + rbf(gv[e] * y[e]));
        if (ep.hint) {
            float hv[W];
            loadw<W>(ep.hint + (long long)m * ep.ld_hint + n, hv);
#pragma unroll
            for (int e = 0; e < W; ++e) y[e] = y[e] + rbf(hv[e] * ep.hint_scale);
        }
    } else if (ep.mode == VS_EPI_RES) {
        float rv[W];
        loadw<W>(ep.res + (long long)m * ep.ld_res + n, rv);
#pragma unroll
        for (int e = 0; e < W; ++e) y[e] = rv[e] + rbf(ep.alpha * y[e]);
    }
    if constexpr (W == 4) {
        *reinterpret_cast<u32x2_t*>(C + (long long)m * ldc + n) = u32x2_t{pack2(y[0], y[1]), pack2(y[2], y[3])};
    } else {
        *reinterpret_cast<u32x4_t*>(C + (long long)m * ldc + n) =
            u32x4_t{pack2(y[0], y[1]), pack2(y[2], y[3]), pack2(y[4], y[5]), pack2(y[6], y[7])};
    }
}

__device__ __forceinline__ void epilogue_store(const f32x4_t& a, int m, int n, bf16_t* C, long long ldc,
                                               const Epi& ep) {
    const float v[4] = {a[0], a[1], a[2], a[3]};
    epilogue_store_w<4>(v, m, n, C, ldc, ep);
}

__global__ __launch_bounds__(NTHR, 2) void gemm_bf16_tn(
    const bf16_t* __restrict__ A, long long lda, const bf16_t* __restrict__ W, long long ldw,
    bf16_t* C, long long ldc, int M, int N, int K, const bf16_t* __restrict__ A2, long long lda2,
    const bf16_t* __restrict__ W2, long long ldw2, int K2, Epi ep, int ntm, int ntn) {
    extern __shared__ __attribute__((aligned(16))) char smem[];

    // grouped tile order (8 m-tiles per group) on top of the XCD remap
    const int pid = xcd_remap(blockIdx.x, gridDim.x);
    constexpr int GM = 8;
    const int per_group = GM * ntn;
    const int group = pid / per_group;
    const int first_m = group * GM;
    const int gsz = min(ntm - first_m, GM);
    const int in_g = pid % per_group;
    const int tm = first_m + in_g % gsz;
    const int tn = in_g / gsz;
    const int m0 = tm * BM, n0 = tn * BN;

    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int wm = wave >> 1, wn = wave & 1;

    f32x4_t acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    // LDS-DMA staging: a wave writes 4 pieces of A and 4 of W; piece p = rows 8p..8p+7 (1 KB),
    // lane L lands at byte 16*L of the piece = row 8p + L/8, physical chunk L%8 -> it fetches
    // logical chunk (L%8) ^ (row%8) = (L%8) ^ (L/8).
    const int srow = lane >> 3;
    const int sch = (lane & 7) ^ srow;
    auto stage = [&](int buf, const bf16_t* Ap, long long ldap, const bf16_t* Wp, long long ldwp,
                     int k0) {
        char* base = smem + buf * STAGE_BYTES;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int piece = wave * 4 + j;
            const int row = piece * 8 + srow;
            const long long ar = min(m0 + row, M - 1);
            const bf16_t* src = Ap + ar * ldap + k0 + sch * 8;
            __builtin_amdgcn_global_load_lds((const GLB_AS void*)src,
                                             (LDS_AS void*)(base + piece * 1024), 16, 0, 0);
            const long long wr = min(n0 + row, N - 1);
            const bf16_t* srcw = Wp + wr * ldwp + k0 + sch * 8;
            __builtin_amdgcn_global_load_lds((const GLB_AS void*)srcw,
                                             (LDS_AS void*)(base + BM * 128 + piece * 1024), 16, 0, 0);
        }
    };

    const int frow = lane & 15, fch = lane >> 4;
    auto compute = [&](int buf) {
        const char* As = smem + buf * STAGE_BYTES;
        const char* Bs = As + BM * 128;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            bf16x8_t af[4], wf[4];
#pragma unroll
            for (int i = 0; i < 4; ++i)
                af[i] = *reinterpret_cast<const bf16x8_t*>(As + g_off(wm * 64 + i * 16 + frow, kk * 4 + fch));
#pragma unroll
            for (int j = 0; j < 4; ++j)
                wf[j] = *reinterpret_cast<const bf16x8_t*>(Bs + g_off(wn * 64 + j * 16 + frow, kk * 4 + fch));
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], af[i], acc[i][j], 0, 0, 0);
        }
    };

    const int nk1 = K / BK;
    const int total = nk1 + K2 / BK;
    stage(0, A, lda, W, ldw, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int kt = 0; kt < total; ++kt) {
        const int kn = kt + 1;
        if (kn < total) {
            if (kn < nk1)
                stage(kn & 1, A, lda, W, ldw, kn * BK);
            else
                stage(kn & 1, A2, lda2, W2, ldw2, (kn - nk1) * BK);
        }
        compute(kt & 1);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }

    // epilogue: acc[i][j][e] = C[m][n], m = m0+wm*64+16i+(lane&15), n = n0+wn*64+16j+4*(lane>>4)+e
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int m = m0 + wm * 64 + i * 16 + (lane & 15);
        if (m >= M) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int n = n0 + wn * 64 + j * 16 + 4 * (lane >> 4);
            if (n >= N) continue;
            epilogue_store(acc[i][j], m, n, C, ldc, ep);
        }
    }
}


// ---------------------------------------------------------------------------------------------
// 256x256 tiles (gemm_bf16_tn_8p, gemm_fp8_tn_8p): shared tile order, split-tail combine, epilogue
// pass of the hipBLASLt route.
// ---------------------------------------------------------------------------------------------
#ifndef VS_GEMM_GM
#define VS_GEMM_GM 4            // M-tiles per raster group (L2 reuse of the weight tile)
#endif
constexpr int BT = 256;

// tile id -> (tm, tn): raster groups of GM M-tiles sweep all N-tiles, so consecutive ids on one
// XCD share the weight tile in L2
__device__ __forceinline__ void tile_of(int pid, int ntm, int ntn, int GM, int& tm, int& tn) {
    const int per_group = GM * ntn;
    const int group = pid / per_group;
    const int first_m = group * GM;
    const int gsz = min(ntm - first_m, GM);
    const int in_g = pid % per_group;
    tm = first_m + in_g % gsz;
    tn = in_g / gsz;
}

// Split-tail combine: one thread per (tail tile, row, 4 columns): sum the ksplit fp32 partials in
// piece order, then the same epilogue as the unsplit kernel
__global__ __launch_bounds__(256) void gemm_split_combine(const float* __restrict__ part, bf16_t* C, long long ldc,
                                                          int M, int N, Epi ep, int ntm, int ntn, int nmain,
                                                          int ntail, int ksplit,
                                                          const float* __restrict__ scale_a = nullptr) {
    const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
    if (idx >= (long long)ntail * BT * (BT / 4)) return;
    const int t = (int)(idx / (BT * (BT / 4)));
    const int rem = (int)(idx % (BT * (BT / 4)));
    const int row = rem / (BT / 4), c4 = rem % (BT / 4);
    int tm, tn;
    tile_of(nmain + t, ntm, ntn, ep.gm, tm, tn);
    const int m = tm * BT + row, n = tn * BT + 4 * c4;
    if (m >= M || n >= N) return;
    const float* pp = part + (long long)t * ksplit * BT * BT + row * BT + 4 * c4;
    f32x4_t a = *reinterpret_cast<const f32x4_t*>(pp);
    for (int j = 1; j < ksplit; ++j) a += *reinterpret_cast<const f32x4_t*>(pp + (long long)j * BT * BT);
    if (scale_a) a *= scale_a[m];
    epilogue_store(a, m, n, C, ldc, ep);
}


// ---------------------------------------------------------------------------------------------
// gemm_bf16_tn_8p: 256x256x64 tile, 8 waves, 4 phases per K-tile (cdna_hip_programming.md §5,
// "The 256² 8-phase template", written for this epilogue / split-tail / LoRA contract).
//
// LDS: two buffers (even / odd K-tile) of four 16-KB half-tiles each: A rows 0-127 (A0), A rows
// 128-255 (A1), W rows 0-127 (B0), W rows 128-255 (B1); 128-B rows (64 bf16 of K) with the 16-B
// chunk swizzle c ^ (row & 7) (conflict-free 16x16x32 fragment reads), filled by LDS-DMA
// (buffer_load ... lds, one 1-KB piece = 8 rows per wave-instruction, swizzle on the source).
// The tile's four 128x128 quadrants are computed one per phase by all 8 waves (wave (wr, wc) =
// rows 64 wr.. of the A half x columns 32 wc.. of the W half: 16 MFMAs per phase):
//   ph0 (A0,B0): read A-frags (8 ds_read_b128) + B0-frags (4)    ph1 (A0,B1): read B1-frags (4)
//   ph2 (A1,B1): read A-frags (8)                                ph3 (A1,B0): no reads
// so half-tile A0/B0 of a buffer is dead after ph0, B1 after ph1, A1 after ph2, and each phase
// restages one half-tile whose last read is >= 1 phase (and one workgroup barrier) behind it:
//   ph0: A1 of tile t+1, ph1: A0 of t+2, ph2: B0 of t+2, ph3: B1 of t+2.
// Phase = [fragment reads; 2 DMA pieces; (ph3: s_waitcnt vmcnt(6)); s_barrier; lgkmcnt(0);
// setprio 1; 16 MFMAs; setprio 0; s_barrier]: the ph3 wait retires tile t+1 while the three
// half-tiles issued after it stay in flight across the barriers (counted vmcnt, raw s_barrier,
// never vmcnt(0) in the main loop).  Waves 4-7 run ONE BARRIER BEHIND waves 0-3 (the template's
// stagger), so on every SIMD one wave's 16 MFMAs pair with its partner's fragment reads and DMA
// issue (matrix beside memory) instead of all 8 waves reading, then all 8 computing: r3, same box,
// 1135-1177 -> 1301-1373 TF/s on the 14B block shapes (profiles/r3/gemm_stagger_ab_s1.log).  With
// the groups a barrier apart, A0 (restaged one phase after its ph0 reads) is protected by a counted
// lgkmcnt(4) (the 8 A reads are issued before the 4 B reads) ahead of ph0's first barrier.
// Product D[n][m] = W.A^T (16x16x32, W fragment as the A operand) so each lane owns 4 consecutive
// output columns for the fused epilogue.
// ---------------------------------------------------------------------------------------------
constexpr int T8 = 256, HT8 = 128 * 128, BUF8 = 4 * HT8, LDS8 = 2 * BUF8;   // 16 KB, 64 KB, 128 KB
// half-tiles (0 A0, 1 A1, 2 B0, 3 B1) of the two buffers interleaved: [A0 b0][A0 b1][A1 b0][A1 b1]
// [B0 b0]...  so every A read of either buffer lies within the 16-bit ds_read offset of one base
// VGPR per k-step, and every B read within that of a second one
constexpr int R_A0 = 0, R_A1 = 1, R_B0 = 2, R_B1 = 3;
__device__ __forceinline__ constexpr int hoff(int which, int b) { return (2 * which + b) * HT8; }

__device__ __forceinline__ int q_off(int row, int ch) { return row * 128 + 16 * (ch ^ (row & 7)); }

template <bool LORA, bool WIDE>    // WIDE: 16-B epilogue accesses (host-checked alignment, N % 8 == 0)
__global__ __launch_bounds__(512, 2) void gemm_bf16_tn_8p(
    const bf16_t* __restrict__ A, long long lda, const bf16_t* __restrict__ W, long long ldw,
    bf16_t* C, long long ldc, int M, int N, int K, const bf16_t* __restrict__ A2, long long lda2,
    const bf16_t* __restrict__ W2, long long ldw2, int K2, Epi ep, int ntm, int ntn, int nmain, int ksplit,
    int piece_k, float* __restrict__ part) {
    extern __shared__ __attribute__((aligned(16))) char smem[];

    // blocks [0, nmain) own whole tiles (XCD-remapped); the blocks after them run the last tiles of
    // the grid as ksplit K ranges of piece_k each (fp32 partial tiles for gemm_split_combine)
    int pid, piece = -1;
    if ((int)blockIdx.x < nmain) {
        pid = xcd_remap(blockIdx.x, nmain);
    } else {
        const int t = blockIdx.x - nmain;
        pid = nmain + t / ksplit;
        piece = t % ksplit;
    }
    int tm, tn;
    tile_of(pid, ntm, ntn, ep.gm, tm, tn);
    const int m0 = tm * T8, n0 = tn * T8;
    const int kb = piece < 0 ? 0 : piece * piece_k;
    const int Kp = piece < 0 ? K : min(K - kb, piece_k);
    const int nk1 = Kp / 64;
    const int nt = nk1 + (piece < 0 ? K2 / 64 : 0);

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wave >> 2, wc = wave & 3;

    f32x4_t acc[2][2][4][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[a][b][i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    // DMA: a half-tile is 16 pieces of 1 KB; wave w issues pieces 2w, 2w+1 = rows 16w + 8j + L/8,
    // lane L lands in physical chunk L%8 of its row and fetches logical chunk (L%8) ^ (L/8).
    // Buffer descriptors are rebased on the tile's first row, so a voffset is < 256 rows x ld.
    const int prow = 16 * wave + (lane >> 3);
    const unsigned pcol = 16u * ((lane & 7) ^ (lane >> 3));
    auto rsrc = [](const void* base) {
        return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
    };
    const __amdgpu_buffer_rsrc_t ra = rsrc(A + (long long)m0 * lda + kb);
    const __amdgpu_buffer_rsrc_t rw = rsrc(W + (long long)n0 * ldw + kb);
    const int alim = M - 1 - m0, wlim = N - 1 - n0;
    const unsigned ldab = (unsigned)(lda * 2), ldwb = (unsigned)(ldw * 2);
    // stage half-tile `which` (0 A0, 1 A1, 2 B0, 3 B1) of K-tile t into buffer t & 1
    // the eight DMA row offsets (half-tile x piece; the K offset goes in soffset) computed once and
    // held in VGPRs across the K loop: forming them per stage cost a 32-bit multiply (v_mad_u64_u32),
    // a clamp and an add per LDS-DMA instruction -- hoisted, +4-5 % on every 14B shape at 59 280 and
    // 7410 rows, 4 more VGPRs (profiles/r3/gemm_preoff_ab.log)
    unsigned voff[4][2];
#pragma unroll
    for (int w = 0; w < 4; ++w)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int r = (w & 1) * 128 + prow + 8 * j;
            voff[w][j] = w >= 2 ? (unsigned)min(r, wlim) * ldwb + pcol : (unsigned)min(r, alim) * ldab + pcol;
        }
    auto stage = [&](int t, int which) {
        char* dst = smem + hoff(which, t & 1) + wave * 2048;
        const bool isw = which >= 2;
        const int h = which & 1;
        if (!LORA || t < nk1) {
            const unsigned ko = (unsigned)t * 128u;
#pragma unroll
            for (int j = 0; j < 2; ++j)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(isw ? rw : ra, (LDS_AS void*)(dst + j * 1024), 16,
                                                         voff[which][j], ko, 0, 0);
        } else {
            // second K phase (un-merged LoRA): A2 . W2^T, rank-sized, addresses formed here
            const unsigned ko = (unsigned)(t - nk1) * 128u;
            const __amdgpu_buffer_rsrc_t r2 = rsrc(isw ? W2 + (long long)n0 * ldw2 : A2 + (long long)m0 * lda2);
            const int lim = (isw ? N : M) - 1, r0 = isw ? n0 : m0;
            const unsigned ld2 = (unsigned)((isw ? ldw2 : lda2) * 2);
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int r = h * 128 + prow + 8 * j;
                __builtin_amdgcn_raw_ptr_buffer_load_lds(r2, (LDS_AS void*)(dst + j * 1024), 16,
                                                         (unsigned)(min(r0 + r, lim) - r0) * ld2 + pcol, ko, 0, 0);
            }
        }
    };

    const int frow = lane & 15, fch = lane >> 4;
    bf16x8_t af[4][2], bf0[2][2], bf1[2][2];
    // fragment addresses: q_off(row0 + 16 i + frow, 4 s + fch) = q_off(row0 + frow, 4 s + fch) + 2048 i
    // (row & 7 = frow & 7); one base per (buffer, operand, k-step) -- the second buffer lies past the
    // 16-bit ds_read offset field -- kept opaque so the compiler keeps exactly these 8 bases
    int abase[2], bbase[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        abase[s] = (int)(uintptr_t)smem + q_off(wr * 64 + frow, 4 * s + fch);
        bbase[s] = (int)(uintptr_t)smem + hoff(R_B0, 0) + q_off(wc * 32 + frow, 4 * s + fch);
        asm volatile("" : "+v"(abase[s]), "+v"(bbase[s]));
    }
    auto lds_frag = [&](int addr) {
        return *reinterpret_cast<const LDS_AS bf16x8_t*>((const LDS_AS char*)(uintptr_t)(unsigned)addr);
    };
    auto read_a = [&](const char* buf, int region) {
        const int b = buf == smem ? 0 : 1;     // (buf: smem or smem + BUF8)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int s = 0; s < 2; ++s) af[i][s] = lds_frag(abase[s] + hoff(region, b) + 2048 * i);
    };
    auto read_b = [&](const char* buf, int region, bf16x8_t (&bf)[2][2]) {
        const int b = buf == smem ? 0 : 1;     // (buf: smem or smem + BUF8)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int s = 0; s < 2; ++s) bf[j][s] = lds_frag(bbase[s] + hoff(region, b) - hoff(R_B0, 0) + 2048 * j);
    };
    auto mfma16 = [&](f32x4_t (&c)[4][2], const bf16x8_t (&bf)[2][2]) {
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    c[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][s], af[i][s], c[i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
    };
    auto bar = [&]() {
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_barrier" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
    };
    auto bar_wait_lgkm = [&]() {
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_barrier" ::: "memory");
        // the builtin form (not asm): the compiler's wait-count pass then knows every earlier LDS read
        // has landed and adds no lgkmcnt(0) of its own in front of this phase's MFMAs
        __builtin_amdgcn_s_waitcnt(0xC07F);     // lgkmcnt(0)
        __builtin_amdgcn_sched_barrier(0);
    };

    // prologue: tile 0 (A0 B0 B1 A1) and tile 1 (A0 B0 B1) in flight, wait for tile 0
    stage(0, 0); stage(0, 2); stage(0, 3); stage(0, 1);
    if (nt > 1) {
        stage(1, 0); stage(1, 2); stage(1, 3);
        asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    bar();

    // one K-tile = 4 phases; the body is written for a pair of tiles so the buffer is a constant
    auto tile4 = [&](int t, const char* buf) __attribute__((always_inline)) {
        // ph0: quadrant (A0, B0); lgkmcnt(4) retires this wave's A0 reads before the barrier
        read_a(buf, R_A0);
        __builtin_amdgcn_sched_barrier(0);
        read_b(buf, R_B0, bf0);
        if (t + 1 < nt) stage(t + 1, 1);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_waitcnt(0xC47F);     // lgkmcnt(4)
        bar_wait_lgkm();
        mfma16(acc[0][0], bf0);
        bar();
        // ph1: quadrant (A0, B1)
        read_b(buf, R_B1, bf1);
        if (t + 2 < nt) stage(t + 2, 0);
        bar_wait_lgkm();
        mfma16(acc[0][1], bf1);
        bar();
        // ph2: quadrant (A1, B1)
        read_a(buf, R_A1);
        if (t + 2 < nt) stage(t + 2, 2);
        bar_wait_lgkm();
        mfma16(acc[1][1], bf1);
        bar();
        // ph3: quadrant (A1, B0); retire tile t+1 (the 3 half-tiles of t+2 stay in flight)
        if (t + 2 < nt) {
            stage(t + 2, 3);
            __builtin_amdgcn_sched_barrier(0);
            asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        } else if (t + 1 < nt) {
            __builtin_amdgcn_sched_barrier(0);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        bar_wait_lgkm();
        mfma16(acc[1][0], bf0);
        bar();
    };
    if (wr == 1) bar();                 // the stagger: waves 4-7 one barrier behind
#pragma nounroll
    for (int t = 0; t < nt; t += 2) {
        tile4(t, smem);
        if (t + 1 < nt) tile4(t + 1, smem + BUF8);
    }
    if (wr == 0) bar();                 // equal barrier counts before the epilogue

    // output: acc[qa][qb][i][j][e] = C[m][n], m = m0 + 128 qa + 64 wr + 16 i + (lane & 15),
    // n = n0 + 128 qb + 32 wc + 16 j + 4 (lane >> 4) + e
    if (piece >= 0) {
        float* pp = part + ((long long)(pid - nmain) * ksplit + piece) * T8 * T8;
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b)
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j)
                        *reinterpret_cast<f32x4_t*>(pp + (128 * a + 64 * wr + 16 * i + (lane & 15)) * T8 + 128 * b +
                                                    32 * wc + 16 * j + 4 * (lane >> 4)) = acc[a][b][i][j];
        return;
    }
    if constexpr (WIDE) {
        // 16-B epilogue (CDNA guide T21): lanes of row groups g, g^1 (lane ^ 16) trade one column
        // block through permlane16_swap, so an even-g lane holds columns 4g .. 4g+7 of block j = 0 and
        // an odd-g lane columns 16 + 4(g-1) .. +7 of block 1: one 8-column epilogue (16-B loads of
        // bias / residual / gate / hint, one 16-B store) instead of two 4-column ones
        const int g = lane >> 4;
        const int nw = 16 * (g & 1) + 4 * (g & ~1);
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int m = m0 + 128 * a + 64 * wr + 16 * i + (lane & 15);
#pragma unroll
                for (int b = 0; b < 2; ++b) {
                    float v[8];
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        // (element first, then __float_as_uint: hipcc 7.2 folds __builtin_bit_cast of a
                        // vector element to element 0 -- every swap then moved the same value)
                        const float x = acc[a][b][i][0][e], y = acc[a][b][i][1][e];
                        const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(y), false, false);
                        v[e] = __uint_as_float(sw[0]);
                        v[4 + e] = __uint_as_float(sw[1]);
                    }
                    const int n = n0 + 128 * b + 32 * wc + nw;
                    if (m < M && n < N) epilogue_store_w<8>(v, m, n, C, ldc, ep);
                }
            }
        return;
    }
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int m = m0 + 128 * a + 64 * wr + 16 * i + (lane & 15);
            if (m >= M) continue;
#pragma unroll
            for (int b = 0; b < 2; ++b)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const int n = n0 + 128 * b + 32 * wc + 16 * j + 4 * (lane >> 4);
                    if (n >= N) continue;
                    epilogue_store(acc[a][b][i][j], m, n, C, ldc, ep);
                }
        }
}


// ---------------------------------------------------------------------------------------------
// gemm_bf16_tn_4w: 256x256x64 tile, 4 waves (one per SIMD), each wave a 128x128 quadrant (8 x 8
// v_mfma_f32_16x16x32_bf16 tiles, 256 accumulator AGPRs).  The issue order is the one ROCm's own
// hipBLASLt uses for this tile on gfx950 (its MT256x256x64_MI16x16 DTLA1_DTLB1 PGR2 kernel, read
// from the disassembly of the image's TensileLibrary code object), written here from scratch
// for this library's epilogue / split-tail contract:
//  * LDS image per operand and buffer: 32 rows of 1056 B = 8 global rows x 128 B (64 k) + 32 B of
//    pad.  LDS row rho, column block q holds global row 128 (rho / 16) + 16 q + rho % 16, so one
//    LDS-DMA instruction (buffer_load_dwordx4 ... lds, 64 lanes x 16 B) fills exactly one LDS row
//    from 8 whole 128-B row segments, and a 16x32 fragment (lane l: row l % 16, 16-B chunk l / 16)
//    of m-tile i is one ds_read_b128 at row (16 wm + l % 16), +128 i, +64 s: the 1056-B stride
//    moves consecutive rows 8 banks apart, conflict-free for every lane group of ds_read_b128.
//  * Two buffers (K-tiles t, t+1); the DMA of K-tile t+2 goes into the buffer of t as soon as the
//    four waves have its fragments in registers: a K-tile's fragments (both k-steps, 128 VGPRs)
//    are held in registers, so each operand region is released by one barrier in the first
//    k-step and refilled during the rest of the iteration (one iteration of latency hiding).
//  * One iteration = 128 MFMAs (k-step 0, then k-step 1); interleaved in the MFMA stream: the
//    k-step-1 fragment reads of the current buffer, the 16 DMA instructions of K-tile t+2 (8 W rows
//    first, then 8 A), the k-step-0 fragment reads of the next buffer, and four barriers
//    (W region free, A region free, W of t+1 landed -- counted vmcnt(18) --, A of t+1 landed --
//    vmcnt(15)).  Every instruction group is fenced (sched_barrier), so issue order = source order.
// Product D[n][m] = W.A^T (W fragment as the A operand): each lane owns 4 consecutive output
// columns for the fused epilogue, as the other kernels.
// ---------------------------------------------------------------------------------------------
// straight-line expansion f(integral_constant<int, 0>) ... f(integral_constant<int, N-1>): every
// index is a compile-time constant (a 128-step #pragma unroll loop is not fully unrolled by hipcc,
// leaving the fragment arrays runtime-indexed, i.e. in scratch)
typedef int i32x4_t __attribute__((ext_vector_type(4)));
typedef int i32x8_t __attribute__((ext_vector_type(8)));

template <class F, int... Q>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, Q...>) {
    (f(std::integral_constant<int, Q>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
    static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// ---------------------------------------------------------------------------------------------
// Tile epilogue of the 4-wave kernels (16-B accesses): a wave owns rows m = m_w + 16 i + (lane & 15)
// (i = 0..7) and, after the permlane16_swap pairing of column blocks (2p, 2p+1), 8 consecutive
// columns n = n_w + 32 p .. +7 (p = 0..3).  The per-element epilogue branch of epilogue_store_w
// (mode tested per 8 columns, each load waited for before its store: 32 serialised HBM round trips
// per wave) becomes one mode-specialised body per launch that issues the residual / hint loads of
// rows i+4 while rows i are computed (4 rows of loads in flight), with the bias and gate rows loaded
// once per tile.  Same arithmetic and rounding points as epilogue_store_w.
// SCALED: the fp8 kernel's per-row activation scale (applied to the accumulator first).
// ---------------------------------------------------------------------------------------------
#ifndef W4_EPI_DEPTH
#define W4_EPI_DEPTH 2
#endif
// cache policy of the tile epilogue's output stores / residual loads (A/B knobs; gfx950 CPol bits:
// 1 sc0, 2 nt, 16 sc1)
#ifndef W4_OUT_CPOL
#define W4_OUT_CPOL 2
#endif
#ifndef W4_RES_CPOL
#define W4_RES_CPOL 0
#endif
#ifndef W4_EPI_DEPTH_BF16       // the bf16 un-hinted residual modes (registers for deeper prefetch)
#define W4_EPI_DEPTH_BF16 2
#endif
__device__ __forceinline__ u32x4_t ld16(const bf16_t* p) { return *reinterpret_cast<const u32x4_t*>(p); }
__device__ __forceinline__ void unpack8(const u32x4_t& w, float* v) {
#pragma unroll
    for (int i = 0; i < 4; ++i) { v[2 * i] = bflo(w[i]); v[2 * i + 1] = bfhi(w[i]); }
}

// v + s in a VGPR, formed at the point of use: a buffer access's row step kept in voffset (the
// resource's range check then covers it, so rows past the matrix load 0 whether or not the
// hardware checks soffset) without the compiler hoisting one VGPR per row step out of the loop
__device__ __forceinline__ int vadd_opq(int v, int s) {
    int r;
#if defined(__HIP_DEVICE_COMPILE__)         // (x86 reads "s" / "a" as register names: device pass only)
    asm volatile("v_add_u32 %0, %1, %2" : "=v"(r) : "s"(s), "v"(v));
#else
    r = v + s;
#endif
    return r;
}

// the store's pack, one v_cvt_pk_bf16_f32 per output pair (RNE, = pack2): from the C expression the
// compiler formed the pairs of its packed arithmetic, packed those and re-shuffled the halves
__device__ __forceinline__ uint32_t pk_store(float lo, float hi) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((float __attribute__((ext_vector_type(2)))){lo, hi}, bf16x2_t));
}
typedef float f32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2_t unpk2(uint32_t w) {
    return f32x2_t{__uint_as_float(w << 16), __uint_as_float(w & 0xffff0000u)};
}
// a bf16 rounding point of a pair (= rbf of each)
__device__ __forceinline__ f32x2_t rbf2(f32x2_t v) { return unpk2(pk_store(v.x, v.y)); }

// one accumulator element AGPR -> VGPR at its point of use: left to the compiler, the copies of
// all 256 accumulators were made at the K loop's exit (the class change from the MFMA asm's "a"
// operands) and the overflow spilled to scratch
__device__ __forceinline__ float acc_rd(float a) {
    float v;
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(v) : "a"(a));
#else
    v = a;
#endif
    return v;
}

// The tile epilogue's shape: W4_EPI_ROWS row steps of 16 x W4_EPI_CBLK column blocks of 32, one
// 16-B store each (+ one 16-B residual load each for the residual modes).  w4_epi_min_vmem is the
// fewest VMEM operations any instantiation issues (bias / gate / hint loads are conditional or
// mode-specific extras): the cross-tile drain of gemm_bf16_tn_4w (EPI_OPS; the fp8 kernel drains) relies
// on at least that many being issued after the tile's last DMAs, and static_asserts against it.
constexpr int W4_EPI_ROWS = 8, W4_EPI_CBLK = 4;
constexpr int w4_epi_min_vmem(int mode) {
    return W4_EPI_ROWS * W4_EPI_CBLK * ((mode == VS_EPI_GATE_RES || mode == VS_EPI_RES) ? 2 : 1);
}

template <int MODE, bool HINT, bool SCALED, class AccT>
__device__ __forceinline__ void tile_epilogue_w4(const AccT& acc, int m_w, int n_w, int lane, bf16_t* C, long long ldc,
                                                 int M, int N, const Epi& ep, const float* __restrict__ scale_a) {
    constexpr bool RESID = MODE == VS_EPI_GATE_RES || MODE == VS_EPI_RES;
    const int g = lane >> 4;
    const int ncol = 16 * (g & 1) + 4 * (g & ~1);         // lane's column within a 32-column pair block
    const int nl = n_w + ncol;                            // + 32 p
    const int r = lane & 15;                              // + 16 i
    // buffer resources rebased on the wave's first row, num_records = the bytes of its rows < M:
    // one voffset per lane plus the row step i (vadd_opq) and the column block p (no 64-bit address
    // per access); rows past M read as 0 and their stores are dropped by the range check
    const int rows = max(0, min(128, M - m_w));
    // (num_records through readfirstlane: the compiler formed the clamp with its 128 in a VGPR and
    // then wrapped every access in a waterfall loop)
    auto rsrc = [&](const bf16_t* base, long long ld, bool load) {
        return __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(base + (long long)m_w * ld), 0,
                                                 load ? __builtin_amdgcn_readfirstlane((int)((long long)rows * ld * 2))
                                                      : 0x7fffffff, 0x00020000);
    };
    const __amdgpu_buffer_rsrc_t rc = rsrc(C, ldc, true);
    const int vo_c = (int)((r * ldc + n_w + ncol) * 2);
    // bias unpacked once per tile (the per-row unpack was 8 of the ~95 VALU per 16-B store)
    float bvf[W4_EPI_CBLK][8];
#pragma unroll
    for (int p = 0; p < W4_EPI_CBLK; ++p)
        unpack8(ep.bias ? ld16(ep.bias + min(nl + 32 * p, N - 8)) : u32x4_t{0, 0, 0, 0}, bvf[p]);
    u32x4_t gw0[4], gw1[4];
    int b_lo = 0;
    if constexpr (MODE == VS_EPI_GATE_RES) {
        b_lo = min(m_w, M - 1) / ep.rows_per_batch;
        const int b_hi = min(m_w + 127, M - 1) / ep.rows_per_batch;
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const int n = min(nl + 32 * p, N - 8);
            gw0[p] = ld16(ep.gate + (long long)b_lo * ep.gate_bstride + n);
            gw1[p] = ld16(ep.gate + (long long)b_hi * ep.gate_bstride + n);
        }
    }
    // (resources of absent operands point at C with an empty range: never read)
    const __amdgpu_buffer_rsrc_t rr = RESID ? rsrc(ep.res, ep.ld_res, true) : rsrc(C, ldc, false);
    const __amdgpu_buffer_rsrc_t rh = HINT ? rsrc(ep.hint, ep.ld_hint, true) : rsrc(C, ldc, false);
    const int vo_r = RESID ? (int)((r * ep.ld_res + n_w + ncol) * 2) : 0;
    const int vo_h = HINT ? (int)((r * ep.ld_hint + n_w + ncol) * 2) : 0;
    // rows of residual / hint loads in flight (1 for the fp8 hint instantiation: its registers)
    constexpr int DEPTH = (HINT && SCALED) ? 1 : (HINT || SCALED) ? W4_EPI_DEPTH : W4_EPI_DEPTH_BF16;
    u32x4_t rs[DEPTH][4], hs[DEPTH][4];
    auto load_rows = [&](auto ic, u32x4_t (&r_)[4], u32x4_t (&h_)[4]) __attribute__((always_inline)) {
        constexpr int i = decltype(ic)::value;
#pragma unroll
        for (int p = 0; p < W4_EPI_CBLK; ++p) {
            r_[p] = __builtin_amdgcn_raw_buffer_load_b128(rr, vadd_opq(vo_r, (int)(16 * i * ep.ld_res * 2)) + 64 * p, 0, W4_RES_CPOL);
            if constexpr (HINT) h_[p] = __builtin_amdgcn_raw_buffer_load_b128(rh, vadd_opq(vo_h, (int)(16 * i * ep.ld_hint * 2)) + 64 * p, 0, 0);
        }
    };
    if constexpr (RESID) {
        static_for<DEPTH>([&](auto ic) __attribute__((always_inline)) {
            constexpr int i = decltype(ic)::value;
            load_rows(ic, rs[i], hs[i]);
        });
    }
    static_for<W4_EPI_ROWS>([&](auto ic) __attribute__((always_inline)) {
        constexpr int i = decltype(ic)::value;
        const int m = m_w + r + 16 * i;
        float sa = 1.f;
        if constexpr (SCALED) sa = scale_a[min(m, M - 1)];
#pragma unroll
        for (int p = 0; p < W4_EPI_CBLK; ++p) {
            float y[8];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float x = acc_rd(acc[i][2 * p][e]), z = acc_rd(acc[i][2 * p + 1][e]);
                const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(z), false, false);
                y[e] = __uint_as_float(sw[0]);
                y[4 + e] = __uint_as_float(sw[1]);
            }
            // pair arithmetic (output pair j = y[2j], y[2j+1] = word j of the 16-B store): packed
            // f32 adds / muls, every bf16 rounding point one v_cvt_pk_bf16_f32 of a pair plus its
            // unpack (rbf2); a value rounded only for the store is left to the store's pack (RNE is
            // idempotent: pack2(rbf(v)) == pack2(v) bit for bit) -- the plain-bias output and the
            // un-hinted gate-residual sum.  Same operations and rounding points as epilogue_store_w.
            f32x2_t y2[4];
            uint32_t wo[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                f32x2_t v = f32x2_t{y[2 * j], y[2 * j + 1]};
                if constexpr (SCALED) v = v * sa;
                v = v + f32x2_t{bvf[p][2 * j], bvf[p][2 * j + 1]};
                y2[j] = v;
            }
            if constexpr (MODE == VS_EPI_GELU || MODE == VS_EPI_SILU) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const f32x2_t v = rbf2(y2[j]);
                    wo[j] = MODE == VS_EPI_GELU ? pk_store(gelu_tanh_f(v.x), gelu_tanh_f(v.y))
                                                : pk_store(silu_f(v.x), silu_f(v.y));
                }
            } else if constexpr (MODE == VS_EPI_GATE_RES) {
                const bool hi = m / ep.rows_per_batch != b_lo;
                const u32x4_t gsel = hi ? gw1[p] : gw0[p];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    f32x2_t v = unpk2(rs[i % DEPTH][p][j]) + rbf2(unpk2(gsel[j]) * rbf2(y2[j]));
                    if constexpr (HINT) v = rbf2(v) + rbf2(unpk2(hs[i % DEPTH][p][j]) * ep.hint_scale);
                    wo[j] = pk_store(v.x, v.y);
                }
            } else if constexpr (MODE == VS_EPI_RES) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const f32x2_t v = unpk2(rs[i % DEPTH][p][j]) + rbf2(ep.alpha * rbf2(y2[j]));
                    wo[j] = pk_store(v.x, v.y);
                }
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j) wo[j] = pk_store(y2[j].x, y2[j].y);
            }
            // rows past M fall outside rc's range, columns past N get an offset outside it: the
            // hardware drops those stores (no per-store branch)
            const int so = vadd_opq(vo_c, (int)(16 * i * ldc * 2)) + 64 * p;
            __builtin_amdgcn_raw_buffer_store_b128(u32x4_t{wo[0], wo[1], wo[2], wo[3]}, rc,
                                                   nl + 32 * p < N ? so : 0x7ffffff0, 0, W4_OUT_CPOL);
            // one column block at a time: the scheduler would otherwise hoist the accumulator reads
            // of later blocks (AGPR -> VGPR copies) and run out of VGPRs
            __builtin_amdgcn_sched_barrier(0);
        }
        if constexpr (RESID && i + DEPTH < W4_EPI_ROWS) load_rows(std::integral_constant<int, i + DEPTH>{}, rs[i % DEPTH], hs[i % DEPTH]);
    });
}

constexpr int W4_ROWB = 1056;                 // LDS row: 8 global rows x 128 B + 32 B pad
constexpr int W4_OPB = 32 * W4_ROWB;          // one operand's K-tile image (256 rows x 64 k)
constexpr int W4_LDS = 4 * W4_OPB;            // [A b0][A b1][W b0][W b1] = 135168 B
static_assert(4 * W4_ROWB == 0x1080, "the 4w kernel's M0 step");

// ---------------------------------------------------------------------------------------------
// Tile schedule of the 4-wave kernels (r5): persistent workgroups fed by XCD-local tile queues.
//
// Blocks [0, npers) are persistent (one per CU): block b sits on XCD x = b % 8 (round-robin
// dispatch) in slot s = b / 8 and computes tiles of its XCD's contiguous id range [x R, (x+1) R),
// R = G8 tp (G8 = npers / 8), as ONE stream of K-tiles: the DMA runs two K-tiles ahead straight
// across tile boundaries, so a tile's first K-tiles land during the previous tile's last K-tiles
// and its epilogue.  A block takes every tile from its XCD's queue (head word q[x]: range positions
// t = 0, 1, ..), then, once that has run dry, from the other XCDs' queues (probed in ring order),
// then from the remainder pool (the nrem whole tiles past npers tp, head q[8]).  A block that starts
// late -- its CU held by another kernel, e.g. RCCL under the Ulysses overlap -- finds the queues
// drained and exits (r5 measured a fixed first tile per block: the held blocks' first tiles then
// ran after the hog, +19 % on an SP = 8 FFN-down with 8-32 CUs held, profiles/r5/cu_hold_s4.log).
//   r4 walked a static list (positions s, s + G8, s + 2 G8, ..).  Over a 54-tile list an XCD's CUs
//   drifted apart, so the 32 tiles in flight on an XCD stopped being one 4 x 8 block sharing its A / W
//   slices in L2 (FFN-up: 23.1 GB of fabric reads per dispatch against the library's 13.1,
//   profiles/r4/pmc_fetch_rows.txt), and a CU held by a concurrent kernel (RCCL under the Ulysses
//   overlap) delayed its whole list.  With the queue the tiles computing on an XCD are always about
//   the 32 most recently taken ids, and a CU that is slow or held simply takes fewer.
// The first tile costs one atomic round trip before the prologue; after that the next tile id is
// known one tile ahead: wave 0 takes it during tile k's epilogue (its atomic issued at the
// epilogue's start and its value used at the end, under the stores) -- the second tile's under the
// prologue's DMAs -- writes it to an LDS word, and every wave reads that word in tile k+1's first
// K-tile behind a barrier, before the DMA cursor crosses into tile k+2 at the end of K-tile nt - 3
// (nt >= 3, host-checked).  The last
// persistent block to finish (exit count q[9]) zeroes the queue words, so every launch finds them
// zero (workspace kind 5: bound zeroed, one per stream, so graph replays and concurrent streams are
// safe).  Without a bound queue the same walk runs the static list and the nrem whole tiles get
// blocks of their own.  The blocks after those run the split-tail K pieces of the last tiles.
// ---------------------------------------------------------------------------------------------
constexpr int WQ_LINE = VS_Q_LINE;            // queue words 128 B apart (a line each, common.h)
constexpr int WQ_BYTES = 11 * WQ_LINE * 4;    // 8 XCD heads, the remainder head, the piece head, the exit count
struct W4Sched {
    unsigned* q;      // queue words (null: static lists)
    int npers;        // persistent blocks (a multiple of 8, or 0)
    int tp;           // tiles per slot of an XCD range
    int nrem;         // whole tiles past npers * tp
    int npiece;       // split-tail pieces taken from the piece pool q[9] by the persistent blocks (r6;
                      // 0: the pieces run as blocks of their own after the persistent ones)
};
struct W4Work {
    int first, second;  // the block's first two tile ids (-1: none)
    int piece;          // split-tail piece (-1: whole tiles)
    int kb, nt;         // K offset (elements) and K-tiles per tile
};
__device__ __forceinline__ W4Work w4_work(const W4Sched& sc, int K, int nmain, int ksplit, int piece_k, int kstep) {
    W4Work w;
    const int b = blockIdx.x;
    w.piece = -1;
    w.kb = 0;
    w.nt = K / kstep;
    w.second = -1;
    const int nstat = sc.q ? 0 : sc.nrem;          // remainder tiles with blocks of their own
    if (b < sc.npers) {
        const int g8 = sc.npers >> 3, base = (b & 7) * g8 * sc.tp, s = b >> 3;
        w.first = base + s;
        if (sc.tp >= 2) w.second = base + g8 + s;
    } else if (b < sc.npers + nstat) {
        w.first = sc.npers * sc.tp + (b - sc.npers);
    } else {
        const int t = b - sc.npers - nstat;
        w.first = nmain + t / ksplit;
        w.piece = t % ksplit;
        w.kb = w.piece * piece_k;
        w.nt = min(K - w.kb, piece_k) / kstep;
    }
    return w;
}
__device__ __forceinline__ unsigned wq_add(unsigned* p) { return vs_queue_add(p); }
// The tile taking of one persistent block (wave 0; see the schedule above).  issue(): the atomic on
// the XCD's head, lane 0 only, at the start of an epilogue; finish<W>(): the tile id (-1: none
// left), wave-uniform, at its end.  The head atomic is inline asm that sets EXEC to lane 0 itself:
// as a compiler-visible atomic, the compiler's wait before its value is used was a vmcnt(0) (it
// cannot count across the epilogue's branches), i.e. the epilogue's stores drained before the next
// tile -- the per-tile wait r4 removed (gemm_drain_ab.log) -- and its atomic optimizer consumed the
// value right after the atomic (Makefile).  finish<W>() waits vmcnt(W) instead: VMEM operations
// complete in issue order and the caller has issued >= W of them since issue() (the epilogue's),
// so the atomic has returned.  The steal / remainder atomics are ordinary ones (rare: once the own
// queue has run dry).
struct W4Grab {
    const W4Sched& sc;
    int k = 2;                  // static list: position of the next tile
    bool local = true;          // the XCD's own queue may still hold tiles
    bool steal = true;          // another XCD's queue may
    bool rem_dry = false;       // the remainder pool has run dry
    unsigned t0 = 0;
    __device__ __forceinline__ explicit W4Grab(const W4Sched& s) : sc(s) {}
    __device__ __forceinline__ void issue() {
        if (sc.q && local) t0 = vs_queue_issue(sc.q + (blockIdx.x & 7) * WQ_LINE);
    }
    template <int W>
    __device__ __forceinline__ int finish(int lane) {
        const int g8 = sc.npers >> 3, x = blockIdx.x & 7;
        if (!sc.q) {
            const int id = k < sc.tp ? x * g8 * sc.tp + k * g8 + (blockIdx.x >> 3) : -1;
            ++k;
            return id;
        }
        const unsigned qlen = (unsigned)(g8 * sc.tp);
        if (local) {
            const unsigned t = vs_queue_value<W>(t0);
            if (t < qlen) return x * g8 * sc.tp + (int)t;
            local = false;
        }
        // other XCDs' queues: lanes 0-6 probe heads x+1 .. x+7, the first live one in ring order is
        // taken from (a lost race just probes again; heads only grow, so this ends)
        for (int it = 0; steal && it < 16; ++it) {
            unsigned h = qlen;
            if (lane < 7) h = __hip_atomic_load(sc.q + ((x + 1 + lane) & 7) * WQ_LINE, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
            const unsigned long long live = __ballot(lane < 7 && h < qlen);
            if (!live) {
                steal = false;
                break;
            }
            const int v = (x + 1 + (int)__builtin_ctzll(live)) & 7;
            unsigned t = 0;
            if (lane == 0) t = wq_add(sc.q + v * WQ_LINE);
            t = (unsigned)__builtin_amdgcn_readfirstlane((int)t);
            if (t < qlen) return v * g8 * sc.tp + (int)t;
        }
        steal = false;
        if (sc.nrem > 0 && !rem_dry) {
            unsigned u = 0;
            if (lane == 0) u = wq_add(sc.q + 8 * WQ_LINE);
            u = (unsigned)__builtin_amdgcn_readfirstlane((int)u);
            if (u < (unsigned)sc.nrem) return sc.npers * sc.tp + (int)u;
            rem_dry = true;
        }
        // then the split-tail pieces (work ids nmain + p, see w4_item), so they run on the CUs that
        // finish their whole tiles first instead of as blocks dispatched behind the persistent ones
        if (sc.npiece > 0) {
            unsigned u = 0;
            if (lane == 0) u = wq_add(sc.q + 9 * WQ_LINE);
            u = (unsigned)__builtin_amdgcn_readfirstlane((int)u);
            if (u < (unsigned)sc.npiece) return sc.npers * sc.tp + sc.nrem + (int)u;
        }
        return -1;
    }
    // after the block's last tile: the last persistent block to finish (exit count q[10]) zeroes the
    // queue words
    __device__ __forceinline__ void done(int tid) {
        if (sc.q && (int)blockIdx.x < sc.npers && tid == 0) vs_queue_done(sc.q, 11, sc.npers);
    }
};

// the DMA issued before MFMA q of a K-tile of gemm_bf16_tn_4w (-1: none): W instructions 0-7 as
// d = 0-7, A instructions 0-7 as d = 8-15 (the library kernel's placement, see the body)
constexpr int w4_dma_at(int q) {
    return (q >= 21 && q <= 37 && (q - 21) % 4 == 0) ? (q - 21) / 4
         : (q == 53 || q == 56 || q == 59)             ? 5 + (q - 53) / 3
         : q == 62                                     ? 8
         : q == 65                                     ? 9
         : (q >= 86 && q <= 98 && (q - 86) % 3 == 0)   ? 10 + (q - 86) / 3
         : q == 122                                    ? 15
                                                       : -1;
}

template <int MODE, bool HINT>
__global__ __launch_bounds__(256, 1) void gemm_bf16_tn_4w(
    const bf16_t* __restrict__ A, long long lda, const bf16_t* __restrict__ W, long long ldw,
    bf16_t* C, long long ldc, int M, int N, int K, Epi ep, int ntm, int ntn, int nmain, int ksplit,
    int piece_k, float* __restrict__ part, W4Sched sc) {
#if defined(__HIP_DEVICE_COMPILE__)     // (the AGPR asm operands are not host constraints)
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const W4Work wk = w4_work(sc, K, nmain, ksplit, piece_k, 64);
    // work ids (r6): id < nmain a whole tile, id >= nmain split-tail piece p = id - nmain (tile
    // nmain + p / ksplit, K range p % ksplit) -- a persistent block takes pieces from the queue's
    // piece pool after the whole tiles (W4Grab), a piece block of its own starts with its piece's id
    const int kt_all = K / 64;
    auto nt_of = [&](int id) {
        return id < nmain ? kt_all : min(K - ((id - nmain) % ksplit) * piece_k, piece_k) / 64;
    };

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 1, wn = wave & 1;

    f32x4_t acc[8][8];

    // DMA: instruction j of wave w fills LDS row 4j + w of an operand image; lane L lands in column
    // block L / 8, chunk L % 8 = global row 128 (rho / 16) + 16 (L / 8) + rho % 16, bytes 16 (L % 8)..
    // i.e. instruction j's rows are those of instruction 0 plus 4j (+112 from j = 4).  As in the
    // library's kernel, a DMA is ONE instruction: the 16 per-lane row offsets are formed once (tile-
    // invariant: the resources are rebased on the tile), the K-tile offset is folded into the
    // resource base (advanced per K-tile, num_records shrunk with it), and M0 (the LDS destination)
    // is written in the MFMA gap before the load -- no address VALU and no s_nop per DMA (r4: the
    // per-DMA v_add + hazard nop were 2 of the 4 instructions of every DMA group).  Rows past the
    // matrix fall outside the resource's range and load 0; their outputs are discarded.  The DMA
    // cursor (K-tile dkt of the tile it is in) runs two K-tiles ahead of the compute; past the
    // block's last K-tile it re-reads that K-tile (into the buffer no later read uses), which keeps
    // every iteration's wait counts identical.  The DMAs are inline asm, invisible to the compiler's
    // wait counting (its own waits only grow stricter with older loads in flight); the protocol
    // waits are the hand-placed vmcnt below (EPI_OPS: the epilogue's stores drain under the next
    // tile's first K-tile) and the vmcnt(0) after the block's last tile.
    const unsigned ldab = (unsigned)(lda * 2), ldwb = (unsigned)(ldw * 2);
    auto rsrc4 = [](const char* base, int bytes) {      // (readfirstlane: an "s" operand)
        const unsigned long long a = (unsigned long long)(uintptr_t)base;
        return i32x4_t{__builtin_amdgcn_readfirstlane((int)(unsigned)a),
                       __builtin_amdgcn_readfirstlane((int)((unsigned)(a >> 32) & 0xffffu)),
                       __builtin_amdgcn_readfirstlane(bytes), 0x00020000};
    };
    auto rows_bytes = [](int rows, unsigned ldb) {
        return (int)((long long)max(0, min(rows, 256)) * (long long)ldb);
    };
    auto jrow = [](int j) { return 4 * j + (j >= 4 ? 112 : 0); };
    const unsigned grow0 = (unsigned)(16 * (lane >> 3) + wave);     // row of instruction 0
    unsigned voa[8], vow[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        voa[j] = (grow0 + (unsigned)jrow(j)) * ldab + 16u * (lane & 7);
        vow[j] = (grow0 + (unsigned)jrow(j)) * ldwb + 16u * (lane & 7);
        asm volatile("" : "+v"(voa[j]), "+v"(vow[j]));     // kept, not re-formed per use
    }
    const char* abp = nullptr;
    const char* wbp = nullptr;
    int arec = 0, wrec = 0;
    int dnt = 0;                    // K-tiles of the work the DMA cursor is in
    auto dma_tile = [&](int id) {
        int tm, tn, tile = id, kb = 0;
        if (id >= nmain) {
            const int p = id - nmain;
            tile = nmain + p / ksplit;
            kb = (p % ksplit) * piece_k;
        }
        dnt = nt_of(id);
        tile_of(tile, ntm, ntn, ep.gm, tm, tn);
        const int m0 = tm * 256, n0 = tn * 256;
        abp = (const char*)(A + (long long)m0 * lda + kb);
        wbp = (const char*)(W + (long long)n0 * ldw + kb);
        arec = __builtin_amdgcn_readfirstlane(rows_bytes(M - m0, ldab));
        wrec = __builtin_amdgcn_readfirstlane(rows_bytes(N - n0, ldwb));
    };
    // tiles: cur (computing), nxt (the next one, read from the LDS word in cur's first K-tile) and
    // dnext (where the DMA cursor goes when it leaves cur; -1: re-read)
    int cur = wk.piece >= 0 ? nmain + (wk.first - nmain) * ksplit + wk.piece : wk.first;
    int nxt = wk.second, dnext = wk.second;
    int dkt = 0;
    auto dma_advance = [&]() {
        if (++dkt == dnt) {
            if (dnext >= 0) {
                dkt = 0;
                dma_tile(dnext);
                dnext = -1;
            } else {
                dkt = dnt - 1;
            }
        }
    };
    W4Grab grab(sc);
    const unsigned slot = (unsigned)(uintptr_t)smem + W4_LDS;     // the next tile id (LDS word)
    auto slot_ref = [&]() -> volatile LDS_AS int& { return *(volatile LDS_AS int*)(uintptr_t)slot; };
    int slotv = 0;
    // LDS-DMA destinations (wave-uniform byte offsets of the wave's first row in the current
    // buffer) and the per-lane fragment bases; both toggle between the two buffers by XOR once per
    // K-tile, so the loop body is one instance with immediate ds_read offsets
    unsigned dw = 2 * W4_OPB + wave * W4_ROWB, da = wave * W4_ROWB;
    const unsigned dw_tog = dw ^ (dw + W4_OPB), da_tog = da ^ (da + W4_OPB);
    const unsigned lds0 = (unsigned)(uintptr_t)smem;
    i32x4_t rsa, rsw;                   // the current K-tile's resources (set at each DMA K-tile)
    auto ktile_rsrc = [&](unsigned ko) {
        rsa = rsrc4(abp + ko, arec - (int)ko);
        rsw = rsrc4(wbp + ko, wrec - (int)ko);
    };
    // DMA d of a K-tile: d < 8 W instruction d, else A instruction d - 8
    auto dma_lds = [&](int d) { return lds0 + (d < 8 ? dw + 4 * d * W4_ROWB : da + 4 * (d - 8) * W4_ROWB); };
    // M0: set at an operand's first instruction, then stepped by one 4-row group (4 x 1056 B) --
    // one SALU per DMA, as the library's kernel (nothing between these statements writes M0).
    // m0_step_note: the step declares no "m0" clobber -- with it the hazard recognizer put an
    // s_nop before every step that follows an MFMA (the library's kernel steps M0 right after
    // MFMAs with no nop); the compiler is told of the M0 write by the s_mov that starts each run,
    // and nothing in this kernel reads M0 but these DMAs
    auto m0_set = [&](int d) {
        if (d == 0 || d == 8) asm volatile("s_mov_b32 m0, %0" :: "s"(dma_lds(d)) : "m0");
        else asm volatile("s_add_u32 m0, m0, 0x1080" ::: "memory");   // (see m0_step_note)
    };
    auto dma_go = [&](int d) {
#ifdef VS_W4_DIAG_NODMA     // diagnostic build only (scripts/build_diag.sh): no operand DMA, garbage results
        (void)d;
#else
        if (d < 8) asm volatile("buffer_load_dwordx4 %0, %1, 0 offen lds" :: "v"(vow[d]), "s"(rsw) : "memory");
        else asm volatile("buffer_load_dwordx4 %0, %1, 0 offen lds" :: "v"(voa[d - 8]), "s"(rsa) : "memory");
#endif
    };
    auto dma_now = [&](int d) {                     // outside the pipelined body: M0, nop, load
        asm volatile("s_mov_b32 m0, %0" :: "s"(dma_lds(d)) : "m0");
        asm volatile("s_nop 0" ::: "memory");
        dma_go(d);
    };

    // fragment bases (lane: row l % 16 of the wave's LDS rows, 16-B chunk l / 16), kept opaque so
    // every read is base + immediate
    int abase = (int)(uintptr_t)smem + (wm * 16 + (lane & 15)) * W4_ROWB + 16 * (lane >> 4);
    int wbase = (int)(uintptr_t)smem + 2 * W4_OPB + (wn * 16 + (lane & 15)) * W4_ROWB + 16 * (lane >> 4);
    int atog = abase ^ (abase + W4_OPB), wtog = wbase ^ (wbase + W4_OPB);
    asm volatile("" : "+v"(abase), "+v"(wbase), "+v"(atog), "+v"(wtog));
    auto frag = [&](int addr) {
#ifdef VS_W4_DIAG_NOREAD    // diagnostic build only: no fragment reads (the MFMAs see constant operands)
        return bf16x8_t{(__bf16)(float)(addr & 1), 0, 0, 0, 0, 0, 0, 0};
#else
        return *reinterpret_cast<const LDS_AS bf16x8_t*>((const LDS_AS char*)(uintptr_t)(unsigned)addr);
#endif
    };
    bf16x8_t fa0[8], fa1[8], fw0[8], fw1[8];
    auto fence = [&]() { __builtin_amdgcn_sched_barrier(0); };
    auto bar = [&]() {
        fence();
        asm volatile("s_barrier" ::: "memory");
        fence();
    };
    auto wait_lgkm_bar = [&]() {
        fence();
        __builtin_amdgcn_s_waitcnt(0xC07F);     // lgkmcnt(0), visible to the compiler's wait-count pass
        asm volatile("s_barrier" ::: "memory");
        fence();
    };
    auto read_k0 = [&]() {
#pragma unroll
        for (int j = 0; j < 8; ++j) fw0[j] = frag(wbase + 128 * j);
#pragma unroll
        for (int i = 0; i < 8; ++i) fa0[i] = frag(abase + 128 * i);
        fence();
    };

    // The counted waits of a tile's first K-tile after an epilogue.  VMEM operations complete in
    // issue order (loads, stores and LDS-DMA alike), and the epilogue's >= EPI_OPS loads / stores
    // were issued after the 16 DMAs it waits on, so while any of those is pending at least EPI_OPS
    // more are: the wait counts grow by EPI_OPS (capped at the counter's 63) and the epilogue's
    // stores drain under the next tile's first K-tile instead of before it (r3-r4: a vmcnt(0)
    // after every epilogue; dropping every store in a diagnostic build was worth +3.8 %, 
    // gemm_epidiag_ab.log).  EPI_OPS = the fewest VMEM operations any epilogue path of this
    // instantiation issues: 32 16-B stores, + 32 residual loads (the split-K piece path: 64 stores).
    constexpr int EPI_OPS = (MODE == VS_EPI_GATE_RES || MODE == VS_EPI_RES) ? 64 : 32;
    static_assert(EPI_OPS <= w4_epi_min_vmem(MODE), "the epilogue issues fewer VMEM operations than the drain counts");
    // prologue: K-tiles 0 and 1 of the stream in flight (W then A each), then the k-step-0 fragments
    const bool dyn = sc.q && (int)blockIdx.x < sc.npers;    // a persistent block fed by the queues
    if (dyn) {              // the first tile from the queues too (a block that starts late: none left)
        if (wave == 0) {
            grab.issue();
            const int id = grab.finish<0>(lane);
            if (lane == 0) slot_ref() = id;
        }
        __syncthreads();
        cur = __builtin_amdgcn_readfirstlane(slot_ref());
        if (cur < 0) {
            grab.done(tid);
            return;
        }
    }
    dma_tile(cur);
    ktile_rsrc(0);
    if (dyn && wave == 0) grab.issue();                       // the second tile, under the prologue
#pragma unroll
    for (int d = 0; d < 16; ++d) dma_now(d);
    dma_advance();
    dw ^= dw_tog;
    da ^= da_tog;
    ktile_rsrc((unsigned)dkt * 128u);
#pragma unroll
    for (int d = 0; d < 16; ++d) dma_now(d);
    dma_advance();
    dw ^= dw_tog;
    da ^= da_tog;
    fence();
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    bar();
    read_k0();
    if (wave == 0) {        // the second tile into the LDS word (read in the first tile's first K-tile)
        const int id = dyn ? grab.finish<32>(lane) : wk.second;     // (the 32 prologue DMAs since issue)
        if (lane == 0) slot_ref() = id;
    }
    // the first tile's first K-tile counts EPI_OPS operations behind K-tile 1's DMAs as every later
    // tile's does: as many stores the buffer range check drops (offset past num_records 0)
    {
        const i32x4_t rz = rsrc4((const char*)C, 0);
        const int vz = 0;
#pragma unroll
        for (int d = 0; d < EPI_OPS; ++d)
            asm volatile("buffer_store_dword %0, %0, %1, 0 offen" :: "v"(vz), "s"(rz) : "memory");
    }

    // one K-tile: 128 MFMAs with, before MFMA q, the reads / DMA / barriers of this table.  FIRST:
    // the tile's first K-tile, whose k-step-0 MFMAs start the accumulators from 0 (no zeroing pass,
    // and no accumulator value live across the tile loop: the register allocator otherwise copied
    // and spilled the 256 accumulators around the epilogue)
    auto ktile = [&](auto firstc) __attribute__((always_inline)) {
            constexpr bool FIRST = decltype(firstc)::value;
            constexpr int W69 = FIRST ? (18 + EPI_OPS < 63 ? 18 + EPI_OPS : 63) : 18;
            constexpr int W101 = FIRST ? (15 + EPI_OPS < 63 ? 15 + EPI_OPS : 63) : 15;
            ktile_rsrc((unsigned)dkt * 128u);
            static_for<128>([&](auto qc) __attribute__((always_inline)) {
                constexpr int q = decltype(qc)::value;
                if constexpr (q < 16 && (q & 1)) fw1[q >> 1] = frag(wbase + 128 * (q >> 1) + 64);
                if constexpr (q == 17) wbase ^= wtog;                          // next buffer's W fragments
                if constexpr (q == 20) wait_lgkm_bar();                        // W region of this buffer free
                if constexpr (FIRST && q == 21) slotv = slot_ref();           // the next tile (behind q 20)
                if constexpr (q >= 23 && q <= 39 && (q - 23) % 4 == 0) fa1[(q - 23) / 4] = frag(abase + 128 * ((q - 23) / 4) + 64);
                if constexpr (q >= 41 && q <= 45 && (q & 1)) fa1[5 + (q - 41) / 2] = frag(abase + 128 * (5 + (q - 41) / 2) + 64);
                if constexpr (q == 47) abase ^= atog;
                if constexpr (q == 52) wait_lgkm_bar();                        // A region of this buffer free
                if constexpr (FIRST && q == 53) {
                    nxt = __builtin_amdgcn_readfirstlane(slotv);
                    dnext = nxt;
                }
                if constexpr (q == 69) {                                       // W of the next K-tile landed
                    fence();
                    asm volatile("s_waitcnt vmcnt(%0)" :: "n"(W69) : "memory");
                    bar();
                }
                if constexpr (q >= 70 && q <= 84 && !(q & 1)) fw0[(q - 70) / 2] = frag(wbase + 128 * ((q - 70) / 2));
                if constexpr (q == 101) {                                      // A of the next K-tile landed
                    fence();
                    asm volatile("s_waitcnt vmcnt(%0)" :: "n"(W101) : "memory");
                    bar();
                }
                if constexpr (q >= 102 && q <= 116 && !(q & 1)) fa0[(q - 102) / 2] = frag(abase + 128 * ((q - 102) / 2));
                // the 16 DMAs of K-tile t+2 (W 0-4 every 4 MFMAs from 21 after the W-free barrier, W 5-7
                // and A 0-1 after the A-free barrier, A 2-6 between the landing waits, A 7 last), each
                // with its M0 written one MFMA earlier
                if constexpr (w4_dma_at(q) >= 0) dma_go(w4_dma_at(q));
                if constexpr (w4_dma_at(q + 1) >= 0) m0_set(w4_dma_at(q + 1));
                // MFMA q: k-step q / 64, tile (i, j) = ((q % 64) / 8, q % 8).  Inline asm with the
                // accumulator tied in place: the 256 accumulators then fill the AGPR file exactly (the
                // builtin let the register allocator rename them per MFMA: AGPR copies and spills)
                constexpr int i = (q & 63) >> 3, j = q & 7;
                if constexpr (q < 64 && FIRST)
                    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(acc[i][j]) : "v"(fw0[j]), "v"(fa0[i]));
                else if constexpr (q < 64)
                    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[i][j]) : "v"(fw0[j]), "v"(fa0[i]));
                else
                    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[i][j]) : "v"(fw1[j]), "v"(fa1[i]));
                fence();
            });
            dw ^= dw_tog;
            da ^= da_tog;
            dma_advance();
    };

#pragma nounroll
    for (;;) {
        const int nt = nt_of(cur);
        ktile(std::true_type{});
#pragma nounroll
        for (int t = 1; t < nt; ++t) ktile(std::false_type{});
        // the accumulators leave through v_accvgpr_read: cover the last MFMAs' write latency by hand
        // (the hazard recognizer does not see into the asm statements)
        asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");

        int tm, tn;
        const int cur_tile = cur < nmain ? cur : nmain + (cur - nmain) / ksplit;
        tile_of(cur_tile, ntm, ntn, ep.gm, tm, tn);
        const int m0 = tm * 256, n0 = tn * 256;
        // the tile after nxt: wave 0's queue atomic goes out under this epilogue
        if (nxt >= 0 && wave == 0) grab.issue();
        // output: acc[i][j][e] = C[m][n], m = m0 + 128 wm + 16 i + (lane & 15), n = n0 + 128 wn + 16 j + 4 (lane >> 4) + e
        if (cur >= nmain) {
            // fp32 partial tile through one buffer resource: a per-lane offset, the row block i in
            // soffset and the column block j in the immediate (64 precomputed 64-bit addresses,
            // hoisted out of the tile loop by the compiler, were spilled)
            const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(
                part + (long long)(cur - nmain) * 256 * 256, 0, 256 * 256 * 4, 0x00020000);
            const int vo = ((128 * wm + (lane & 15)) * 256 + 128 * wn + 4 * (lane >> 4)) * 4;
#pragma unroll
            for (int i = 0; i < 8; ++i)
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    __builtin_amdgcn_raw_buffer_store_b128(
                        u32x4_t{__float_as_uint(acc_rd(acc[i][j][0])), __float_as_uint(acc_rd(acc[i][j][1])),
                                __float_as_uint(acc_rd(acc[i][j][2])), __float_as_uint(acc_rd(acc[i][j][3]))},
                        rp, vo, 16 * i * 256 * 4 + 64 * j, 0);
        } else {
            // 16-B epilogue (host-checked alignment): column blocks (2p, 2p+1) traded between lane
            // groups g, g^1 (permlane16_swap): an even-g lane ends with columns 32p + 4g .. +7, an
            // odd-g lane with 32p + 16 + 4(g-1) .. +7; loads issued ahead (tile_epilogue_w4).  One
            // epilogue mode per kernel instantiation (the runtime switch's six bodies beside the
            // 256 live accumulators overflowed the register file)
            tile_epilogue_w4<MODE, HINT, false>(acc, m0 + 128 * wm, n0 + 128 * wn, lane, C, ldc, M, N, ep, nullptr);
        }
        if (nxt < 0) break;
        // the id of the tile after nxt into the LDS word (read in nxt's first K-tile, behind its
        // q = 20 barrier; the readers of the previous id passed this K-tile's q = 52 barrier long ago)
        if (wave == 0) {
            const int id = grab.finish<(EPI_OPS < 63 ? EPI_OPS : 63)>(lane);   // (>= EPI_OPS issued since)
            if (lane == 0) slot_ref() = id;
        }
        cur = nxt;
        // the next tile's k-step-0 fragments (its first K-tile has landed); the epilogue's stores stay
        // in flight (EPI_OPS above)
        read_k0();
    }
    // after the last tile everything drains, the re-read DMAs into LDS included, before the
    // workgroup's LDS is released
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    grab.done(tid);
#endif
}



// ---------------------------------------------------------------------------------------------
// gemm_fp8_tn_8p: the 8-phase skeleton of gemm_bf16_tn_8p for the fp8 path (config 5;
// AutoWrappedLinear.fp8_linear, diffsynth/vram_management/layers.py:115-151):
// C = epilogue(scale_a[m] * (A8 . W8^T)), e4m3 (OCP) operands, activations quantised per row by
// vs_quant_fp8_rows, unscaled weights.  A K-tile is 128 fp8 = the same 128-B LDS rows, half-tiles,
// DMA pieces and phase schedule as the bf16 kernel; per phase a wave runs 4 MX-rate
// v_mfma_scale_f32_32x32x64_f8f6f4 (unit E8M0 scales; two 64-deep k-steps x two 32-row m-tiles
// x one 32-column n-tile) = twice the bf16 FLOPs in the same MFMA cycles.  Fragment (32x32x64 map,
// as the r2 kernel): lane l holds row l & 31, k = 32 (l >> 5) .. +31 of the k-step, i.e. 16-B chunks
// 4s + 2(l >> 5) + {0, 1}; chunk swizzle c ^ ((row & 7) ^ ((row >> 3) & 1)) makes these reads
// conflict-free (the bf16 kernel's c ^ (row & 7) would be 2-way here).
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ int q8_off(int row, int ch) {
    return row * 128 + 16 * (ch ^ (row & 7) ^ ((row >> 3) & 1));
}

__global__ __launch_bounds__(512, 2) void gemm_fp8_tn_8p(
    const uint8_t* __restrict__ A, long long lda, const float* __restrict__ scale_a, const uint8_t* __restrict__ W,
    long long ldw, bf16_t* C, long long ldc, int M, int N, int K, Epi ep, int ntm, int ntn, int nmain, int ksplit,
    int piece_k, float* __restrict__ part) {
    extern __shared__ __attribute__((aligned(16))) char smem[];

    int pid, piece = -1;
    if ((int)blockIdx.x < nmain) {
        pid = xcd_remap(blockIdx.x, nmain);
    } else {
        const int t = blockIdx.x - nmain;
        pid = nmain + t / ksplit;
        piece = t % ksplit;
    }
    int tm, tn;
    tile_of(pid, ntm, ntn, ep.gm, tm, tn);
    const int m0 = tm * T8, n0 = tn * T8;
    const int kb = piece < 0 ? 0 : piece * piece_k;
    const int Kp = piece < 0 ? K : min(K - kb, piece_k);
    const int nt = Kp / 128;

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wave >> 2, wc = wave & 3;

    f32x16_t acc[2][2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[a][b][i][r] = 0.f;

    // DMA: as gemm_bf16_tn_8p; piece j of a wave covers rows 16w + 8j + L/8, whose (row >> 3) & 1 = j
    const int prow = 16 * wave + (lane >> 3);
    auto rsrc = [](const void* base) {
        return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
    };
    const __amdgpu_buffer_rsrc_t ra = rsrc(A + (long long)m0 * lda + kb);
    const __amdgpu_buffer_rsrc_t rw = rsrc(W + (long long)n0 * ldw + kb);
    const unsigned pcol = 16u * ((lane & 7) ^ (lane >> 3));
    const int alim = M - 1 - m0, wlim = N - 1 - n0;
    // row offsets formed per stage from two opaque VGPRs (kept for the fragment prefetch's registers;
    // a variant holding the eight offsets across the K loop compiles without spills but has not been
    // A/B-tested on a GPU yet: scripts/ab/ab_fp8_preoff.sh)
    auto stage = [&](int t, int which) {
        char* dst = smem + hoff(which, t & 1) + wave * 2048;
        const bool isw = which >= 2;
        const int h = which & 1;
        const unsigned ko = (unsigned)t * 128u;
        int pr = prow;
        unsigned pc = pcol;
        asm volatile("" : "+v"(pr), "+v"(pc));
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int r = h * 128 + pr + 8 * j;
            const unsigned pcj = pc ^ (16u * j);
            const unsigned vo = isw ? (unsigned)min(r, wlim) * (unsigned)ldw + pcj : (unsigned)min(r, alim) * (unsigned)lda + pcj;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(isw ? rw : ra, (LDS_AS void*)(dst + j * 1024), 16, vo, ko, 0, 0);
        }
    };

    const int frow = lane & 31, fh = lane >> 5;
    i32x8_t af[2][2], ag[2][2], bf0[2], bg0[2], bf1[2];
    // fragment bases per (buffer, k-step): q8_off(row0 + 32 i + frow, c) = q8_off(row0 + frow, c) + 4096 i,
    // and the second 16-B chunk of a lane's 32 bytes sits at (address ^ 16) (bit 4 of the address =
    // bit 0 of the swizzled chunk; every other term is a multiple of 128)
    int abase[2], bbase[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        abase[s] = (int)(uintptr_t)smem + q8_off(wr * 64 + frow, 4 * s + 2 * fh);
        bbase[s] = (int)(uintptr_t)smem + hoff(R_B0, 0) + q8_off(wc * 32 + frow, 4 * s + 2 * fh);
        asm volatile("" : "+v"(abase[s]), "+v"(bbase[s]));
    }
    auto frag = [&](int base, int imm) {
        int base2;      // (asm: formed where it is used, not hoisted into a register live across the loop)
        asm volatile("v_xor_b32 %0, 16, %1" : "=v"(base2) : "v"(base));
        const u32x4_t lo = *reinterpret_cast<const LDS_AS u32x4_t*>((const LDS_AS char*)(uintptr_t)(unsigned)(base + imm));
        const u32x4_t hi = *reinterpret_cast<const LDS_AS u32x4_t*>((const LDS_AS char*)(uintptr_t)(unsigned)(base2 + imm));
        return i32x8_t{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
    };
    auto read_a = [&](int b, int region, i32x8_t (&a)[2][2]) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int s = 0; s < 2; ++s) a[i][s] = frag(abase[s], hoff(region, b) + 4096 * i);
    };
    auto read_b = [&](int b, int region, i32x8_t (&bf)[2]) {
#pragma unroll
        for (int s = 0; s < 2; ++s) bf[s] = frag(bbase[s], hoff(region, b) - hoff(R_B0, 0));
    };
    auto mfma4 = [&](f32x16_t (&c)[2], const i32x8_t (&a)[2][2], const i32x8_t (&bf)[2]) {
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int i = 0; i < 2; ++i)
                c[i] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(bf[s], a[i][s], c[i], 0, 0, 0, 0x7f, 0, 0x7f);
        // pin the cluster inside its phase: the IR passes may otherwise sink these register-only
        // MFMAs past the phase's barrier (and keep every fragment set live across phases)
        asm volatile("" : "+v"(c[0]), "+v"(c[1]));
        __builtin_amdgcn_s_setprio(0);
    };
    auto bar = [&]() {
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_barrier" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
    };
    auto bar_wait_lgkm = [&]() {
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_barrier" ::: "memory");
        __builtin_amdgcn_s_waitcnt(0xC07F);     // lgkmcnt(0), visible to the compiler's wait-count pass
        __builtin_amdgcn_sched_barrier(0);
    };

    stage(0, 0); stage(0, 2); stage(0, 3); stage(0, 1);
    if (nt > 1) {
        stage(1, 0); stage(1, 2); stage(1, 3);
        asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    bar();
    // the phase schedule of gemm_bf16_tn_8p without the stagger, with a fragment prefetch: each phase
    // waits for the fragments the previous one read, reads the next phase's new ones and runs its 4
    // MX MFMAs under them (the bf16 kernel's stagger measured +-0 here: profiles/r3/
    // gemm_fp8_stagger_ab_s1.log, the 4 MX MFMAs of a phase already cover its reads)
    auto tile4p = [&](int t, int b, i32x8_t (&b0)[2], i32x8_t (&b0n)[2]) __attribute__((always_inline)) {
        if (t + 1 < nt) stage(t + 1, 1);
        bar_wait_lgkm();
        read_b(b, R_B1, bf1);
        __builtin_amdgcn_sched_barrier(0);
        mfma4(acc[0][0], af, b0);
        bar();
        if (t + 2 < nt) stage(t + 2, 0);
        bar_wait_lgkm();
        read_a(b, R_A1, ag);
        __builtin_amdgcn_sched_barrier(0);
        mfma4(acc[0][1], af, bf1);
        bar();
        if (t + 2 < nt) stage(t + 2, 2);
        bar_wait_lgkm();
        mfma4(acc[1][1], ag, bf1);
        bar();
        if (t + 2 < nt) {
            stage(t + 2, 3);
            __builtin_amdgcn_sched_barrier(0);
            asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        } else if (t + 1 < nt) {
            __builtin_amdgcn_sched_barrier(0);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        bar_wait_lgkm();
        if (t + 1 < nt) {
            read_a(b ^ 1, R_A0, af);
            read_b(b ^ 1, R_B0, b0n);
        }
        __builtin_amdgcn_sched_barrier(0);
        mfma4(acc[1][0], ag, b0);
        bar();
    };
    read_a(0, R_A0, af);
    read_b(0, R_B0, bf0);
#pragma nounroll
    for (int t = 0; t < nt; t += 2) {
        tile4p(t, 0, bf0, bg0);
        if (t + 1 < nt) tile4p(t + 1, 1, bg0, bf0);
    }

    // acc[qa][qb][i][4g + e] = D[n][m]: m = m0 + 128 qa + 64 wr + 32 i + (lane & 31),
    // n = n0 + 128 qb + 32 wc + 8 g + 4 (lane >> 5) + e
    if (piece >= 0) {
        float* pp = part + ((long long)(pid - nmain) * ksplit + piece) * T8 * T8;
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b)
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int g = 0; g < 4; ++g)
                        *reinterpret_cast<f32x4_t*>(pp + (128 * a + 64 * wr + 32 * i + frow) * T8 + 128 * b + 32 * wc +
                                                    8 * g + 4 * fh) =
                            f32x4_t{acc[a][b][i][4 * g], acc[a][b][i][4 * g + 1], acc[a][b][i][4 * g + 2],
                                    acc[a][b][i][4 * g + 3]};
        return;
    }
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int m = m0 + 128 * a + 64 * wr + 32 * i + frow;
            if (m >= M) continue;
            const float sa = scale_a[m];
#pragma unroll
            for (int b = 0; b < 2; ++b)
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int n = n0 + 128 * b + 32 * wc + 8 * g + 4 * fh;
                    if (n >= N) continue;
                    epilogue_store(f32x4_t{acc[a][b][i][4 * g] * sa, acc[a][b][i][4 * g + 1] * sa,
                                           acc[a][b][i][4 * g + 2] * sa, acc[a][b][i][4 * g + 3] * sa},
                                   m, n, C, ldc, ep);
                }
        }
}


// ---------------------------------------------------------------------------------------------
// gemm_fp8_tn_4w: the 4-wave 256x256 schedule of gemm_bf16_tn_4w for the fp8 path (config 5;
// AutoWrappedLinear.fp8_linear, layers.py:115-151): C = epilogue(scale_a[m] * (A8 . W8^T)), e4m3
// operands.  A K-tile is 128 fp8 = the same 128-B row segments, LDS-DMA pieces and 1-KB LDS rows
// as the bf16 kernel; per wave and K-tile 64 MX-rate v_mfma_scale_f32_16x16x128_f8f6f4 (unit E8M0
// scales, 32 cycles each: twice the bf16 FLOPs per cycle).  A 16x16x128 fragment is 32 B per lane
// (row l % 16, bytes 32 (l / 16) ..), one K-tile's 16 fragments are all 128 VGPRs, so instead of
// holding two k-steps the MFMA order lets fragments die early: rows 0-3 of the 8x8 tile grid
// i-major (q < 32), then rows 4-7 column by column; the next K-tile's fragments are read into the
// dead registers (A 0-3 from q = 32, W column j after its last use at q = 35 + 4j, W 7 and A 4-7 at
// the top of the next iteration).  LDS rows of 1088 B (64-B pad) with the 16-B chunk XOR
// 3 (r >> 3) on rows r % 16 >= 8 (applied on the DMA source address): conflict-free for both 16-B
// halves of every fragment read (tests/probes: searched over pads and XOR swizzles).
// Per iteration: top reads of K-tile t, one barrier (buffer of t free), the 16 DMA instructions of
// K-tile t+2 into it (every 3 MFMAs from q = 11), vmcnt(6) + barrier at q = 29 (K-tile t+1 landed),
// then the next K-tile's reads.
// ---------------------------------------------------------------------------------------------
constexpr int F4_ROWB = 1088;
constexpr int F4_OPB = 32 * F4_ROWB;
constexpr int F4_LDS = 4 * F4_OPB;            // [A b0][A b1][W b0][W b1] = 139264 B
static_assert(4 * F4_ROWB == 0x1100, "the fp8 4w kernel's M0 step");
__device__ __forceinline__ int f4_swz(int r) { return ((r >> 3) & 1) * 3; }

template <bool WIDE, int MODE, bool HINT>      // MODE / HINT: the 16-B epilogue's (WIDE) mode
__global__ __launch_bounds__(256, 1) void gemm_fp8_tn_4w(
    const uint8_t* __restrict__ A, long long lda, const float* __restrict__ scale_a, const uint8_t* __restrict__ W,
    long long ldw, bf16_t* C, long long ldc, int M, int N, int K, Epi ep, int ntm, int ntn, int nmain, int ksplit,
    int piece_k, float* __restrict__ part, W4Sched sc) {
#if defined(__HIP_DEVICE_COMPILE__)     // (the AGPR asm operands are not host constraints)
    extern __shared__ __attribute__((aligned(16))) char smem[];
    // persistent as gemm_bf16_tn_4w (w4_work / W4Grab: one workgroup per CU fed by its XCD's tile
    // queue, the DMA cursor running across tile boundaries, split pieces after)
    const W4Work wk = w4_work(sc, K, nmain, ksplit, piece_k, 128);
    const int nt = wk.nt;

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 1, wn = wave & 1;

    f32x4_t acc[8][8];

    // DMA instruction j of wave w: LDS row 4j + w, global row 128 (rho / 16) + 16 (lane / 8) + rho % 16
    // (rho = 4j + w), 16-B chunk lane % 8 taken from the swizzled source chunk; the row offsets are
    // tile-invariant (resources rebased on the tile, num_records = its rows' bytes: rows past the
    // matrix load 0), the K-tile offset goes in soffset.  One instruction per DMA: M0 (the LDS
    // destination) is set at an operand's first instruction and stepped by 4 rows (4 x 1088 B) one
    // MFMA ahead of the next (the bf16 kernel's r4 form, see gemm_bf16_tn_4w)
    auto rsrc4 = [](const uint8_t* base, int bytes) {
        const unsigned long long a = (unsigned long long)(uintptr_t)base;
        return i32x4_t{__builtin_amdgcn_readfirstlane((int)(unsigned)a),
                       __builtin_amdgcn_readfirstlane((int)((unsigned)(a >> 32) & 0xffffu)),
                       __builtin_amdgcn_readfirstlane(bytes), 0x00020000};
    };
    unsigned voa[8], vow[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int rho = 4 * j + wave;
        const unsigned g = (unsigned)((rho >> 4) * 128 + 16 * (lane >> 3) + (rho & 15));
        const unsigned ch = 16u * (unsigned)((lane & 7) ^ f4_swz(rho & 15));
        voa[j] = g * (unsigned)lda + ch;
        vow[j] = g * (unsigned)ldw + ch;
        asm volatile("" : "+v"(voa[j]), "+v"(vow[j]));     // kept, not re-formed per use
    }
    i32x4_t ra, rw;
    auto dma_tile = [&](int id) {
        int tm, tn;
        tile_of(id, ntm, ntn, ep.gm, tm, tn);
        const int m0 = tm * 256, n0 = tn * 256;
        ra = rsrc4(A + (long long)m0 * lda + wk.kb, (int)((long long)max(0, min(M - m0, 256)) * lda));
        rw = rsrc4(W + (long long)n0 * ldw + wk.kb, (int)((long long)max(0, min(N - n0, 256)) * ldw));
    };
    // tiles: cur (computing), nxt (the next one, from the LDS word in cur's first K-tile), dnext
    // (where the DMA cursor goes when it leaves cur; -1: re-read), as in gemm_bf16_tn_4w
    int cur = wk.first, nxt = wk.second, dnext = wk.second;
    int dkt = 0;
    auto dma_advance = [&]() {
        if (++dkt == nt) {
            if (dnext >= 0) {
                dkt = 0;
                dma_tile(dnext);
                dnext = -1;
            } else {
                dkt = nt - 1;           // past the block's last K-tile: re-read it (unused buffer)
            }
        }
    };
    W4Grab grab(sc);
    const unsigned slot = (unsigned)(uintptr_t)smem + F4_LDS;     // the next tile id (LDS word)
    auto slot_ref = [&]() -> volatile LDS_AS int& { return *(volatile LDS_AS int*)(uintptr_t)slot; };
    int slotv = 0;
    unsigned dw = 2 * F4_OPB + wave * F4_ROWB, da = wave * F4_ROWB;
    const unsigned dw_tog = dw ^ (dw + F4_OPB), da_tog = da ^ (da + F4_OPB);
    const unsigned lds0 = (unsigned)(uintptr_t)smem;
    // DMA d: W instruction d (d < 8) or A instruction d - 8
    auto m0_set = [&](int d) {
        if (d == 0 || d == 8) asm volatile("s_mov_b32 m0, %0" :: "s"(lds0 + (d == 0 ? dw : da)) : "m0");
        else asm volatile("s_add_u32 m0, m0, 0x1100" ::: "memory");   // (see m0_step_note)
    };
    auto dma_go = [&](unsigned ko, int d) {
        if (d < 8) asm volatile("buffer_load_dwordx4 %0, %1, %2 offen lds" :: "v"(vow[d]), "s"(rw), "s"(ko) : "memory");
        else asm volatile("buffer_load_dwordx4 %0, %1, %2 offen lds" :: "v"(voa[d - 8]), "s"(ra), "s"(ko) : "memory");
    };
    auto dma_now = [&](unsigned ko, int d) {
        asm volatile("s_mov_b32 m0, %0" :: "s"(lds0 + (d < 8 ? dw + 4 * d * F4_ROWB : da + 4 * (d - 8) * F4_ROWB)) : "m0");
        asm volatile("s_nop 0" ::: "memory");
        dma_go(ko, d);
    };

    // fragment bases: the two 16-B halves of a lane's 32 B (logical chunks 2c, 2c+1 of row r)
    const int fr = lane & 15, fc = lane >> 4, sw = f4_swz(fr);
    int a0 = (int)(uintptr_t)smem + (wm * 16 + fr) * F4_ROWB + 16 * ((2 * fc) ^ sw);
    int a1 = (int)(uintptr_t)smem + (wm * 16 + fr) * F4_ROWB + 16 * ((2 * fc + 1) ^ sw);
    int w0 = (int)(uintptr_t)smem + 2 * F4_OPB + (wn * 16 + fr) * F4_ROWB + 16 * ((2 * fc) ^ sw);
    int w1 = (int)(uintptr_t)smem + 2 * F4_OPB + (wn * 16 + fr) * F4_ROWB + 16 * ((2 * fc + 1) ^ sw);
    int a0t = a0 ^ (a0 + F4_OPB), a1t = a1 ^ (a1 + F4_OPB), w0t = w0 ^ (w0 + F4_OPB), w1t = w1 ^ (w1 + F4_OPB);
    asm volatile("" : "+v"(a0), "+v"(a1), "+v"(w0), "+v"(w1));
    asm volatile("" : "+v"(a0t), "+v"(a1t), "+v"(w0t), "+v"(w1t));
    auto frag = [&](int lo, int hi, int off) {
        const u32x4_t x = *reinterpret_cast<const LDS_AS u32x4_t*>((const LDS_AS char*)(uintptr_t)(unsigned)(lo + off));
        const u32x4_t y = *reinterpret_cast<const LDS_AS u32x4_t*>((const LDS_AS char*)(uintptr_t)(unsigned)(hi + off));
        return i32x8_t{(int)x[0], (int)x[1], (int)x[2], (int)x[3], (int)y[0], (int)y[1], (int)y[2], (int)y[3]};
    };
    // the same read from inline asm: invisible to the compiler's wait-count pass, waited for by the
    // hand-placed lgkmcnt of the loop body (the pass would otherwise wait for it at the loop top)
    auto frag_asm = [&](int lo, int hi, int off) {
        u32x4_t x, y;
        asm volatile("ds_read_b128 %0, %2 offset:%4\n\tds_read_b128 %1, %3 offset:%4"
                     : "=&v"(x), "=&v"(y) : "v"(lo), "v"(hi), "i"(off) : "memory");
        return i32x8_t{(int)x[0], (int)x[1], (int)x[2], (int)x[3], (int)y[0], (int)y[1], (int)y[2], (int)y[3]};
    };
    i32x8_t fa[8], fw[8];
    const int unit = 0x7f7f7f7f;        // E8M0 scale 2^0 in every byte
    auto fence = [&]() { __builtin_amdgcn_sched_barrier(0); };
    auto bar = [&]() {
        fence();
        asm volatile("s_barrier" ::: "memory");
        fence();
    };
    // the fragments a K-tile's loop top does not read itself (A 0-3, W 0-6), of the K-tile the
    // fragment bases point at
    auto read_early = [&]() {
#pragma unroll
        for (int i = 0; i < 4; ++i) fa[i] = frag(a0, a1, 128 * i);
#pragma unroll
        for (int j = 0; j < 7; ++j) fw[j] = frag(w0, w1, 128 * j);
        fence();
    };

    // prologue: K-tiles 0 and 1 of the stream in flight, then the early fragments of K-tile 0
    const bool dyn = sc.q && (int)blockIdx.x < sc.npers;    // a persistent block fed by the queues
    if (dyn) {              // the first tile from the queues too (a block that starts late: none left)
        if (wave == 0) {
            grab.issue();
            const int id = grab.finish<0>(lane);
            if (lane == 0) slot_ref() = id;
        }
        __syncthreads();
        cur = __builtin_amdgcn_readfirstlane(slot_ref());
        if (cur < 0) {
            grab.done(tid);
            return;
        }
    }
    dma_tile(cur);
    if (dyn && wave == 0) grab.issue();                       // the second tile, under the prologue
#pragma unroll
    for (int d = 0; d < 16; ++d) dma_now(0u, d);
    dma_advance();
    dw ^= dw_tog;
    da ^= da_tog;
#pragma unroll
    for (int d = 0; d < 16; ++d) dma_now((unsigned)dkt * 128u, d);
    dma_advance();
    dw ^= dw_tog;
    da ^= da_tog;
    fence();
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    bar();
    read_early();
    if (wave == 0) {        // the second tile into the LDS word (read in the first tile's first K-tile)
        const int id = dyn ? grab.finish<32>(lane) : wk.second;     // (the 32 prologue DMAs since issue)
        if (lane == 0) slot_ref() = id;
    }

    // one K-tile: top reads of this K-tile (W 7, A 4-7), one barrier (its buffer free for the DMA of
    // the stream's K-tile two ahead, every 3 MFMAs from q = 11), vmcnt(6) + barrier at q = 29 (the
    // next K-tile landed), then the next K-tile's early reads into the fragments that died.  FIRST:
    // the tile's first K-tile, whose MFMAs start the accumulators from 0
    auto ktile = [&](auto firstc) __attribute__((always_inline)) {
        constexpr bool FIRST = decltype(firstc)::value;
        const unsigned ko = (unsigned)dkt * 128u;
        fence();
        __builtin_amdgcn_s_waitcnt(0xC07F);     // lgkmcnt(0): the early reads landed
        fence();
        static_for<64>([&](auto qc) __attribute__((always_inline)) {
            constexpr int q = decltype(qc)::value;
            if constexpr (q == 0) fw[7] = frag_asm(w0, w1, 128 * 7);                // this K-tile, this buffer
            if constexpr (q >= 1 && q <= 4) fa[3 + q] = frag_asm(a0, a1, 128 * (3 + q));
            if constexpr (q == 7) {                  // W 7 landed (the 8 reads of A 4-7 may still fly)
                fence();
                asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
                fence();
            }
            if constexpr (q == 5) {                                                  // to the next buffer
                a0 ^= a0t; a1 ^= a1t; w0 ^= w0t; w1 ^= w1t;
            }
            if constexpr (q == 10) {                                                 // this buffer free
                fence();
                __builtin_amdgcn_s_waitcnt(0xC07F);     // lgkmcnt(0)
                asm volatile("s_barrier" ::: "memory");
                fence();
            }
            if constexpr (q >= 11 && q <= 56 && (q - 11) % 3 == 0) dma_go(ko, (q - 11) / 3);
            if constexpr (FIRST && q == 11) slotv = slot_ref();           // the next tile (behind q 10)
            if constexpr (q == 29) {                                                 // next K-tile landed
                fence();
                asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
                bar();
            }
            if constexpr (FIRST && q == 30) {
                nxt = __builtin_amdgcn_readfirstlane(slotv);
                dnext = nxt;
            }
            if constexpr (q >= 32 && q <= 35) fa[q - 32] = frag(a0, a1, 128 * (q - 32));
            if constexpr (q >= 36 && q <= 60 && (q - 36) % 4 == 0) fw[(q - 36) / 4] = frag(w0, w1, 128 * ((q - 36) / 4));
            // MFMA q: rows 0-3 i-major, then rows 4-7 column by column
            constexpr int i = q < 32 ? (q >> 3) : 4 + ((q - 32) & 3);
            constexpr int j = q < 32 ? (q & 7) : (q - 32) >> 2;
            if constexpr (q >= 10 && q <= 55 && (q - 10) % 3 == 0) m0_set((q - 10) / 3);   // DMA of MFMA q + 1
            if constexpr (FIRST)
                asm volatile("v_mfma_scale_f32_16x16x128_f8f6f4 %0, %1, %2, 0, %3, %3 op_sel_hi:[0,0,0]"
                             : "=a"(acc[i][j]) : "v"(fw[j]), "v"(fa[i]), "v"(unit));
            else
                asm volatile("v_mfma_scale_f32_16x16x128_f8f6f4 %0, %1, %2, %0, %3, %3 op_sel_hi:[0,0,0]"
                             : "+a"(acc[i][j]) : "v"(fw[j]), "v"(fa[i]), "v"(unit));
            fence();
        });
        dw ^= dw_tog;
        da ^= da_tog;
        dma_advance();
    };

#pragma nounroll
    for (;;) {
        ktile(std::true_type{});
#pragma nounroll
        for (int t = 1; t < nt; ++t) ktile(std::false_type{});
        // the accumulators leave through v_accvgpr_read (acc_rd): cover the last MFMAs' write latency
        asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");
        int tm, tn;
        tile_of(cur, ntm, ntn, ep.gm, tm, tn);
        const int m0 = tm * 256, n0 = tn * 256;
        if (nxt >= 0 && wave == 0) grab.issue();            // the tile after nxt, under the epilogue
        // acc[i][j][e] = D[n][m]: m = m0 + 128 wm + 16 i + (lane & 15), n = n0 + 128 wn + 16 j + 4 (lane >> 4) + e
        if (wk.piece >= 0) {
            const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(
                part + ((long long)(cur - nmain) * ksplit + wk.piece) * 256 * 256, 0, 256 * 256 * 4, 0x00020000);
            const int vo = ((128 * wm + (lane & 15)) * 256 + 128 * wn + 4 * (lane >> 4)) * 4;
#pragma unroll
            for (int i = 0; i < 8; ++i)
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    __builtin_amdgcn_raw_buffer_store_b128(
                        u32x4_t{__float_as_uint(acc_rd(acc[i][j][0])), __float_as_uint(acc_rd(acc[i][j][1])),
                                __float_as_uint(acc_rd(acc[i][j][2])), __float_as_uint(acc_rd(acc[i][j][3]))},
                        rp, vo, 16 * i * 256 * 4 + 64 * j, 0);
        } else if constexpr (WIDE) {
            tile_epilogue_w4<MODE, HINT, true>(acc, m0 + 128 * wm, n0 + 128 * wn, lane, C, ldc, M, N, ep, scale_a);
        } else {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int m = m0 + 128 * wm + 16 * i + (lane & 15);
                const float sa = scale_a[min(m, M - 1)];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int n = n0 + 128 * wn + 16 * j + 4 * (lane >> 4);
                    // (plain reads: the 8-B path, for N % 8 != 0 only, leaves the copies to the
                    // compiler -- through acc_rd its AGPR round trips came back stale)
                    if (m < M && n < N) epilogue_store(acc[i][j] * sa, m, n, C, ldc, ep);
                }
            }
        }
        // the epilogue's loads and stores leave the counted DMA waits of the next tile exact
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (nxt < 0) break;
        if (wave == 0) {                // the id of the tile after nxt into the LDS word
            const int id = grab.finish<0>(lane);
            if (lane == 0) slot_ref() = id;
        }
        cur = nxt;
        read_early();   // the next tile's early fragments (its first K-tile landed: the last q = 29 wait)
    }
    grab.done(tid);
#endif
}


// fp8_linear's activation quantisation (vram_management/layers.py:115-151): per row s = max(bf16(max|x| /
// 448), 1), x8 = e4m3(x / (s + 1e-8)).  One wave per row.  NC > 0: the row stays in registers
// between the max and the conversion (NC 16-B chunks per lane: cols <= 512 NC) -- one HBM read of x
// instead of two (r5; r1-r4 re-read the row: 249 us per 59 280 x 5120 launch, 4.1 % of a config-5
// step, profiles/r5/prof_fp8_r5s17); NC == 0: the two-pass form for wider rows.
template <int NC>
__global__ __launch_bounds__(256) void quant_fp8_rows_kernel(const bf16_t* __restrict__ x, long long ldx,
                                                             uint8_t* __restrict__ x8, long long ld8,
                                                             float* __restrict__ scale, int rows, int cols) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= rows) return;
    const bf16_t* xr = x + (long long)row * ldx;
    uint8_t* yr = x8 + (long long)row * ld8;
    float mx = 0.f;
    auto absmax = [&](const u32x4_t& w) {
#pragma unroll
        for (int e = 0; e < 4; ++e) mx = fmaxf(mx, fmaxf(fabsf(bflo(w[e])), fabsf(bfhi(w[e]))));
    };
    auto convert = [&](const u32x4_t& w, float d, int c) {
        u32x2_t o;
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            int v = __builtin_amdgcn_cvt_pk_fp8_f32(bflo(w[2 * e]) / d, bfhi(w[2 * e]) / d, 0, false);
            v = __builtin_amdgcn_cvt_pk_fp8_f32(bflo(w[2 * e + 1]) / d, bfhi(w[2 * e + 1]) / d, v, true);
            o[e] = (uint32_t)v;
        }
        *reinterpret_cast<u32x2_t*>(yr + c) = o;
    };
    u32x4_t w[NC > 0 ? NC : 1];
    if constexpr (NC > 0) {
#pragma unroll
        for (int i = 0; i < NC; ++i) {
            const int c = lane * 8 + 512 * i;
            w[i] = c < cols ? *reinterpret_cast<const u32x4_t*>(xr + c) : u32x4_t{0, 0, 0, 0};
        }
#pragma unroll
        for (int i = 0; i < NC; ++i) absmax(w[i]);
    } else {
        for (int c = lane * 8; c < cols; c += 512) absmax(*reinterpret_cast<const u32x4_t*>(xr + c));
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    const float s = fmaxf(rbf(mx / 448.0f), 1.0f);
    const float d = s + 1e-8f;
    if (lane == 0) scale[row] = s;
    if constexpr (NC > 0) {
#pragma unroll
        for (int i = 0; i < NC; ++i) {
            const int c = lane * 8 + 512 * i;
            if (c < cols) convert(w[i], d, c);
        }
    } else {
        for (int c = lane * 8; c < cols; c += 512) convert(*reinterpret_cast<const u32x4_t*>(xr + c), d, c);
    }
}

// The same quantisation for wide rows (the FFN-down input, 13 824 columns): one 256-thread block per
// row, NC 16-B chunks per thread in registers, the row max through LDS (one wave per row held 28
// chunks = 281 VGPRs per lane, one wave per SIMD: 3.8 TB/s).
template <int NC>
__global__ __launch_bounds__(256) void quant_fp8_rows_wide_kernel(const bf16_t* __restrict__ x, long long ldx,
                                                                  uint8_t* __restrict__ x8, long long ld8,
                                                                  float* __restrict__ scale, int cols) {
    __shared__ float red[4];
    const long long row = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63;
    const bf16_t* xr = x + row * ldx;
    uint8_t* yr = x8 + row * ld8;
    u32x4_t w[NC];
    float mx = 0.f;
#pragma unroll
    for (int i = 0; i < NC; ++i) {
        const int c = tid * 8 + 2048 * i;
        w[i] = c < cols ? *reinterpret_cast<const u32x4_t*>(xr + c) : u32x4_t{0, 0, 0, 0};
    }
#pragma unroll
    for (int i = 0; i < NC; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) mx = fmaxf(mx, fmaxf(fabsf(bflo(w[i][e])), fabsf(bfhi(w[i][e]))));
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    if (lane == 0) red[tid >> 6] = mx;
    __syncthreads();
    mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    const float s = fmaxf(rbf(mx / 448.0f), 1.0f);
    const float d = s + 1e-8f;
    if (tid == 0) scale[row] = s;
#pragma unroll
    for (int i = 0; i < NC; ++i) {
        const int c = tid * 8 + 2048 * i;
        if (c >= cols) continue;
        u32x2_t o;
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            int v = __builtin_amdgcn_cvt_pk_fp8_f32(bflo(w[i][2 * e]) / d, bfhi(w[i][2 * e]) / d, 0, false);
            v = __builtin_amdgcn_cvt_pk_fp8_f32(bflo(w[i][2 * e + 1]) / d, bfhi(w[i][2 * e + 1]) / d, v, true);
            o[e] = (uint32_t)v;
        }
        *reinterpret_cast<u32x2_t*>(yr + c) = o;
    }
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }
bool aligned8(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 7) == 0; }

}  // namespace


// Split tail.  One 256x256 workgroup fills a CU, so a grid of T tiles runs in ceil(T / CUs)
// rounds and the last, partial one leaves CUs idle: the 14B N=5120 GEMMs on 2 x 29640 tokens are
// 4640 tiles = 18.1 rounds on 256 CUs, and under Ulysses SP=8 (7410 rows) 580 tiles = 2.27.  The
// last T % CUs tiles instead run as ksplit K ranges each (fp32 partial tiles in a caller-bound
// per-(device, stream) workspace, then one combine launch that applies the epilogue), ksplit
// chosen by the measured cost model below.
constexpr int MAX_SPLIT_PIECES = 512;        // 512 x 256 KB fp32 partial tiles
struct KSplit { int nmain = 0, ntail = 0, ksplit = 1, piece_k = 0; };

KSplit plan_ksplit(int ntiles, int nh, int cus, int step = 64) {
    // Cost model in microseconds, calibrated on MI355X (tests/probes/split_ab.py): a whole tile
    // takes t = K * 0.029 us at ~1150 TF/s; a round of pieces costs t/f plus ~18 us (prologue and
    // the fp32 partial-tile writes, 256 KB per piece); the combine ~5 us + 0.065 us per partial
    // tile read.  Split only when the tail drops below 0.85 t.
    KSplit p;
    p.nmain = ntiles;
    if (cus <= 0 || ntiles < cus) return p;
    const int tail = ntiles % cus;
    if (tail == 0) return p;
    const double t = nh * step * 0.029;
    double best = 0.85 * t;
    int bf = 1;
    for (int f = 2; f <= 16 && tail * f <= MAX_SPLIT_PIECES && nh * step / f >= 512; ++f) {
        const int rounds = (tail * f + cus - 1) / cus;
        const double cost = rounds * (t / f + 18.0) + 5.0 + 0.065 * tail * f;
        if (cost < best) { best = cost; bf = f; }
    }
    if (bf == 1) return p;
    const int piece_h = (nh + bf - 1) / bf;
    p.ntail = tail;
    p.nmain = ntiles - tail;
    p.piece_k = piece_h * step;
    p.ksplit = (nh + piece_h - 1) / piece_h;
    return p;
}

// r6, with the piece pool (VS_OPT_PIECE_QUEUE): a GEMM of 1-3 whole rounds also keeps 1/16 of every
// round's capacity as K pieces.  Under the Ulysses overlap RCCL's all-to-all kernels hold some CUs;
// with exactly R rounds of whole tiles the tiles those CUs cannot take form an extra round of WHOLE
// tiles on the others (the SP = 8 FFN-down: 580 tiles = 2 rounds + 68, 1.17x its unheld time with
// 16 CUs held), while pieces of a quarter tile spread over every CU that is free.  Larger grids
// (>= 4 rounds) balance through the queues alone (profiles/r5/cu_hold_s5.log).
KSplit plan_ksplit_held(int ntiles, int nh, int cus, int step) {
    KSplit p = plan_ksplit(ntiles, nh, cus, step);
    const int R = cus > 0 ? ntiles / cus : 0;
    if (R < 1 || R > 3 || cus < 16) return p;
    const int tail = ntiles % cus + R * (cus / 16);
    int f = 0;
    for (int c = 4; c >= 2 && !f; --c)
        if (tail * c <= MAX_SPLIT_PIECES && nh * step / c >= 512) f = c;
    if (!f) return p;
    const int piece_h = (nh + f - 1) / f;
    p.ntail = tail;
    p.nmain = ntiles - tail;
    p.piece_k = piece_h * step;
    p.ksplit = (nh + piece_h - 1) / piece_h;
    return p;
}

// Routing (r5): every GEMM of the path runs on the kernels of this file.  r1-r4 sent the plain-bias
// q|k|v / cross-q projections, the GELU FFN-up and the context GEMMs at SP = 1 to a private copy of
// ROCm's hipBLASLt (+ a separate epilogue pass), which beat the hand-written kernels there (r4: q|k|v
// 1551 vs 1501 TF/s).  With the XCD tile queues the 4-wave kernel matches it on q|k|v (1529-1544 vs
// 1547-1556 TF/s, within run-to-run spread), leads on every fused-epilogue shape (FFN-up 1488-1496
// vs 1410-1413, o-proj 1438-1441 vs 1291-1296), reads fewer L2->fabric bytes on q|k|v (16.8 vs
// 17.9 GB per dispatch), and the whole step is as fast: 0.3906 / 0.3882 vs 0.3888 / 0.3881 steps/s
// with the library routes, same box, interleaved (profiles/r5/queue_ab_s2.log,
// pmc_fetch_queue_s2.txt, bench_own_vs_lt_ab_s2.log).  r6 removed the A/B build's library route.

// which 256x256 kernel runs the un-split-phase (k2 == 0) GEMMs: the 4-wave kernel (default since
// r4: 1-5 % over the 8-phase kernel on every 14B shape at 59 280 and 7410 rows) | VS_OPT_GEMM_KERNEL 8
static bool use_4w() { return vs_opt(VS_OPT_GEMM_KERNEL) == 4; }

// the schedule of a 4-wave launch (W4Sched): one persistent block per CU when the main tiles fill
// every CU and a tile has >= 3 K-tiles (the tile-id hand-off, see the schedule's comment), fed by the
// XCD tile queues when the stream has a queue workspace (kind 5) bound (VS_OPT_QUEUE 0: the
// static lists)
// npiece: the launch's split-tail pieces, taken by the persistent blocks from the queue's piece pool
// after the whole tiles (the bf16 kernel, r6); 0 (the fp8 kernel, or no queue): blocks of their own
static W4Sched w4_sched(int nmain, int nt, hipStream_t stream, int npiece = 0) {
    W4Sched s{nullptr, 0, 0, 0, 0};
    const int cus = vs_cus_for_split(false);
    if (cus >= 8 && cus % 8 == 0 && nmain >= cus && nt >= 3) {
        s.npers = cus;
        s.tp = nmain / cus;
    }
    s.nrem = nmain - s.npers * s.tp;
    if (s.npers && vs_opt(VS_OPT_QUEUE)) s.q = (unsigned*)vs_split_workspace(5, WQ_BYTES, stream);
    if (s.q) s.npiece = npiece;
    return s;
}
static unsigned w4_grid(const W4Sched& s, const KSplit& sp) {
    return (unsigned)(s.npers + (s.q ? 0 : s.nrem) + (s.npiece ? 0 : sp.ntail * sp.ksplit));
}

static int fill_epi(Epi& ep, int epilogue, const vs_epilogue* epi, int m, int n) {
    if (epilogue < VS_EPI_BIAS || epilogue > VS_EPI_RES) return VS_E_INVALID;
    ep = Epi{};
    ep.mode = epilogue;
    ep.rows_per_batch = m;
    ep.alpha = 1.f;
    ep.hint_scale = 1.f;
    ep.gm = VS_GEMM_GM;
    if (epi) {
        ep.bias = (const bf16_t*)epi->bias;
        ep.res = (const bf16_t*)epi->residual;
        ep.ld_res = epi->ld_res;
        ep.gate = (const bf16_t*)epi->gate;
        ep.gate_bstride = epi->gate_bstride;
        ep.hint = (const bf16_t*)epi->hint;
        ep.ld_hint = epi->ld_hint;
        ep.hint_scale = epi->hint_scale;
        ep.alpha = epi->alpha;
        if (epi->rows_per_batch > 0) ep.rows_per_batch = epi->rows_per_batch;
    }
    if ((epilogue == VS_EPI_GATE_RES || epilogue == VS_EPI_RES) && (!ep.res || ep.ld_res < n)) return VS_E_INVALID;
    if (epilogue == VS_EPI_GATE_RES && !ep.gate) return VS_E_INVALID;
    if (ep.hint && ep.ld_hint < n) return VS_E_INVALID;
    return VS_OK;
}


extern "C" int vs_gemm(const void* a, long long lda, const void* w, long long ldw, void* c,
                       long long ldc, int m, int n, int k, int epilogue, const vs_epilogue* epi,
                       const void* a2, long long lda2, const void* w2, long long ldw2, int k2,
                       void* stream) {
    if (!a || !w || !c || m <= 0 || n <= 0 || k <= 0) return VS_E_INVALID;
    if (k % BK || k2 % BK || k2 < 0 || n % 4) return VS_E_INVALID;
    if (lda < k || ldw < k || ldc < n || (lda & 7) || (ldw & 7) || (ldc & 3)) return VS_E_INVALID;
    if (!aligned16(a) || !aligned16(w) || !aligned8(c)) return VS_E_INVALID;
    if (k2 > 0) {
        if (!a2 || !w2 || lda2 < k2 || ldw2 < k2 || (lda2 & 7) || (ldw2 & 7)) return VS_E_INVALID;
        if (!aligned16(a2) || !aligned16(w2)) return VS_E_INVALID;
    }
    Epi ep;
    const int rc = fill_epi(ep, epilogue, epi, m, n);
    if (rc) return rc;
    // 256x256 schedule once the grid holds >= half a round of tiles (the 4-wave kernel from K = 1024:
    // persistent from one full round, its next tile's first K-tiles loading under the current one's
    // epilogue; the 8-phase kernel of the LoRA second phase from K = 4096), 128x128 otherwise
    // (VS_OPT_GEMM_TILE forces one).  r5: the 1.3B model's K = 1536 block GEMMs run 1314-1497 TF/s on
    // the 4-wave kernel against 606-861 on the 128x128 one (profiles/r5/gemm_ab_1p3b_s3.log), and the
    // 160-tile context k|v GEMM (M = 1024, K = 4096) is one 4-wave round instead of 218 us of 128x128
    const int force = vs_opt(VS_OPT_GEMM_TILE);
    const long long tiles256 = (long long)((m + BT - 1) / BT) * ((n + BT - 1) / BT);
    const bool big = force ? force == 256
                           : (tiles256 >= 240 && k >= 4096) || (tiles256 >= 128 && k >= 1024 && k2 == 0 && use_4w());
    if (big) {
        // 256x256 staggered 8-phase kernel (LoRA second phase included); the last partial round of
        // tiles runs as K pieces + combine (split tail)
        const int tm = (m + BT - 1) / BT, tn = (n + BT - 1) / BT;
        static bool attr8 = false;
        if (!attr8) {
            for (const void* f : {(const void*)gemm_bf16_tn_8p<false, false>, (const void*)gemm_bf16_tn_8p<true, false>,
                                  (const void*)gemm_bf16_tn_8p<false, true>, (const void*)gemm_bf16_tn_8p<true, true>})
                (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, LDS8);
            attr8 = true;
        }
        // 16-B epilogue accesses when every epilogue operand allows them
        const bool wide = n % 8 == 0 && ldc % 8 == 0 && aligned16(c) &&
                          (!ep.bias || aligned16(ep.bias)) && (!ep.res || (ep.ld_res % 8 == 0 && aligned16(ep.res))) &&
                          (!ep.gate || (ep.gate_bstride % 8 == 0 && aligned16(ep.gate))) &&
                          (!ep.hint || (ep.ld_hint % 8 == 0 && aligned16(ep.hint)));
        KSplit sp = k2 ? KSplit{tm * tn, 0, 1, 0} : plan_ksplit(tm * tn, k / 64, vs_cus_for_split(!vs_opt(VS_OPT_GEMM_SPLIT)), 64);
        float* part = nullptr;
        if (sp.ntail) {
            part = vs_split_workspace(1, (size_t)sp.ntail * sp.ksplit * BT * BT * sizeof(float), (hipStream_t)stream);
            if (!part) sp = KSplit{tm * tn, 0, 1, 0};
        }
        if (k2 == 0 && wide && use_4w() && vs_opt(VS_OPT_QUEUE) && vs_opt(VS_OPT_PIECE_QUEUE) == 2 &&
            vs_opt(VS_OPT_GEMM_SPLIT)) {
            const KSplit held = plan_ksplit_held(tm * tn, k / 64, vs_cus_for_split(false), 64);
            if (held.ntail > sp.ntail) {
                float* p2 = vs_split_workspace(1, (size_t)held.ntail * held.ksplit * BT * BT * sizeof(float),
                                               (hipStream_t)stream);
                if (p2) {
                    sp = held;
                    part = p2;
                }
            }
        }
        if (k2 == 0 && wide && use_4w()) {
            using K4 = void (*)(const bf16_t*, long long, const bf16_t*, long long, bf16_t*, long long, int, int, int,
                                Epi, int, int, int, int, int, float*, W4Sched);
            // (a static table's constant initializer left the kernels' host stubs un-instantiated)
            const K4 kern4[6] = {gemm_bf16_tn_4w<VS_EPI_BIAS, false>, gemm_bf16_tn_4w<VS_EPI_GELU, false>,
                                        gemm_bf16_tn_4w<VS_EPI_SILU, false>, gemm_bf16_tn_4w<VS_EPI_GATE_RES, false>,
                                        gemm_bf16_tn_4w<VS_EPI_RES, false>, gemm_bf16_tn_4w<VS_EPI_GATE_RES, true>};
            static bool attr4 = false;
            if (!attr4) {
                for (const K4 f : kern4)
                    (void)hipFuncSetAttribute((const void*)f, hipFuncAttributeMaxDynamicSharedMemorySize, W4_LDS + 16);
                attr4 = true;
            }
            const K4 kf = kern4[(ep.mode == VS_EPI_GATE_RES && ep.hint) ? 5 : ep.mode];
            // raster groups of 2 M-tiles for the deep-K FFN-down (K 13 824: 5.47-5.48 vs 5.54-5.57 ms at
            // 59 280 rows), 4 elsewhere (q|k|v / FFN-up 1-1.5 % slower at 2, 5-15 % at 8-16;
            // profiles/r6/gemm_gm_s10.log).  The split combine below reads the same ep.gm
            if (k >= 8192) ep.gm = 2;
            const W4Sched sc = w4_sched(sp.nmain, k / 64, (hipStream_t)stream,
                                        vs_opt(VS_OPT_PIECE_QUEUE) ? sp.ntail * sp.ksplit : 0);
            hipLaunchKernelGGL(kf, dim3(w4_grid(sc, sp)), dim3(256), W4_LDS + 16,
                               (hipStream_t)stream, (const bf16_t*)a, lda, (const bf16_t*)w, ldw, (bf16_t*)c, ldc, m,
                               n, k, ep, tm, tn, sp.nmain, sp.ksplit, sp.piece_k, part, sc);
            VS_CHECK_LAUNCH();
        } else {
        hipLaunchKernelGGL(k2 ? (wide ? gemm_bf16_tn_8p<true, true> : gemm_bf16_tn_8p<true, false>)
                              : (wide ? gemm_bf16_tn_8p<false, true> : gemm_bf16_tn_8p<false, false>),
                           dim3((unsigned)(sp.nmain + sp.ntail * sp.ksplit)),
                           dim3(512), LDS8, (hipStream_t)stream, (const bf16_t*)a, lda, (const bf16_t*)w, ldw,
                           (bf16_t*)c, ldc, m, n, k, (const bf16_t*)a2, lda2, (const bf16_t*)w2, ldw2, k2, ep, tm, tn,
                           sp.nmain, sp.ksplit, sp.piece_k, part);
        VS_CHECK_LAUNCH();
        }
        if (sp.ntail) {
            const long long threads = (long long)sp.ntail * BT * (BT / 4);
            hipLaunchKernelGGL(gemm_split_combine, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0,
                               (hipStream_t)stream, part, (bf16_t*)c, ldc, m, n, ep, tm, tn, sp.nmain, sp.ntail,
                               sp.ksplit);
            VS_CHECK_LAUNCH();
        }
        return VS_OK;
    }
    const int ntm = (m + BM - 1) / BM, ntn = (n + BN - 1) / BN;
    const long long nwg = (long long)ntm * ntn;
    if (nwg > 0x7fffffff) return VS_E_INVALID;
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)gemm_bf16_tn,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 2 * STAGE_BYTES);
        attr_set = true;
    }
    hipLaunchKernelGGL(gemm_bf16_tn, dim3((unsigned)nwg), dim3(NTHR), 2 * STAGE_BYTES,
                       (hipStream_t)stream, (const bf16_t*)a, lda, (const bf16_t*)w, ldw,
                       (bf16_t*)c, ldc, m, n, k, (const bf16_t*)a2, lda2, (const bf16_t*)w2, ldw2,
                       k2, ep, ntm, ntn);
    VS_CHECK_LAUNCH();
    return VS_OK;
}

extern "C" int vs_gemm_fp8(const void* a8, long long lda, const float* scale_a, const void* w8, long long ldw,
                           void* c, long long ldc, int m, int n, int k, int epilogue, const vs_epilogue* epi,
                           void* stream) {
    if (!a8 || !scale_a || !w8 || !c || m <= 0 || n <= 0 || k <= 0) return VS_E_INVALID;
    // K % 128: the MFMA kernel's K-tile
    if (k % 128 || n % 4 || lda < k || ldw < k || ldc < n || (lda & 15) || (ldw & 15) || (ldc & 3))
        return VS_E_INVALID;
    if (!aligned16(a8) || !aligned16(w8) || !aligned8(c)) return VS_E_INVALID;
    Epi ep;
    const int rc = fill_epi(ep, epilogue, epi, m, n);
    if (rc) return rc;
    // r4 kept hipBLASLt fp8 for the plain-bias q|k|v (2807 vs 3067 TF/s); with the XCD tile queues
    // the 4-wave kernel runs it at 3013 vs 3068 and every fused-epilogue shape ahead of the library
    // + its epilogue pass (FFN-up 2839 vs 2500, o-proj 2652 vs 2225: profiles/r5/
    // gemm_fp8_queue_ab_s1.log), so every fp8 GEMM runs here (the library only in the A/B build)
    // the fp8 MFMA kernels (K-tiles of 128 fp8)
    const int tm = (m + BT - 1) / BT, tn = (n + BT - 1) / BT;
    static bool attr8 = false;
    if (!attr8) {
        (void)hipFuncSetAttribute((const void*)gemm_fp8_tn_8p, hipFuncAttributeMaxDynamicSharedMemorySize, LDS8);
        attr8 = true;
    }
    KSplit sp = plan_ksplit(tm * tn, k / 128, vs_cus_for_split(!vs_opt(VS_OPT_GEMM_SPLIT)), 128);
    float* part = nullptr;
    if (sp.ntail) {
        part = vs_split_workspace(1, (size_t)sp.ntail * sp.ksplit * BT * BT * sizeof(float), (hipStream_t)stream);
        if (!part) sp = KSplit{tm * tn, 0, 1, 0};
    }
    if (use_4w()) {                 // the 4-wave kernel unless VS_OPT_GEMM_KERNEL 8
        using KF4 = void (*)(const uint8_t*, long long, const float*, const uint8_t*, long long, bf16_t*, long long,
                             int, int, int, Epi, int, int, int, int, int, float*, W4Sched);
        // one instantiation per 16-B epilogue mode (index: mode, 5 = gate-residual + hint), 6: 8-B path
        const KF4 kf4[7] = {gemm_fp8_tn_4w<true, VS_EPI_BIAS, false>, gemm_fp8_tn_4w<true, VS_EPI_GELU, false>,
                            gemm_fp8_tn_4w<true, VS_EPI_SILU, false>, gemm_fp8_tn_4w<true, VS_EPI_GATE_RES, false>,
                            gemm_fp8_tn_4w<true, VS_EPI_RES, false>, gemm_fp8_tn_4w<true, VS_EPI_GATE_RES, true>,
                            gemm_fp8_tn_4w<false, VS_EPI_BIAS, false>};
        static bool attr4 = false;
        if (!attr4) {
            for (const KF4 f : kf4)
                (void)hipFuncSetAttribute((const void*)f, hipFuncAttributeMaxDynamicSharedMemorySize, F4_LDS + 16);
            attr4 = true;
        }
        const bool wide = n % 8 == 0 && ldc % 8 == 0 && aligned16(c) && (!ep.bias || aligned16(ep.bias)) &&
                          (!ep.res || (ep.ld_res % 8 == 0 && aligned16(ep.res))) &&
                          (!ep.gate || (ep.gate_bstride % 8 == 0 && aligned16(ep.gate))) &&
                          (!ep.hint || (ep.ld_hint % 8 == 0 && aligned16(ep.hint)));
        // persistent blocks fed by the XCD tile queues, as the bf16 kernel (w4_sched)
        const W4Sched sc = w4_sched(sp.nmain, k / 128, (hipStream_t)stream);
        const KF4 kf = kf4[!wide ? 6 : (ep.mode == VS_EPI_GATE_RES && ep.hint) ? 5 : ep.mode];
        hipLaunchKernelGGL(kf, dim3(w4_grid(sc, sp)), dim3(256), F4_LDS + 16,
                           (hipStream_t)stream, (const uint8_t*)a8, lda, scale_a, (const uint8_t*)w8, ldw, (bf16_t*)c,
                           ldc, m, n, k, ep, tm, tn, sp.nmain, sp.ksplit, sp.piece_k, part, sc);
    } else
    hipLaunchKernelGGL(gemm_fp8_tn_8p, dim3((unsigned)(sp.nmain + sp.ntail * sp.ksplit)), dim3(512), LDS8,
                       (hipStream_t)stream, (const uint8_t*)a8, lda, scale_a, (const uint8_t*)w8, ldw, (bf16_t*)c,
                       ldc, m, n, k, ep, tm, tn, sp.nmain, sp.ksplit, sp.piece_k, part);
    VS_CHECK_LAUNCH();
    if (sp.ntail) {
        const long long threads = (long long)sp.ntail * BT * (BT / 4);
        hipLaunchKernelGGL(gemm_split_combine, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0,
                           (hipStream_t)stream, part, (bf16_t*)c, ldc, m, n, ep, tm, tn, sp.nmain, sp.ntail,
                           sp.ksplit, scale_a);
        VS_CHECK_LAUNCH();
    }
    return VS_OK;
}

extern "C" int vs_quant_fp8_rows(const void* x, long long ldx, void* x8, long long ld8, float* scale, int rows,
                                 int cols, void* stream) {
    if (!x || !x8 || !scale || rows <= 0 || cols <= 0 || cols % 8 || ldx < cols || ld8 < cols || (ldx & 7) ||
        (ld8 & 7) || !aligned16(x) || !aligned8(x8))
        return VS_E_INVALID;
    const int nc = (cols + 511) / 512;
    if (nc > 12 && cols <= 2048 * 8) {        // wide rows: a block per row (up to 16 384 columns)
        hipLaunchKernelGGL(quant_fp8_rows_wide_kernel<8>, dim3((unsigned)rows), dim3(256), 0, (hipStream_t)stream,
                           (const bf16_t*)x, ldx, (uint8_t*)x8, ld8, scale, cols);
        VS_CHECK_LAUNCH();
        return VS_OK;
    }
    void (*kern)(const bf16_t*, long long, uint8_t*, long long, float*, int, int) =
        nc <= 4 ? quant_fp8_rows_kernel<4> : nc <= 12 ? quant_fp8_rows_kernel<12> : quant_fp8_rows_kernel<0>;
    hipLaunchKernelGGL(kern, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, (hipStream_t)stream,
                       (const bf16_t*)x, ldx, (uint8_t*)x8, ld8, scale, rows, cols);
    VS_CHECK_LAUNCH();
    return VS_OK;
}

// the route of a GEMM (include/vstyler.h): 0 = the MFMA kernels with the fused epilogue, the only
// route there is (r1-r4's vendor-library route, 1, is gone)
extern "C" int vs_gemm_route_epi(int m, int n, int k, int epilogue, int fp8) {
    if (m <= 0 || n <= 0 || k <= 0 || epilogue < VS_EPI_BIAS || epilogue > VS_EPI_RES) return -VS_E_INVALID;
    (void)fp8;
    return 0;
}
extern "C" int vs_gemm_route(int m, int n, int k) { return vs_gemm_route_epi(m, n, k, VS_EPI_BIAS, 0); }

extern "C" int vs_gemm_split_plan(int m, int n, int k, int cus, int* out) {
    if (!out || m <= 0 || n <= 0 || k <= 0 || k % BK || cus < 0) return VS_E_INVALID;
    const KSplit p = plan_ksplit(((m + BT - 1) / BT) * ((n + BT - 1) / BT), k / 64, cus);
    out[0] = p.nmain;
    out[1] = p.ntail;
    out[2] = p.ksplit;
    out[3] = p.piece_k;
    return VS_OK;
}

long long vs_gemm_split_workspace_bytes_impl() { return (long long)MAX_SPLIT_PIECES * BT * BT * (long long)sizeof(float); }
