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
// Two schedules share the epilogue:
//  * gemm_bf16_tn_256 (large M*N, K >= 4096): 256x256 tile, 8 waves in a ping-pong pair per SIMD
//    (see its header) -- the DiT projections and FFN;
//  * gemm_bf16_tn (everything else): the structure described below.
// Structure: 128x128x64 tile, 4 waves (2x2, 64x64 each), v_mfma_f32_16x16x32_bf16 computing the
// transposed tile (W rows as the A operand) so every lane owns 4 consecutive output columns;
// both operands are K-contiguous ([rows][K]) and staged by global_load_lds_dwordx4 (LDS-DMA,
// no VGPR round trip) into a 2-stage LDS ring whose 128-B rows carry a 16-B-chunk XOR swizzle
// (chunk ^ (row & 7)) applied on the global SOURCE address, which makes the fragment
// ds_read_b128 conflict free; grouped (8 m-tiles) + XCD-aware tile order for L2 reuse.
#include "common.h"
#include <stdlib.h>

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
__device__ __forceinline__ void load4(const bf16_t* p, float* v) { loadw<4>(p, v); }

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
// 256x256 tile, 8 waves, ping-pong schedule.  K is consumed in 32-wide half-steps through a
// 4-slot LDS ring (4 x 32 KB, LDS-DMA filled three half-steps ahead).  Waves 0-3 (rows 0-127)
// and waves 4-7 (rows 128-255) share SIMDs pairwise (w, w+4) and run one barrier-phase apart:
// in every phase one wave of each SIMD executes its 32 MFMAs (setprio 1) while its partner reads
// the next fragments from LDS and issues its LDS-DMA, so the matrix pipe alternates between the
// two waves instead of idling at every barrier.  Counted vmcnt (never 0 in the main loop), raw
// s_barrier.  64-B LDS rows, 16-B chunk swizzle c ^ ((3*(row>>2)) & 3) (conflict-free 16x16x32
// fragment reads).
// ---------------------------------------------------------------------------------------------
#ifndef VS_GEMM_RING
#define VS_GEMM_RING 4
#endif
#ifndef VS_GEMM_GM
#define VS_GEMM_GM 4            // M-tiles per raster group (L2 reuse of the weight tile)
#endif
constexpr int BT = 256, HK = 32, NTHR8 = 512, SLOT = 2 * BT * HK * 2;   // 32 KB per slot
constexpr int RING = VS_GEMM_RING;          // LDS slots (<= 5: 160 KB); prefetch distance RING-1

__device__ __forceinline__ int h_off(int row, int ch) {
    return row * 64 + 16 * (ch ^ ((3 * (row >> 2)) & 3));
}

__device__ __forceinline__ void wait_barrier(int n_after) {
    // The LDS-DMA of the needed half-step (vmcnt) must land before the barrier makes it visible;
    // the wave's own fragment reads (lgkmcnt) only have to land before its MFMAs, so with
    // this order they are waited for after the barrier (the slot they read is restaged two
    // phases later at the earliest).  Measured +0.5..1 % (VS_GEMM_EARLY_LGKM restores the old order).
    __builtin_amdgcn_sched_barrier(0);
#ifndef VS_GEMM_EARLY_LGKM
    if (n_after >= 3)
        asm volatile("s_waitcnt vmcnt(12)\n\ts_barrier\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
    else if (n_after == 2)
        asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
    else if (n_after == 1)
        asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
    else
        asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
#else
    if (n_after >= 3)
        asm volatile("s_waitcnt vmcnt(12) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else if (n_after == 2)
        asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else if (n_after == 1)
        asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
#endif
    __builtin_amdgcn_sched_barrier(0);
}

#ifdef VS_GEMM_STAMPS
// debug: s_memtime stamps of wave 0 and wave 4 of workgroup 0 (5 per half-step, 32 half-steps)
__device__ unsigned long long g_gemm_stamps[2][5 * 32];
#define STAMP(slot)                                                                             \
    do {                                                                                        \
        if (blockIdx.x == 0 && lane == 0 && (wave & 3) == 0 && h < 32) {                        \
            unsigned long long t_;                                                              \
            __builtin_amdgcn_sched_barrier(0);                                                  \
            asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");          \
            __builtin_amdgcn_sched_barrier(0);                                                  \
            g_gemm_stamps[wave >> 2][5 * h + (slot)] = t_;                                      \
        }                                                                                       \
    } while (0)
#else
#define STAMP(slot) do {} while (0)
#endif

// tile id -> (tm, tn): raster groups of GM M-tiles sweep all N-tiles, so consecutive ids on one
// XCD share the weight tile in L2
__device__ __forceinline__ void tile_of(int pid, int ntm, int ntn, int& tm, int& tn) {
    constexpr int GM = VS_GEMM_GM;
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
    tile_of(nmain + t, ntm, ntn, tm, tn);
    const int m = tm * BT + row, n = tn * BT + 4 * c4;
    if (m >= M || n >= N) return;
    const float* pp = part + (long long)t * ksplit * BT * BT + row * BT + 4 * c4;
    f32x4_t a = *reinterpret_cast<const f32x4_t*>(pp);
    for (int j = 1; j < ksplit; ++j) a += *reinterpret_cast<const f32x4_t*>(pp + (long long)j * BT * BT);
    if (scale_a) a *= scale_a[m];
    epilogue_store(a, m, n, C, ldc, ep);
}

// Epilogue continuation after a hipBLASLt GEMM: y = bf16(acc + bias) is already materialised in
// Y; feed it to the fused epilogue with no bias (rbf(y + 0) == y) so GELU / SiLU / gate-residual
// [+ hint] / residual round exactly as in the fused kernels.  One thread per 4 columns.
__global__ __launch_bounds__(256) void gemm_epi_apply(const bf16_t* Y, long long ldy, bf16_t* C, long long ldc,
                                                      int M, int N, Epi ep) {
    const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
    const int n4 = N / 4;
    if (idx >= (long long)M * n4) return;
    const int m = (int)(idx / n4), n = 4 * (int)(idx % n4);
    float v[4];
    load4(Y + (long long)m * ldy + n, v);
    epilogue_store(f32x4_t{v[0], v[1], v[2], v[3]}, m, n, C, ldc, ep);
}

// The same, 8 columns per thread with 16-B accesses and a (row, column-chunk) grid: no 64-bit
// index division, one pass at the HBM rate (N % 8 == 0 and 16-B aligned rows; host-checked).
__global__ __launch_bounds__(256) void gemm_epi_apply8(const bf16_t* Y, long long ldy, bf16_t* C, long long ldc,
                                                       int N, Epi ep) {
    const int m = blockIdx.x;
    const int n = 8 * (blockIdx.y * 256 + threadIdx.x);
    if (n >= N) return;
    float v[8];
    loadw<8>(Y + (long long)m * ldy + n, v);
    epilogue_store_w<8>(v, m, n, C, ldc, ep);
}

template <bool BUF>
__global__ __launch_bounds__(NTHR8, 2) void gemm_bf16_tn_256(
    const bf16_t* __restrict__ A, long long lda, const bf16_t* __restrict__ W, long long ldw,
    bf16_t* C, long long ldc, int M, int N, int K, const bf16_t* __restrict__ A2, long long lda2,
    const bf16_t* __restrict__ W2, long long ldw2, int K2, Epi ep, int ntm, int ntn, int nmain, int ksplit,
    int piece_k, float* __restrict__ part) {
    extern __shared__ __attribute__((aligned(16))) char smem[];

    // blocks [0, nmain) own whole tiles (XCD-remapped); the blocks after them run the last tiles
    // of the grid as ksplit K ranges of piece_k each and leave fp32 partial tiles for
    // gemm_split_combine (split tail, see vs_gemm; never with a LoRA second phase)
    int pid, piece = -1;
    if ((int)blockIdx.x < nmain) {
        pid = xcd_remap(blockIdx.x, nmain);
    } else {
        const int t = blockIdx.x - nmain;
        pid = nmain + t / ksplit;
        piece = t % ksplit;
    }
    int tm, tn;
    tile_of(pid, ntm, ntn, tm, tn);
    const int m0 = tm * BT, n0 = tn * BT;
    const int kb = piece < 0 ? 0 : piece * piece_k;
    const int Kp = piece < 0 ? K : min(K - kb, piece_k);

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 2, wn = wave & 3;      // wm = ping-pong group

    f32x4_t acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    // LDS-DMA: piece p (1 KB) = 16 rows x 64 B; lane L -> row 16p + L/4, physical chunk L%4,
    // logical chunk (L%4) ^ ((3*((L/4)>>2))&3).  Per half-step 32 pieces (16 A, 16 W):
    // wave w issues pieces 4w..4w+3 (waves 0-3: A, waves 4-7: W).
    const int prow = lane >> 2;
    const int pch = (lane & 3) ^ ((3 * (prow >> 2)) & 3);
    const int nh1 = Kp / HK;
    const int nh = nh1 + (piece < 0 ? K2 / HK : 0);
    // operand this wave streams (group 0: activations A/A2 rows m0.., group 1: weights W/W2 rows n0..)
    const bf16_t* Pm = (wm == 0 ? A : W) + kb;
    const bf16_t* Pl = wm == 0 ? A2 : W2;
    const long long ldm = wm == 0 ? lda : ldw;
    const long long ldl = wm == 0 ? lda2 : ldw2;
    const int lim = (wm == 0 ? M : N) - 1;
    const int r0 = wm == 0 ? m0 : n0;
    const int dst_off = wm * (BT * 64) + wn * 4 * 1024;
    const int rbase = r0 + wn * 64 + prow;
    int issued = -1;                                // highest half-step this wave has issued
    // BUF (every byte offset of the operands fits 31 bits; host-checked): buffer-addressed DMA with
    // the 4 row offsets loop-invariant in VGPRs and the half-step's K offset in soffset.  Otherwise
    // 64-bit flat addresses, recomputed per piece (2 v_mul_lo_u32 + v_mad_u64_u32 each: ~4x the
    // issue cost of the DMA itself).
    unsigned vo[4] = {0, 0, 0, 0};
    const __amdgpu_buffer_rsrc_t rm = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(Pm), 0, 0x7fffffff,
                                                                        0x00020000);
    if constexpr (BUF) {
#pragma unroll
        for (int j = 0; j < 4; ++j) vo[j] = (unsigned)min(rbase + j * 16, lim) * (unsigned)(ldm * 2) + pch * 16;
    }
    auto issue = [&](int h) {
        char* dst = smem + (h % RING) * SLOT + dst_off;
        const bool lora = h >= nh1;
        if (BUF && !lora) {
            const unsigned ko = (unsigned)h * HK * 2;
#pragma unroll
            for (int j = 0; j < 4; ++j)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rm, (LDS_AS void*)(dst + j * 1024), 16, vo[j], ko, 0, 0);
        } else {
            const bf16_t* P = (lora ? Pl : Pm) + (lora ? h - nh1 : h) * HK + pch * 8;
            const long long ld = lora ? ldl : ldm;
#pragma unroll
            for (int j = 0; j < 4; ++j)
                __builtin_amdgcn_global_load_lds((const GLB_AS void*)(P + (long long)min(rbase + j * 16, lim) * ld),
                                                 (LDS_AS void*)(dst + j * 1024), 16, 0, 0);
        }
        issued = h;
    };

    const int frow = lane & 15, fch = lane >> 4;
    bf16x8_t wf[4], af[8];
    auto load_frags = [&](int h) {
        const char* As = smem + (h % RING) * SLOT;
        const char* Bs = As + BT * 64;
#pragma unroll
        for (int j = 0; j < 4; ++j)
            wf[j] = *reinterpret_cast<const bf16x8_t*>(Bs + h_off(wn * 64 + j * 16 + frow, fch));
#pragma unroll
        for (int i = 0; i < 8; ++i)
            af[i] = *reinterpret_cast<const bf16x8_t*>(As + h_off(wm * 128 + i * 16 + frow, fch));
    };
    auto mfmas = [&]() {
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], af[i], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
    };

#ifdef VS_GEMM_PIPE
    // Register-pipelined variant: every wave runs [barrier_h; DMA(h+RING-1); frags(h+1) -> other
    // register set; MFMAs(h)], one barrier per half-step, no ping-pong.  barrier_h retires (vmcnt)
    // the wave's DMA of half-step h+1 and, because each wave reaches it only after consuming
    // frags(h-1), frees slot (h-1) % RING for the DMA issued right after it.
    bf16x8_t wf2[4], af2[8];
    auto load_frags2 = [&](int h, bf16x8_t* w, bf16x8_t* a) {
        const char* As = smem + (h % RING) * SLOT;
        const char* Bs = As + BT * 64;
#pragma unroll
        for (int j = 0; j < 4; ++j)
            w[j] = *reinterpret_cast<const bf16x8_t*>(Bs + h_off(wn * 64 + j * 16 + frow, fch));
#pragma unroll
        for (int i = 0; i < 8; ++i)
            a[i] = *reinterpret_cast<const bf16x8_t*>(As + h_off(wm * 128 + i * 16 + frow, fch));
    };
    auto mfmas2 = [&](const bf16x8_t* w, const bf16x8_t* a) {
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[j], a[i], acc[i][j], 0, 0, 0);
    };
#pragma unroll
    for (int j = 0; j < RING - 1; ++j)
        if (j < nh) issue(j);
    wait_barrier(issued);                           // half-step 0 landed and visible
    load_frags2(0, wf, af);
    for (int h = 0; h < nh; h += 2) {
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const int hc = h + e;
            if (hc >= nh) break;
            // barrier: half-step hc+1 visible (all but the DMAs issued after it may be pending)
            wait_barrier(issued - min(hc + 1, nh - 1));
            if (hc + RING - 1 < nh) issue(hc + RING - 1);
            if (e == 0) {
                if (hc + 1 < nh) load_frags2(hc + 1, wf2, af2);
                mfmas2(wf, af);
            } else {
                if (hc + 1 < nh) load_frags2(hc + 1, wf, af);
                mfmas2(wf2, af2);
            }
        }
    }
#else
    // prologue: half-steps 0..RING-2 in flight, then wait for half-step 0
#pragma unroll
    for (int j = 0; j < RING - 1; ++j)
        if (j < nh) issue(j);
    wait_barrier(issued);                           // needed = 0
    // Every wave runs the same body [L(h); barrier; C(h); barrier]; group 1 executes one extra
    // barrier first, so its L phases coincide with group 0's C phases (s_barrier counts arrivals,
    // not code positions) and group 0 balances the count at the end.  Global phase q = barriers
    // passed since the prologue; the barrier into phase q+1 needs half-step (q+1)/2 on every wave.
    int q = 0;
    auto bar = [&]() {
        wait_barrier(issued - min((q + 1) >> 1, nh - 1));
        ++q;
    };
    if (wm == 1) bar();
#pragma nounroll
    for (int h = 0; h < nh; ++h) {
        STAMP(0);
#ifndef VS_GEMM_DIAG_NOREADS      // diagnostics only (wrong results): time without fragment reads
        load_frags(h);
#endif
#ifndef VS_GEMM_DIAG_NODMA        // diagnostics only (wrong results): time without in-loop LDS-DMA
        if (h + RING - 1 < nh) issue(h + RING - 1);
#endif
        STAMP(1);
        bar();
        STAMP(2);
        mfmas();
        STAMP(3);
        bar();
        STAMP(4);
    }
    if (wm == 0) bar();
#endif

    if (piece >= 0) {
        float* pp = part + ((long long)(pid - nmain) * ksplit + piece) * BT * BT;
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                *reinterpret_cast<f32x4_t*>(pp + (wm * 128 + i * 16 + (lane & 15)) * BT + wn * 64 + j * 16 +
                                            4 * (lane >> 4)) = acc[i][j];
        return;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int m = m0 + wm * 128 + i * 16 + (lane & 15);
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
// never vmcnt(0) in the main loop).  Product D[n][m] = W.A^T (16x16x32, W fragment as the A
// operand) so each lane owns 4 consecutive output columns for the fused epilogue.
// ---------------------------------------------------------------------------------------------
constexpr int T8 = 256, HT8 = 128 * 128, BUF8 = 4 * HT8, LDS8 = 2 * BUF8;   // 16 KB, 64 KB, 128 KB
// half-tiles (0 A0, 1 A1, 2 B0, 3 B1) of the two buffers interleaved: [A0 b0][A0 b1][A1 b0][A1 b1]
// [B0 b0]...  so every A read of either buffer lies within the 16-bit ds_read offset of one base
// VGPR per k-step, and every B read within that of a second one
constexpr int R_A0 = 0, R_A1 = 1, R_B0 = 2, R_B1 = 3;
__device__ __forceinline__ constexpr int hoff(int which, int b) { return (2 * which + b) * HT8; }

__device__ __forceinline__ int q_off(int row, int ch) { return row * 128 + 16 * (ch ^ (row & 7)); }

template <bool LORA, int SCHED>     // SCHED 0: reads at phase start, 1: prefetch, 2: prefetch + one barrier
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
    tile_of(pid, ntm, ntn, tm, tn);
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
    // stage half-tile `which` (0 A0, 1 A1, 2 B0, 3 B1) of K-tile t into buffer t & 1.  The two row
    // offsets are formed here from two live VGPRs (row, chunk) -- kept opaque so the compiler does
    // not hoist eight loop-invariant offsets into registers the fragment prefetch needs
    auto stage = [&](int t, int which) {
        char* dst = smem + hoff(which, t & 1) + wave * 2048;
        const bool isw = which >= 2;
        const int h = which & 1;
        if (!LORA || t < nk1) {
            const unsigned ko = (unsigned)t * 128u;
            int pr = prow;
            unsigned pc = pcol;
            asm volatile("" : "+v"(pr), "+v"(pc));
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int r = h * 128 + pr + 8 * j;
                const unsigned vo = isw ? (unsigned)min(r, wlim) * ldwb + pc : (unsigned)min(r, alim) * ldab + pc;
                __builtin_amdgcn_raw_ptr_buffer_load_lds(isw ? rw : ra, (LDS_AS void*)(dst + j * 1024), 16, vo, ko,
                                                         0, 0);
            }
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
    bf16x8_t ag[4][2], bg0[2][2];       // PRE: the A1 set and the next tile's B0 set
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
    auto read_a_to = [&](const char* buf, int region, bf16x8_t (&a)[4][2]) {
        const int b = buf == smem ? 0 : 1;     // (buf: smem or smem + BUF8)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int s = 0; s < 2; ++s) a[i][s] = lds_frag(abase[s] + hoff(region, b) + 2048 * i);
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
    auto mfma16x = [&](f32x4_t (&c)[4][2], const bf16x8_t (&a)[4][2], const bf16x8_t (&bf)[2][2]) {
#ifdef VS_G8_DIAG_NOMFMA    // timing diagnostics only: operands consumed, no MFMA issued
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
                asm volatile("" : "+v"(c[i][j]) : "v"(a[i][0]), "v"(a[i][1]), "v"(bf[j][0]), "v"(bf[j][1]));
        return;
#endif
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    c[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][s], a[i][s], c[i][j], 0, 0, 0);
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
    // SCHED 2: wait for my own reads BEFORE the barrier (the barrier then proves every wave's)
    auto bar_wait_lgkm_pre = [&]() {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_waitcnt(0xC07F);     // lgkmcnt(0)
#ifndef VS_G8_DIAG_NOBAR    // timing diagnostics only (races): no phase barrier
        asm volatile("s_barrier" ::: "memory");
#endif
        __builtin_amdgcn_sched_barrier(0);
    };

    constexpr bool PRE = SCHED == 1 || SCHED == 2;
    if constexpr (SCHED == 2) {
        // prologue: tiles 0 and 1 in flight (A0 B0 B1 A1 each), wait for tile 0
        stage(0, 0); stage(0, 2); stage(0, 3); stage(0, 1);
        if (nt > 1) {
            stage(1, 0); stage(1, 2); stage(1, 3); stage(1, 1);
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    } else {
        // prologue: tile 0 (A0 B0 B1 A1) and tile 1 (A0 B0 B1) in flight, wait for tile 0
        stage(0, 0); stage(0, 2); stage(0, 3); stage(0, 1);
        if (nt > 1) {
            stage(1, 0); stage(1, 2); stage(1, 3);
            asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    }
    bar();

    // SCHED 3 (the template's stagger): waves 4-7 run one barrier behind waves 0-3, so on every SIMD
    // one wave's 16 MFMAs pair with its partner's fragment reads + DMA issue (matrix beside memory)
    // instead of all 8 waves reading, then all 8 computing.  A0 is restaged one phase after its ph0
    // reads; with the groups a barrier apart the other group's reads are retired by a counted
    // lgkmcnt(4) (the 8 A reads, issued first) before ph0's first barrier.
    constexpr bool STAG = SCHED == 3;
    // one K-tile = 4 phases; the body is written for a pair of tiles so the buffer is a constant
    auto tile4 = [&](int t, const char* buf) __attribute__((always_inline)) {
        // ph0: quadrant (A0, B0)
        read_a(buf, R_A0);
        if constexpr (STAG) __builtin_amdgcn_sched_barrier(0);
        read_b(buf, R_B0, bf0);
        if (t + 1 < nt) stage(t + 1, 1);
        if constexpr (STAG) {
            __builtin_amdgcn_sched_barrier(0);
            __builtin_amdgcn_s_waitcnt(0xC47F);     // lgkmcnt(4): this wave's A0 reads landed
        }
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
    // PRE: every phase first waits for the fragments the previous phase prefetched, then issues the
    // reads of the NEXT phase's new fragments and runs its MFMAs under them (the LDS reads of a tile,
    // 192 KB per CU, then overlap the matrix pipe instead of preceding it).  Register sets: af = A0
    // rows, ag = A1 rows, bf1 = B1, bf0 / bg0 = B0 of even / odd tiles (ph3 reads the next tile's A0
    // and B0 while its own A1 x B0 MFMAs still need the current B0).  Last reads of a half-tile:
    // A0, B0 in ph3 of the previous tile, B1 in ph0, A1 in ph1, each waited for one phase later --
    // so the restaging schedule (ph1: A0, ph2: B0, ph3: B1, next ph0: A1 of tile t+2) stays one phase
    // and one barrier behind every read of the same half-tile.
    auto tile4p = [&](int t, const char* buf, const char* nbuf, bf16x8_t (&b0)[2][2],
                      bf16x8_t (&b0n)[2][2]) __attribute__((always_inline)) {
        // ph0: (A0, B0); prefetch B1
        if (t + 1 < nt) stage(t + 1, 1);
        bar_wait_lgkm();
        read_b(buf, R_B1, bf1);
        __builtin_amdgcn_sched_barrier(0);
        mfma16x(acc[0][0], af, b0);
        bar();
        // ph1: (A0, B1); prefetch A1
        if (t + 2 < nt) stage(t + 2, 0);
        bar_wait_lgkm();
        read_a_to(buf, R_A1, ag);
        __builtin_amdgcn_sched_barrier(0);
        mfma16x(acc[0][1], af, bf1);
        bar();
        // ph2: (A1, B1)
        if (t + 2 < nt) stage(t + 2, 2);
        bar_wait_lgkm();
        mfma16x(acc[1][1], ag, bf1);
        bar();
        // ph3: (A1, B0); retire tile t+1, then prefetch its A0 and B0
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
            read_a_to(nbuf, R_A0, af);
            read_b(nbuf, R_B0, b0n);
        }
        __builtin_amdgcn_sched_barrier(0);
        mfma16x(acc[1][0], ag, b0);
        bar();
    };
    // SCHED 2: ONE barrier per phase.  Phase p = [lgkmcnt(0): my phase p-1 reads landed; (ph3:
    // vmcnt(6): tile t+1 landed); s_barrier; DMA; reads for phase p+1; 16 MFMAs].  Passing the
    // barrier proves every wave's phase p-1 reads complete (so the half-tile they last touched may be
    // restaged) and, in ph3, tile t+1 visible.  Last reads of tile t's half-tiles: A0, B0 in ph3 of
    // tile t-1, B1 in ph0, A1 in ph1 -> tile t+2 restaged ph0: A0, ph1: B0, ph2: B1, ph3: A1 (each
    // at least one phase, i.e. one barrier, after the last read).  The ph3 wait leaves the three
    // half-tiles of t+2 issued in ph0-ph2 in flight.  The waves run a phase's MFMAs straight into
    // the next phase's barrier: the pipe is not drained by a second barrier behind them.
    auto tile4b = [&](int t, const char* buf, const char* nbuf, bf16x8_t (&b0)[2][2],
                      bf16x8_t (&b0n)[2][2]) __attribute__((always_inline)) {
#ifdef VS_G8_DIAG_NODMA     // timing diagnostics only (wrong results): no in-loop DMA / waits
        const bool more = false;
        if (nt < 0) t = 0;
#else
        const bool more = t + 2 < nt;
#endif
        // ph0: (A0, B0); restage A0 of t+2; prefetch B1
        bar_wait_lgkm_pre();
        if (more) stage(t + 2, 0);
        read_b(buf, R_B1, bf1);
        __builtin_amdgcn_sched_barrier(0);
        mfma16x(acc[0][0], af, b0);
        // ph1: (A0, B1); restage B0 of t+2; prefetch A1
        bar_wait_lgkm_pre();
        if (more) stage(t + 2, 2);
        read_a_to(buf, R_A1, ag);
        __builtin_amdgcn_sched_barrier(0);
        mfma16x(acc[0][1], af, bf1);
        // ph2: (A1, B1); restage B1 of t+2
        bar_wait_lgkm_pre();
        if (more) stage(t + 2, 3);
        __builtin_amdgcn_sched_barrier(0);
        mfma16x(acc[1][1], ag, bf1);
        // ph3: (A1, B0); retire tile t+1, restage A1 of t+2, prefetch A0 / B0 of t+1
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_waitcnt(0xC07F);                       // lgkmcnt(0)
        if (more)
            asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
#ifndef VS_G8_DIAG_NODMA
        else if (t + 1 < nt)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
        bar_wait_lgkm_pre();
        if (more) stage(t + 2, 1);
        if (t + 1 < nt) {
            read_a_to(nbuf, R_A0, af);
            read_b(nbuf, R_B0, b0n);
        }
        __builtin_amdgcn_sched_barrier(0);
        mfma16x(acc[1][0], ag, b0);
    };
    if constexpr (SCHED == 2) {
        read_a_to(smem, R_A0, af);
        read_b(smem, R_B0, bf0);
#pragma nounroll
        for (int t = 0; t < nt; t += 2) {
            tile4b(t, smem, smem + BUF8, bf0, bg0);
            if (t + 1 < nt) tile4b(t + 1, smem + BUF8, smem, bg0, bf0);
        }
    } else if constexpr (PRE) {
        read_a_to(smem, R_A0, af);
        read_b(smem, R_B0, bf0);
#pragma nounroll
        for (int t = 0; t < nt; t += 2) {
            tile4p(t, smem, smem + BUF8, bf0, bg0);
            if (t + 1 < nt) tile4p(t + 1, smem + BUF8, smem, bg0, bf0);
        }
    } else {
        if (STAG && wr == 1) bar();
#pragma nounroll
        for (int t = 0; t < nt; t += 2) {
            tile4(t, smem);
            if (t + 1 < nt) tile4(t + 1, smem + BUF8);
        }
        if (STAG && wr == 0) bar();
    }

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


typedef int i32x8_t __attribute__((ext_vector_type(8)));

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

template <bool STAG>     // STAG: the staggered schedule of gemm_bf16_tn_8p<false, 3>
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
    tile_of(pid, ntm, ntn, tm, tn);
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
    // row offsets formed per stage from two opaque VGPRs (see gemm_bf16_tn_8p)
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
    // the phase schedule and fragment prefetch of gemm_bf16_tn_8p<PRE>: each phase waits for the
    // fragments the previous one read, reads the next phase's new ones and runs its 4 MX MFMAs
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
    // STAG: reads at phase start, waves 4-7 one barrier behind waves 0-3 (see gemm_bf16_tn_8p
    // SCHED 3; A0 is restaged one phase after its ph0 reads, retired by lgkmcnt(4) before ph0's
    // first barrier: read_a issues its 8 reads before read_b's 4)
    auto tile4s = [&](int t, int b) __attribute__((always_inline)) {
        read_a(b, R_A0, af);
        __builtin_amdgcn_sched_barrier(0);
        read_b(b, R_B0, bf0);
        if (t + 1 < nt) stage(t + 1, 1);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_waitcnt(0xC47F);     // lgkmcnt(4)
        bar_wait_lgkm();
        mfma4(acc[0][0], af, bf0);
        bar();
        read_b(b, R_B1, bf1);
        if (t + 2 < nt) stage(t + 2, 0);
        bar_wait_lgkm();
        mfma4(acc[0][1], af, bf1);
        bar();
        read_a(b, R_A1, af);
        if (t + 2 < nt) stage(t + 2, 2);
        bar_wait_lgkm();
        mfma4(acc[1][1], af, bf1);
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
        mfma4(acc[1][0], af, bf0);
        bar();
    };
    if constexpr (STAG) {
        if (wr == 1) bar();
#pragma nounroll
        for (int t = 0; t < nt; t += 2) {
            tile4s(t, 0);
            if (t + 1 < nt) tile4s(t + 1, 1);
        }
        if (wr == 0) bar();
    } else {
        read_a(0, R_A0, af);
        read_b(0, R_B0, bf0);
#pragma nounroll
        for (int t = 0; t < nt; t += 2) {
            tile4p(t, 0, bf0, bg0);
            if (t + 1 < nt) tile4p(t + 1, 1, bg0, bf0);
        }
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
// 256x256 tile, 4 waves (one per SIMD), 128x128 output per wave: the accumulators (256 fp32 per
// lane) live in AGPRs, which the MFMAs read and write directly, so a wave owns 64 MFMAs
// (16x16x32) per 32-deep K half-step against 16 fragment reads (vs 32 against 12 in the 8-wave
// ping-pong kernel).  Same LDS ring (RING x 32 KB slots, LDS-DMA three half-steps ahead, 64-B rows,
// chunk swizzle) as gemm_bf16_tn_256.  Per half-step h, every wave runs
//   [vmcnt: own DMA of h+1 landed; s_barrier] [DMA h+RING-1 -> slot of h-1] [frags(h+1) -> other
//   register set] [64 MFMAs(h)]
// one barrier per half-step: passing it proves (a) every wave's pieces of h+1 have landed (RAW)
// and (b) every wave has consumed frags(h-1) (their lgkmcnt wait precedes MFMAs(h-1)), so slot
// (h-1) % RING is free for the DMA issued right after it (WAR).
// ---------------------------------------------------------------------------------------------
constexpr int NTHR4 = 256;

__global__ __launch_bounds__(NTHR4, 1) void gemm_bf16_tn_w4(
    const bf16_t* __restrict__ A, long long lda, const bf16_t* __restrict__ W, long long ldw,
    bf16_t* C, long long ldc, int M, int N, int K, const bf16_t* __restrict__ A2, long long lda2,
    const bf16_t* __restrict__ W2, long long ldw2, int K2, Epi ep, int ntm, int ntn) {
    extern __shared__ __attribute__((aligned(16))) char smem[];

    const int pid = xcd_remap(blockIdx.x, gridDim.x);
    constexpr int GM = VS_GEMM_GM;
    const int per_group = GM * ntn;
    const int group = pid / per_group;
    const int first_m = group * GM;
    const int gsz = min(ntm - first_m, GM);
    const int in_g = pid % per_group;
    const int tm = first_m + in_g % gsz;
    const int tn = in_g / gsz;
    const int m0 = tm * BT, n0 = tn * BT;

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 1, wn = wave & 1;

    f32x4_t acc[8][8];

    // LDS-DMA: a half-step is 32 pieces of 1 KB (16 rows x 64 B); wave w issues A rows
    // 64w..64w+63 (pieces 4w..4w+3 of the A half) and W rows 64w..64w+63.  Lane L -> row
    // 16j + L/4 of its piece, physical chunk L%4, logical chunk (L%4) ^ ((3*((L/4)>>2))&3).
    const int prow = lane >> 2;
    const int pch = (lane & 3) ^ ((3 * (prow >> 2)) & 3);
    const int nh1 = K / HK;
    const int nh = nh1 + K2 / HK;
    const int arow = m0 + wave * 64 + prow, wrow = n0 + wave * 64 + prow;
    const int alim = M - 1, wlim = N - 1;
    // buffer-addressed DMA (host guarantees every byte offset fits 32 bits): the per-lane row
    // offsets are 8 loop-invariant VGPRs, the K offset of a half-step goes to soffset
    auto rsrc = [](const void* base) {
        return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
    };
    const __amdgpu_buffer_rsrc_t ra = rsrc(A), rw = rsrc(W);
    unsigned voa[4], vow[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        voa[j] = (unsigned)min(arow + j * 16, alim) * (unsigned)(lda * 2) + pch * 16;
        vow[j] = (unsigned)min(wrow + j * 16, wlim) * (unsigned)(ldw * 2) + pch * 16;
    }
    int issued = -1;
    auto issue = [&](int h) {
        char* dst = smem + (h % RING) * SLOT + wave * 4 * 1024;
        if (h < nh1) {
            const unsigned ko = (unsigned)h * HK * 2;
#pragma unroll
            for (int j = 0; j < 4; ++j)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (LDS_AS void*)(dst + j * 1024), 16, voa[j], ko, 0, 0);
#pragma unroll
            for (int j = 0; j < 4; ++j)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (LDS_AS void*)(dst + BT * 64 + j * 1024), 16, vow[j], ko,
                                                         0, 0);
        } else {
            // second K phase (un-merged LoRA): A2 . W2^T
            const unsigned ko = (unsigned)(h - nh1) * HK * 2;
            const __amdgpu_buffer_rsrc_t ra2 = rsrc(A2), rw2 = rsrc(W2);
#pragma unroll
            for (int j = 0; j < 4; ++j)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    ra2, (LDS_AS void*)(dst + j * 1024), 16,
                    (unsigned)min(arow + j * 16, alim) * (unsigned)(lda2 * 2) + pch * 16, ko, 0, 0);
#pragma unroll
            for (int j = 0; j < 4; ++j)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    rw2, (LDS_AS void*)(dst + BT * 64 + j * 1024), 16,
                    (unsigned)min(wrow + j * 16, wlim) * (unsigned)(ldw2 * 2) + pch * 16, ko, 0, 0);
        }
        issued = h;
    };
    // barrier after this wave's DMA of half-step `need` has landed (8 pieces per half-step)
    auto bar_for = [&](int need) {
        const int after = issued - need;
        __builtin_amdgcn_sched_barrier(0);
        if (after >= 2)
            asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
        else if (after == 1)
            asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
        else
            asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
    };

    const int frow = lane & 15, fch = lane >> 4;
    auto read_frags = [&](int h, bf16x8_t* af, bf16x8_t* wf) {
        const char* As = smem + (h % RING) * SLOT;
        const char* Bs = As + BT * 64;
#pragma unroll
        for (int j = 0; j < 8; ++j)
            wf[j] = *reinterpret_cast<const bf16x8_t*>(Bs + h_off(wn * 128 + j * 16 + frow, fch));
#pragma unroll
        for (int i = 0; i < 8; ++i)
            af[i] = *reinterpret_cast<const bf16x8_t*>(As + h_off(wm * 128 + i * 16 + frow, fch));
    };
    // accumulators pinned to AGPRs ("+a"), fragments in VGPRs: left to itself hipcc splits the
    // 512-register file badly (fragments in AGPRs, ~1200 accvgpr copies and 355 spilled registers)
    // accumulators live in AGPRs ("+a"; born there from the srcC = 0 form of the first half-step),
    // fragments and addresses in VGPRs.  Left to itself hipcc splits the 512-register file badly
    // (fragments in AGPRs and ~1200 accvgpr copies per tile, or accumulators spilled to AGPRs).
    auto mfmas = [&](const bf16x8_t* af, const bf16x8_t* wf) {
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 8; ++j)
                asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[i][j]) : "v"(wf[j]), "v"(af[i]));
    };
    auto mfmas_first = [&](const bf16x8_t* af, const bf16x8_t* wf) {
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 8; ++j)
                asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(acc[i][j]) : "v"(wf[j]), "v"(af[i]));
    };

    bf16x8_t a0[8], w0[8], a1[8], w1[8];
#pragma unroll
    for (int j = 0; j < RING - 1; ++j)
        if (j < nh) issue(j);
    bar_for(0);
    read_frags(0, a0, w0);
    // half-step 0 (peeled: it creates the accumulators)
    if (1 < nh) bar_for(1);
    if (RING - 1 < nh) issue(RING - 1);
    if (1 < nh) read_frags(1, a1, w1);
    mfmas_first(a0, w0);
    for (int h = 1; h < nh; h += 2) {
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const int hc = h + e;
            if (hc >= nh) break;
            if (hc + 1 < nh) bar_for(hc + 1);
            if (hc + RING - 1 < nh) issue(hc + RING - 1);
            if (e == 0) {
                if (hc + 1 < nh) read_frags(hc + 1, a0, w0);
                mfmas(a1, w1);
            } else {
                if (hc + 1 < nh) read_frags(hc + 1, a1, w1);
                mfmas(a0, w0);
            }
        }
    }

    // the last inline-asm MFMAs' results are read by VALU (accvgpr reads): the hazard recognizer
    // does not see through inline asm, so wait out the 16x16x32 pipeline explicitly
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int m = m0 + wm * 128 + i * 16 + (lane & 15);
        if (m >= M) continue;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int n = n0 + wn * 128 + j * 16 + 4 * (lane >> 4);
            if (n >= N) continue;
            epilogue_store(acc[i][j], m, n, C, ldc, ep);
        }
    }
}


// ---------------------------------------------------------------------------------------------
// gemm_bf16_tn_w4r: 256x256x64 tile, 4 waves = one per SIMD, 128x128 output per wave (2 x 2 waves),
// accumulators (256 fp32 per lane) in AGPRs, operands REGISTER-staged: each K-tile's A and W rows
// arrive by buffer_load_dwordx4 into 16 staging VGPR quads per wave and are written to LDS by
// ds_write_b128 one K-tile later.  Why not LDS-DMA as the 8-wave kernels: a wave alone on its SIMD
// issues its own DMA between its own MFMAs, and a DMA piece costs ~60 issue cycles there
// (MI355X_MICROARCH 'LDS-DMA piece issue cost'): 16 pieces per K-tile are ~960 of the 2048 MFMA
// cycles, which is what held the r2 one-wave kernel (DMA-staged) at 845-902 TF/s.
//
// LDS: two buffers (K-tile parity) of [A 256 x 128 B | W 256 x 128 B], 16-B chunk c of row r at
// q_off(r, c) = r * 128 + 16 (c ^ (r & 7)) (the 8-phase kernel's conflict-free image).  Per K-tile t
// (buffer b = t & 1; staging regs hold tile t+1, loaded during tile t-1):
//   S0: 64 MFMAs on the k 0..31 fragments f0 | reads of the k 32..63 fragments f1 (buffer b) |
//       ds_write of tile t+1 (staging regs -> buffer b^1) | loads of tile t+2 (-> staging regs)
//   lgkmcnt(0); s_barrier            (tile t+1 in LDS for every wave; buffer b's f1 reads retired)
//   S1: 64 MFMAs on f1 | reads of tile t+1's f0 (buffer b^1)
// One barrier per K-tile.  WAR: buffer b^1 was last read for tile t-1's f1, issued in tile t-1's S0
// and retired before tile t-1's barrier, which every wave passes before tile t's writes.  RAW: the
// writes of tile t+1 retire (lgkmcnt) before tile t's barrier, the reads of tile t+1 come after it.
// Product D[n][m] = W . A^T (16x16x32, W fragment as the A operand), as gemm_bf16_tn_8p.
// ---------------------------------------------------------------------------------------------
constexpr int W4R_THR = 256, W4R_LDS = 2 * 2 * 256 * 128;     // 128 KB

__global__ __launch_bounds__(W4R_THR, 1) void gemm_bf16_tn_w4r(
    const bf16_t* __restrict__ A, long long lda, const bf16_t* __restrict__ W, long long ldw,
    bf16_t* C, long long ldc, int M, int N, int K, Epi ep, int ntm, int ntn, int nmain, int ksplit,
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
    tile_of(pid, ntm, ntn, tm, tn);
    const int m0 = tm * 256, n0 = tn * 256;
    const int kb = piece < 0 ? 0 : piece * piece_k;
    const int Kp = piece < 0 ? K : min(K - kb, piece_k);
    const int nt = Kp / 64;

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 1, wn = wave & 1;

    // loader: wave w moves rows 64w .. 64w+63 of the A tile and of the W tile, 8 rows (1 KB) per
    // instruction: lane L -> row 64w + 8j + (L >> 3), 16-B chunk L & 7 of the K-tile's 128 B.  The
    // descriptors are rebased on the tile's first row and end after its last valid row, so rows past
    // M / N load zeros (their products are dropped): no per-lane branch around any load (a
    // lane-dependent select there makes hipcc wrap each load in an exec branch).  Row step 8j goes to
    // soffset.
    const int alim = M - 1 - m0, wlim = N - 1 - n0;
    auto rsrc_n = [](const void* base, long long bytes) {
        return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0,
                                                 (int)min(bytes, (long long)0x7fffffff), 0x00020000);
    };
    const __amdgpu_buffer_rsrc_t ra = rsrc_n(A + (long long)m0 * lda + kb, (long long)alim * lda * 2 + (long long)Kp * 2);
    const __amdgpu_buffer_rsrc_t rw = rsrc_n(W + (long long)n0 * ldw + kb, (long long)wlim * ldw * 2 + (long long)Kp * 2);
    const int lrow = 64 * wave + (lane >> 3), lch = lane & 7;
    const unsigned goa = (unsigned)lrow * (unsigned)(lda * 2) + 16u * lch;
    const unsigned gow = (unsigned)lrow * (unsigned)(ldw * 2) + 16u * lch;
    const unsigned ga_step = 8u * (unsigned)(lda * 2), gw_step = 8u * (unsigned)(ldw * 2);
    u32x4_t st[16];
    auto load_q = [&](int q, int t) __attribute__((always_inline)) {
        const unsigned ko = (unsigned)t * 128u;
        const int j = q & 7;
        st[q] = __builtin_bit_cast(u32x4_t, q < 8 ? __builtin_amdgcn_raw_buffer_load_b128(ra, goa, ko + j * ga_step, 0)
                                                  : __builtin_amdgcn_raw_buffer_load_b128(rw, gow, ko + j * gw_step, 0));
    };
    auto load_tile = [&](int t) __attribute__((always_inline)) {
#pragma unroll
        for (int q = 0; q < 16; ++q) load_q(q, t);
    };
    // LDS destinations of the staging quads: row 64w + 8j + (L >> 3), chunk L & 7 (swizzled)
    const unsigned sbase = (unsigned)(uintptr_t)smem;
    const unsigned wdst = (unsigned)q_off(lrow, lch);        // (lrow + 8j) & 7 == lrow & 7
    auto write_q = [&](int b, int q) __attribute__((always_inline)) {
        const unsigned addr = sbase + b * 65536 + (q >= 8 ? 32768 : 0) + wdst + (q & 7) * 1024;
        *reinterpret_cast<LDS_AS u32x4_t*>((LDS_AS char*)(uintptr_t)addr) = st[q];
    };
    // fragments: A rows wm*128 + 16i + (L & 15), W rows wn*128 + 16j + (L & 15); k-half s = 0, 1:
    // chunk 4s + (L >> 4)
    const int frow = lane & 15, fch = lane >> 4;
    unsigned fa[2], fw[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        fa[s] = sbase + (unsigned)q_off(wm * 128 + frow, 4 * s + fch);
        fw[s] = sbase + 32768u + (unsigned)q_off(wn * 128 + frow, 4 * s + fch);
    }
    auto rd = [&](unsigned addr) {
        return *reinterpret_cast<const LDS_AS bf16x8_t*>((const LDS_AS char*)(uintptr_t)addr);
    };
    f32x4_t acc[8][8];
    bf16x8_t a0[8], w0[8], a1[8], w1[8];
    auto fence = [] { __builtin_amdgcn_sched_barrier(0); };
    auto mf = [&](f32x4_t& c, const bf16x8_t& w, const bf16x8_t& a, bool first) __attribute__((always_inline)) {
        if (first)
            asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(c) : "v"(w), "v"(a));
        else
            asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(w), "v"(a));
    };

    // prologue: tile 0 -> regs -> LDS buffer 0, tile 1 -> regs, barrier, f0 of tile 0
    load_tile(0);
#pragma unroll
    for (int q = 0; q < 16; ++q) write_q(0, q);
    load_tile(min(1, nt - 1));
    fence();
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    fence();
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        a0[i] = rd(fa[0] + 2048 * i);
        w0[i] = rd(fw[0] + 2048 * i);
    }
    auto ktile = [&](int t, bool first) __attribute__((always_inline)) {
        const unsigned bo = (unsigned)(t & 1) * 65536u, bn = bo ^ 65536u;
        // S0: row block i of f0 x the 8 column blocks; fillers: f1 reads (steps 0-3), writes of tile
        // t+1 and loads of tile t+2 (steps 4-7, each quad written before it is reloaded).  Past the
        // last K-tile the writes land in the idle buffer and the loads re-read the last tile:
        // branch-free
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (i < 4) {       // the W fragments first (S1's first step needs all of them)
#pragma unroll
                for (int u = 0; u < 2; ++u) w1[2 * i + u] = rd(fw[1] + bo + 2048 * (2 * i + u));
#pragma unroll
                for (int u = 0; u < 2; ++u) a1[2 * i + u] = rd(fa[1] + bo + 2048 * (2 * i + u));
            } else {
#pragma unroll
                for (int u = 0; u < 4; ++u) write_q(bn >> 16, 4 * (i - 4) + u);
#pragma unroll
                for (int u = 0; u < 4; ++u) load_q(4 * (i - 4) + u, min(t + 2, nt - 1));
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) mf(acc[i][j], w0[j], a0[i], first);
            fence();
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        fence();
        // S1: f1; fillers: tile t+1's f0 reads (buffer b^1): the W fragments, which the next S0's
        // first step needs all of, in steps 0-3, the A fragments (one per next-S0 step) in steps 4-7
#pragma unroll
        for (int i = 0; i < 8; ++i) {
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                if (i < 4)
                    w0[2 * i + u] = rd(fw[0] + bn + 2048 * (2 * i + u));
                else
                    a0[2 * (i - 4) + u] = rd(fa[0] + bn + 2048 * (2 * (i - 4) + u));
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) mf(acc[i][j], w1[j], a1[i], false);
            fence();
        }
    };
    ktile(0, true);
#pragma nounroll
    for (int t = 1; t < nt; ++t) ktile(t, false);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");     // the last prefetch (a re-read) has landed

    // the last inline-asm MFMAs' results are read by VALU (accvgpr reads): the hazard recognizer
    // does not see through inline asm, so wait out the 16x16x32 pipeline explicitly
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
    // acc[i][j][e] = C[m][n], m = m0 + 128 wm + 16 i + (L & 15), n = n0 + 128 wn + 16 j + 4 (L >> 4) + e
    if (piece >= 0) {
        float* pp = part + ((long long)(pid - nmain) * ksplit + piece) * 256 * 256;
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 8; ++j)
                *reinterpret_cast<f32x4_t*>(pp + (128 * wm + 16 * i + frow) * 256 + 128 * wn + 16 * j + 4 * fch) =
                    acc[i][j];
        return;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int m = m0 + 128 * wm + 16 * i + frow;
        if (m >= M) continue;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int n = n0 + 128 * wn + 16 * j + 4 * fch;
            if (n >= N) continue;
            epilogue_store(acc[i][j], m, n, C, ldc, ep);
        }
    }
}


// ---------------------------------------------------------------------------------------------
// fp8 e4m3 (OCP) GEMM for the fp8 path (config 5; AutoWrappedLinear.fp8_linear,
// diffsynth/vram_management/layers.py:115-151): C = epilogue(scale_a[m] * (A8 . W8^T)) with the
// activations quantised per row by vs_quant_fp8_rows and unscaled fp8 weights (scale_b = 1).
// Same 256x256 ping-pong skeleton as gemm_bf16_tn_256: a slot row holds 64 fp8 (64 B), so the
// LDS ring, LDS-DMA pieces and swizzle are unchanged; each half-step is 8 MX-rate
// v_mfma_scale_f32_32x32x64_f8f6f4 per wave (unit E8M0 scales) = twice the bf16 FLOPs in the same
// MFMA cycles.  The product is formed transposed (D[n][m] = W8 . A8^T) so each lane owns 4
// consecutive output columns per register group and the bf16 epilogue is reused unchanged.
// ---------------------------------------------------------------------------------------------

template <bool BUF>
__global__ __launch_bounds__(NTHR8, 2) void gemm_fp8_tn_256(
    const uint8_t* __restrict__ A, long long lda, const float* __restrict__ scale_a,
    const uint8_t* __restrict__ W, long long ldw, bf16_t* C, long long ldc, int M, int N, int K, Epi ep,
    int ntm, int ntn) {
    extern __shared__ __attribute__((aligned(16))) char smem[];

    const int pid = xcd_remap(blockIdx.x, gridDim.x);
    constexpr int GM = VS_GEMM_GM;
    const int per_group = GM * ntn;
    const int group = pid / per_group;
    const int first_m = group * GM;
    const int gsz = min(ntm - first_m, GM);
    const int in_g = pid % per_group;
    const int tm = first_m + in_g % gsz;
    const int tn = in_g / gsz;
    const int m0 = tm * BT, n0 = tn * BT;

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 2, wn = wave & 3;

    f32x16_t acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int prow = lane >> 2;
    const int pch = (lane & 3) ^ ((3 * (prow >> 2)) & 3);
    constexpr int HB = 64;                            // fp8 per half-step = bytes per slot row
    const int nh = K / HB;
    const uint8_t* P = wm == 0 ? A : W;
    const long long ld = wm == 0 ? lda : ldw;
    const int lim = (wm == 0 ? M : N) - 1;
    const int r0 = wm == 0 ? m0 : n0;
    const int dst_off = wm * (BT * 64) + wn * 4 * 1024;
    const int rbase = r0 + wn * 64 + prow;
    int issued = -1;
    // BUF: buffer-addressed DMA with loop-invariant 32-bit row offsets (see gemm_bf16_tn_256)
    unsigned vo[4] = {0, 0, 0, 0};
    const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(P), 0, 0x7fffffff,
                                                                        0x00020000);
    if constexpr (BUF) {
#pragma unroll
        for (int j = 0; j < 4; ++j) vo[j] = (unsigned)min(rbase + j * 16, lim) * (unsigned)ld + pch * 16;
    }
    auto issue = [&](int h) {
        char* dst = smem + (h % RING) * SLOT + dst_off;
        if constexpr (BUF) {
#pragma unroll
            for (int j = 0; j < 4; ++j)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rp, (LDS_AS void*)(dst + j * 1024), 16, vo[j],
                                                         (unsigned)h * HB, 0, 0);
        } else {
            const uint8_t* src = P + (long long)h * HB + pch * 16;
#pragma unroll
            for (int j = 0; j < 4; ++j)
                __builtin_amdgcn_global_load_lds((const GLB_AS void*)(src + (long long)min(rbase + j * 16, lim) * ld),
                                                 (LDS_AS void*)(dst + j * 1024), 16, 0, 0);
        }
        issued = h;
    };

    // fragments: lane (r = l&31, hf = l>>5) holds row r, k = 32 hf .. 32 hf + 31 (chunks 2hf, 2hf+1)
    const int fr = lane & 31, fh = lane >> 5;
    i32x8_t wfr[2], afr[4];
    auto load_frags = [&](int h) {
        const char* As = smem + (h % RING) * SLOT;
        const char* Bs = As + BT * 64;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int row = wn * 64 + j * 32 + fr;
            const u32x4_t lo = *reinterpret_cast<const u32x4_t*>(Bs + h_off(row, 2 * fh));
            const u32x4_t hi = *reinterpret_cast<const u32x4_t*>(Bs + h_off(row, 2 * fh + 1));
            wfr[j] = i32x8_t{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int row = wm * 128 + i * 32 + fr;
            const u32x4_t lo = *reinterpret_cast<const u32x4_t*>(As + h_off(row, 2 * fh));
            const u32x4_t hi = *reinterpret_cast<const u32x4_t*>(As + h_off(row, 2 * fh + 1));
            afr[i] = i32x8_t{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
        }
    };
    auto mfmas = [&]() {
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(wfr[j], afr[i], acc[i][j], 0, 0, 0, 0x7f,
                                                                           0, 0x7f);
        __builtin_amdgcn_s_setprio(0);
    };

#pragma unroll
    for (int j = 0; j < RING - 1; ++j)
        if (j < nh) issue(j);
    wait_barrier(issued);
    int q = 0;
    auto bar = [&]() {
        wait_barrier(issued - min((q + 1) >> 1, nh - 1));
        ++q;
    };
    if (wm == 1) bar();
#pragma nounroll
    for (int h = 0; h < nh; ++h) {
        load_frags(h);
        if (h + RING - 1 < nh) issue(h + RING - 1);
        bar();
        mfmas();
        bar();
    }
    if (wm == 0) bar();

    // D[n][m]: lane column m = m0 + wm*128 + 32i + (l&31); rows n = n0 + wn*64 + 32j + 8g + 4hf + {0..3}
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int m = m0 + wm * 128 + i * 32 + fr;
        if (m >= M) continue;
        const float sa = scale_a[m];
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int n = n0 + wn * 64 + j * 32 + 8 * g + 4 * fh;
                if (n >= N) continue;
                const f32x4_t a = f32x4_t{acc[i][j][4 * g] * sa, acc[i][j][4 * g + 1] * sa, acc[i][j][4 * g + 2] * sa,
                                          acc[i][j][4 * g + 3] * sa};
                epilogue_store(a, m, n, C, ldc, ep);
            }
    }
}

// Per-row activation quantisation of fp8_linear (layers.py:124-137): s = max(bf16(max|x| / 448), 1)
// (the reference divides and clamps the bf16 row max, so the quotient is rounded to bf16 before the
// clamp), x8 = e4m3(x / (s + 1e-8)) (fp32 division, round-to-nearest-even), one wave per row.
__global__ __launch_bounds__(256) void quant_fp8_rows_kernel(const bf16_t* __restrict__ x, long long ldx,
                                                             uint8_t* __restrict__ x8, long long ld8,
                                                             float* __restrict__ scale, int rows, int cols) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= rows) return;
    const bf16_t* xr = x + (long long)row * ldx;
    float mx = 0.f;
    for (int c = lane * 8; c < cols; c += 512) {
        const u32x4_t w = *reinterpret_cast<const u32x4_t*>(xr + c);
#pragma unroll
        for (int e = 0; e < 4; ++e) mx = fmaxf(mx, fmaxf(fabsf(bflo(w[e])), fabsf(bfhi(w[e]))));
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    const float s = fmaxf(rbf(mx / 448.0f), 1.0f);
    const float d = s + 1e-8f;
    if (lane == 0) scale[row] = s;
    uint8_t* yr = x8 + (long long)row * ld8;
    for (int c = lane * 8; c < cols; c += 512) {
        const u32x4_t w = *reinterpret_cast<const u32x4_t*>(xr + c);
        u32x2_t o;
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            int v = __builtin_amdgcn_cvt_pk_fp8_f32(bflo(w[2 * e]) / d, bfhi(w[2 * e]) / d, 0, false);
            v = __builtin_amdgcn_cvt_pk_fp8_f32(bflo(w[2 * e + 1]) / d, bfhi(w[2 * e + 1]) / d, v, true);
            o[e] = (uint32_t)v;
        }
        *reinterpret_cast<u32x2_t*>(yr + c) = o;
    }
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }
bool aligned8(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 7) == 0; }

}  // namespace

#ifdef VS_GEMM_STAMPS
extern "C" int vs_debug_gemm_stamps(unsigned long long* host_out) {
    return hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_gemm_stamps), sizeof(g_gemm_stamps)) == hipSuccess ? 0 : 2;
}
#endif

// Split tail.  One 256x256 workgroup fills a CU, so a grid of T tiles runs in ceil(T / CUs)
// rounds and the last, partial one leaves CUs idle: the 14B N=5120 GEMMs on 2 x 29640 tokens are
// 4640 tiles = 18.1 rounds on 256 CUs, and under Ulysses SP=8 (7410 rows) 580 tiles = 2.27.  The
// last T % CUs tiles instead run as ksplit K ranges each (fp32 partial tiles in a caller-bound
// per-(device, stream) workspace, then one combine launch that applies the epilogue), ksplit
// chosen by the measured cost model below.
constexpr int MAX_SPLIT_PIECES = 512;        // 512 x 256 KB fp32 partial tiles
struct KSplit { int nmain = 0, ntail = 0, ksplit = 1, piece_k = 0; };

KSplit plan_ksplit(int ntiles, int nh, int cus, int step = HK) {
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

// Which GEMMs go to hipBLASLt (VS_GEMM_BACKEND=vstyler|lt overrides).  Measured per block GEMM
// of the 14B model with its real epilogue (profiles/r1/gemm_backend_ab_r1g.log): at 2 x 29640 rows
// (4640-13920 tiles of 256^2) hipBLASLt + epilogue pass is 1.14-1.35x the MFMA kernels on all six,
// staged gate-residual / residual included; at the SP=8 row count (7410) it wins only the >= 1566-
// tile GEMMs (qkv 1.12x, FFN-up 1.05x) and loses the 580-tile ones (0.85-0.97x).  So: hipBLASLt
// when the grid holds >= 1024 tiles (4 full rounds on 256 CUs), at any K (the 1.3B model's K = 1536
// GEMMs: 1217-1300 TF/s against 707-797 on the 128^2 kernel, profiles/r1/gemm_bench_r1f.log).
// hipBLASLt (autotuned per shape, blaslt.hip) vs the 256^2 MFMA kernel with its split tail, measured
// per 14B block GEMM (profiles/r1/gemm_lt_tune_r1i.log, gemm_backend_ab_r1j.log): hipBLASLt wins on
// every grid of >= 1024 256^2 tiles, and on 256-1023-tile grids (the SP=8 row counts 7410 and, per
// CFG micro-batch, 3705) while K <= 8192 (1.01-1.32x); the K = 13824 FFN-down GEMM at those sizes
// stays on the MFMA kernel (0.88-0.96x on hipBLASLt).  Grids of < 256 tiles with N >= 2048 and
// 1024 <= K <= 8192 -- the per-step context GEMMs (fused cross k|v over 2 x 512 context rows, text
// embedding), the time projection (M = 2) and the UMT5 layers -- also go to hipBLASLt: 1.05-2.4x
// the 128^2 kernel (profiles/r1/gemm_backend_ab_ctx_r1s.log); the narrow head (N = 64) and the
// patch embeddings (K = 64 / 384) are unmeasured there and stay on the MFMA kernels.
// r2: on the private ROCm-7.2 hipBLASLt copy (blaslt.hip) the K = 13824 FFN-down at 3705 rows runs
// at 0.404-0.411 ms against 0.466-0.474 on the MFMA kernel (profiles/r2/lt_lib_ab_r2l.log), so with
// that library the 256-1023-tile grids go to hipBLASLt at any K.
bool vs_lt_is_private();
static bool lt_route(int m, int n, int k) {
    const char* e = getenv("VS_GEMM_BACKEND");
    const int mode = !e ? 2 : (e[0] == 'v' ? 0 : (e[0] == 'l' ? 1 : 2));   // 0 never, 1 always, 2 auto
    if (mode != 2) return mode == 1;
    const long long tiles = (long long)((m + 255) / 256) * ((n + 255) / 256);
    return tiles >= 1024 || (tiles >= 256 && (k <= 8192 || vs_lt_is_private())) ||
           (k <= 8192 && n >= 2048 && k >= 1024);
}

// hipBLASLt for bf16(A W^T [* scale] + bias) (gemm(y, ldy)), then the rest of the epilogue with
// the fused kernels' code (see blaslt.hip).  false: no workspace bound or hipBLASLt declined the
// shape -- the caller falls through to the MFMA kernels.
template <class Gemm>
static bool lt_with_epilogue(void* c, long long ldc, int m, int n, int epilogue, const Epi& ep, hipStream_t stream,
                             Gemm gemm) {
    const bool staged = epilogue == VS_EPI_GATE_RES || epilogue == VS_EPI_RES;
    bf16_t* y = (bf16_t*)c;
    long long ldy = ldc;
    if (staged) {
        y = (bf16_t*)vs_split_workspace(3, (size_t)m * n * 2, stream);
        ldy = n;
    }
    if (!y || gemm((void*)y, ldy) != VS_OK) return false;
    if (epilogue != VS_EPI_BIAS) {
        Epi e2 = ep;
        e2.bias = nullptr;
        const bool w8 = n % 8 == 0 && ldy % 8 == 0 && ldc % 8 == 0 && aligned16(y) && aligned16(c) &&
                        (!e2.res || (e2.ld_res % 8 == 0 && aligned16(e2.res))) &&
                        (!e2.gate || (e2.gate_bstride % 8 == 0 && aligned16(e2.gate))) &&
                        (!e2.hint || (e2.ld_hint % 8 == 0 && aligned16(e2.hint)));
        if (w8) {
            hipLaunchKernelGGL(gemm_epi_apply8, dim3((unsigned)m, (unsigned)((n / 8 + 255) / 256)), dim3(256), 0,
                               stream, y, ldy, (bf16_t*)c, ldc, n, e2);
        } else {
            const long long threads = (long long)m * (n / 4);
            hipLaunchKernelGGL(gemm_epi_apply, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, stream, y, ldy,
                               (bf16_t*)c, ldc, m, n, e2);
        }
        if (hipGetLastError() != hipSuccess) return false;
    }
    return true;
}

static int fill_epi(Epi& ep, int epilogue, const vs_epilogue* epi, int m, int n) {
    if (epilogue < VS_EPI_BIAS || epilogue > VS_EPI_RES) return VS_E_INVALID;
    ep = Epi{};
    ep.mode = epilogue;
    ep.rows_per_batch = m;
    ep.alpha = 1.f;
    ep.hint_scale = 1.f;
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
    // 256x256 schedule once there are enough tiles to fill the chip, 128x128 otherwise
    // (VSTYLER_GEMM_TILE=128|256 forces one for A/B measurements)
    const char* tile_env = getenv("VSTYLER_GEMM_TILE");
    const int force = tile_env ? atoi(tile_env) : 0;
    const bool big = force ? force == 256
                          : k >= 4096 && (long long)((m + BT - 1) / BT) * ((n + BT - 1) / BT) >= 240;
    // GELU on the hipBLASLt route: the library's fused GELU_BIAS epilogue (GELU-tanh of the fp32
    // acc + bias, one bf16 rounding) instead of bf16(acc + bias) + the gemm_epi_apply8 GELU pass: the
    // 14B FFN-up 6.18 -> 5.79 ms (profiles/r2/lt_gelu_ab.log).  It drops the reference's bf16 rounding
    // of the linear output before F.gelu: 35 % of outputs move by one bf16 ulp, closer to the exact
    // GELU (0.8 % off its rounding vs 35 %).  Off by default (r3): the default keeps the reference's
    // rounding points (bf16 linear output, then the GELU pass); VS_LT_GELU=1 selects the fused epilogue.
    const char* lt_gelu = getenv("VS_LT_GELU");
    if (k2 == 0 && epilogue == VS_EPI_GELU && (lt_gelu && lt_gelu[0] == '1') && lt_route(m, n, k) &&
        vs_lt_gemm_bias_gelu(a, lda, w, ldw, c, ldc, m, n, k, ep.bias, (hipStream_t)stream) == VS_OK)
        return VS_OK;
    if (k2 == 0 && lt_route(m, n, k) &&
        lt_with_epilogue(c, ldc, m, n, epilogue, ep, (hipStream_t)stream, [&](void* y, long long ldy) {
            return vs_lt_gemm_bias(a, lda, w, ldw, y, ldy, m, n, k, ep.bias, (hipStream_t)stream);
        }))
        return VS_OK;
    if (big) {
        const int tm = (m + BT - 1) / BT, tn = (n + BT - 1) / BT;
        static int impl = -1;
        if (impl < 0) {
            (void)hipFuncSetAttribute((const void*)gemm_bf16_tn_256<true>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, RING * SLOT);
            (void)hipFuncSetAttribute((const void*)gemm_bf16_tn_256<false>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, RING * SLOT);
            (void)hipFuncSetAttribute((const void*)gemm_bf16_tn_w4,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, RING * SLOT);
            const char* e = getenv("VS_GEMM_IMPL");     // 4: one-wave-per-SIMD kernel (A/B)
            impl = (e && e[0] == '4') ? 4 : 8;
        }
        const bool fits32 = (long long)(m - 1) * lda * 2 + (long long)k * 2 < 0x7fffffffLL &&
                            (long long)(n - 1) * ldw * 2 + (long long)k * 2 < 0x7fffffffLL &&
                            (k2 == 0 || ((long long)(m - 1) * lda2 * 2 + (long long)k2 * 2 < 0x7fffffffLL &&
                                         (long long)(n - 1) * ldw2 * 2 + (long long)k2 * 2 < 0x7fffffffLL));
        if (impl == 4 && fits32) {
            hipLaunchKernelGGL(gemm_bf16_tn_w4, dim3((unsigned)(tm * tn)), dim3(NTHR4), RING * SLOT,
                               (hipStream_t)stream, (const bf16_t*)a, lda, (const bf16_t*)w, ldw,
                               (bf16_t*)c, ldc, m, n, k, (const bf16_t*)a2, lda2, (const bf16_t*)w2, ldw2,
                               k2, ep, tm, tn);
            VS_CHECK_LAUNCH();
            return VS_OK;
        }
        static bool attr8 = false;
        if (!attr8) {
            for (const void* f : {(const void*)gemm_bf16_tn_8p<false, 0>, (const void*)gemm_bf16_tn_8p<true, 0>,
                                  (const void*)gemm_bf16_tn_8p<false, 1>, (const void*)gemm_bf16_tn_8p<false, 2>,
                                  (const void*)gemm_bf16_tn_8p<false, 3>})
                (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, LDS8);
            attr8 = true;
        }
        // VS_GEMM_IMPL (A/B only): pp = the r2 ping-pong kernel, 8p = the 8-phase kernel without the
        // fragment prefetch; default: 8-phase with prefetch
        const char* impl_env = getenv("VS_GEMM_IMPL");
        const bool pp = impl_env && impl_env[0] == 'p' && impl_env[1] == 'p';
        // 8p: reads at phase start; pre: fragment prefetch, two barriers per phase; default: 1b
        const int sched = (impl_env && impl_env[0] == '8') ? 0 : (impl_env && impl_env[0] == 'p') ? 1
                        : (impl_env && impl_env[0] == 's') ? 3 : (impl_env && impl_env[0] == 'r') ? 4 : 2;
        if (!pp) {
            KSplit sp = k2 ? KSplit{tm * tn, 0, 1, 0}
                           : plan_ksplit(tm * tn, k / 64, vs_cus_for_split("VS_GEMM_NO_SPLIT"), 64);
            float* part = nullptr;
            if (sp.ntail) {
                part = vs_split_workspace(1, (size_t)sp.ntail * sp.ksplit * BT * BT * sizeof(float), (hipStream_t)stream);
                if (!part) sp = KSplit{tm * tn, 0, 1, 0};
            }
            if (sched == 4 && k2 == 0) {
                static bool attr_r = false;
                if (!attr_r) {
                    (void)hipFuncSetAttribute((const void*)gemm_bf16_tn_w4r, hipFuncAttributeMaxDynamicSharedMemorySize,
                                              W4R_LDS);
                    attr_r = true;
                }
                hipLaunchKernelGGL(gemm_bf16_tn_w4r, dim3((unsigned)(sp.nmain + sp.ntail * sp.ksplit)), dim3(W4R_THR),
                                   W4R_LDS, (hipStream_t)stream, (const bf16_t*)a, lda, (const bf16_t*)w, ldw,
                                   (bf16_t*)c, ldc, m, n, k, ep, tm, tn, sp.nmain, sp.ksplit, sp.piece_k, part);
                VS_CHECK_LAUNCH();
            } else {
            // (the LoRA second phase needs a few more VGPRs than the prefetch leaves: no prefetch there)
            auto kern = k2 ? gemm_bf16_tn_8p<true, 0>
                           : sched == 3 ? gemm_bf16_tn_8p<false, 3>
                           : sched == 2 ? gemm_bf16_tn_8p<false, 2>
                                        : sched == 1 ? gemm_bf16_tn_8p<false, 1> : gemm_bf16_tn_8p<false, 0>;
            hipLaunchKernelGGL(kern, dim3((unsigned)(sp.nmain + sp.ntail * sp.ksplit)), dim3(512), LDS8, (hipStream_t)stream, (const bf16_t*)a, lda, (const bf16_t*)w, ldw, (bf16_t*)c, ldc, m,
                               n, k, (const bf16_t*)a2, lda2, (const bf16_t*)w2, ldw2, k2, ep, tm, tn, sp.nmain,
                               sp.ksplit, sp.piece_k, part);
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
        static int buf_ok = -1;
        if (buf_ok < 0) {
            const char* e = getenv("VS_GEMM_FLAT_DMA");   // 1: flat-address DMA (A/B)
            buf_ok = !(e && e[0] == '1');
        }
        KSplit sp = k2 ? KSplit{tm * tn, 0, 1, 0}
                       : plan_ksplit(tm * tn, k / HK, vs_cus_for_split("VS_GEMM_NO_SPLIT"));
        float* part = nullptr;
        if (sp.ntail) {
            part = vs_split_workspace(1, (size_t)sp.ntail * sp.ksplit * BT * BT * sizeof(float), (hipStream_t)stream);
            if (!part) sp = KSplit{tm * tn, 0, 1, 0};
        }
        const unsigned grid = (unsigned)(sp.nmain + sp.ntail * sp.ksplit);
        if (buf_ok && fits32)
            hipLaunchKernelGGL(gemm_bf16_tn_256<true>, dim3(grid), dim3(NTHR8), RING * SLOT,
                               (hipStream_t)stream, (const bf16_t*)a, lda, (const bf16_t*)w, ldw,
                               (bf16_t*)c, ldc, m, n, k, (const bf16_t*)a2, lda2, (const bf16_t*)w2, ldw2,
                               k2, ep, tm, tn, sp.nmain, sp.ksplit, sp.piece_k, part);
        else
            hipLaunchKernelGGL(gemm_bf16_tn_256<false>, dim3(grid), dim3(NTHR8), RING * SLOT,
                               (hipStream_t)stream, (const bf16_t*)a, lda, (const bf16_t*)w, ldw,
                               (bf16_t*)c, ldc, m, n, k, (const bf16_t*)a2, lda2, (const bf16_t*)w2, ldw2,
                               k2, ep, tm, tn, sp.nmain, sp.ksplit, sp.piece_k, part);
        VS_CHECK_LAUNCH();
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
    if (k % 64 || n % 4 || lda < k || ldw < k || ldc < n || (lda & 15) || (ldw & 15) || (ldc & 3))
        return VS_E_INVALID;
    if (!aligned16(a8) || !aligned16(w8) || !aligned8(c)) return VS_E_INVALID;
    Epi ep;
    const int rc = fill_epi(ep, epilogue, epi, m, n);
    if (rc) return rc;
    // hipBLASLt fp8 (OCP e4m3 operands, per-token fp32 scale vector as hipBLASLt's outer B scale)
    // + the epilogue pass: 1.3-1.6x the fp8 MFMA kernel on every 14B block shape at SP=1 and SP=8
    // and bit-identical to it, epilogues included (profiles/r1/gemm_fp8_lt_r1j.log).
    // VS_FP8_BACKEND=vstyler forces the MFMA kernel, which also runs when no workspace is bound.
    // GELU as in vs_gemm: hipBLASLt's fused GELU_BIAS epilogue only with VS_LT_GELU=1.
    const char* fb = getenv("VS_FP8_BACKEND");      // lt | vstyler (8-phase MFMA kernel) | pp (r2 kernel, A/B)
    const char* lt_gelu = getenv("VS_LT_GELU");
    const bool use_lt = !(fb && (fb[0] == 'v' || fb[0] == 'p'));
    if (use_lt && epilogue == VS_EPI_GELU && (lt_gelu && lt_gelu[0] == '1') &&
        vs_lt_gemm_fp8(a8, lda, scale_a, w8, ldw, c, ldc, m, n, k, ep.bias, true, (hipStream_t)stream) == VS_OK)
        return VS_OK;
    if (use_lt &&
        lt_with_epilogue(c, ldc, m, n, epilogue, ep, (hipStream_t)stream, [&](void* y, long long ldy) {
            return vs_lt_gemm_fp8(a8, lda, scale_a, w8, ldw, y, ldy, m, n, k, ep.bias, false, (hipStream_t)stream);
        }))
        return VS_OK;
    const int tm = (m + BT - 1) / BT, tn = (n + BT - 1) / BT;
    if (k % 128 == 0 && !(fb && fb[0] == 'p')) {
        static bool attr8 = false;
        if (!attr8) {
            (void)hipFuncSetAttribute((const void*)gemm_fp8_tn_8p<false>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS8);
            (void)hipFuncSetAttribute((const void*)gemm_fp8_tn_8p<true>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS8);
            attr8 = true;
        }
        KSplit sp = plan_ksplit(tm * tn, k / 128, vs_cus_for_split("VS_GEMM_NO_SPLIT"), 128);
        float* part = nullptr;
        if (sp.ntail) {
            part = vs_split_workspace(1, (size_t)sp.ntail * sp.ksplit * BT * BT * sizeof(float), (hipStream_t)stream);
            if (!part) sp = KSplit{tm * tn, 0, 1, 0};
        }
        // VS_FP8_BACKEND=vs: the staggered schedule (A/B)
        hipLaunchKernelGGL((fb && fb[0] == 'v' && fb[1] == 's') ? gemm_fp8_tn_8p<true> : gemm_fp8_tn_8p<false>, dim3((unsigned)(sp.nmain + sp.ntail * sp.ksplit)), dim3(512), LDS8,
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
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)gemm_fp8_tn_256<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  RING * SLOT);
        (void)hipFuncSetAttribute((const void*)gemm_fp8_tn_256<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  RING * SLOT);
        attr = true;
    }
    const bool fits32 = (long long)(m - 1) * lda + k < 0x7fffffffLL && (long long)(n - 1) * ldw + k < 0x7fffffffLL;
    if (fits32)
        hipLaunchKernelGGL(gemm_fp8_tn_256<true>, dim3((unsigned)(tm * tn)), dim3(NTHR8), RING * SLOT,
                           (hipStream_t)stream, (const uint8_t*)a8, lda, scale_a, (const uint8_t*)w8, ldw, (bf16_t*)c,
                           ldc, m, n, k, ep, tm, tn);
    else
        hipLaunchKernelGGL(gemm_fp8_tn_256<false>, dim3((unsigned)(tm * tn)), dim3(NTHR8), RING * SLOT,
                           (hipStream_t)stream, (const uint8_t*)a8, lda, scale_a, (const uint8_t*)w8, ldw, (bf16_t*)c,
                           ldc, m, n, k, ep, tm, tn);
    VS_CHECK_LAUNCH();
    return VS_OK;
}

extern "C" int vs_quant_fp8_rows(const void* x, long long ldx, void* x8, long long ld8, float* scale, int rows,
                                 int cols, void* stream) {
    if (!x || !x8 || !scale || rows <= 0 || cols <= 0 || cols % 8 || ldx < cols || ld8 < cols || (ldx & 7) ||
        (ld8 & 7) || !aligned16(x) || !aligned8(x8))
        return VS_E_INVALID;
    hipLaunchKernelGGL(quant_fp8_rows_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, (hipStream_t)stream,
                       (const bf16_t*)x, ldx, (uint8_t*)x8, ld8, scale, rows, cols);
    VS_CHECK_LAUNCH();
    return VS_OK;
}

extern "C" int vs_gemm_route(int m, int n, int k) {
    if (m <= 0 || n <= 0 || k <= 0) return VS_E_INVALID;
    return lt_route(m, n, k) ? 1 : 0;
}

extern "C" int vs_gemm_split_plan(int m, int n, int k, int cus, int* out) {
    if (!out || m <= 0 || n <= 0 || k <= 0 || k % BK || cus < 0) return VS_E_INVALID;
    const KSplit p = plan_ksplit(((m + BT - 1) / BT) * ((n + BT - 1) / BT), k / HK, cus);
    out[0] = p.nmain;
    out[1] = p.ntail;
    out[2] = p.ksplit;
    out[3] = p.piece_k;
    return VS_OK;
}

long long vs_gemm_split_workspace_bytes_impl() { return (long long)MAX_SPLIT_PIECES * BT * BT * (long long)sizeof(float); }
