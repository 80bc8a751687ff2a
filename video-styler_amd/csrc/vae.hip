// Causal 3-D VAE kernels (Wan2.1 VAE, diffsynth/models/wan_video_vae.py) for gfx950.
//
// vae_conv_kernel: one implicit-GEMM MFMA kernel covers every convolution of the VAE
//   (CausalConv3d 3x3x3 / 1x1x1 / (3,1,1) time convs, the 3x3 stride-1/2 Conv2d of Resample with
//   the nearest-x2 upsample fused into its gather, the 1x1 convs of AttentionBlock) and the two
//   batched GEMMs of the VAE attention (fp32 scores, P.V).
//   Tile: 128 output pixels x 32*NB output channels, K-step 32 (one 64-B row chunk group), 4 waves
//   of 32 pixels each.  Operands are register-staged global->LDS (double buffered, loads of step
//   s+1 in flight during the MFMAs of step s, one barrier per step); LDS rows are 64 B with the
//   16-B chunk swizzle c ^ ((row>>1)&3), conflict-free for the 32-row ds_read_b128 fragments.
//   The product is computed transposed, D[co][pix] = W . X^T with v_mfma_f32_32x32x16_bf16, so
//   each lane owns one pixel and 4 consecutive channels per register group (8-byte stores into
//   the channels-last output).  Padding (causal time pad, spatial pad, ZeroPad2d) is a predicate
//   on the gather, never a padded copy.
// The elementwise kernels (channel RMS norm + SiLU, softmax, transpose, tile gather/blend) are
// HBM-bound one-pass kernels.
#include "common.h"
#include <algorithm>

namespace {

constexpr int BM = 128, BK = 32, CNTHR = 256;

// LDS image of a 64-B row chunk: chunk c of row R at c ^ f(R), f(R) = (R1 ^ R2) | 2 R3 (bits of R).
// Conflict-free for both accesses of the kernel (MI355X_MICROARCH §LDS lane groups): the
// ds_write_b128 of the register-staged A rows (8 contiguous lanes = 4 rows x 2 lanes, one 128-B bank
// window: the 8 (row parity, chunk) slots distinct) and the 32-row ds_read_b128 fragments (16-lane
// groups {0-3,12-15,20-27} / {4-11,16-19,28-31}, one 256-B window: per row & 3 the four lanes' f
// distinct).  r1-r4 used f = (R >> 1) & 3, conflict-free for the writes only: the fragment reads ran
// 2-way, SQ_LDS_BANK_CONFLICT 32 % of the LDS cycles (profiles/r5/pmc_vae_r5).
__device__ __forceinline__ int swz(int row, int ch) {
    return row * 64 + 16 * (ch ^ ((((row >> 1) ^ (row >> 2)) & 1) | ((row >> 2) & 2)));
}

// The conv's output store for one pixel (n, to, yo, xo) of slice z: a lane's NB accumulator blocks hold
// channels n0 + 32j + 8g + 4h + {0..3} (h = lane >> 5) -- bias, residual, the time interleave of
// `split`, bf16 rounding (or fp32 alpha * acc) as vs_conv3d documents.
template <int NB, bool F32>
__device__ __forceinline__ void conv_store(const vs_conv3d& p, const f32x16_t (&acc)[NB], int z, long long nn, int to,
                                           int yo, int xo, int n0, int lane) {
    const int h = lane >> 5;
#pragma unroll
    for (int j = 0; j < NB; ++j) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int n = n0 + 32 * j + 8 * g + 4 * h;
            if (n >= p.cout) continue;
            int co = n, sub = 0;
            if (p.split > 0 && n >= p.split) { co = n - p.split; sub = 1; }
            const int tt = to * p.t_mul + p.t_add + sub;
            const long long off = z * p.y_zs + nn * p.y_ns + ((long long)(tt * p.h_out + yo) * p.w_out + xo) * p.ldy + co;
            const int nv = min(4, p.cout - n);
            if constexpr (F32) {
                float* y = (float*)p.y + off;
                if (nv == 4) {
                    *(f32x4_t*)y = f32x4_t{p.alpha * acc[j][4 * g], p.alpha * acc[j][4 * g + 1],
                                           p.alpha * acc[j][4 * g + 2], p.alpha * acc[j][4 * g + 3]};
                } else {
                    for (int e = 0; e < nv; ++e) y[e] = p.alpha * acc[j][4 * g + e];
                }
            } else {
                float v[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    float a = acc[j][4 * g + e];
                    if (p.bias && e < nv) a += bf2f(((const bf16_t*)p.bias)[n + e]);
                    v[e] = rbf(a);
                }
                bf16_t* y = (bf16_t*)p.y + off;
                if (p.res) {
                    const bf16_t* r = (const bf16_t*)p.res + off;
                    for (int e = 0; e < nv; ++e) v[e] = rbf(v[e] + bf2f(r[e]));
                }
                if (nv == 4) {
                    *(u32x2_t*)y = u32x2_t{pack2(v[0], v[1]), pack2(v[2], v[3])};
                } else {
                    for (int e = 0; e < nv; ++e) y[e] = (bf16_t)f2bf(v[e]);
                }
            }
        }
    }
}

template <int NB, bool F32, int PXB, int PRE>
__global__ __launch_bounds__(CNTHR, 2) void vae_conv_kernel(vs_conv3d p, long long M, int ntn) {
    // PRE = 2: two register stages, the global loads of step s+2 issued before step s's MFMAs (two
    // steps of latency cover instead of one).
    // PXB pixel blocks of 32 per wave: the workgroup tile is 128*PXB pixels x 32*NB channels and each
    // wave's W fragment feeds PXB MFMAs (PXB = 2: 0.83 LDS fragment reads per MFMA at NB = 3 instead
    // of 1.33).  The K order of every output's accumulation is the same for both PXB: bit-identical.
    constexpr int BN = 32 * NB, BMT = BM * PXB;
    constexpr int NBL = (BN * 4 + CNTHR - 1) / CNTHR;
    constexpr int STAGE = (BMT + BN) * 64;
    __shared__ __attribute__((aligned(16))) char lds[2 * STAGE];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const long long mt = blockIdx.x / ntn;
    const int n0 = (blockIdx.x % ntn) * BN;
    const int z = blockIdx.y;
    const long long m0 = mt * BMT;

    // ---- A (pixel) loader state: rows tid>>1 + 128*b, chunks 2*(tid&1)+{0,1}
    const int arow = tid >> 1, ach = (tid & 1) * 2;
    bool avalid[PXB];
    int ti0[PXB], yi0[PXB], xi0[PXB];
    const bf16_t* xb[PXB];
#pragma unroll
    for (int b = 0; b < PXB; ++b) {
        const long long am = m0 + arow + BM * b;
        avalid[b] = am < M;
        long long q = avalid[b] ? am : 0;
        int xo = (int)(q % p.w_out); q /= p.w_out;
        int yo = (int)(q % p.h_out); q /= p.h_out;
        int to = (int)(q % p.t_out);
        long long nn = q / p.t_out;
        xb[b] = (const bf16_t*)p.x + z * p.x_zs + nn * p.x_ns + ach * 8;
        ti0[b] = to * p.st - p.pt;
        yi0[b] = yo * p.sh - p.ph;
        xi0[b] = xo * p.sw - p.pw;
    }
    const int hv = p.up2 ? 2 * p.h_in : p.h_in, wv = p.up2 ? 2 * p.w_in : p.w_in;
    const bf16_t* wb = (const bf16_t*)p.w + z * p.w_zs;

    const int csteps = p.cin / BK;
    const int nsteps = p.kt * p.kh * p.kw * csteps;
    int lc = 0, lkx = 0, lky = 0, lkt = 0;  // loader position (uniform)

    struct Stage { u32x4_t a0[PXB], a1[PXB], b[NBL]; };
    // the gather source of the current tap (kt, ky, kx): validity and pixel address are recomputed
    // when the loader enters a tap (lc == 0, a uniform branch) and stepped by BK channels within it
    // (r1-r4 recomputed both every K-step: ~10 VALU per MFMA, profiles/r5/pmc_vae_r5)
    // (the source pixel's index in its slice, ~0u: outside the input)
    unsigned toff[PXB];
    auto tap = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int b = 0; b < PXB; ++b) {
            const int ti = ti0[b] + lkt, yi = yi0[b] + lky, xi = xi0[b] + lkx;
            const bool v = avalid[b] && ti >= p.t_lo && ti < p.t_in && yi >= 0 && yi < hv && xi >= 0 && xi < wv;
            const int ys = p.up2 ? (yi >> 1) : yi, xs = p.up2 ? (xi >> 1) : xi;
            toff[b] = v ? (unsigned)((ti * p.h_in + ys) * p.w_in + xs) : ~0u;
        }
    };
    auto load = [&](Stage& r) {
        if (lc == 0) tap();
#pragma unroll
        for (int b = 0; b < PXB; ++b) {
            if (toff[b] != ~0u) {
                const bf16_t* src = xb[b] + (unsigned long long)toff[b] * (unsigned)p.ldx + lc;
                r.a0[b] = *(const u32x4_t*)src;
                r.a1[b] = *(const u32x4_t*)(src + 8);
            } else {
                r.a0[b] = u32x4_t{0, 0, 0, 0};
                r.a1[b] = r.a0[b];
            }
        }
        const int kofs = ((lkt * p.kh + lky) * p.kw + lkx) * p.cin + lc;
#pragma unroll
        for (int i = 0; i < NBL; ++i) {
            const int c = tid + CNTHR * i;
            r.b[i] = u32x4_t{0, 0, 0, 0};
            if (c < BN * 4) {
                const int nr = n0 + (c >> 2);
                if (nr < p.cout) r.b[i] = *(const u32x4_t*)(wb + (long long)nr * p.ldw + kofs + (c & 3) * 8);
            }
        }
        // advance (c0, kx, ky, kt)
        lc += BK;
        if (lc == p.cin) {
            lc = 0;
            if (++lkx == p.kw) {
                lkx = 0;
                if (++lky == p.kh) { lky = 0; ++lkt; }
            }
        }
    };
    auto store = [&](const Stage& r, int buf) {
        char* A = lds + buf * STAGE;
        char* B = A + BMT * 64;
#pragma unroll
        for (int b = 0; b < PXB; ++b) {
            *(u32x4_t*)(A + swz(arow + BM * b, ach)) = r.a0[b];
            *(u32x4_t*)(A + swz(arow + BM * b, ach + 1)) = r.a1[b];
        }
#pragma unroll
        for (int i = 0; i < NBL; ++i) {
            const int c = tid + CNTHR * i;
            if (c < BN * 4) *(u32x4_t*)(B + swz(c >> 2, c & 3)) = r.b[i];
        }
    };

    f32x16_t acc[PXB][NB];
#pragma unroll
    for (int b = 0; b < PXB; ++b)
#pragma unroll
        for (int j = 0; j < NB; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[b][j][r] = 0.f;

    // wave w computes pixel blocks w*32 + 128*b of the tile
    auto compute = [&](int buf) {
        const char* A = lds + buf * STAGE;
        const char* B = A + BMT * 64;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const int ch = 2 * s + (lane >> 5);
            bf16x8_t xa[PXB];
#pragma unroll
            for (int b = 0; b < PXB; ++b) xa[b] = *(const bf16x8_t*)(A + swz(BM * b + wave * 32 + (lane & 31), ch));
#pragma unroll
            for (int j = 0; j < NB; ++j) {
                const bf16x8_t wf = *(const bf16x8_t*)(B + swz(j * 32 + (lane & 31), ch));
#pragma unroll
                for (int b = 0; b < PXB; ++b)
                    acc[b][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf, xa[b], acc[b][j], 0, 0, 0);
            }
        }
    };

    if constexpr (PRE == 1) {
        Stage r;
        load(r);
        store(r, 0);
        __syncthreads();
        for (int s = 0; s < nsteps; ++s) {
            const bool more = s + 1 < nsteps;
            if (more) load(r);
            compute(s & 1);
            if (more) store(r, (s + 1) & 1);
            __syncthreads();
        }
    } else if constexpr (PRE == 2) {
        // step s's data is in LDS buffer s&1, step s+1's in flight in stage (s+1)&1
        Stage r0, r1;
        load(r0);
        if (nsteps > 1) load(r1);
        store(r0, 0);
        __syncthreads();
        auto step = [&](int s, Stage& mine, Stage& next) __attribute__((always_inline)) {
            if (s + 2 < nsteps) load(mine);        // mine (step s) is already in LDS
            compute(s & 1);
            if (s + 1 < nsteps) store(next, (s + 1) & 1);
            __syncthreads();
        };
        for (int s = 0; s < nsteps; s += 2) {
            step(s, r0, r1);
            if (s + 1 < nsteps) step(s + 1, r1, r0);
        }
    } else {
        // three stages: steps s+1 and s+2 in flight while step s computes
        Stage r0, r1, r2;
        load(r0);
        if (nsteps > 1) load(r1);
        if (nsteps > 2) load(r2);
        store(r0, 0);
        __syncthreads();
        auto step = [&](int s, Stage& mine, Stage& next) __attribute__((always_inline)) {
            if (s + 3 < nsteps) load(mine);
            compute(s & 1);
            if (s + 1 < nsteps) store(next, (s + 1) & 1);
            __syncthreads();
        };
        for (int s = 0; s < nsteps; s += 3) {
            step(s, r0, r1);
            if (s + 1 < nsteps) step(s + 1, r1, r2);
            if (s + 2 < nsteps) step(s + 2, r2, r0);
        }
    }

    // ---- epilogue: lane owns pixel m, channels n0 + 32j + 8g + 4h + {0..3}
#pragma unroll
    for (int b = 0; b < PXB; ++b) {
        const long long me = m0 + BM * b + wave * 32 + (lane & 31);
        if (me >= M) continue;
        long long q = me;
        const int xo = (int)(q % p.w_out); q /= p.w_out;
        const int yo = (int)(q % p.h_out); q /= p.h_out;
        const int to = (int)(q % p.t_out);
        const long long nn = q / p.t_out;
        conv_store<NB, F32>(p, acc[b], z, nn, to, yo, xo, n0, lane);
    }
}

// ------------------------------------------------------------------------------------------
// vae_conv_halo_kernel (r5): the 3x3(x3) stride-1 convs (ResidualBlock / middle / head CausalConv3d,
// 71 % + of the VAE's conv time) with the input read ONCE per (input frame, channel chunk) instead
// of once per tap.  The implicit GEMM above gathers a 256-pixel x 32-channel A tile per tap: 27
// gathers of every input pixel per output (N = 96 channels gives 96 FLOP per byte gathered, and a
// plain GEMM of the same K with contiguous rows runs slower still, HBM-bound:
// profiles/r5/vae_conv_probe_s26.log).  Here a workgroup (8 waves) owns a 16 x 32 output tile of
// one frame and 32 * NB output channels; per stage (16-channel chunk c, time tap kt) it LDS-DMAs the
// 18 x 34 input patch of frame t + kt - pt (pitch 40 pixels, 32 B each) and the 9 spatial taps'
// weights (9 x 32NB rows x 32 B), and runs all 9 taps from LDS.  A ring of three stages (150 KB:
// one workgroup per CU), the DMA two stages ahead.  The LDS-DMA bytes bound this kernel (diagnostic
// builds of the first, 32-channel / 256-pixel version: the DMA alone 0.82 ms, the MFMAs alone
// 1.05 ms, both 1.28 ms -- profiles/r5/vae_halo_diag_s29.log -- at the chip's LDS-DMA rate,
// MI355X_MICROARCH 'ldsdma-fill'); 512-pixel tiles halve the weight bytes per FLOP, and 16-channel
// stages fit the deeper ring.  Padding and the causal time pad: a patch pixel outside the frame
// loads through an out-of-range buffer offset, which the buffer unit returns as zero; a time tap
// outside [t_lo, t_in) is skipped (its contribution is zero).
// LDS swizzle: half k of patch pixel (row, col) at k ^ ((col >> 3) & 1), of weight row r at
// k ^ ((r >> 3) & 1): with the 1280-B patch row pitch (a multiple of the 256-B bank window) every
// fragment read -- 32 consecutive columns from any start column 0..2 -- is conflict-free for both
// ds_read_b128 lane groups ({0-3,12-15,20-27}, {4-11,16-19,28-31}: the two lanes of each column
// residue mod 8 sit 8 or 24 columns apart, so in opposite halves).  The K order per output differs
// from vae_conv_kernel's (chunk-major instead of tap-major): results agree to bf16 rounding of the
// fp32 sums.
typedef int i32x4h_t __attribute__((ext_vector_type(4)));
constexpr int HTHR = 512, HT = 16, HW = 32, HPITCH = 40, HPROWS = HT + 2;
constexpr int HPATCH_Q = (HPROWS * HPITCH + 31) / 32;          // 23 DMA instructions of 1 KB (32 slots)
constexpr int HPATCH_B = HPATCH_Q * 1024;
template <int NB> constexpr int halo_w_bytes() { return 9 * 32 * NB * 32; }
template <int NB> constexpr int halo_buf_bytes() { return HPATCH_B + halo_w_bytes<NB>(); }
constexpr int HSLOTS = 3;

template <int NB, bool F32>
__global__ __launch_bounds__(HTHR, 1) void vae_conv_halo_kernel(vs_conv3d p, int tiles_x, int tiles_y) {
    constexpr int BN = 32 * NB, WQ = 9 * BN / 32, BUF = halo_buf_bytes<NB>();
    constexpr int PQW = (HPATCH_Q + 7) / 8, WQW = (WQ + 7) / 8;   // DMA instructions per wave (at most)
    extern __shared__ __attribute__((aligned(16))) char hsmem[];
    const unsigned smem_base = (unsigned)(uintptr_t)hsmem;
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int n0 = blockIdx.y * BN, z = blockIdx.z;
    // XCD-aware order: workgroup b runs on XCD b % 8, which takes a contiguous eighth of the work
    // list (n, tile row, tile column, output frame -- frame fastest), so one XCD's CUs work on
    // consecutive frames of the same tile at once and the three frames each input frame feeds read
    // its patch from that XCD's L2 instead of HBM (HBM bytes 2.74 -> 0.52 GB per launch of the
    // dominant shape, profiles/r5/pmc_vaeconv_halo{,2})
    const long long nblk = (long long)p.n * tiles_y * tiles_x * p.t_out, per = (nblk + 7) / 8;
    long long bid = (long long)(blockIdx.x & 7) * per + (blockIdx.x >> 3);
    if (bid >= nblk) return;
    const int to = (int)(bid % p.t_out); bid /= p.t_out;
    const int tx = (int)(bid % tiles_x); bid /= tiles_x;
    const int ty = (int)(bid % tiles_y);
    const long long nn = bid / tiles_y;
    const int x0 = tx * HW, y0 = ty * HT;
    const int tb = to - p.pt;                                   // input frame of time tap 0 (st = 1)
    const int kt_lo = max(0, p.t_lo - tb), kt_hi = min(p.kt, p.t_in - tb);
    const int nkt = max(0, kt_hi - kt_lo);
    const int nst = nkt * (p.cin / 16);

    auto rsrc = [](const void* base, unsigned bytes) {
        const unsigned long long a = (unsigned long long)(uintptr_t)base;
        return i32x4h_t{(int)(unsigned)a, (int)((unsigned)(a >> 32) & 0xffffu), (int)bytes, 0x00020000};
    };
    // the input buffer resource spans ONE frame, rebased per stage (any t_in; offsets < 2^31 per frame)
    const long long plane = (long long)p.h_in * p.w_in * p.ldx;          // elements per input frame
    const bf16_t* const xs = (const bf16_t*)p.x + z * p.x_zs + nn * p.x_ns;
    i32x4h_t wr = rsrc((const bf16_t*)p.w + z * p.w_zs + (long long)n0 * p.ldw,
                       (unsigned)((long long)(p.cout - n0) * p.ldw * 2));
#pragma unroll
    for (int e = 0; e < 4; ++e) wr[e] = __builtin_amdgcn_readfirstlane(wr[e]);
    // per-lane DMA source offsets (the uniform frame / chunk / tap-plane part goes in soffset); lane l
    // fills 16-B half (l & 1) of slot 32q + (l >> 1)
    unsigned pvo[PQW], wvo[WQW];
#pragma unroll
    for (int i = 0; i < PQW; ++i) {
        const int P = 32 * (wave + 8 * i) + (lane >> 1);
        const int pr = P / HPITCH, pc = P % HPITCH;
        // (yi, xi): the conv's input grid -- with up2 the nearest-x2 upsample of the frame, read as
        // source pixel (yi / 2, xi / 2): the Resample upsample convs gather through it, no copy
        const int yi = y0 - p.ph + pr, xi = x0 - p.pw + pc;
        const int hv = p.up2 ? 2 * p.h_in : p.h_in, wv = p.up2 ? 2 * p.w_in : p.w_in;
        const int ys = p.up2 ? yi >> 1 : yi, xs = p.up2 ? xi >> 1 : xi;
        const int lc = (lane & 1) ^ ((pc >> 3) & 1);
        const bool v = pr < HPROWS && pc < HW + 2 && yi >= 0 && yi < hv && xi >= 0 && xi < wv;
        pvo[i] = v ? (unsigned)(((long long)ys * p.w_in + xs) * p.ldx * 2 + lc * 16) : 0x80000000u;
    }
#pragma unroll
    for (int i = 0; i < WQW; ++i) {
        const int R = 32 * (wave + 8 * i) + (lane >> 1);
        const int tap = R / BN, co = R % BN;
        const int lc = (lane & 1) ^ ((co >> 3) & 1);
        wvo[i] = (unsigned)((long long)co * p.ldw * 2 + tap * p.cin * 2 + lc * 16);
    }
    // this wave's DMA instructions per stage (the counted wait below)
    const int nq = (wave < HPATCH_Q % 8 || HPATCH_Q % 8 == 0 ? PQW : PQW - 1) + (wave < WQ % 8 || WQ % 8 == 0 ? WQW : WQW - 1);
    auto dma = [](unsigned lds, unsigned voff, i32x4h_t rs, int soff) __attribute__((always_inline)) {
        asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
                     :: "s"(lds), "v"(voff), "s"(rs), "s"(soff) : "m0", "memory");
    };
    auto issue = [&](int s) __attribute__((always_inline)) {
        // (uniform values the compiler may hold in VGPRs: the asm's "s" operands take readfirstlane)
        const int c = s / nkt, kt = kt_lo + s % nkt;
        const unsigned buf = __builtin_amdgcn_readfirstlane(smem_base + (s % HSLOTS) * BUF);
        i32x4h_t xr = rsrc(xs + (tb + kt) * plane, (unsigned)(plane * 2));
#pragma unroll
        for (int e = 0; e < 4; ++e) xr[e] = __builtin_amdgcn_readfirstlane(xr[e]);
        const int sx = __builtin_amdgcn_readfirstlane(c * 32);
        const int sw = __builtin_amdgcn_readfirstlane((kt * 9 * p.cin + c * 16) * 2);
#pragma unroll
        for (int i = 0; i < PQW; ++i)
            if (wave + 8 * i < HPATCH_Q) dma(buf + (wave + 8 * i) * 1024, pvo[i], xr, sx);
#pragma unroll
        for (int i = 0; i < WQW; ++i)
            if (wave + 8 * i < WQ) dma(buf + HPATCH_B + (wave + 8 * i) * 1024, wvo[i], wr, sw);
    };

    f32x16_t acc[2][NB];
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int j = 0; j < NB; ++j) {
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[b][j][r] = 0.f;
            asm volatile("" : "+a"(acc[b][j]));
        }

    // wave w: output rows 2w, 2w + 1 of the tile (pixel blocks b), 32 columns, all NB channel blocks
    const int hi = lane >> 5, l32 = lane & 31;
    auto lds16 = [](unsigned addr) { return *reinterpret_cast<const LDS_AS bf16x8_t*>((const LDS_AS char*)(uintptr_t)addr); };
    auto compute = [&](int s) __attribute__((always_inline)) {
        const unsigned buf = smem_base + (s % HSLOTS) * BUF;
        unsigned xb[3], wb1;
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
            const int col = kx + l32;
            xb[kx] = buf + (2 * wave * HPITCH + col) * 32 + 16 * (hi ^ ((col >> 3) & 1));
            asm volatile("" : "+v"(xb[kx]));        // (row / tap displacements fold into ds offsets)
        }
        wb1 = buf + HPATCH_B + l32 * 32 + 16 * (hi ^ ((l32 >> 3) & 1));
        asm volatile("" : "+v"(wb1));
        // 9 steps (taps); the fragments of step i + 1 are read before step i's MFMAs (with the
        // reads issued right before their MFMAs -- the compiler's schedule -- every step waited
        // out the LDS latency with the MFMA pipe empty)
        bf16x8_t xa[2][2], wf[2][NB];
        auto rd = [&](int tap, int buf2) __attribute__((always_inline)) {
            const int ky = tap / 3, kx = tap % 3;
#pragma unroll
            for (int b = 0; b < 2; ++b) xa[buf2][b] = lds16(xb[kx] + (b + ky) * HPITCH * 32);
#pragma unroll
            for (int j = 0; j < NB; ++j) wf[buf2][j] = lds16(wb1 + (tap * BN + 32 * j) * 32);
        };
        rd(0, 0);
#pragma unroll
        for (int i = 0; i < 9; ++i) {
            if (i + 1 < 9) rd(i + 1, (i + 1) & 1);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int j = 0; j < NB; ++j)
#pragma unroll
                for (int b = 0; b < 2; ++b) {
                    acc[b][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[i & 1][j], xa[i & 1][b], acc[b][j], 0, 0, 0);
                    // (pinned to AGPRs: held in VGPRs across the stage loop, the accumulators
                    // were copied into AGPRs and back every stage)
                    asm volatile("" : "+a"(acc[b][j]));
                }
            __builtin_amdgcn_sched_barrier(0);
        }
    };

    // ring of HSLOTS stages, DMA two ahead: before stage s, wait for this wave's stage-s pieces
    // (its stage-(s+1) pieces, issued later, may stay in flight: vmcnt(nq)), then the barrier makes
    // every wave's pieces visible and frees slot (s+2) % 3 (stage s-1's, read by all waves)
    if (nst > 0) issue(0);
    if (nst > 1) issue(1);
    for (int s = 0; s < nst; ++s) {
        if (s + 1 < nst) {
            switch (nq) {          // (an immediate operand: one wait per possible count)
                case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
                case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
                case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
                case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
                case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
                default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
            }
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        asm volatile("s_barrier" ::: "memory");
        if (s + 2 < nst) issue(s + 2);
        compute(s);
    }
    // epilogue through LDS (halo_ok: bf16 output, no time split, ldy % 8 == 0, 16-B aligned y / res,
    // 8-B aligned bias): bias + rounding in the accumulator layout (lane = pixel, 4-channel groups),
    // then the wave's 64 pixels x 96 channels are transposed through LDS (pixel pitch 208 B:
    // conflict-free 8-B writes) so each global store / residual load instruction moves 64
    // consecutive 16-B chunks (a pixel's 192 B, then the next pixel's) -- stored straight from the
    // accumulator layout, every instruction touched 64 lines at 8 B each, and the epilogue cost as
    // much as 16 % of the kernel (profiles/r5/vae_halo2_compute_diag_s38.log)
    if constexpr (NB != 3) {
        // (NB = 1: the conv_out / head convs with at most 32 output channels -- few bytes out, the
        // generic store with its channel and stride predicates)
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            const int yo = y0 + 2 * wave + b, xo = x0 + l32;
            if (yo < p.h_out && xo < p.w_out) conv_store<NB, F32>(p, acc[b], z, nn, to, yo, xo, n0, lane);
        }
        return;
    }
    constexpr int EP = 208;
    asm volatile("s_barrier" ::: "memory");                    // every wave is done with the ring
    const bf16_t* bias = (const bf16_t*)p.bias;
    const unsigned eb = smem_base + wave * 64 * EP;
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int j = 0; j < NB; ++j)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int c = 32 * j + 8 * g + 4 * hi;
                float a[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) a[e] = acc[b][j][4 * g + e];
                if (bias) {
                    const u32x2_t bb = *(const u32x2_t*)(bias + n0 + c);
                    a[0] += bf2f(bb[0] & 0xffffu); a[1] += bf2f(bb[0] >> 16);
                    a[2] += bf2f(bb[1] & 0xffffu); a[3] += bf2f(bb[1] >> 16);
                }
                *reinterpret_cast<LDS_AS u32x2_t*>((LDS_AS char*)(uintptr_t)(eb + (32 * b + l32) * EP + 2 * c)) =
                    u32x2_t{pack2(a[0], a[1]), pack2(a[2], a[3])};
            }
    // chunk q = 64 i + lane of the wave's 64 x 12 (pixel, 16-B chunk) pairs
#pragma unroll
    for (int i = 0; i < 12; ++i) {
        const int q = 64 * i + lane, px = q / 12, k = q % 12;
        const int yo = y0 + 2 * wave + (px >> 5), xo = x0 + (px & 31);
        u32x4_t v = *reinterpret_cast<const LDS_AS u32x4_t*>((const LDS_AS char*)(uintptr_t)(eb + px * EP + 16 * k));
        if (yo >= p.h_out || xo >= p.w_out) continue;
        const long long off = z * p.y_zs + nn * p.y_ns +
                              ((long long)((to * p.t_mul + p.t_add) * p.h_out + yo) * p.w_out + xo) * p.ldy + n0 + 8 * k;
        if (p.res) {
            const u32x4_t rr = *(const u32x4_t*)((const bf16_t*)p.res + off);
#pragma unroll
            for (int e = 0; e < 4; ++e)
                v[e] = pack2(bf2f(v[e] & 0xffffu) + bf2f(rr[e] & 0xffffu), bf2f(v[e] >> 16) + bf2f(rr[e] >> 16));
        }
        *(u32x4_t*)((bf16_t*)p.y + off) = v;
    }
}

// The halo kernel's shapes: 3x3 spatial taps, stride 1, spatial pad 1, kt <= 3 (any time pad), with
// or without the nearest-x2 upsample, bf16 output, one input frame and the weight rows addressable
// with 31-bit buffer offsets; then either whole 96-channel blocks (NB = 3, the LDS-transposed
// epilogue: ldy % 8, 16-B aligned y / res) or at most 32 output channels (NB = 1: the decoder's
// 96 -> 3 conv_out and the encoder's 32-channel head, the generic epilogue).  0: not eligible.
int halo_nb(const vs_conv3d& p) {
    const bool base = vs_opt(VS_OPT_VAE_HALO) && p.kh == 3 && p.kw == 3 && p.sh == 1 && p.sw == 1 && p.st == 1 &&
                      p.ph == 1 && p.pw == 1 && p.kt <= 3 && !p.out_f32 && p.cin % 16 == 0 && p.split == 0 &&
                      (p.x_zs | p.x_ns) % 8 == 0 && (long long)p.h_in * p.w_in * p.ldx * 2 < (1LL << 31) &&
                      (long long)p.cout * p.ldw * 2 < (1LL << 31);
    if (!base) return 0;
    if (p.cout % 96 == 0 && p.ldy % 8 == 0 && !(((uintptr_t)p.y | (uintptr_t)p.res) & 15) &&
        !((uintptr_t)p.bias & 7) && (p.y_zs | p.y_ns) % 8 == 0)
        return 3;
    return p.cout <= 32 ? 1 : 0;
}

template <int NB>
int launch_conv_halo(const vs_conv3d& p, hipStream_t st) {
    const int tiles_x = (p.w_out + HW - 1) / HW, tiles_y = (p.h_out + HT - 1) / HT;
    const long long nblk = (long long)p.n * p.t_out * tiles_y * tiles_x;
    if (nblk > 0x7ffffff0LL) return VS_E_UNSUPPORTED;
    const int lds = HSLOTS * halo_buf_bytes<NB>();
    // (once per process and instance, thread-safe: a function-local static's initialiser)
    static const bool attr = [lds] {
        return hipFuncSetAttribute((const void*)vae_conv_halo_kernel<NB, false>,
                                   hipFuncAttributeMaxDynamicSharedMemorySize, lds) == hipSuccess;
    }();
    (void)attr;
    hipLaunchKernelGGL((vae_conv_halo_kernel<NB, false>),
                       dim3((unsigned)((nblk + 7) / 8 * 8), (p.cout + 32 * NB - 1) / (32 * NB), p.nz), dim3(HTHR), lds,
                       st, p, tiles_x, tiles_y);
    VS_CHECK_LAUNCH();
    return VS_OK;
}

template <int NB, int PXB, int PRE>
int launch_conv_px(const vs_conv3d& p, long long M, hipStream_t st) {
    const int ntn = (p.cout + 32 * NB - 1) / (32 * NB);
    const long long mt = (M + BM * PXB - 1) / (BM * PXB);
    if (mt * ntn > 0x7fffffffLL) return VS_E_UNSUPPORTED;
    dim3 grid((unsigned)(mt * ntn), p.nz);
    if (p.out_f32)
        hipLaunchKernelGGL((vae_conv_kernel<NB, true, PXB, PRE>), grid, dim3(CNTHR), 0, st, p, M, ntn);
    else
        hipLaunchKernelGGL((vae_conv_kernel<NB, false, PXB, PRE>), grid, dim3(CNTHR), 0, st, p, M, ntn);
    VS_CHECK_LAUNCH();
    return VS_OK;
}

// VS_OPT_VAE_PXB 1 | 2 pixel blocks per wave, VS_OPT_VAE_PRE 1 | 2 | 3 register stages of the global->LDS
// pipeline (the im2col gathers are latency-bound: with one stage 256-pixel tiles ran 0.68x of
// 128-pixel ones).  Default 2 / 3, measured at 832x480x73 (profiles/r2/vae_conv_ab.log): tiled encode
// 452 -> 498 TF/s, decode 467 -> 518 TF/s.  All variants are bit-identical (same K order per output).
template <int NB>
int launch_conv(const vs_conv3d& p, long long M, hipStream_t st) {
    const bool px2 = vs_opt(VS_OPT_VAE_PXB) == 2;
    // (NB = 4 with three stages and two pixel blocks needs more than 256 VGPRs: two stages there)
    const int pre = NB == 4 && px2 ? std::min(vs_opt(VS_OPT_VAE_PRE), 2) : vs_opt(VS_OPT_VAE_PRE);
    if (px2) return pre == 3 ? launch_conv_px<NB, 2, 3>(p, M, st) : pre == 2 ? launch_conv_px<NB, 2, 2>(p, M, st)
                                                                             : launch_conv_px<NB, 2, 1>(p, M, st);
    return pre == 3 ? launch_conv_px<NB, 1, 3>(p, M, st) : pre == 2 ? launch_conv_px<NB, 1, 2>(p, M, st)
                                                                   : launch_conv_px<NB, 1, 1>(p, M, st);
}

// ------------------------------------------------------------------------------------------
// Channel RMS norm (+SiLU): 4 lanes per pixel, lane q owns 16-B chunks q, q+4, q+8, ...
__global__ __launch_bounds__(256) void vae_rmsnorm_kernel(const bf16_t* __restrict__ x, long long ldx,
                                                          bf16_t* __restrict__ y, long long ldy,
                                                          const bf16_t* __restrict__ gamma, long long npix,
                                                          int c, int silu, float scale) {
    // r5: 16 lanes per pixel, lane q owning 16-B chunks q, q + 16, q + 32 (c <= 384), so one load /
    // store instruction moves 4 whole consecutive pixel rows (768 contiguous B at c = 96) -- with 4
    // lanes per pixel each instruction took 64-B pieces at the pixel stride and the kernel ran at
    // 2.2 TB/s (profiles/r5/vae_rmsnorm_s43.log); the row stays in registers between the norm and the
    // write (one read of x); one correctly rounded division per pixel (1 / ||x||) and a multiply per
    // element instead of an fp32 division per element; SiLU as v * rcp(1 + exp2(-v log2 e)).  Agrees
    // with the reference's bf16 ops to the test's bar (<= 1 bf16 ulp, > 99.5 % bit-equal: the fp32
    // values differ by a few ulp before the bf16 rounding).
    constexpr int MAXN = 3;
    const long long gid = (long long)blockIdx.x * 256 + threadIdx.x;
    const long long pix = gid >> 4;
    const int q = (int)(gid & 15);
    const bool valid = pix < npix;
    const int nck = c >> 3;  // 16-B chunks per pixel
    const bf16_t* xr = x + (valid ? pix : 0) * ldx;
    u32x4_t w[MAXN];
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < MAXN; ++i) {
        const int k = q + 16 * i;
        if (k < nck) {
            w[i] = *(const u32x4_t*)(xr + k * 8);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float a = bflo(w[i][e]), b = bfhi(w[i][e]);
                ss += a * a + b * b;
            }
        }
    }
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) ss += __shfl_xor(ss, o);
    if (!valid) return;
    const float nrm = fmaxf(rbf(sqrtf(ss)), 1e-12f);  // F.normalize: x / max(||x||, eps), norm in bf16
    const float rn = 1.0f / nrm;
    bf16_t* yr = y + pix * ldy;
#pragma unroll
    for (int i = 0; i < MAXN; ++i) {
        const int k = q + 16 * i;
        if (k >= nck) continue;
        const u32x4_t gw = *(const u32x4_t*)(gamma + k * 8);
        u32x4_t o;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            float v0 = rbf(rbf(rbf(bflo(w[i][e]) * rn) * scale) * bflo(gw[e]));
            float v1 = rbf(rbf(rbf(bfhi(w[i][e]) * rn) * scale) * bfhi(gw[e]));
            if (silu) {
                v0 = v0 * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.4426950408889634f * v0));
                v1 = v1 * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.4426950408889634f * v1));
            }
            o[e] = pack2(v0, v1);
        }
        *(u32x4_t*)(yr + k * 8) = o;
    }
}

// One wave per row.
__global__ __launch_bounds__(256) void vae_softmax_kernel(const float* __restrict__ s, long long ld_s,
                                                          bf16_t* __restrict__ p, long long ld_p,
                                                          long long rows, int ncols) {
    const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= rows) return;
    const float* sr = s + row * ld_s;
    bf16_t* pr = p + row * ld_p;
    float mx = -INFINITY;
    for (int j = lane; j < ncols; j += 64) mx = fmaxf(mx, sr[j]);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    float sum = 0.f;
    for (int j = lane; j < ncols; j += 64) sum += expf(sr[j] - mx);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) sum += __shfl_xor(sum, o);
    const float inv = 1.0f / sum;
    for (int j = lane; j < ld_p; j += 64) pr[j] = j < ncols ? (bf16_t)f2bf(expf(sr[j] - mx) * inv) : (bf16_t)0;
}

__global__ __launch_bounds__(256) void vae_transpose_kernel(const bf16_t* __restrict__ v, long long v_zs,
                                                            long long ld_v, bf16_t* __restrict__ vt,
                                                            long long vt_zs, long long ld_vt, int rows,
                                                            int cols) {
    __shared__ bf16_t tile[32][33];
    const int z = blockIdx.z;
    const int r0 = blockIdx.x * 32, c0 = blockIdx.y * 32;
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
    for (int i = ty; i < 32; i += 8) {
        const int r = r0 + i, c = c0 + tx;
        tile[i][tx] = (r < rows && c < cols) ? v[z * v_zs + (long long)r * ld_v + c] : (bf16_t)0;
    }
    __syncthreads();
    for (int i = ty; i < 32; i += 8) {
        const int c = c0 + i, r = r0 + tx;
        if (c < cols && r < ld_vt) vt[z * vt_zs + (long long)c * ld_vt + r] = tile[tx][i];
    }
}

__device__ __forceinline__ float affine(float x, int mode, const bf16_t* a, const bf16_t* b, int c) {
    if (mode == 1) return rbf(rbf(x - bf2f(a[c])) * bf2f(b[c]));
    if (mode == 2) return rbf(rbf(x / bf2f(b[c])) + bf2f(a[c]));
    return x;
}

__global__ __launch_bounds__(256) void vae_tile_gather_kernel(const bf16_t* __restrict__ src, int c, int t_src,
                                                              int h, int w, int t, int h0, int w0, int th, int tw,
                                                              bf16_t* __restrict__ dst, int cpad, int mode,
                                                              const bf16_t* a, const bf16_t* b) {
    const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;  // (t, i, j)
    const long long npix = (long long)t * th * tw;
    if (idx >= npix) return;
    const int j = (int)(idx % tw);
    const int i = (int)((idx / tw) % th);
    const int tt = (int)(idx / ((long long)tw * th));
    const long long plane = (long long)t_src * h * w;
    const long long so = ((long long)tt * h + h0 + i) * w + w0 + j;
    bf16_t* d = dst + idx * cpad;
    for (int cc = 0; cc < cpad; cc += 2) {
        float v0 = 0.f, v1 = 0.f;
        if (cc < c) v0 = affine(bf2f(src[cc * plane + so]), mode, a, b, cc);
        if (cc + 1 < c) v1 = affine(bf2f(src[(cc + 1) * plane + so]), mode, a, b, cc + 1);
        *(uint32_t*)(d + cc) = pack2(v0, v1);
    }
}

__device__ __forceinline__ float ramp(int i, int len, bool lo_bound, bool hi_bound, int bw) {
    float m = 1.0f;
    if (!lo_bound && i < bw) m = (float)(i + 1) / (float)bw;
    if (!hi_bound && i >= len - bw) m = (float)(len - i) / (float)bw;
    return m;
}

__global__ __launch_bounds__(256) void vae_tile_blend_kernel(const bf16_t* __restrict__ tile, long long ldc,
                                                             int c, int t, int th, int tw,
                                                             bf16_t* __restrict__ values, bf16_t* __restrict__ weight,
                                                             int h, int w, int h0, int w0, int bound, int bw_h,
                                                             int bw_w, int mode, const bf16_t* a, const bf16_t* b) {
    const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
    const long long npix = (long long)t * th * tw;
    if (idx >= npix) return;
    const int j = (int)(idx % tw);
    const int i = (int)((idx / tw) % th);
    const int tt = (int)(idx / ((long long)tw * th));
    const float mh = ramp(i, th, bound & 1, bound & 2, bw_h);
    const float mw = ramp(j, tw, bound & 4, bound & 8, bw_w);
    const float mask = rbf(fminf(mh, mw));
    const long long plane = (long long)t * h * w;
    const long long o = ((long long)tt * h + h0 + i) * w + w0 + j;
    const bf16_t* tr = tile + idx * ldc;
    for (int cc = 0; cc < c; ++cc) {
        const float v = affine(bf2f(tr[cc]), mode, a, b, cc);
        values[cc * plane + o] = (bf16_t)f2bf(bf2f(values[cc * plane + o]) + rbf(v * mask));
    }
    weight[o] = (bf16_t)f2bf(bf2f(weight[o]) + mask);
}

__global__ __launch_bounds__(256) void vae_blend_finish_kernel(const bf16_t* __restrict__ values,
                                                               const bf16_t* __restrict__ weight,
                                                               bf16_t* __restrict__ out, int c, long long plane,
                                                               int clamp) {
    const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
    if (idx >= plane * c) return;
    float v = rbf(bf2f(values[idx]) / bf2f(weight[idx % plane]));
    if (clamp) v = fminf(fmaxf(v, -1.0f), 1.0f);
    out[idx] = (bf16_t)f2bf(v);
}

// vae_output_to_video: bf16 (x - (-1)) * 127.5, clip [0, 255], truncating uint8 cast, CTHW -> THWC.
__global__ __launch_bounds__(256) void vae_to_u8_kernel(const bf16_t* __restrict__ v, uint8_t* __restrict__ out,
                                                        long long plane) {
    const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
    if (idx >= plane) return;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        float x = rbf(rbf(bf2f(v[c * plane + idx]) + 1.0f) * 127.5f);
        x = fminf(fmaxf(x, 0.0f), 255.0f);
        out[idx * 3 + c] = (uint8_t)(int)x;
    }
}

// WanVideoUnit_VACE.process (wan_video_new.py:878-888) on uint8 frames [T][H][W][3]:
// preprocess_video (utils/__init__.py:60-73) then inactive = v*(1-m) + 0*m, reactive = v*m + 0*(1-m),
// every op a bf16 tensor op.  video == NULL -> zeros, mask == NULL -> ones (:880-886).
__global__ __launch_bounds__(256) void vace_prepare_kernel(const uint8_t* __restrict__ video,
                                                           const uint8_t* __restrict__ mask,
                                                           bf16_t* __restrict__ inactive, bf16_t* __restrict__ reactive,
                                                           bf16_t* __restrict__ mask0, long long plane) {
    const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
    if (idx >= plane) return;
    const float sv = 2.0f / 255.0f, sm = 1.0f / 255.0f;  // (max - min) / 255 as fp32 opmath scalars
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const float v = video ? rbf(rbf((float)video[idx * 3 + c] * sv) - 1.0f) : 0.0f;
        const float m = mask ? rbf(rbf((float)mask[idx * 3 + c] * sm) + 0.0f) : 1.0f;
        const float om = rbf(1.0f - m);
        inactive[c * plane + idx] = (bf16_t)f2bf(rbf(v * om) + rbf(0.0f * m));
        reactive[c * plane + idx] = (bf16_t)f2bf(rbf(v * m) + rbf(0.0f * om));
        if (c == 0) mask0[idx] = (bf16_t)f2bf(m);
    }
}

// vace_mask_latents (wan_video_new.py:893-894): rearrange "T (H 8) (W 8) -> (8 8) T H W" and
// nearest-exact resize of T to t_out = (T + 3) // 4 (src = min(floor((j + 0.5) * T / t_out), T - 1)).
__global__ __launch_bounds__(256) void vace_mask_latents_kernel(const bf16_t* __restrict__ mask0,
                                                                bf16_t* __restrict__ out, int t, int h, int w,
                                                                int t_out) {
    const int hl = h / 8, wl = w / 8;
    const long long n = 64LL * t_out * hl * wl;
    const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
    if (idx >= n) return;
    const int ww = (int)(idx % wl);
    const int hh = (int)((idx / wl) % hl);
    const int j = (int)((idx / ((long long)wl * hl)) % t_out);
    const int c = (int)(idx / ((long long)wl * hl * t_out));
    const float scale = (float)t / (float)t_out;
    const int src = min((int)floorf(((float)j + 0.5f) * scale), t - 1);
    out[idx] = mask0[((long long)src * h + hh * 8 + c / 8) * w + ww * 8 + c % 8];
}

}  // namespace

extern "C" int vs_vace_prepare(const void* video_u8, const void* mask_u8, void* inactive, void* reactive,
                               void* mask0, int t, int h, int w, void* stream) {
    if (!inactive || !reactive || !mask0 || t <= 0 || h <= 0 || w <= 0) return VS_E_INVALID;
    const long long plane = (long long)t * h * w;
    hipLaunchKernelGGL(vace_prepare_kernel, dim3((unsigned)((plane + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       (const uint8_t*)video_u8, (const uint8_t*)mask_u8, (bf16_t*)inactive, (bf16_t*)reactive,
                       (bf16_t*)mask0, plane);
    VS_CHECK_LAUNCH();
    return VS_OK;
}

extern "C" int vs_vace_mask_latents(const void* mask0, void* out, int t, int h, int w, int t_out, void* stream) {
    if (!mask0 || !out || t <= 0 || h <= 0 || w <= 0 || h % 8 || w % 8 || t_out <= 0) return VS_E_INVALID;
    const long long n = 64LL * t_out * (h / 8) * (w / 8);
    hipLaunchKernelGGL(vace_mask_latents_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       (const bf16_t*)mask0, (bf16_t*)out, t, h, w, t_out);
    VS_CHECK_LAUNCH();
    return VS_OK;
}

extern "C" int vs_vae_to_u8(const void* video, void* out, int t, int h, int w, void* stream) {
    if (!video || !out || t <= 0 || h <= 0 || w <= 0) return VS_E_INVALID;
    const long long plane = (long long)t * h * w;
    hipLaunchKernelGGL(vae_to_u8_kernel, dim3((unsigned)((plane + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       (const bf16_t*)video, (uint8_t*)out, plane);
    VS_CHECK_LAUNCH();
    return VS_OK;
}

extern "C" int vs_vae_conv(const vs_conv3d* pp, void* stream) {
    if (!pp) return VS_E_INVALID;
    const vs_conv3d& p = *pp;
    if (!p.x || !p.w || !p.y || p.cin <= 0 || p.cin % BK || p.ldx % 8 || p.ldw % 8 || p.cout <= 0 ||
        p.n <= 0 || p.nz <= 0 || p.t_out < 0 || p.h_out <= 0 || p.w_out <= 0 || p.kt <= 0 || p.kh <= 0 ||
        p.kw <= 0 || p.st <= 0 || p.sh <= 0 || p.sw <= 0 || p.ldy % 4 || (p.split > 0 && p.split % 4) ||
        (p.out_f32 && (p.bias || p.res)))
        return VS_E_INVALID;
    if (((uintptr_t)p.x | (uintptr_t)p.w) & 15) return VS_E_INVALID;
    if (p.t_out == 0) return VS_OK;
    const long long M = (long long)p.n * p.t_out * p.h_out * p.w_out;
    hipStream_t st = (hipStream_t)stream;
    switch (halo_nb(p)) {
        case 3: return launch_conv_halo<3>(p, st);
        case 1: return launch_conv_halo<1>(p, st);
        default: break;
    }
    if (p.cout <= 32) return launch_conv<1>(p, M, st);
    if (p.cout <= 64) return launch_conv<2>(p, M, st);
    if (p.cout <= 96) return launch_conv<3>(p, M, st);
    const int w4 = (p.cout + 127) / 128 * 128 - p.cout, w3 = (p.cout + 95) / 96 * 96 - p.cout;
    return w3 < w4 ? launch_conv<3>(p, M, st) : launch_conv<4>(p, M, st);
}

extern "C" int vs_vae_rmsnorm(const void* x, long long ldx, void* y, long long ldy, const void* gamma,
                              long long npix, int c, int silu, void* stream) {
    if (!x || !y || !gamma || c <= 0 || c % 32 || c > 384 || ldx % 8 || ldy % 8 || npix < 0) return VS_E_INVALID;
    if (npix == 0) return VS_OK;
    const long long threads = npix * 16;
    hipLaunchKernelGGL(vae_rmsnorm_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, (const bf16_t*)x, ldx, (bf16_t*)y, ldy, (const bf16_t*)gamma, npix,
                       c, silu, (float)sqrt((double)c));
    VS_CHECK_LAUNCH();
    return VS_OK;
}

extern "C" int vs_vae_softmax(const float* s, long long ld_s, void* p, long long ld_p, long long rows, int ncols,
                              void* stream) {
    if (!s || !p || ncols <= 0 || ld_s < ncols || ld_p < ncols || rows < 0) return VS_E_INVALID;
    if (rows == 0) return VS_OK;
    hipLaunchKernelGGL(vae_softmax_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, (hipStream_t)stream,
                       s, ld_s, (bf16_t*)p, ld_p, rows, ncols);
    VS_CHECK_LAUNCH();
    return VS_OK;
}

extern "C" int vs_vae_transpose(const void* v, long long v_zs, long long ld_v, void* vt, long long vt_zs,
                                long long ld_vt, int nz, int rows, int cols, void* stream) {
    if (!v || !vt || nz <= 0 || rows <= 0 || cols <= 0 || ld_vt < rows || ld_v < cols) return VS_E_INVALID;
    dim3 grid((unsigned)((ld_vt + 31) / 32), (unsigned)((cols + 31) / 32), nz);
    hipLaunchKernelGGL(vae_transpose_kernel, grid, dim3(256), 0, (hipStream_t)stream, (const bf16_t*)v, v_zs, ld_v,
                       (bf16_t*)vt, vt_zs, ld_vt, rows, cols);
    VS_CHECK_LAUNCH();
    return VS_OK;
}

extern "C" int vs_vae_tile_gather(const void* src, int c, int t_src, int h, int w, int t, int h0, int w0, int th,
                                  int tw, void* dst, int cpad, int mode, const void* a, const void* b, void* stream) {
    if (!src || !dst || c <= 0 || cpad < c || cpad % 2 || t <= 0 || t > t_src || th <= 0 || tw <= 0 || h0 < 0 || w0 < 0 ||
        h0 + th > h || w0 + tw > w || mode < 0 || mode > 2 || (mode && (!a || !b)))
        return VS_E_INVALID;
    const long long n = (long long)t * th * tw;
    hipLaunchKernelGGL(vae_tile_gather_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       (const bf16_t*)src, c, t_src, h, w, t, h0, w0, th, tw, (bf16_t*)dst, cpad, mode, (const bf16_t*)a,
                       (const bf16_t*)b);
    VS_CHECK_LAUNCH();
    return VS_OK;
}

extern "C" int vs_vae_tile_blend(const void* tile, long long ldc, int c, int t, int th, int tw, void* values,
                                 void* weight, int h, int w, int h0, int w0, int bound, int bw_h, int bw_w,
                                 int mode, const void* a, const void* b, void* stream) {
    if (!tile || !values || !weight || c <= 0 || ldc < c || t <= 0 || th <= 0 || tw <= 0 || h0 < 0 || w0 < 0 ||
        h0 + th > h || w0 + tw > w || mode < 0 || mode > 2 || (mode && (!a || !b)) ||
        ((bound & 3) != 3 && bw_h <= 0) || ((bound & 12) != 12 && bw_w <= 0))
        return VS_E_INVALID;
    const long long n = (long long)t * th * tw;
    hipLaunchKernelGGL(vae_tile_blend_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       (const bf16_t*)tile, ldc, c, t, th, tw, (bf16_t*)values, (bf16_t*)weight, h, w, h0, w0, bound,
                       bw_h, bw_w, mode, (const bf16_t*)a, (const bf16_t*)b);
    VS_CHECK_LAUNCH();
    return VS_OK;
}

extern "C" int vs_vae_blend_finish(const void* values, const void* weight, void* out, int c, long long plane,
                                   int clamp, void* stream) {
    if (!values || !weight || !out || c <= 0 || plane <= 0) return VS_E_INVALID;
    const long long n = plane * c;
    hipLaunchKernelGGL(vae_blend_finish_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       (const bf16_t*)values, (const bf16_t*)weight, (bf16_t*)out, c, plane, clamp);
    VS_CHECK_LAUNCH();
    return VS_OK;
}

extern "C" int vs_vae_copy_frames(const void* src, long long src_ns, void* dst, long long dst_ns, int n,
                                  long long frame_elems, void* stream) {
    if (!src || !dst || n <= 0 || frame_elems <= 0 || src_ns < frame_elems || dst_ns < frame_elems)
        return VS_E_INVALID;
    if (hipMemcpy2DAsync(dst, dst_ns * 2, src, src_ns * 2, frame_elems * 2, n, hipMemcpyDeviceToDevice,
                         (hipStream_t)stream) != hipSuccess)
        return VS_E_LAUNCH;
    return VS_OK;
}
