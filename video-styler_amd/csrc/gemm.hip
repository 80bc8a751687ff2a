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
// Structure: 128x128x64 tile, 4 waves (2x2, 64x64 each), v_mfma_f32_16x16x32_bf16 computing the
// transposed tile (W rows as the A operand) so every lane owns 4 consecutive output columns;
// both operands are K-contiguous ([rows][K]) and staged by global_load_lds_dwordx4 (LDS-DMA,
// no VGPR round trip) into a 2-stage LDS ring whose 128-B rows carry a 16-B-chunk XOR swizzle
// (chunk ^ (row & 7)) applied on the global SOURCE address, which makes the fragment
// ds_read_b128 conflict free; grouped (8 m-tiles) + XCD-aware tile order for L2 reuse.
#include "common.h"

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

__device__ __forceinline__ void load4(const bf16_t* p, float* v) {
    const u32x2_t w = *reinterpret_cast<const u32x2_t*>(p);
    v[0] = bflo(w[0]);
    v[1] = bfhi(w[0]);
    v[2] = bflo(w[1]);
    v[3] = bfhi(w[1]);
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
        const int bidx = m / ep.rows_per_batch;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int n = n0 + wn * 64 + j * 16 + 4 * (lane >> 4);
            if (n >= N) continue;
            float bv[4] = {0.f, 0.f, 0.f, 0.f};
            if (ep.bias) load4(ep.bias + n, bv);
            float y[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) y[e] = rbf(acc[i][j][e] + bv[e]);
            if (ep.mode == VS_EPI_GELU) {
#pragma unroll
                for (int e = 0; e < 4; ++e) y[e] = gelu_tanh_f(y[e]);
            } else if (ep.mode == VS_EPI_SILU) {
#pragma unroll
                for (int e = 0; e < 4; ++e) y[e] = silu_f(y[e]);
            } else if (ep.mode == VS_EPI_GATE_RES) {
                float rv[4], gv[4];
                load4(ep.res + (long long)m * ep.ld_res + n, rv);
                load4(ep.gate + (long long)bidx * ep.gate_bstride + n, gv);
#pragma unroll
                for (int e = 0; e < 4; ++e) y[e] = rbf(rv[e] + rbf(gv[e] * y[e]));
                if (ep.hint) {
                    float hv[4];
                    load4(ep.hint + (long long)m * ep.ld_hint + n, hv);
#pragma unroll
                    for (int e = 0; e < 4; ++e) y[e] = y[e] + rbf(hv[e] * ep.hint_scale);
                }
            } else if (ep.mode == VS_EPI_RES) {
                float rv[4];
                load4(ep.res + (long long)m * ep.ld_res + n, rv);
#pragma unroll
                for (int e = 0; e < 4; ++e) y[e] = rv[e] + rbf(ep.alpha * y[e]);
            }
            u32x2_t w;
            w[0] = pack2(y[0], y[1]);
            w[1] = pack2(y[2], y[3]);
            *reinterpret_cast<u32x2_t*>(C + (long long)m * ldc + n) = w;
        }
    }
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }
bool aligned8(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 7) == 0; }

}  // namespace

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
    if (epilogue < VS_EPI_BIAS || epilogue > VS_EPI_RES) return VS_E_INVALID;
    Epi ep{};
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
    if ((epilogue == VS_EPI_GATE_RES || epilogue == VS_EPI_RES) && (!ep.res || ep.ld_res < n))
        return VS_E_INVALID;
    if (epilogue == VS_EPI_GATE_RES && !ep.gate) return VS_E_INVALID;
    if (ep.hint && ep.ld_hint < n) return VS_E_INVALID;
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
