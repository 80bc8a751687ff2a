/*
 * vstyler.h -- C ABI of the MI355X (gfx950) kernel library `libvstyler.so`.
 *
 * The library replaces the GPU operators of the Wan2.1(-VACE) denoising path of the reference
 * (Ditto / DiffSynth-Studio 1.1.8, paths relative to the reference root).  Every entry point is
 * stream-ordered, allocation-free and graph-capturable; pointers are caller-owned device buffers
 * (bf16 unless stated, row-major), sizes/strides are in ELEMENTS.  No C++ types cross the ABI.
 *
 * Error convention: every call returns 0 (VS_OK) or a VS_E_* code; shape/alignment violations are
 * rejected up front with VS_E_INVALID before anything is launched.  vs_strerror() names a code.
 */
#ifndef VSTYLER_H
#define VSTYLER_H

#ifdef __cplusplus
extern "C" {
#endif

#define VS_OK 0
#define VS_E_INVALID 1     /* bad shape / stride / alignment / null pointer            */
#define VS_E_LAUNCH 2      /* hipGetLastError() after the launch was not hipSuccess   */
#define VS_E_UNSUPPORTED 3 /* valid request this build does not implement (e.g. d!=128) */

const char* vs_strerror(int code);
int vs_abi_version(void);

/* Epilogue selector for vs_gemm (fp32 accumulator -> bf16, rounding points of the reference). */
#define VS_EPI_BIAS 0      /* y = bf16(acc + bias)                                           */
#define VS_EPI_GELU 1      /* bf16(gelu_tanh(y))            : nn.GELU(approximate='tanh')      */
#define VS_EPI_SILU 2      /* bf16(silu(y))                 : nn.SiLU                          */
#define VS_EPI_GATE_RES 3  /* bf16(res + bf16(gate*y)) [+ bf16(hint*hint_scale)] : GateModule  */
#define VS_EPI_RES 4       /* bf16(res + bf16(alpha*y))     : residual add / LoRA merge        */

typedef struct vs_epilogue {
    const void* bias;        /* [N] or NULL                                                  */
    const void* residual;    /* [M x ld_res] (may alias C: each element read then written)   */
    long long ld_res;
    const void* gate;        /* [batches x N] (row m uses batch m / rows_per_batch)          */
    long long gate_bstride;
    const void* hint;        /* [M x ld_hint] or NULL (VACE hint add, wan_video_new.py:1450)  */
    long long ld_hint;
    float hint_scale;
    float alpha;
    int rows_per_batch;
    int reserved;
} vs_epilogue;

/*
 * C[M,N] = epilogue(A[M,K] . W[N,K]^T (+ A2[M,K2] . W2[N,K2]^T)).
 * Replaces torch.nn.functional.linear in AutoWrappedLinear.forward
 * (diffsynth/vram_management/layers.py:173-188) incl. the un-merged LoRA term out + x A^T B^T
 * (layers.py:180-182): pass A2 = alpha * x A^T (computed by a previous vs_gemm) and W2 = B.
 * K and K2 must be multiples of 64, lda/ldw/lda2/ldw2 multiples of 8, N a multiple of 4.
 */
int vs_gemm(const void* a, long long lda, const void* w, long long ldw, void* c, long long ldc,
            int m, int n, int k, int epilogue, const vs_epilogue* epi,
            const void* a2, long long lda2, const void* w2, long long ldw2, int k2, void* stream);

/*
 * O = softmax(Q K^T * scale) V per (batch, head), non-causal, no mask.  head_dim must be 128.
 * Q: [batch][sq] rows of stride ldq (head h at columns h*128..), K/V: [batch][skv], O like Q.
 * Replaces flash_attention() / AttentionModule.forward (diffsynth/models/wan_video_dit.py:28-61,
 * 114-121) for self-attention (skv = sq) and T5 cross-attention (skv = 512).
 */
int vs_attn_fwd(const void* q, const void* k, const void* v, void* o,
                int batch, int sq, int skv, int heads, int head_dim,
                long long ldq, long long ldk, long long ldv, long long ldo,
                long long bsq, long long bsk, long long bsv, long long bso,
                float scale, void* stream);

/*
 * out = bf16(LN(x)) [affine: weight/bias] then, if shift/scale given, modulate:
 * bf16(bf16(n * bf16(1+scale)) + shift) with shift/scale rows selected per batch.
 * Replaces WanAutoCastLayerNorm (layers.py:63-92) + modulate (wan_video_dit.py:64-65,225,228,268).
 */
int vs_layernorm_modulate(const void* x, long long ldx, void* out, long long ldo, int rows, int dim,
                          int rows_per_batch, const void* shift, const void* scale,
                          long long mod_bstride, const void* weight, const void* bias, float eps,
                          void* stream);

/*
 * In place: x = bf16(bf16(x * rsqrt(mean(x^2)+eps)) * weight) over the full row (all heads), then
 * (if rope != NULL) the interleaved 3-D RoPE of each head_dim slice with table rope[pos][pair]
 * (float2 cos,sin; pair axes 22 t / 21 h / 21 w).  Token index = (row % rows_per_batch) +
 * token_offset, decomposed as (f, h, w) over grid (gf, gh, gw).
 * Replaces RMSNorm (wan_video_dit.py:100-111) + rope_apply (:92-97; SP slice
 * diffsynth/distributed/xdit_context_parallel.py:27-40).
 */
int vs_rmsnorm_rope(void* x, long long ldx, int rows, int dim, int head_dim, const void* weight,
                    float eps, const void* rope, int rope_len, int gf, int gh, int gw,
                    int rows_per_batch, int token_offset, void* stream);

/* lat [B,C,T,H,W] -> tokens [B*T*(H/2)*(W/2), C*4], column c*4+kh*2+kw (Conv3d k=s=(1,2,2) im2col,
 * wan_video_dit.py:306-307 / wan_video_vace.py:51, token order of wan_video_new.py:1381-1382). */
int vs_patchify(const void* lat, void* tokens, int batch, int channels, int frames, int height,
                int width, void* stream);

/* tokens [B*S, 4*C] -> lat [B,C,T,H,W] ('b (f h w) (x y z c) -> b c (f x) (h y) (w z)',
 * wan_video_dit.py:347-352). height/width are the latent (output) sizes. */
int vs_unpatchify(const void* tokens, void* lat, int batch, int channels, int frames, int height,
                  int width, void* stream);

/* x = bf16(x + bf16(v * dsigma)), v = use_cfg ? bf16(vn + bf16(cfg*bf16(vp - vn))) : vp.
 * Replaces the CFG combine (wan_video_new.py:535) + FlowMatchScheduler.step (flow_match.py:72-82). */
int vs_cfg_euler(const void* v_pos, const void* v_neg, void* x, long long n, float cfg_scale,
                 float dsigma, int use_cfg, void* stream);

/* out[b] = bf16([cos(t*10000^(-i/(dim/2))) || sin(...)]) in fp64, t = bf16 timestep[b]
 * (sinusoidal_embedding_1d, wan_video_dit.py:68-72). */
int vs_time_sinusoid(const void* t, void* out, int batch, int dim, void* stream);

/* out[b][r][d] = bf16(param[r][d] + tv[b*tv_bstride + r*tv_rstride + d]) -- the AdaLN modulation
 * add (wan_video_dit.py:218-219) and the head's (modulation + t) (wan_video_dit.py:267). */
int vs_mod_add(const void* param, const void* tv, void* out, int batch, int rows, int dim,
               long long tv_bstride, long long tv_rstride, void* stream);

/* x = bf16(x + bf16(y * scale)) elementwise (VACE hint injection, wan_video_new.py:1450). */
int vs_axpy(void* x, const void* y, float scale, long long n, void* stream);

/* Ulysses SP row permutation (one 16-B vector per thread); index (j,b,t,c) with rank chunk j:
 *   packed = j*jstride + (b*s_local + t)*cols_per_rank + c   (all_to_all_single chunk j)
 *   local  = (b*s_local + t)*ld_local + j*cols_per_rank + c  (token shard, all heads)
 *   full   = (b*world*s_local + j*s_local + t)*cols_per_rank + c (head shard, all tokens)
 * mode 0 local->packed, 1 packed->local, 2 packed->full, 3 full->packed.  Replaces the layout
 * transforms inside xFuserLongContextAttention / yunchang all-to-all
 * (diffsynth/distributed/xdit_context_parallel.py:117-127) and the head-output all_gather
 * reassembly (diffsynth/pipelines/wan_video_new.py:1459-1462). */
int vs_ulysses_permute(const void* src, void* dst, int batch, int s_local, int world,
                       int cols_per_rank, long long ld_local, long long jstride, int mode, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* VSTYLER_H */
