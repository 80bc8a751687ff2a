/*
 * vstyler.h -- C ABI of the MI355X (gfx950) kernel library `libvstyler.so`.
 *
 * The library replaces the GPU operators of the Wan2.1(-VACE) denoising path of the reference
 * (Ditto / DiffSynth-Studio 1.1.8, paths relative to the reference root).  Every entry point is
 * stream-ordered and graph-capturable; pointers are caller-owned device buffers
 * (bf16 unless stated, row-major), sizes/strides are in ELEMENTS.  No C++ types cross the ABI.
 *
 * Allocation: none.  vs_gemm and vs_attn_fwd use a caller-owned fp32 split-tail workspace per
 * (device, stream) bound with vs_split_workspace_bind; on a stream without one they launch
 * unsplit (same results up to fp32 summation order).
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
#define VS_E_COMM 4        /* RCCL missing or returned an error (vs_sp_last_error)     */

const char* vs_strerror(int code);
/* 2 since r6: vs_blaslt_library is gone (r5) and workspace kinds 2 / 3 are unused
 * (vs_split_workspace_bytes returns 0); 1: r1-r5. */
int vs_abi_version(void);

/*
 * Path-selection options.  The library reads no environment variable: every launch takes its
 * kernel / schedule from this process-wide table, whose defaults are the product configuration.
 * Tests and A/B probes select the alternate paths (each bit-identical or within its stated tolerance
 * of the default) through vs_set_option, which returns the previous value (-VS_E_INVALID for an
 * unknown id or value).  Not for concurrent use with launches that depend on the changed option.
 */
#define VS_OPT_GEMM_TILE 0     /* 0 auto (default); 128 / 256: force the 128x128 / 256x256 schedule   */
#define VS_OPT_GEMM_KERNEL 1   /* 4: the 4-wave 256x256 kernels (default); 8: the 8-phase ones         */
#define VS_OPT_GEMM_SPLIT 2    /* 1: split tails (default); 0: whole-tile grids                        */
#define VS_OPT_QUEUE 3         /* 1: XCD work queues of the persistent GEMMs / self-attention (default; a kind-5 workspace); 0: static lists */
#define VS_OPT_ATTN_IMPL 4     /* 0: auto (default: 4-wave for >= 16 key tiles); 4 / 8 force a kernel  */
#define VS_OPT_ATTN_MFMA 5     /* 16 (default) / 32: the 8-wave kernel's MFMA shape                     */
#define VS_OPT_ATTN_NC 6       /* 1: optimistic softmax + checked redo (default); 0: checked only       */
#define VS_OPT_ATTN_SPLIT 7    /* 1: split tails (default); 0: whole-item grids                        */
#define VS_OPT_ATTN_PERSIST 8  /* 1: persistent item walk (default); 0: one block per item             */
#define VS_OPT_VAE_PXB 9       /* 2 (default) / 1: 128-pixel blocks per wave of the VAE conv            */
#define VS_OPT_VAE_PRE 10      /* 3 (default) / 2 / 1: register stages of the VAE conv's gathers        */
#define VS_OPT_VAE_HALO 11     /* 1 (default): the VAE's 3x3(x3) stride-1 convs on the patch-resident kernel; 0: per-tap gathers */
#define VS_OPT_PIECE_QUEUE 12  /* 1 (default, r6): the 4-wave bf16 GEMM's split-tail pieces taken by its persistent blocks from the queue after the whole tiles; 0: blocks of their own; 2: 1 + grids of 1-3 rounds keep 1/16 of each round as pieces (held-CU reserve) */
#define VS_OPT_COUNT 13
int vs_set_option(int id, int value);
int vs_get_option(int id);

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
 * Execution: every GEMM runs on the hand-written MFMA kernels: grids of >= 240 256x256 tiles with
 * K >= 1024 on the 256x256 schedule (the persistent 4-wave kernel fed by XCD tile queues when a
 * kind-5 workspace is bound; with the kind-1 split tail), the un-merged LoRA second phase on the
 * 8-phase 256x256 kernel, everything else on the 128x128 kernel (vs_set_option overrides).  Every
 * path keeps the reference's rounding points and differs only in fp32 summation order.
 */
int vs_gemm(const void* a, long long lda, const void* w, long long ldw, void* c, long long ldc,
            int m, int n, int k, int epilogue, const vs_epilogue* epi,
            const void* a2, long long lda2, const void* w2, long long ldw2, int k2, void* stream);

/*
 * The split-tail plan vs_gemm uses for its 256x256 schedule on a device with `cus` compute units
 * (no LoRA second phase): out[0] = whole-tile workgroups, out[1] = tail tiles split along K,
 * out[2] = K pieces per tail tile, out[3] = K per piece (out[1] = 0: no split).  Host-only.
 */
int vs_gemm_split_plan(int m, int n, int k, int cus, int* out);

/*
 * The route vs_gemm (fp8 = 0) / vs_gemm_fp8 (fp8 = 1) takes for an (m, n, k) GEMM with epilogue
 * `epilogue`: 0 = the MFMA kernels with the epilogue fused -- the only route of this build (r5: the
 * vendor-library route and its separate epilogue pass are gone) -- or -VS_E_INVALID for non-positive
 * sizes or an unknown epilogue.  vs_gemm_route(m, n, k) = vs_gemm_route_epi(m, n, k, VS_EPI_BIAS, 0).
 * Host-only.  (A binding fuses a residual epilogue with the next LayerNorm only on a route != 0.)
 */
int vs_gemm_route(int m, int n, int k);
int vs_gemm_route_epi(int m, int n, int k, int epilogue, int fp8);

/*
 * fp8 path (config 5; AutoWrappedLinear.fp8_linear, diffsynth/vram_management/layers.py:115-151):
 * vs_quant_fp8_rows quantises activations per row, s[m] = max(max_k |x[m][k]| / 448, 1),
 * x8 = e4m3fn(x / (s + 1e-8)) (OCP e4m3, round-to-nearest-even); vs_gemm_fp8 computes
 * C = epilogue(s[m] * (A8 . W8^T)) with unscaled e4m3 weights W8 [N][K] (scale_b = 1, as the
 * reference) and the same epilogues as vs_gemm (bias added in fp32 before the single bf16 rounding,
 * as torch._scaled_mm).  K % 128 == 0 on every route (the MFMA kernel's K-tile is 128 fp8; the 14B
 * shapes K = 5120 / 13824 qualify), N % 4 == 0, lda/ldw multiples of 16 bytes.
 */
int vs_quant_fp8_rows(const void* x, long long ldx, void* x8, long long ld8, float* scale, int rows, int cols,
                      void* stream);
int vs_gemm_fp8(const void* a8, long long lda, const float* scale_a, const void* w8, long long ldw, void* c,
                long long ldc, int m, int n, int k, int epilogue, const vs_epilogue* epi, void* stream);

/*
 * O = softmax(Q K^T * scale) V per (batch, head), non-causal, no mask.  head_dim must be 128.
 * Q: [batch][sq] rows of stride ldq (head h at columns h*128..), K/V: [batch][skv], O like Q.
 * Replaces flash_attention() / AttentionModule.forward (diffsynth/models/wan_video_dit.py:28-61,
 * 114-121) for self-attention (skv = sq) and T5 cross-attention (skv = 512).
 * With a kind-4 workspace bound on the stream (and O not overlapping Q/K/V) the launch runs the
 * optimistic softmax (no running max; row sums on MFMA) and recomputes, with the checked online
 * softmax, every (batch, head, 256-query) item whose row sum left [2^-64, 2^64] (VS_ATTN_NC=0:
 * checked kernel only).
 */
int vs_attn_fwd(const void* q, const void* k, const void* v, void* o,
                int batch, int sq, int skv, int heads, int head_dim,
                long long ldq, long long ldk, long long ldv, long long ldo,
                long long bsq, long long bsk, long long bsv, long long bso,
                float scale, void* stream);

/*
 * The split-tail plan vs_attn_fwd uses on a device with `cus` compute units: out[0] = whole-item
 * workgroups, out[1] = tail items split over key ranges, out[2] = pieces per tail item,
 * out[3] = 64-key tiles per piece (out[1] = 0: no split).  Host-only, no device call.
 */
int vs_attn_split_plan(int batch, int sq, int skv, int heads, int cus, int* out);

/*
 * Library scratch (kind 0: vs_attn_fwd split tail, 1: vs_gemm split tail, 2 and 3: unused by this
 * build (vs_split_workspace_bytes 0; were the vendor-library route's workspace / staging), 4: vs_attn_fwd
 * item flags, one int per item, ZERO-FILLED by the caller when bound -- every launch leaves it zero;
 * 5: the tile queues of vs_gemm / vs_gemm_fp8's persistent 256x256 kernels, ZERO-FILLED when bound,
 * left zero by every launch -- without one those kernels walk static per-CU tile lists).
 * vs_split_workspace_bytes(kind) is the size that covers every plan of kind 0, 1, 4 or 5 (0: not used);
 * vs_split_workspace_bind(kind, ptr, bytes, stream) registers a caller-owned
 * device buffer (16-B aligned) for launches of that kind on `stream` of the current device
 * (ptr = NULL unbinds).  The buffer must stay valid while bound, including in captured graphs.
 */
long long vs_split_workspace_bytes(int kind);
int vs_split_workspace_bind(int kind, void* ptr, long long bytes, void* stream);

/*
 * Row kernels (vs_layernorm_modulate, _fp8, vs_residual_layernorm, vs_rmsnorm_rope): one 128-thread
 * block per row, 5 chunks of 8 elements per thread up to dim 5120 (every Wan width: 1536 / 5120),
 * 8 chunks up to 8192 (r6; r1-r4 accepted up to 6144, r5 only 5120); dim % 8 == 0 and dim <= 8192,
 * VS_E_INVALID otherwise.
 *
 * out = bf16(LN(x)) [affine: weight/bias] then, if shift/scale given, modulate:
 * bf16(bf16(n * bf16(1+scale)) + shift) with shift/scale rows selected per batch.
 * Replaces WanAutoCastLayerNorm (layers.py:63-92) + modulate (wan_video_dit.py:64-65,225,228,268).
 */
int vs_layernorm_modulate(const void* x, long long ldx, void* out, long long ldo, int rows, int dim,
                          int rows_per_batch, const void* shift, const void* scale,
                          long long mod_bstride, const void* weight, const void* bias, float eps,
                          void* stream);

/* vs_layernorm_modulate into fp8_linear's quantised activation instead of a bf16 row (config 5):
 * x8 [rows, >=dim] e4m3fn bytes and qscale [rows] fp32, exactly vs_quant_fp8_rows of the bf16 rows
 * vs_layernorm_modulate would write (layers.py:115-151). */
int vs_layernorm_modulate_fp8(const void* x, long long ldx, void* x8, long long ld8, float* qscale, int rows,
                              int dim, int rows_per_batch, const void* shift, const void* scale,
                              long long mod_bstride, const void* weight, const void* bias, float eps,
                              void* stream);

/*
 * x = epilogue(y, x) then out = vs_layernorm_modulate(x): the gate-residual / residual epilogue of a
 * projection whose bf16(A W^T + bias) was staged in y, fused with the
 * LayerNorm [+ affine] [+ modulate] that reads the updated row next (wan_video_dit.py:225-228).
 * epilogue: VS_EPI_GATE_RES (epi->gate, gate_bstride, rows_per_batch, optional hint) or VS_EPI_RES
 * (epi->alpha); epi->residual is ignored (x is the residual).  Same rounding points as vs_gemm's
 * epilogue followed by vs_layernorm_modulate: bit-identical to the two calls.  (Used with a GEMM route
 * that stages its output, vs_gemm_route_epi != 0; none in this build.)
 */
int vs_residual_layernorm(const void* y, long long ldy, void* x, long long ldx, void* out, long long ldo, int rows,
                          int dim, int epilogue, const vs_epilogue* epi, int rows_per_batch, const void* shift,
                          const void* scale, long long mod_bstride, const void* weight, const void* bias,
                          float eps, void* stream);

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
/* Same, with dsigma read from device memory (one fp32): lets a hipGraph-captured denoising step
 * be replayed for every step index with the step's dsigma written to that slot before launch. */
int vs_cfg_euler_dev(const void* v_pos, const void* v_neg, void* x, long long n, float cfg_scale,
                     const float* dsigma, int use_cfg, void* stream);

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
/* The same with the packed rows `packed_ld` elements apart (>= cols_per_rank):
 *   packed = j*jstride + (b*s_local + t)*packed_ld + c.
 * With packed_ld = 3*cols_per_rank and q / k / v at column offsets 0 / cpr / 2cpr of each row, the
 * all-to-all of one CFG sample delivers q|k|v rows of the whole sequence in token order, which the
 * attention reads in place (no packed->full pass). */
int vs_ulysses_permute_rows(const void* src, void* dst, int batch, int s_local, int world, int cols_per_rank,
                            long long ld_local, long long jstride, long long packed_ld, int mode, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Ulysses SP collectives over RCCL (xGMI), for hosts without torch.distributed.  Replace the
 * reference's initialize_usp (diffsynth/pipelines/wan_video_new.py:313-323: init_process_group
 * "nccl") and the xfuser/yunchang all-to-all + all_gather of the Ulysses attention and head
 * output (diffsynth/distributed/xdit_context_parallel.py:110-131, wan_video_new.py:1459-1462).
 * One communicator per process and GPU.  RCCL is opened at vs_sp_init (dlopen "librccl.so.1":
 * inside a PyTorch process the copy torch loaded), so the rest of the library does not depend on it.
 * Byte counts are per peer; buffers hold world * bytes_per_rank bytes, chunk j at j*bytes_per_rank
 * (the vs_ulysses_permute packing).  Calls are stream-ordered and enqueue only (no host sync).
 * ------------------------------------------------------------------------------------------- */
#define VS_SP_UNIQUE_ID_BYTES 128
typedef struct vs_sp_comm vs_sp_comm;
/* rank 0 creates the id and hands it to every rank out of band (the torch store, MPI, a file) */
int vs_sp_unique_id(void* out_id);
/* collective over all `world` ranks; binds the communicator to HIP device `device` (the calling
 * thread's current device is restored before returning) */
int vs_sp_init(int rank, int world, const void* unique_id, int device, vs_sp_comm** out);
/* recv chunk j <- chunk `rank` of rank j's send (grouped send/recv, all_to_all_single semantics) */
int vs_sp_all_to_all(vs_sp_comm* comm, const void* send, void* recv, long long bytes_per_rank, void* stream);
/* recv chunk j <- rank j's send (all_gather_into_tensor semantics) */
int vs_sp_all_gather(vs_sp_comm* comm, const void* send, void* recv, long long bytes_per_rank, void* stream);
int vs_sp_comm_destroy(vs_sp_comm* comm);
/* the text of the last RCCL / loader failure of this thread ("" if none) */
const char* vs_sp_last_error(void);

/* ---------------------------------------------------------------------------------------------
 * UMT5-XXL text encoder (diffsynth/models/wan_video_text_encoder.py; GEMMs / norms / per-head
 * products go through vs_gemm, vs_rmsnorm_rope and the batched mode of vs_vae_conv).
 * ------------------------------------------------------------------------------------------- */

/* out[r] = table[ids[r]] (nn.Embedding, :233); ids int64, rows of dim bf16. */
int vs_embed_rows(const long long* ids, const void* table, long long ld_table, long long vocab, void* out,
                  long long ld_out, long long rows, int dim, void* stream);

/* T5Attention scores -> probabilities (:69-83): for head z (global head head0 + z), query i, key j:
 * v = bf16(bf16(s) + bias), bias = emb[buckets[i*L + j]][head0 + z] (bf16, per-block relative
 * position embedding) or the bf16 lowest value where keymask[j] == 0; p = bf16(softmax_j(v)) in
 * fp32.  s fp32 [nz][L][ld_s], p bf16 [nz][L][ld_p] (columns >= L written 0), buckets int32 [L][L]. */
int vs_t5_bias_softmax(const float* s, long long zs_s, long long ld_s, void* p, long long zs_p, long long ld_p,
                       const int* buckets, const void* emb, int nheads, int head0, const int* keymask, int L, int nz,
                       void* stream);

/* out = bf16(a * gelu(g)) with the tanh-GELU evaluated op by op in bf16 (GELU :15-19,
 * T5FeedForward :105-110). */
int vs_t5_gelu_mul(const void* a, const void* g, void* out, long long n, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Causal 3-D VAE (diffsynth/models/wan_video_vae.py, Wan2.1 part).  Activations are channels-last
 * "NTHWC" tiles: element (n, t, y, x, c) of a tensor lives at base + n*ns + ((t*H + y)*W + x)*ld + c.
 * ------------------------------------------------------------------------------------------- */

/* Implicit-GEMM convolution (MFMA), one call per CausalConv3d / Conv2d / 1x1 conv of the VAE:
 *   y(z, n, t, yo, xo, co) = bf16(bias[co] + sum_{kt,ky,kx,ci} X(z, n, t*st+kt-pt, ...)*W[co][kt][ky][kx][ci])
 * X is read as zero outside [t_lo, t_in) x [0, H) x [0, W) (causal time pad, spatial zero pad,
 * ZeroPad2d), through a fused nearest-x2 spatial upsample when up2 (wan_video_vae.py:73-79,94,98).
 * Output frame = t*t_mul + t_add (+1 for co >= split when split > 0: the channel->time interleave
 * of Resample upsample3d, :153-156); res (same geometry as y) adds the ResidualBlock shortcut
 * bf16(bf16(conv) + res) (:301).  out_f32 = 1 writes fp32 alpha*acc instead (attention scores).
 * Also a batched plain GEMM (kt=kh=kw=1, t_in=h_in=1, w_in=rows) over nz slices with *_zs strides.
 * Requires cin % 32 == 0, ldx/ldw % 8 == 0; weights are [cout][kt*kh*kw*cin] (ci fastest).
 * Replaces CausalConv3d.forward (:33-52) and the nn.Conv2d of Resample / AttentionBlock. */
typedef struct vs_conv3d {
    const void* x; long long x_zs, x_ns, ldx;
    int n, t_in, h_in, w_in, cin;
    int kt, kh, kw, st, sh, sw, pt, ph, pw, up2, t_lo;
    int t_out, h_out, w_out;
    const void* w; long long w_zs, ldw;
    const void* bias;           /* bf16 [cout] or NULL */
    int cout;
    void* y; long long y_zs, y_ns, ldy;
    int t_mul, t_add, split, out_f32;
    float alpha;
    const void* res;            /* bf16, geometry of y, or NULL */
    int nz;
} vs_conv3d;
int vs_vae_conv(const vs_conv3d* p, void* stream);

/* RMS_norm over channels (F.normalize(x, dim=C) * sqrt(C) * gamma, wan_video_vae.py:55-70) with
 * the bf16 rounding points of the reference, optionally followed by nn.SiLU (:276-278); the fp32
 * division and SiLU are evaluated with a per-row reciprocal and exp2/rcp (within one bf16 ulp).
 * x, y: npix rows of c channels (row strides ldx, ldy); c % 32 == 0, c <= 384. */
int vs_vae_rmsnorm(const void* x, long long ldx, void* y, long long ldy, const void* gamma,
                   long long npix, int c, int silu, void* stream);

/* Row softmax of fp32 scores s[rows][ld_s] over the first ncols columns -> bf16 p[rows][ld_p],
 * columns ncols..ld_p-1 written as 0 (AttentionBlock F.scaled_dot_product_attention, :331). */
int vs_vae_softmax(const float* s, long long ld_s, void* p, long long ld_p, long long rows, int ncols,
                   void* stream);

/* Flash form of the same attention (csrc/vae_attention.hip): for each of nz frames z,
 * out[z][r][:c] = softmax(q k^T / sqrt(c)) v over `rows` pixels, with q | k | v the columns [0, c) |
 * [c, 2c) | [2c, 3c) of qkv[z][r] (the to_qkv output, row stride ld_qkv, frame stride qkv_zs); the
 * softmax exact (two passes over K), rounded to bf16 before P.V as vs_vae_softmax; no score
 * buffer.  c % 128 == 0, c <= 384; ld_qkv % 8 == 0, qkv 16-B aligned, ld_o % 4 == 0.
 * Replaces AttentionBlock's F.scaled_dot_product_attention (wan_video_vae.py:330-335). */
int vs_vae_attention(const void* qkv, long long qkv_zs, long long ld_qkv, void* out, long long o_zs,
                     long long ld_o, int nz, int rows, int c, void* stream);

/* vt[z][c][r] = v[z][r][c] for r < rows, 0 for rows <= r < ld_vt (V^T operand of P.V). */
int vs_vae_transpose(const void* v, long long v_zs, long long ld_v, void* vt, long long vt_zs,
                     long long ld_vt, int nz, int rows, int cols, void* stream);

/* Tile cut of the first t frames of an NCTHW bf16 tensor src[C][t_src][H][W] into an NTHWC tile
 * dst[t][th][tw][cpad]
 * (channels >= C zero) with an optional per-channel affine (mode 0 none; 1: bf16(bf16(x-a)*b),
 * the encode latent normalisation :1004-1005; 2: bf16(bf16(x/b)+a), the decode de-normalisation
 * :1016-1017).  Replaces the video[:, :, :, h:h_, w:w_] slicing of tiled_encode/tiled_decode. */
int vs_vae_tile_gather(const void* src, int c, int t_src, int h, int w, int t, int h0, int w0, int th,
                       int tw, void* dst, int cpad, int mode, const void* a, const void* b, void* stream);

/* One step of the tiled blend (wan_video_vae.py:1081-1101,1128-1149,1180-1201), in the reference's
 * bf16 arithmetic and task order: values[c][t][h0+i][w0+j] += bf16(tile * mask), weight += mask,
 * mask = bf16(min(ramp_h(i), ramp_w(j))) with linear ramps of widths bw_h/bw_w on the non-bound
 * edges (bound = bit0 top, bit1 bottom, bit2 left, bit3 right).  tile is NTHWC [t][th][tw][ldc]
 * (with the per-channel affine `mode` of vs_vae_tile_gather applied first); values is NCTHW
 * [c][t][H][W], weight [t][H][W], both bf16. */
int vs_vae_tile_blend(const void* tile, long long ldc, int c, int t, int th, int tw, void* values,
                      void* weight, int h, int w, int h0, int w0, int bound, int bw_h, int bw_w,
                      int mode, const void* a, const void* b, void* stream);

/* out = bf16(values / weight) (weight broadcast over channels), clamped to [-1, 1] if clamp. */
int vs_vae_blend_finish(const void* values, const void* weight, void* out, int c, long long plane,
                        int clamp, void* stream);

/* BasePipeline.vae_output_to_video (diffsynth/pipelines/wan_video_new.py:557 -> utils/__init__.py:76-91) for B = 1:
 * video bf16 [3][t][h][w] in [-1, 1] -> out uint8 [t][h][w][3] = trunc(clip(bf16(bf16(x+1)*127.5))). */
int vs_vae_to_u8(const void* video, void* out, int t, int h, int w, void* stream);

/* WanVideoUnit_VACE.process (diffsynth/pipelines/wan_video_new.py:878-888): uint8 frames
 * [t][h][w][3] (video_u8 NULL = zeros, mask_u8 NULL = ones) -> preprocess_video to bf16 in [-1, 1]
 * (mask in [0, 1]), inactive = v*(1-m) + 0*m and reactive = v*m + 0*(1-m) as NCTHW [3][t][h][w]
 * bf16, and mask channel 0 as mask0 [t][h][w] bf16 -- the reference's bf16 rounding points. */
int vs_vace_prepare(const void* video_u8, const void* mask_u8, void* inactive, void* reactive, void* mask0,
                    int t, int h, int w, void* stream);

/* VACE mask latents (wan_video_new.py:893-894): out [64][t_out][h/8][w/8] bf16 (a channel slice of
 * vace_context) = nearest-exact temporal resize of rearrange(mask0, "T (H 8) (W 8) -> (8 8) T H W"). */
int vs_vace_mask_latents(const void* mask0, void* out, int t, int h, int w, int t_out, void* stream);

/* UniPC multistep tensor update (FlowUniPCMultistepScheduler,
 * denoising_enhancing/wan/utils/fm_solvers_unipc.py:281-628; config 5's 4-step sampler), fp32 with the reference's op order:
 * mode 0 convert out = x - c1*mt; 1 UniP order 1; 2 UniP order 2; 3 UniC order 1; 4 UniC order 2
 * (formulas at the kernel).  coef = host array {c1, c2, c3, r0, r1, rk} computed by the scheduler.
 * Pointers not used by a mode may be NULL. */
int vs_unipc_update(float* out, const float* x, const float* m0, const float* m1, const float* mt, long long n,
                    int mode, const float* coef, void* stream);

/* Elementwise dtype cast: to_bf16 = 1: fp32 -> bf16 (RNE), 0: bf16 -> fp32. */
int vs_cast(const void* src, void* dst, long long n, int to_bf16, void* stream);

/* Copy n frames of frame_elems elements (src/dst strides per n in elements): the pass-through
 * first frame of Resample downsample3d/upsample3d (:125-127,165-167). */
int vs_vae_copy_frames(const void* src, long long src_ns, void* dst, long long dst_ns, int n,
                       long long frame_elems, void* stream);


#ifdef __cplusplus
}
#endif
#endif /* VSTYLER_H */
