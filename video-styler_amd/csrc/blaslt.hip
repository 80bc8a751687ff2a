// hipBLASLt for the plain part of the block GEMMs (host code only).
//
// The task's rule for MI355X: hand-written MFMA kernels for fused hot ops, the vendor library for
// plain library GEMMs.  Measured on MI355X (profiles/r1/gemm_backend_ab_*.log), hipBLASLt's
// stream-K 256x256x64 kernels run the 14B block GEMMs at 1240-1500 TF/s where gemm_bf16_tn_256
// reaches 1040-1210, so vs_gemm routes C = A W^T + bias to hipBLASLt (one bf16 rounding of
// acc + bias, exactly the first rounding point of every vs_gemm epilogue) and finishes any
// further epilogue (GELU, SiLU, gate-residual [+ VACE hint], residual) with gemm_epi_apply,
// which continues from that rounded value with the same code as the fused epilogue -- so both
// paths have the reference's rounding points and differ only in fp32 summation order.
//
// Column-major view: C[m][n] row-major is D = W^T(op T on the [k x n] col-major view of W[n][k])
// times A (op N on the [k x m] col-major view of A[m][k]): D is n x m col-major with ld = ldc,
// and the bias runs along D's rows (n), hipBLASLt's BIAS epilogue.
#include "common.h"

#include <hipblaslt/hipblaslt.h>

#include <algorithm>
#include <cstdlib>
#include <vector>

namespace {

struct LtKey {
    int dev, m, n, k;
    long long lda, ldw, ldc;
    bool bias;
    bool fp8;          // e4m3fn operands with a per-row (per-token) fp32 scale on A
    bool gelu;         // hipBLASLt's GELU epilogue on the fp32 acc + bias (one bf16 rounding)
    bool operator<(const LtKey& o) const {
        return std::tie(dev, m, n, k, lda, ldw, ldc, bias, fp8, gelu) <
               std::tie(o.dev, o.m, o.n, o.k, o.lda, o.ldw, o.ldc, o.bias, o.fp8, o.gelu);
    }
};

struct LtPlan {
    hipblasLtMatmulDesc_t desc = nullptr;
    hipblasLtMatrixLayout_t lw = nullptr, la = nullptr, lc = nullptr;
    hipblasLtMatmulAlgo_t algo;
    size_t ws_need = 0;
    bool ok = false, tuned = false;
    int pick = 0;                                       // index of the algorithm in use in cand
    std::vector<hipblasLtMatmulHeuristicResult_t> cand;
};

std::mutex g_mu;
std::map<int, hipblasLtHandle_t> g_handles;
std::map<LtKey, LtPlan> g_plans;

hipblasLtHandle_t handle_for(int dev) {
    auto it = g_handles.find(dev);
    if (it != g_handles.end()) return it->second;
    hipblasLtHandle_t h = nullptr;
    if (hipblasLtCreate(&h) != HIPBLAS_STATUS_SUCCESS) h = nullptr;
    g_handles[dev] = h;
    return h;
}

// builds (once per shape) the descriptor, the layouts and the heuristic's first algorithm that
// fits `ws_bytes` of workspace
LtPlan* plan_for(const LtKey& key, size_t ws_bytes) {
    auto it = g_plans.find(key);
    if (it != g_plans.end()) return it->second.ok ? &it->second : nullptr;
    LtPlan& p = g_plans[key];
    hipblasLtHandle_t h = handle_for(key.dev);
    if (!h) return nullptr;
    if (hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F) != HIPBLAS_STATUS_SUCCESS) return nullptr;
    const hipblasOperation_t opT = HIPBLAS_OP_T, opN = HIPBLAS_OP_N;
    hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &opT, sizeof(opT));
    hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &opN, sizeof(opN));
    if (key.bias || key.gelu) {
        const hipblasLtEpilogue_t epi = key.gelu ? (key.bias ? HIPBLASLT_EPILOGUE_GELU_BIAS : HIPBLASLT_EPILOGUE_GELU)
                                                 : HIPBLASLT_EPILOGUE_BIAS;
        hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &epi, sizeof(epi));
    }
    if (key.bias) {
        const hipDataType bt = HIP_R_16BF;
        hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt));
    }
    const hipDataType in_t = key.fp8 ? HIP_R_8F_E4M3 : HIP_R_16BF;
    if (key.fp8) {
        // fp8_linear (layers.py:115-151): (x8 . w8^T) * scale_x[row] + bias, one bf16 rounding; the
        // token axis is D's column axis here, hipBLASLt's "B" outer scale vector
        const hipblasLtMatmulMatrixScale_t vec = HIPBLASLT_MATMUL_MATRIX_SCALE_OUTER_VEC_32F;
        hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_B_SCALE_MODE, &vec, sizeof(vec));
    }
    if (hipblasLtMatrixLayoutCreate(&p.lw, in_t, key.k, key.n, key.ldw) != HIPBLAS_STATUS_SUCCESS ||
        hipblasLtMatrixLayoutCreate(&p.la, in_t, key.k, key.m, key.lda) != HIPBLAS_STATUS_SUCCESS ||
        hipblasLtMatrixLayoutCreate(&p.lc, HIP_R_16BF, key.n, key.m, key.ldc) != HIPBLAS_STATUS_SUCCESS)
        return nullptr;
    hipblasLtMatmulPreference_t pref = nullptr;
    if (hipblasLtMatmulPreferenceCreate(&pref) != HIPBLAS_STATUS_SUCCESS) return nullptr;
    const uint64_t wsb = ws_bytes;
    hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb, sizeof(wsb));
    // candidates the autotune times: 16 (VS_LT_NCAND = 1..64 for A/B runs)
    constexpr int MAXCAND = 64;
    int ncand = 16;
    if (const char* e = std::getenv("VS_LT_NCAND")) ncand = std::min(MAXCAND, std::max(1, std::atoi(e)));
    hipblasLtMatmulHeuristicResult_t res[MAXCAND];
    int found = 0;
    const hipblasStatus_t st =
        hipblasLtMatmulAlgoGetHeuristic(h, p.desc, p.lw, p.la, p.lc, p.lc, pref, ncand, res, &found);
    hipblasLtMatmulPreferenceDestroy(pref);
    if (st != HIPBLAS_STATUS_SUCCESS || found < 1) return nullptr;
    p.cand.assign(res, res + found);
    p.algo = res[0].algo;
    p.ws_need = res[0].workspaceSize;
    p.ok = true;
    return &p;
}

// Autotune (once per shape, on its first eager call): time every candidate of the heuristic's
// list on the call's own operands and keep the fastest.  The heuristic's first pick is not the
// fastest on every block shape (profiles/r1/gemm_lt_tune_*.log).  Skipped while the stream is
// being captured into a graph (no host sync possible) and with VS_LT_TUNE=0.
void autotune(LtPlan& p, hipblasLtHandle_t h, const void* a, const void* w, void* c, float* ws, size_t ws_bytes,
              hipStream_t stream) {
    if (p.cand.size() < 2) { p.tuned = true; return; }
    const char* env = std::getenv("VS_LT_TUNE");
    if (env && env[0] == '0') { p.tuned = true; return; }
    // inside a graph capture: keep the heuristic pick for now and tune on a later eager call
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(stream, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return;
    p.tuned = true;
    hipEvent_t e0, e1;
    if (hipEventCreate(&e0) != hipSuccess) return;
    if (hipEventCreate(&e1) != hipSuccess) { (void)hipEventDestroy(e0); return; }
    const float alpha = 1.f, beta = 0.f;
    float best = 1e30f, first = 1e30f;
    size_t bi = 0;
    for (size_t i = 0; i < p.cand.size(); ++i) {
        if (p.cand[i].workspaceSize > ws_bytes) continue;
        auto run = [&]() {
            return hipblasLtMatmul(h, p.desc, &alpha, w, p.lw, a, p.la, &beta, c, p.lc, c, p.lc, &p.cand[i].algo, ws,
                                   ws_bytes, stream);
        };
        if (run() != HIPBLAS_STATUS_SUCCESS) continue;
        (void)hipEventRecord(e0, stream);
        bool ok = true;
        for (int r = 0; r < 3 && ok; ++r) ok = run() == HIPBLAS_STATUS_SUCCESS;
        (void)hipEventRecord(e1, stream);
        if (!ok || hipEventSynchronize(e1) != hipSuccess) continue;
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (i == 0) first = ms;
        if (ms < best) { best = ms; bi = i; }
    }
    // keep the heuristic's (deterministic) first pick unless another candidate is clearly faster,
    // so that timing noise between near-equal candidates does not change the algorithm -- and the
    // fp32 summation order -- from run to run or rank to rank
    if (best > 0.97f * first) bi = 0;
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    p.algo = p.cand[bi].algo;
    p.ws_need = p.cand[bi].workspaceSize;
    p.pick = (int)bi;
}

}  // namespace

namespace {
int lt_gemm(const void* a, long long lda, const void* w, long long ldw, void* c, long long ldc, int m, int n, int k,
            const void* bias, const float* scale_a, bool gelu, hipStream_t stream) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return VS_E_LAUNCH;
    long long ws_bytes = 0;
    float* ws = vs_bound_workspace(2, dev, stream, &ws_bytes);
    if (!ws) return VS_E_UNSUPPORTED;
    std::lock_guard<std::mutex> lock(g_mu);
    const LtKey key{dev, m, n, k, lda, ldw, ldc, bias != nullptr, scale_a != nullptr, gelu};
    LtPlan* p = plan_for(key, (size_t)ws_bytes);
    if (!p || p->ws_need > (size_t)ws_bytes) return VS_E_UNSUPPORTED;
    if (bias)
        hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias));
    if (scale_a)
        hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_B_SCALE_POINTER, &scale_a, sizeof(scale_a));
    if (!p->tuned) autotune(*p, handle_for(dev), a, w, c, ws, (size_t)ws_bytes, stream);
    const float alpha = 1.f, beta = 0.f;
    const hipblasStatus_t st = hipblasLtMatmul(handle_for(dev), p->desc, &alpha, w, p->lw, a, p->la, &beta, c, p->lc,
                                               c, p->lc, &p->algo, ws, (size_t)ws_bytes, stream);
    return st == HIPBLAS_STATUS_SUCCESS ? VS_OK : VS_E_LAUNCH;
}
}  // namespace

// C[m][n] (ld ldc) = bf16(A W^T + bias) on `stream` with hipBLASLt; 0 on success, VS_E_UNSUPPORTED
// when hipBLASLt has no algorithm for the shape or the bound workspace (kind 2) is too small.
int vs_lt_gemm_bias(const void* a, long long lda, const void* w, long long ldw, void* c, long long ldc, int m,
                    int n, int k, const void* bias, hipStream_t stream) {
    return lt_gemm(a, lda, w, ldw, c, ldc, m, n, k, bias, nullptr, false, stream);
}

// C[m][n] = bf16(GELU_tanh(A W^T + bias)) with hipBLASLt's fused GELU epilogue (the GELU of the fp32
// acc + bias, not of its bf16 rounding); same contract.
int vs_lt_gemm_bias_gelu(const void* a, long long lda, const void* w, long long ldw, void* c, long long ldc, int m,
                         int n, int k, const void* bias, hipStream_t stream) {
    return lt_gemm(a, lda, w, ldw, c, ldc, m, n, k, bias, nullptr, true, stream);
}

// C[m][n] = bf16((A8 W8^T) * scale_a[row] + bias), e4m3fn operands (fp8_linear), with `gelu` the
// GELU-tanh of that fp32 value before the rounding; same contract.
int vs_lt_gemm_fp8(const void* a8, long long lda, const float* scale_a, const void* w8, long long ldw, void* c,
                   long long ldc, int m, int n, int k, const void* bias, bool gelu, hipStream_t stream) {
    return lt_gemm(a8, lda, w8, ldw, c, ldc, m, n, k, bias, scale_a, gelu, stream);
}
