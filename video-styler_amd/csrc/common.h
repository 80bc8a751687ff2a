// Shared device helpers for the gfx950 kernels of libvstyler.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/vstyler.h"

typedef uint16_t bf16_t;  // raw bf16 bits in global memory
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef short i16x4_t __attribute__((ext_vector_type(4)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));

#define LDS_AS __attribute__((address_space(3)))
#define GLB_AS __attribute__((address_space(1)))

__device__ __forceinline__ float bf2f(uint32_t h) { return __uint_as_float(h << 16); }
__device__ __forceinline__ float bflo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bfhi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

// round-to-nearest-even fp32 -> bf16 (hipcc lowers the __bf16 cast to v_cvt_pk_bf16_f32 on gfx950)
__device__ __forceinline__ uint32_t f2bf(float f) {
    return (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)f);
}
__device__ __forceinline__ uint32_t pack2(float lo, float hi) { return f2bf(lo) | (f2bf(hi) << 16); }
// materialise a bf16 rounding point inside fp32 arithmetic
__device__ __forceinline__ float rbf(float f) { return bf2f(f2bf(f)); }

__device__ __forceinline__ float gelu_tanh_f(float x) {
    // 0.5*x*(1+tanh(sqrt(2/pi)*(x+0.044715x^3)))  (torch GELU approximate='tanh')
    const float k0 = 0.7978845608028654f, k1 = 0.044715f;
    float u = k0 * (x + k1 * x * x * x);
    // 0.5 x (1 + tanh u) == x * sigmoid(2u) == x / (1 + 2^(-2 log2(e) u)): one v_exp_f32 and one
    // v_rcp_f32 (~3 fp32 ulp) instead of the ~40-instruction libm tanhf, which made the GELU pass
    // of the hipBLASLt route VALU-bound (0.93 ms for 1.6 GB in + out at 59280 x 13824); the tanh
    // form's cancellation-free limits hold (u -> -inf: x * rcp(inf) = -0; u -> +inf: x)
    return x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-2.8853900817779268f * u));
}
__device__ __forceinline__ float silu_f(float x) { return x / (1.0f + expf(-x)); }

// Bijective XCD-aware remap of a linear workgroup id (MI355X deals workgroups round-robin over
// 8 XCDs; this gives each XCD a contiguous chunk of the logical id space so that neighbouring
// tiles share that XCD's L2).  cdna_hip_programming.md §5 "XCD swizzle must be bijective".
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
    const int nx = 8;
    int q = nwg / nx, r = nwg % nx;
    int xcd = orig % nx, loc = orig / nx;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
}

#define VS_CHECK_LAUNCH()                                            \
    do {                                                             \
        if (hipGetLastError() != hipSuccess) return VS_E_LAUNCH;     \
    } while (0)

// ---- host helpers shared by the split-tail launches (attention.hip, gemm.hip) ----------------
#include <cstdlib>
#include <map>
#include <mutex>
#include <tuple>

// Path-selection options (include/vstyler.h VS_OPT_*; set by vs_set_option, attention.hip): one
// process-wide table, product defaults; the library reads no environment variable.
inline volatile int g_vs_opt[VS_OPT_COUNT] = {0, 4, 1, 1, 0, 16, 1, 1, 1, 2, 3, 1, 1};
inline int vs_opt(int id) { return g_vs_opt[id]; }

// ---- work queues of the persistent kernels (gemm.hip W4Grab, attention_w4.hip): head words in a
// caller-bound zeroed workspace (kind 5), one 128-B line each; the last block of a launch zeroes them.
constexpr int VS_Q_LINE = 32;                 // words per line
constexpr int VS_Q_ATTN = 16 * VS_Q_LINE;     // attention's words start 2 KB into the workspace

// One returning device-scope atomic add of 1 by lane 0 of the calling wave (EXEC set to lane 0 inside
// the asm, so no exec-masked region for the compiler to merge around the result).  Inline asm: as a
// compiler-visible atomic its value's first use made the compiler drain every in-flight load first
// (vmcnt(0)); the caller retires it with a counted wait instead (vs_queue_value).
__device__ __forceinline__ unsigned vs_queue_issue(unsigned* p) {
    unsigned t;
    unsigned long long sv;
    asm volatile("s_mov_b64 %1, exec\n\t"
                 "s_mov_b64 exec, 1\n\t"
                 "global_atomic_add %0, %2, %3, %4 sc0\n\t"
                 "s_mov_b64 exec, %1"
                 : "=&v"(t), "=&s"(sv)
                 : "v"(0), "v"(1u), "s"(p)
                 : "memory");
    return t;
}
// lane 0's returned value, wave-uniform, after vmcnt(W): the caller has issued at least W vector
// memory operations since vs_queue_issue (they complete in issue order)
template <int W>
__device__ __forceinline__ unsigned vs_queue_value(unsigned t0) {
    unsigned t;
    asm volatile("s_waitcnt vmcnt(%1)\n\tv_readfirstlane_b32 %0, %2" : "=s"(t) : "n"(W), "v"(t0) : "memory");
    return t;
}
__device__ __forceinline__ unsigned vs_queue_add(unsigned* p) {
    return __hip_atomic_fetch_add(p, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// after a persistent block's last item: the last of `nblocks` to get here zeroes `nlines` lines
__device__ __forceinline__ void vs_queue_done(unsigned* q, int nlines, int nblocks) {
    if (vs_queue_add(q + (nlines - 1) * VS_Q_LINE) == (unsigned)nblocks - 1)
        for (int i = 0; i < nlines; ++i) __hip_atomic_store(q + i * VS_Q_LINE, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// compute units of the current device (0 when unknown or when `off`: no split)
inline int vs_cus_for_split(bool off) {
    if (off) return 0;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    static std::mutex mu;
    static std::map<int, int> cache;
    std::lock_guard<std::mutex> lock(mu);
    auto it = cache.find(dev);
    if (it != cache.end()) return it->second;
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) n = 0;
    cache[dev] = n;
    return n;
}

// Split-tail scratch is caller-owned (the library never allocates): the host binds one fp32
// workspace per (kind, device, stream) with vs_split_workspace_bind; a launch on a stream without
// one runs unsplit.  kind 0: attention split tail, 1: GEMM split tail, 2 / 3: unused (r1-r5's
// vendor-library workspace and epilogue staging),
// 4: attention item flags, 5: the 4-wave GEMMs' tile-queue words (4 and 5 bound zero-filled; the
// kernels leave them zero).
struct VsWs { float* ptr; long long bytes; };
inline std::map<std::tuple<int, int, hipStream_t>, VsWs>& vs_ws_registry(std::mutex*& mu) {
    static std::mutex m;
    static std::map<std::tuple<int, int, hipStream_t>, VsWs> reg;
    mu = &m;
    return reg;
}
inline float* vs_bound_workspace(int kind, int dev, hipStream_t stream, long long* bytes) {
    std::mutex* mu;
    auto& reg = vs_ws_registry(mu);
    std::lock_guard<std::mutex> lock(*mu);
    auto it = reg.find({kind, dev, stream});
    if (it == reg.end()) return nullptr;
    if (bytes) *bytes = it->second.bytes;
    return it->second.ptr;
}
inline float* vs_split_workspace(int kind, size_t bytes, hipStream_t stream) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    long long have = 0;
    float* p = vs_bound_workspace(kind, dev, stream, &have);
    return (p && have >= (long long)bytes) ? p : nullptr;
}

long long vs_gemm_split_workspace_bytes_impl();   // gemm.hip
