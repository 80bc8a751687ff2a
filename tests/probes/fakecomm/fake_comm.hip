// Probe only: a stand-in for RCCL's all-to-all kernel on a one-GPU box -- `nblocks` long-lived
// workgroups (RCCL's channels) copying src -> dst, launched on a side stream beside the compute
// kernels, to see how the persistent / full-chip compute grids share the CUs with it.
#include <hip/hip_runtime.h>
#include <cstddef>

__global__ __launch_bounds__(256) void fake_copy(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) dst[i] = src[i];
}

extern "C" int fake_comm(const void* src, void* dst, size_t bytes, int nblocks, void* stream) {
    hipLaunchKernelGGL(fake_copy, dim3(nblocks), dim3(256), 0, (hipStream_t)stream, (const uint4*)src, (uint4*)dst,
                       bytes / 16);
    return hipGetLastError() == hipSuccess ? 0 : 1;
}

// Probe only: `nblocks` workgroups that each hold a CU (64 KB of LDS: a 256x256 GEMM or attention
// workgroup no longer fits beside one) for `usec` microseconds of wall clock -- a collective kernel
// occupying CUs while a persistent compute grid launches (tests/probes/cu_hold.py).
__global__ __launch_bounds__(64) void cu_hog(long long ticks) {
    extern __shared__ char lds[];
    const long long t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
    if (threadIdx.x == 0 && ticks < 0) lds[0] = 1;          // (keeps the LDS allocation)
}

// a short delay on the compute stream, so the hog is resident before the measured launch
__global__ void spin_us(long long ticks) {
    const long long t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

extern "C" int cu_hold(int nblocks, double usec, void* stream) {
    const long long ticks = (long long)(usec * 100.0);      // wall_clock64: 100 MHz
    (void)hipFuncSetAttribute((const void*)cu_hog, hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
    hipLaunchKernelGGL(cu_hog, dim3(nblocks), dim3(64), 65536, (hipStream_t)stream, ticks);
    return hipGetLastError() == hipSuccess ? 0 : 1;
}

extern "C" int delay_us(double usec, void* stream) {
    hipLaunchKernelGGL(spin_us, dim3(1), dim3(64), 0, (hipStream_t)stream, (long long)(usec * 100.0));
    return hipGetLastError() == hipSuccess ? 0 : 1;
}
