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
