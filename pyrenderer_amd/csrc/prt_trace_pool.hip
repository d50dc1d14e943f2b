// prt_trace_pool.hip — the block-pooled shadow-query trace kernel (prt_device.h trace_kernel_pool)
// in its own compilation unit: pyrenderer_amd/build.py compiles it with LLVM's AMDGPU
// register-pressure trackers (-mllvm --amdgpu-use-amdgpu-trackers), under which the kernel fits
// the 72 VGPRs of 7 waves per SIMD with 4 spilled registers instead of 39 (the other trace
// kernels keep the default scheduler: the global-scene kernel is slower with the trackers,
// DESIGN.md §2).
#pragma clang fp contract(off)

#include "prt_device.h"

namespace prt {

hipError_t launch_trace_pool(const TraceParams& P, bool stats, int wpe, int grid, size_t smem, hipStream_t stream) {
    if (stats) {
        if (wpe == 7) trace_kernel_pool<true, 7><<<grid, kBlock, smem, stream>>>(P);
        else if (wpe == 6) trace_kernel_pool<true, 6><<<grid, kBlock, smem, stream>>>(P);
        else return hipErrorInvalidValue;
    } else {
        if (wpe == 7) trace_kernel_pool<false, 7><<<grid, kBlock, smem, stream>>>(P);
        else if (wpe == 6) trace_kernel_pool<false, 6><<<grid, kBlock, smem, stream>>>(P);
        else return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

int trace_occ_pool(bool stats, int wpe, size_t smem) {
    int n = 0;
    if (stats) {
        if (wpe == 7) (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, trace_kernel_pool<true, 7>, kBlock, smem);
        else if (wpe == 6) (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, trace_kernel_pool<true, 6>, kBlock, smem);
    } else {
        if (wpe == 7) (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, trace_kernel_pool<false, 7>, kBlock, smem);
        else if (wpe == 6) (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, trace_kernel_pool<false, 6>, kBlock, smem);
    }
    return n;
}

}  // namespace prt
