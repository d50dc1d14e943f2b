// prt_trace_pool.hip — the block-pooled shadow-query trace kernel (prt_device.h trace_kernel_pool)
// in its own compilation unit: pyrenderer_amd/build.py compiles it with LLVM's AMDGPU
// register-pressure trackers (-mllvm --amdgpu-use-amdgpu-trackers), under which the kernel fits
// the 72 VGPRs of 7 waves per SIMD with 3 spilled registers instead of 39 (the other trace
// kernels keep the default scheduler: the global-scene kernel is slower with the trackers,
// DESIGN.md §2).  One schedule: extension traversals, then the pooled shadow rays in 64-ray
// chunks after the block barrier (round 5's fused, packed-leaf and split-arrival schedules were
// removed in round 6: none became the default).
#pragma clang fp contract(off)

#include "prt_device.h"

namespace prt {

namespace {
template <bool STATS, int WPE>
hipError_t launch_pool(const TraceParams& P, int grid, size_t smem, hipStream_t stream) {
    if (P.plain) trace_kernel_pool<STATS, WPE, true><<<grid, kBlock, smem, stream>>>(P);
    else trace_kernel_pool<STATS, WPE, false><<<grid, kBlock, smem, stream>>>(P);
    return hipGetLastError();
}
}  // namespace

hipError_t launch_trace_pool(const TraceParams& P, bool stats, int wpe, int grid, size_t smem, hipStream_t stream) {
    if (wpe != 7 && wpe != 6) return hipErrorInvalidValue;
    if (stats)
        return wpe == 7 ? launch_pool<true, 7>(P, grid, smem, stream) : launch_pool<true, 6>(P, grid, smem, stream);
    return wpe == 7 ? launch_pool<false, 7>(P, grid, smem, stream) : launch_pool<false, 6>(P, grid, smem, stream);
}

// both builds of one (stats, waves per EU) fit the same blocks per CU (the waves-per-EU target and
// the LDS size set it)
int trace_occ_pool(bool stats, int wpe, size_t smem) {
    int n = 0;
    if (stats && wpe == 7)
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, trace_kernel_pool<true, 7, false>, kBlock, smem);
    else if (stats && wpe == 6)
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, trace_kernel_pool<true, 6, false>, kBlock, smem);
    else if (wpe == 7)
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, trace_kernel_pool<false, 7, false>, kBlock, smem);
    else if (wpe == 6)
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, trace_kernel_pool<false, 6, false>, kBlock, smem);
    return n;
}

}  // namespace prt
