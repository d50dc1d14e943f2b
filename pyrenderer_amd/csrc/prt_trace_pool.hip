// prt_trace_pool.hip — the block-pooled shadow-query trace kernel (prt_device.h trace_kernel_pool)
// in its own compilation unit: pyrenderer_amd/build.py compiles it with LLVM's AMDGPU
// register-pressure trackers (-mllvm --amdgpu-use-amdgpu-trackers), under which the kernel fits
// the 72 VGPRs of 7 waves per SIMD with 3 spilled registers instead of 39 (the other trace
// kernels keep the default scheduler: the global-scene kernel is slower with the trackers,
// DESIGN.md §2).  Two schedules: the two-phase kernel (extension traversals, then the pooled
// shadow rays in 64-ray chunks after the block barrier) and FUSED (round 5: idle lanes of the
// extension traversals take the previous iteration's pooled shadow rays).
#pragma clang fp contract(off)

#include "prt_device.h"

namespace prt {

namespace {
template <bool STATS, int WPE, bool FUSED>
hipError_t launch_pool(const TraceParams& P, int grid, size_t smem, hipStream_t stream) {
    if (P.plain) trace_kernel_pool<STATS, WPE, true, FUSED><<<grid, kBlock, smem, stream>>>(P);
    else trace_kernel_pool<STATS, WPE, false, FUSED><<<grid, kBlock, smem, stream>>>(P);
    return hipGetLastError();
}
template <bool FUSED>
hipError_t launch_pool_f(const TraceParams& P, bool stats, int wpe, int grid, size_t smem, hipStream_t stream) {
    if (stats)
        return wpe == 7 ? launch_pool<true, 7, FUSED>(P, grid, smem, stream) : launch_pool<true, 6, FUSED>(P, grid, smem, stream);
    return wpe == 7 ? launch_pool<false, 7, FUSED>(P, grid, smem, stream) : launch_pool<false, 6, FUSED>(P, grid, smem, stream);
}
template <bool STATS, int WPE, bool FUSED>
int occ_pool(size_t smem) {
    int n = 0;
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, trace_kernel_pool<STATS, WPE, false, FUSED>, kBlock, smem);
    return n;
}
}  // namespace

hipError_t launch_trace_pool(const TraceParams& P, bool stats, int wpe, bool fused, int grid, size_t smem,
                             hipStream_t stream) {
    if (wpe != 7 && wpe != 6) return hipErrorInvalidValue;
    return fused ? launch_pool_f<true>(P, stats, wpe, grid, smem, stream)
                 : launch_pool_f<false>(P, stats, wpe, grid, smem, stream);
}

// every build of one schedule fits the same blocks per CU (the waves-per-EU target and the LDS size set it)
int trace_occ_pool(bool stats, int wpe, bool fused, size_t smem) {
    if (wpe != 7 && wpe != 6) return 0;
    if (fused) {
        if (stats) return wpe == 7 ? occ_pool<true, 7, true>(smem) : occ_pool<true, 6, true>(smem);
        return wpe == 7 ? occ_pool<false, 7, true>(smem) : occ_pool<false, 6, true>(smem);
    }
    if (stats) return wpe == 7 ? occ_pool<true, 7, false>(smem) : occ_pool<true, 6, false>(smem);
    return wpe == 7 ? occ_pool<false, 7, false>(smem) : occ_pool<false, 6, false>(smem);
}

}  // namespace prt
