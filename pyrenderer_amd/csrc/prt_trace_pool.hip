// prt_trace_pool.hip — the block-pooled shadow-query trace kernel (prt_device.h trace_kernel_pool)
// in its own compilation unit: pyrenderer_amd/build.py compiles it with LLVM's AMDGPU
// register-pressure trackers (-mllvm --amdgpu-use-amdgpu-trackers), under which the kernel fits
// the 72 VGPRs of 7 waves per SIMD with 3 spilled registers instead of 39 (the other trace
// kernels keep the default scheduler: the global-scene kernel is slower with the trackers,
// DESIGN.md §2).  Four schedules: the two-phase kernel (extension traversals, then the pooled
// shadow rays in 64-ray chunks after the block barrier), FUSED (round 5: idle lanes of the
// extension traversals take the previous iteration's pooled shadow rays), the two-phase kernel
// with packed leaf trips (round 5, traverse_pk) and the two-phase kernel without the block barrier
// (round 5, split arrival).
#pragma clang fp contract(off)

#include "prt_device.h"

#ifndef PRT_PACK_HOLD
#define PRT_PACK_HOLD 2   // leaves a lane holds before the packed leaf phase (traverse_pk's NP)
#endif

namespace prt {

namespace {
constexpr int kHold = PRT_PACK_HOLD;

template <bool STATS, int WPE, bool FUSED, int PK, bool SPLIT>
hipError_t launch_pool(const TraceParams& P, int grid, size_t smem, hipStream_t stream) {
    if (P.plain) trace_kernel_pool<STATS, WPE, true, FUSED, PK, SPLIT><<<grid, kBlock, smem, stream>>>(P);
    else trace_kernel_pool<STATS, WPE, false, FUSED, PK, SPLIT><<<grid, kBlock, smem, stream>>>(P);
    return hipGetLastError();
}
template <bool FUSED, int PK, bool SPLIT = false>
hipError_t launch_pool_f(const TraceParams& P, bool stats, int wpe, int grid, size_t smem, hipStream_t stream) {
    if (stats)
        return wpe == 7 ? launch_pool<true, 7, FUSED, PK, SPLIT>(P, grid, smem, stream)
                        : launch_pool<true, 6, FUSED, PK, SPLIT>(P, grid, smem, stream);
    return wpe == 7 ? launch_pool<false, 7, FUSED, PK, SPLIT>(P, grid, smem, stream)
                    : launch_pool<false, 6, FUSED, PK, SPLIT>(P, grid, smem, stream);
}
template <bool FUSED, int PK, bool SPLIT = false>
int occ_pool(bool stats, int wpe, size_t smem) {
    int n = 0;
    if (stats && wpe == 7)
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, trace_kernel_pool<true, 7, false, FUSED, PK, SPLIT>, kBlock, smem);
    else if (stats)
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, trace_kernel_pool<true, 6, false, FUSED, PK, SPLIT>, kBlock, smem);
    else if (wpe == 7)
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, trace_kernel_pool<false, 7, false, FUSED, PK, SPLIT>, kBlock, smem);
    else
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, trace_kernel_pool<false, 6, false, FUSED, PK, SPLIT>, kBlock, smem);
    return n;
}
}  // namespace

hipError_t launch_trace_pool(const TraceParams& P, bool stats, int wpe, int sched, int grid, size_t smem,
                             hipStream_t stream) {
    if (wpe != 7 && wpe != 6) return hipErrorInvalidValue;
    switch (sched) {
        case kPoolTwoPhase: return launch_pool_f<false, 0>(P, stats, wpe, grid, smem, stream);
        case kPoolFused: return launch_pool_f<true, 0>(P, stats, wpe, grid, smem, stream);
        case kPoolPacked: return launch_pool_f<false, kHold>(P, stats, wpe, grid, smem, stream);
        case kPoolSplit: return launch_pool_f<false, 0, true>(P, stats, wpe, grid, smem, stream);
        default: return hipErrorInvalidValue;
    }
}

// every build of one schedule fits the same blocks per CU (the waves-per-EU target and the LDS size set it)
int trace_occ_pool(bool stats, int wpe, int sched, size_t smem) {
    if (wpe != 7 && wpe != 6) return 0;
    switch (sched) {
        case kPoolTwoPhase: return occ_pool<false, 0>(stats, wpe, smem);
        case kPoolFused: return occ_pool<true, 0>(stats, wpe, smem);
        case kPoolPacked: return occ_pool<false, kHold>(stats, wpe, smem);
        case kPoolSplit: return occ_pool<false, 0, true>(stats, wpe, smem);
        default: return 0;
    }
}

}  // namespace prt
