// prt_trace_inst.hip — one instantiation set of the persistent trace kernel
// (prt_device.h): every variant of PRT_VARIANTS for traversal stack PRT_STACK and
// stats flag PRT_STATS.  pyrenderer_amd/build.py compiles this file once per
// (stack, stats) pair, in parallel, and links the objects into libprt.so.
#pragma clang fp contract(off)

#include "prt_device.h"

#ifndef PRT_STACK
#error "PRT_STACK (traversal stack entries) must be defined"
#endif
#ifndef PRT_STATS
#error "PRT_STATS (0 or 1) must be defined"
#endif

#define PRT_CAT2(a, c, d) a##c##_##d
#define PRT_CAT(a, c, d) PRT_CAT2(a, c, d)

namespace prt {

hipError_t PRT_CAT(launch_trace_, PRT_STACK, PRT_STATS)(const TraceParams& P, int var, int grid, size_t smem,
                                                         hipStream_t stream) {
    return launch_var<PRT_STACK, PRT_STATS != 0>(P, var, grid, smem, stream);
}

int PRT_CAT(trace_occ_, PRT_STACK, PRT_STATS)(int var, size_t smem) {
    return occ_var<PRT_STACK, PRT_STATS != 0>(var, smem);
}

}  // namespace prt
