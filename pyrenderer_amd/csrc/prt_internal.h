// prt_internal.h — structures shared by the host builder, the C-ABI layer and
// the HIP kernels of libprt.  Not part of the public ABI (see include/prt.h).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace prt {

// ---------------------------------------------------------------- BVH2 layout
// One node = 4 x float4 = 64 B, both child boxes stored in the parent so a
// single node fetch decides the traversal order (coalesced 64-B records):
//   f[0] = (L.lo.x, L.hi.x, L.lo.y, L.hi.y)
//   f[1] = (L.lo.z, L.hi.z, R.lo.x, R.hi.x)
//   f[2] = (R.lo.y, R.hi.y, R.lo.z, R.hi.z)
//   f[3] = (bits(child L), bits(child R), 0, 0)
// Child reference: >= 0 inner node index; < 0 leaf, v = -ref-1,
// first = v >> 3 (index into the BVH-ordered triangle array), count = (v&7)+1.
constexpr int kMaxLeaf = 8;
constexpr int kNodeF4 = 4;
constexpr int kTriF4 = 3;  // (v0, id bits) (e1, 0) (e2, 0)

inline int32_t leaf_ref(int64_t first, int count) {
    return -(int32_t)(((first << 3) | (int64_t)(count - 1)) + 1);
}

struct BvhHost {
    std::vector<float> nodes;      // n_nodes * 16
    std::vector<float> tris;       // n_tri * 12, BVH order
    std::vector<int32_t> order;    // BVH slot -> original triangle index
    int32_t depth = 0;             // max root-to-leaf edge count
    int64_t n_nodes = 0;
    int64_t n_leaves = 0;
    float pad = 0.0f;              // absolute box padding applied
    double sah_cost = 0.0;
};

// Builds a binned-SAH BVH2 over triangles (tri_v: n x 9 f32 world vertices).
// Box padding keeps the slab test conservative w.r.t. Moller-Trumbore's own
// rounding so traversal returns exactly the brute-force closest hit.
bool build_bvh(const float* tri_v, int64_t n_tri, int max_leaf, BvhHost* out, std::string* err);

}  // namespace prt
