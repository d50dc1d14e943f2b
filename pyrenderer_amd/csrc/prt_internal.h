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
    std::vector<int32_t> order;    // BVH slot -> original triangle index (a triangle split by early
                                   // split clipping occupies several slots)
    int64_t n_refs = 0;            // triangle records in BVH order (>= n_tri)
    int32_t depth = 0;             // max root-to-leaf edge count
    int64_t n_nodes = 0;
    int64_t n_leaves = 0;
    float pad = 0.0f;              // absolute box padding applied
    double sah_cost = 0.0;
    int64_t n_spatial = 0;         // spatial splits taken (SBVH, prt_bvh.cpp)
};

// BVH4 collapsed from the BVH2 (same triangle order and leaf encoding).
// One node = 8 x float4 = 128 B, children in SoA so one node fetch tests
// four boxes: f[0..5] = lo.x[4], hi.x[4], lo.y[4], hi.y[4], lo.z[4], hi.z[4];
// f[6] = child refs (int bits); f[7] = unused.  Empty slots: lo = +inf, hi = -inf,
// ref = 0x7FFFFFFF (the traversal sentinel).
constexpr int kNode4F4 = 8;
struct Bvh4Host {
    std::vector<float> nodes;      // n_nodes * 32
    int64_t n_nodes = 0;
    int32_t depth = 0;             // max root-to-leaf node count - 1
    int32_t stack_need = 0;        // worst-case traversal stack entries (collapse_bvh4)
};
void collapse_bvh4(const BvhHost& b2, Bvh4Host* out);

// Quantised BVH4 for scenes read from HBM: one node = 4 x float4 = 64 B (two per
// 128-B cache line, half the BVH4 footprint):
//   f[0] = (origin.x, origin.y, origin.z, s.x)    s = grid step per axis (range / 254, rounded up)
//   f[1] = (s.y, s.z, qlo.x[4], qhi.x[4])         q = u8 per child packed in a u32
//   f[2] = (qlo.y[4], qhi.y[4], qlo.z[4], qhi.z[4])
//   f[3] = child refs (as Bvh4Host), empty slots = 0x7FFFFFFF (masked by the kernel)
// Child box = origin + q * s, rounded outward so that it contains the float box
// with at least `pad` to spare on every side (conservative: traversal unchanged).
constexpr int kNodeQF4 = 4;
void quantize_bvh4(const Bvh4Host& b4, float pad, std::vector<float>* out);


// Builds a binned-SAH BVH2 over triangles (tri_v: n x 9 f32 world vertices).
// Box padding keeps the slab test conservative w.r.t. Moller-Trumbore's own
// rounding so traversal returns exactly the brute-force closest hit.
bool build_bvh(const float* tri_v, int64_t n_tri, int max_leaf, BvhHost* out, std::string* err);

}  // namespace prt
