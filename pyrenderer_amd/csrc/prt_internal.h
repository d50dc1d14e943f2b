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

// Compact quantised BVH4 for scenes read from HBM (round 4): ONE array of 48-B records holding
// both the nodes and the triangle records (3 float4 each, the BVH2 triangle layout), so a node
// visit loads 3 x 16 B per lane instead of 4 (global-scene traversal is bound by the CU's vector
// L1 / address path: every wave load costs one tag lookup per distinct line its lanes touch).
// A node's children live in one contiguous block at `base`: its inner children's node records
// first (in slot order), then each leaf child's triangle records.  Node record:
//   f[0] = (origin.x, origin.y, origin.z, bits(base))
//   f[1] = (qlo.x[4], qhi.x[4], qlo.y[4], qhi.y[4])   u8 grid coordinates per child
//   f[2] = (qlo.z[4], qhi.z[4], bits(exps), bits(meta))
// exps: bytes 0..2 = the f32 exponent field of the grid step 2^e per axis (a power of two at
// or above range / 254), byte 3 = inner-child mask (bits 0..3) | empty-slot mask (bits 4..7);
// meta byte k = child k's offset from base (inner child: its rank among the inner children;
// leaf: (record offset << 3) | (count - 1)).  Child refs therefore decode without a load:
// inner = base + off, leaf = ~((base << 3) + off) (= leaf_ref(base + (off >> 3), (off & 7) + 1)).
// Boxes are rounded outward with the same >= 2 pad of slack as quantize_bvh4 (conservative).
constexpr int kCRecF4 = 3;
// returns false (and *err) when the array would exceed the kernel's 32-bit byte offsets
bool compact_bvh4(const Bvh4Host& b4, const BvhHost& b2, std::vector<float>* out, std::string* err);

// Builds a binned-SAH BVH2 over triangles (tri_v: n x 9 f32 world vertices).
// Box padding keeps the slab test conservative w.r.t. Moller-Trumbore's own
// rounding so traversal returns exactly the brute-force closest hit.
bool build_bvh(const float* tri_v, int64_t n_tri, int max_leaf, BvhHost* out, std::string* err);

}  // namespace prt
