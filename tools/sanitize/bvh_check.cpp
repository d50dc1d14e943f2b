// bvh_check — host driver for the sanitizer build of libprt's BVH builder (VERDICT r05
// item 4).  pyrenderer_amd/csrc/prt_bvh.cpp is pure C++ (standard library + prt_internal.h), so
// tools/sanitize/Makefile compiles it with g++ -fsanitize=address,undefined,float-cast-overflow
// next to this driver, which runs the whole host pipeline a scene takes in prt_scene_create —
// binned-SAH BVH2 with spatial splits and treelet restructuring (build_bvh), the SAH-optimal BVH4
// collapse (collapse_bvh4) and the 8-bit quantisation (quantize_bvh4) — and checks the results
// structurally, so that a sanitizer finding and a wrong tree both fail the run:
//   * BVH2: every inner node reached once, leaf ranges inside the reference array, every reference
//     slot in exactly one leaf, every triangle referenced, child boxes nested in their parent's;
//     every triangle's vertices and interior points inside the box of one of its references (the
//     conservative hit_aabb of /root/reference/accelerators/bvh_taichi.py:168-190);
//   * BVH4: every BVH2 leaf appears once, with a box containing its BVH2 box; inner child boxes
//     contain their node's four boxes; stack_need covers the deepest ancestor chain;
//   * quantised BVH4: the same refs, and every dequantised child box contains the f32 one.
// The reference's own debug mode (ti.init(debug=True), /root/reference/debug/run.py:7) is the
// nearest equivalent there: bounds-checked field accesses.
//
//   bvh_check <soup.f32> [max_leaf]      n x 9 float32 triangle vertices (raw, little endian)
//   bvh_check --random <n> <seed> [max_leaf]
// Prints one JSON line; exit status 0 = every check passed.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <unordered_map>
#include <vector>

#include "prt_internal.h"

namespace {

int g_fail = 0;
#define CHECK(cond, ...)                                         \
    do {                                                         \
        if (!(cond)) {                                           \
            if (g_fail++ < 10) {                                 \
                std::fprintf(stderr, "check failed: %s: ", #cond); \
                std::fprintf(stderr, __VA_ARGS__);               \
                std::fprintf(stderr, "\n");                      \
            }                                                    \
        }                                                        \
    } while (0)

struct Box {
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    bool empty() const { return !(lo[0] <= hi[0] && lo[1] <= hi[1] && lo[2] <= hi[2]); }
    bool contains(const Box& b) const {
        if (b.empty()) return true;
        for (int a = 0; a < 3; ++a)
            if (!(lo[a] <= b.lo[a] && b.hi[a] <= hi[a])) return false;
        return true;
    }
    bool has(const double p[3]) const {
        for (int a = 0; a < 3; ++a)
            if (!(lo[a] <= p[a] && p[a] <= hi[a])) return false;
        return true;
    }
};

int32_t ibits(float f) { int32_t v; std::memcpy(&v, &f, 4); return v; }
uint32_t ubits(float f) { uint32_t v; std::memcpy(&v, &f, 4); return v; }

// BVH2 child `side` of node n (prt_internal.h layout)
Box child2(const float* n, int side) {
    Box b;
    const float* f = n + 6 * side;
    for (int a = 0; a < 3; ++a) { b.lo[a] = f[2 * a]; b.hi[a] = f[2 * a + 1]; }
    return b;
}

std::vector<float> random_soup(int64_t n, unsigned seed) {
    // clustered slivers and large triangles: exercises early split clipping and spatial splits
    std::mt19937 g(seed);
    std::uniform_real_distribution<float> u(-5.0f, 5.0f);
    std::normal_distribution<float> small(0.0f, 0.2f), big(0.0f, 2.5f);
    std::vector<float> tv((size_t)n * 9);
    for (int64_t i = 0; i < n; ++i) {
        const float c[3] = {u(g), u(g), u(g)};
        const bool large = (i % 50) == 0;
        for (int k = 0; k < 9; ++k) tv[(size_t)(9 * i + k)] = c[k % 3] + (large ? big(g) : small(g));
    }
    return tv;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s <soup.f32> [max_leaf] | --random <n> <seed> [max_leaf]\n", argv[0]);
        return 2;
    }
    std::vector<float> tv;
    int max_leaf = 4;
    if (std::strcmp(argv[1], "--random") == 0) {
        if (argc < 4) return 2;
        tv = random_soup(std::atoll(argv[2]), (unsigned)std::atoi(argv[3]));
        if (argc > 4) max_leaf = std::atoi(argv[4]);
    } else {
        FILE* f = std::fopen(argv[1], "rb");
        if (!f) { std::perror(argv[1]); return 2; }
        std::fseek(f, 0, SEEK_END);
        const long bytes = std::ftell(f);
        std::fseek(f, 0, SEEK_SET);
        tv.resize((size_t)bytes / sizeof(float));
        if (std::fread(tv.data(), sizeof(float), tv.size(), f) != tv.size()) { std::fclose(f); return 2; }
        std::fclose(f);
        if (argc > 2) max_leaf = std::atoi(argv[2]);
    }
    const int64_t n_tri = (int64_t)(tv.size() / 9);

    prt::BvhHost b2;
    std::string err;
    if (!prt::build_bvh(tv.data(), n_tri, max_leaf, &b2, &err)) {
        std::fprintf(stderr, "build_bvh: %s\n", err.c_str());
        return 1;
    }
    const int64_t n2 = b2.n_nodes, n_ref = b2.n_refs;
    CHECK((int64_t)b2.nodes.size() == 16 * n2, "node array %zu vs %lld nodes", b2.nodes.size(), (long long)n2);
    CHECK((int64_t)b2.order.size() == n_ref && (int64_t)b2.tris.size() == 12 * n_ref, "reference arrays");

    // ---- BVH2: reachability, leaves, nesting
    std::vector<int> reached((size_t)n2, 0), slot_seen((size_t)n_ref, 0);
    std::vector<Box> slot_box((size_t)n_ref);
    std::unordered_map<int32_t, Box> leaf_box;   // leaf ref -> its box (BVH4 check)
    reached[0] = 1;
    for (int64_t i = 0; i < n2; ++i) {
        const float* nd = b2.nodes.data() + 16 * i;
        for (int side = 0; side < 2; ++side) {
            const int32_t r = ibits(nd[12 + side]);
            const Box cb = child2(nd, side);
            // an inverted (empty) box never passes the slab test: the root of a 0- or 1-triangle tree
            // fills its unused side with one, over a dummy leaf ref
            if (cb.empty()) { CHECK(r < 0, "inner node %d behind an empty box", r); continue; }
            if (r >= 0) {
                CHECK(r > 0 && r < n2, "inner ref %d of node %lld", r, (long long)i);
                if (r <= 0 || r >= n2) continue;
                reached[(size_t)r]++;
                const float* cn = b2.nodes.data() + 16 * (int64_t)r;
                CHECK(cb.contains(child2(cn, 0)) && cb.contains(child2(cn, 1)), "node %d not nested in %lld", r,
                      (long long)i);
            } else {
                const int64_t v = -(int64_t)r - 1, first = v >> 3, cnt = (v & 7) + 1;
                CHECK(cnt <= prt::kMaxLeaf && first >= 0 && first + cnt <= n_ref, "leaf %lld+%lld", (long long)first,
                      (long long)cnt);
                if (first < 0 || first + cnt > n_ref) continue;
                leaf_box[r] = cb;
                for (int64_t s = first; s < first + cnt; ++s) { slot_seen[(size_t)s]++; slot_box[(size_t)s] = cb; }
            }
        }
    }
    if (n_tri > 0)
        for (int64_t i = 0; i < n2; ++i) CHECK(reached[(size_t)i] == 1, "node %lld reached %d times", (long long)i,
                                               reached[(size_t)i]);
    for (int64_t s = 0; s < n_ref; ++s) CHECK(slot_seen[(size_t)s] == 1, "slot %lld in %d leaves", (long long)s,
                                              slot_seen[(size_t)s]);

    // ---- cover: vertices + interior points of every triangle inside one of its references' boxes
    static const double W[9][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}, {1. / 3, 1. / 3, 1. / 3}, {.5, .5, 0},
                                   {0, .5, .5}, {.5, 0, .5}, {.8, .1, .1}, {.05, .25, .7}};
    std::vector<uint16_t> covered((size_t)n_tri, 0);
    std::vector<int> refs_of((size_t)n_tri, 0);
    for (int64_t s = 0; s < n_ref; ++s) {
        const int32_t t = b2.order[(size_t)s];
        CHECK(t >= 0 && t < n_tri, "order[%lld] = %d", (long long)s, t);
        if (t < 0 || t >= n_tri) continue;
        refs_of[(size_t)t]++;
        const float* v = tv.data() + 9 * (int64_t)t;
        const float* rec = b2.tris.data() + 12 * s;
        CHECK(rec[0] == v[0] && rec[1] == v[1] && rec[2] == v[2] && ibits(rec[3]) == t &&
                  rec[4] == v[3] - v[0] && rec[9] == v[7] - v[1], "record of slot %lld", (long long)s);
        for (int m = 0; m < 9; ++m) {
            double p[3];
            for (int a = 0; a < 3; ++a)
                p[a] = W[m][0] * (double)v[a] + W[m][1] * (double)v[3 + a] + W[m][2] * (double)v[6 + a];
            if (slot_box[(size_t)s].has(p)) covered[(size_t)t] |= (uint16_t)(1u << m);
        }
    }
    int64_t uncovered = 0, dup = 0;
    for (int64_t t = 0; t < n_tri; ++t) {
        CHECK(refs_of[(size_t)t] >= 1, "triangle %lld unreferenced", (long long)t);
        uncovered += covered[(size_t)t] != 0x1FF;
        dup += refs_of[(size_t)t] - 1;
    }
    CHECK(uncovered == 0, "%lld triangles not covered by their references' boxes", (long long)uncovered);

    // ---- BVH4 collapse
    prt::Bvh4Host b4;
    prt::collapse_bvh4(b2, &b4);
    const int64_t n4 = b4.n_nodes;
    CHECK((int64_t)b4.nodes.size() == 32 * n4 && n4 >= 1, "BVH4 arrays");
    auto child4 = [&](int64_t n, int k) {
        const float* f = b4.nodes.data() + 32 * n;
        Box b;
        for (int a = 0; a < 3; ++a) { b.lo[a] = f[(2 * a) * 4 + k]; b.hi[a] = f[(2 * a + 1) * 4 + k]; }
        return b;
    };
    std::vector<int> reached4((size_t)n4, 0);
    std::unordered_map<int32_t, int> leaf_seen;
    int max_depth4 = 0, max_anc = 0;
    // depth-first from the root: (node, depth, stack entries its ancestors may have pushed: the
    // valid siblings of every child taken, <= 3 per level)
    struct Item { int64_t n; int depth, anc; };
    std::vector<Item> todo = {{0, 0, 0}};
    reached4[0] = 1;
    while (!todo.empty()) {
        const Item it = todo.back();
        todo.pop_back();
        const float* f = b4.nodes.data() + 32 * it.n;
        int valid = 0;
        for (int k = 0; k < 4; ++k) valid += ibits(f[24 + k]) != 0x7FFFFFFF;
        max_depth4 = std::max(max_depth4, it.depth);
        max_anc = std::max(max_anc, it.anc);
        for (int k = 0; k < 4; ++k) {
            const int32_t r = ibits(f[24 + k]);
            const Box cb = child4(it.n, k);
            if (r == 0x7FFFFFFF) { CHECK(cb.empty(), "sentinel slot of node %lld has a box", (long long)it.n); continue; }
            if (r >= 0) {
                CHECK(r > 0 && r < n4, "BVH4 inner ref %d of node %lld", r, (long long)it.n);
                if (r <= 0 || r >= n4) continue;
                if (reached4[(size_t)r]++ == 0) todo.push_back({r, it.depth + 1, it.anc + valid - 1});
                for (int c = 0; c < 4; ++c)
                    CHECK(cb.contains(child4(r, c)), "BVH4 node %d child %d outside its box", r, c);
            } else {
                leaf_seen[r]++;
                auto lb = leaf_box.find(r);
                CHECK(lb != leaf_box.end(), "BVH4 leaf ref %d is no BVH2 leaf", r);
                if (lb != leaf_box.end()) CHECK(cb.contains(lb->second), "BVH4 leaf %d box smaller than BVH2's", r);
            }
        }
    }
    for (int64_t i = 1; i < n4; ++i) CHECK(reached4[(size_t)i] == 1, "BVH4 node %lld reached %d times", (long long)i,
                                           reached4[(size_t)i]);
    if (n_tri > 0) {
        CHECK(leaf_seen.size() == leaf_box.size(), "BVH4 holds %zu of %zu leaves", leaf_seen.size(), leaf_box.size());
        for (auto& kv : leaf_seen) CHECK(kv.second == 1, "leaf %d appears %d times in the BVH4", kv.first, kv.second);
    }
    // the traversal stack: the sentinel, the entries every ancestor level may have pushed, and the
    // <= 3 slots a visit writes above the top (collapse_bvh4's bound; the LDS kernels size to it)
    CHECK(b4.stack_need >= 1 + max_anc + 3, "stack_need %d below 1 + %d + 3", b4.stack_need, max_anc);

    // ---- quantised BVH4
    std::vector<float> q4;
    prt::quantize_bvh4(b4, b2.pad, &q4);
    CHECK((int64_t)q4.size() == 16 * n4, "quantised array");
    for (int64_t i = 0; i < n4; ++i) {
        const float* q = q4.data() + 16 * i;
        const float* f = b4.nodes.data() + 32 * i;
        const double org[3] = {q[0], q[1], q[2]}, st[3] = {q[3], q[4], q[5]};
        const uint32_t ql[3] = {ubits(q[6]), ubits(q[8]), ubits(q[10])}, qh[3] = {ubits(q[7]), ubits(q[9]), ubits(q[11])};
        for (int k = 0; k < 4; ++k) {
            const int32_t r = ibits(f[24 + k]), rq = ibits(q[12 + k]);
            CHECK(r == rq, "quantised ref of node %lld slot %d: %d vs %d", (long long)i, k, rq, r);
            if (r == 0x7FFFFFFF) continue;
            Box d;
            for (int a = 0; a < 3; ++a) {
                d.lo[a] = org[a] + (double)((ql[a] >> (8 * k)) & 0xFFu) * st[a];
                d.hi[a] = org[a] + (double)((qh[a] >> (8 * k)) & 0xFFu) * st[a];
            }
            CHECK(d.contains(child4(i, k)), "quantised box of node %lld slot %d smaller than the f32 box",
                  (long long)i, k);
        }
    }

    std::printf("{\"triangles\": %lld, \"references\": %lld, \"duplicates\": %lld, \"bvh2_nodes\": %lld, "
                "\"bvh2_depth\": %d, \"bvh4_nodes\": %lld, \"bvh4_depth\": %d, \"stack_need\": %d, "
                "\"sah\": %.4f, \"spatial_splits\": %lld, \"failures\": %d}\n",
                (long long)n_tri, (long long)n_ref, (long long)dup, (long long)n2, b2.depth, (long long)n4,
                max_depth4, b4.stack_need, b2.sah_cost, (long long)b2.n_spatial, g_fail);
    return g_fail ? 1 : 0;
}
