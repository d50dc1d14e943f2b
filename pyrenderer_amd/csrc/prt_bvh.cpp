// prt_bvh.cpp — host-side binned-SAH BVH2 builder over triangles.
//
// The reference builds its BVH over *primitives* (median split in insertion
// order, accelerators/bvh_taichi.py:58-161) and brute-forces each primitive's
// triangles (mathematics/shapes.py:76-110).  That does not scale past a few
// primitives, so libprt builds a triangle-level SAH tree (the intent of the
// reference's unused CPU builder, accelerators/bvh.py:28-215, 12 buckets) and
// lays it out for the GPU: 64-B nodes with both child boxes, triangles as
// (v0, e1, e2) in leaf order.  Closest-hit results do not depend on the tree:
// ties resolve to the lowest original triangle index, which is also the
// reference's first-found order (leaves visited in insertion order).
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <vector>

#include "prt_internal.h"

namespace prt {
namespace {

struct Box {
    float lo[3] = {FLT_MAX, FLT_MAX, FLT_MAX};
    float hi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    void grow(const Box& b) {
        for (int k = 0; k < 3; ++k) { lo[k] = std::min(lo[k], b.lo[k]); hi[k] = std::max(hi[k], b.hi[k]); }
    }
    void grow(const float* p) {
        for (int k = 0; k < 3; ++k) { lo[k] = std::min(lo[k], p[k]); hi[k] = std::max(hi[k], p[k]); }
    }
    bool valid() const { return lo[0] <= hi[0]; }
    double area() const {
        if (!valid()) return 0.0;
        double dx = (double)hi[0] - lo[0], dy = (double)hi[1] - lo[1], dz = (double)hi[2] - lo[2];
        return 2.0 * (dx * dy + dy * dz + dz * dx);
    }
};

struct TNode {
    Box box;
    int32_t left = -1, right = -1;   // temp node ids
    int64_t first = 0;
    int32_t count = 0;               // > 0 for leaves
};

constexpr int kMaxBins = 128;

// ---------------------------------------------------------- early split clipping
// A triangle far larger than the scene's typical one (the Cornell walls among config 4's
// million small cube faces) would otherwise sit deep in the tree and inflate the box of
// every ancestor to the wall's size, so every ray near the wall walks those subtrees
// (config 4: up to 2067 node visits in one query against 25 on average).  Such a
// triangle enters the build as several references, each the triangle clipped to one cell
// of a recursive midpoint split of its box (Ernst & Greiner 2007, "early split
// clipping").  The triangle record is the same for every reference, so traversal tests
// the same Moller-Trumbore on it, possibly more than once, and the closest (t, id) is
// unchanged; the reference boxes only have to cover the triangle, which they do: each
// is the bound of the triangle clipped to its cell (Sutherland-Hodgman in double),
// rounded outward to f32, and then padded like every other box.
struct RefBox { double lo[3], hi[3]; };

// bounds of triangle `v` (3 x xyz, double) clipped to box `c`; false when they do not meet
bool clip_bounds(const double v[3][3], const RefBox& c, RefBox* out) {
    double poly[16][3], tmp[16][3];
    int n = 3;
    for (int i = 0; i < 3; ++i)
        for (int k = 0; k < 3; ++k) poly[i][k] = v[i][k];
    for (int ax = 0; ax < 3 && n > 0; ++ax)
        for (int side = 0; side < 2 && n > 0; ++side) {
            const double b = side == 0 ? c.lo[ax] : c.hi[ax];
            auto inside = [&](const double* p) { return side == 0 ? p[ax] >= b : p[ax] <= b; };
            int m = 0;
            for (int i = 0; i < n; ++i) {
                const double* a = poly[i];
                const double* q = poly[(i + 1) % n];
                const bool ia = inside(a), iq = inside(q);
                if (ia) { for (int k = 0; k < 3; ++k) tmp[m][k] = a[k]; ++m; }
                if (ia != iq && m < 15) {
                    const double t = (b - a[ax]) / (q[ax] - a[ax]);
                    for (int k = 0; k < 3; ++k) tmp[m][k] = a[k] + t * (q[k] - a[k]);
                    tmp[m][ax] = b;
                    ++m;
                }
            }
            n = m;
            for (int i = 0; i < n; ++i)
                for (int k = 0; k < 3; ++k) poly[i][k] = tmp[i][k];
        }
    if (n == 0) return false;
    for (int k = 0; k < 3; ++k) { out->lo[k] = INFINITY; out->hi[k] = -INFINITY; }
    for (int i = 0; i < n; ++i)
        for (int k = 0; k < 3; ++k) {
            out->lo[k] = std::min(out->lo[k], poly[i][k]);
            out->hi[k] = std::max(out->hi[k], poly[i][k]);
        }
    for (int k = 0; k < 3; ++k) {   // the polygon lies in the cell up to rounding
        out->lo[k] = std::max(out->lo[k], c.lo[k]);
        out->hi[k] = std::min(out->hi[k], c.hi[k]);
    }
    return true;
}

double ref_area(const RefBox& b) {
    double dx = b.hi[0] - b.lo[0], dy = b.hi[1] - b.lo[1], dz = b.hi[2] - b.lo[2];
    return 2.0 * (dx * dy + dy * dz + dz * dx);
}

void split_refs(const double v[3][3], const RefBox& cell, double thr, int depth, std::vector<RefBox>* out) {
    RefBox b;
    if (!clip_bounds(v, cell, &b)) return;
    if (ref_area(b) <= thr || depth >= 12) {
        out->push_back(b);
        return;
    }
    int ax = 0;
    for (int k = 1; k < 3; ++k)
        if (b.hi[k] - b.lo[k] > b.hi[ax] - b.lo[ax]) ax = k;
    const double mid = 0.5 * (b.lo[ax] + b.hi[ax]);
    RefBox l = b, r = b;
    l.hi[ax] = mid;
    r.lo[ax] = mid;
    split_refs(v, l, thr, depth + 1, out);
    split_refs(v, r, thr, depth + 1, out);
}

inline Box outward_f32(const RefBox& r, const Box& tri_box) {
    Box b;
    for (int k = 0; k < 3; ++k) {
        float lo = (float)r.lo[k], hi = (float)r.hi[k];
        if ((double)lo > r.lo[k]) lo = std::nextafter(lo, -INFINITY);
        if ((double)hi < r.hi[k]) hi = std::nextafter(hi, INFINITY);
        b.lo[k] = std::max(lo, tri_box.lo[k]);   // never beyond the triangle's own box
        b.hi[k] = std::min(hi, tri_box.hi[k]);
    }
    return b;
}


// Binned-SAH builder over references (a triangle, or an early-split-clipping piece of one), with
// spatial splits (Stich, Friedrich & Dietrich 2009, "Spatial Splits in Bounding Volume
// Hierarchies"; env PRT_SBVH=0 turns them off): where the best object split's two children overlap
// (their intersection's area > alpha x the root's, env PRT_SBVH_ALPHA, default 1e-5), the node's
// box is also cut by 32 planes per axis, every reference chopped into the bins it spans (its triangle
// clipped to the reference box and the bin, bounds in double rounded outward to f32), and the
// cheaper of the two splits is taken.  A reference straddling a spatial split plane goes to both
// sides as two references, each bounding the triangle's part on its side — unless moving it whole
// to one side costs less (reference unsplitting).  Duplicates stop at a budget of references
// (env PRT_SBVH_BUDGET x the initial count, default 1.3).  Every reference's record is its whole
// triangle, so a leaf tests the same Moller-Trumbore on it and the closest (t, id) is unchanged;
// the union of a triangle's reference boxes covers it.
struct Builder {
    const float* tv;           // triangle vertices (n_tri x 9)
    int max_leaf;
    int bins = 32;             // SAH bins per axis (env PRT_SAH_BINS, 2..128; 64 for large scenes)
    double ct = 0.5;           // SAH cost of a node step relative to one triangle test (env PRT_SAH_CT)
    int leaf_min = 2;          // ranges of <= leaf_min triangles always become leaves (env PRT_LEAF_MIN)
    bool sbvh = true;          // spatial splits (env PRT_SBVH=0 turns them off)
    double alpha = 1e-5;       // overlap threshold relative to the root's area (env PRT_SBVH_ALPHA)
    double min_overlap = 0.0;  // alpha x root area
    int64_t ref_budget = 0;    // spatial splits stop once the references reach this count
    std::vector<Box> tb;       // per reference: box
    std::vector<float> cen;    // per reference: box centre (3)
    std::vector<int32_t> ref_tri;   // per reference: original triangle
    std::vector<int32_t> order;     // leaf order of the references (output)
    std::vector<TNode> nodes;
    int32_t max_depth = 0;
    int64_t leaves = 0, spatial_splits = 0;

    void set_centre(int32_t r) {
        for (int k = 0; k < 3; ++k) cen[3 * (size_t)r + k] = 0.5f * (tb[(size_t)r].lo[k] + tb[(size_t)r].hi[k]);
    }
    // the part of reference r's triangle inside box `cell` (intersected with the reference's box),
    // rounded outward; false when empty
    bool clip_ref(int32_t r, double lo_ax, double hi_ax, int ax, Box* out) const {
        const float* t = tv + 9 * (size_t)ref_tri[(size_t)r];
        double v[3][3];
        for (int a = 0; a < 3; ++a)
            for (int k = 0; k < 3; ++k) v[a][k] = (double)t[3 * a + k];
        const Box& rb = tb[(size_t)r];
        RefBox cell;
        for (int k = 0; k < 3; ++k) { cell.lo[k] = rb.lo[k]; cell.hi[k] = rb.hi[k]; }
        cell.lo[ax] = std::max(cell.lo[ax], lo_ax);
        cell.hi[ax] = std::min(cell.hi[ax], hi_ax);
        if (!(cell.lo[ax] <= cell.hi[ax])) return false;
        RefBox cb;
        if (!clip_bounds(v, cell, &cb)) return false;
        Box tri_box;
        tri_box.grow(t); tri_box.grow(t + 3); tri_box.grow(t + 6);
        *out = outward_f32(cb, tri_box);
        // never beyond the reference's own box (the parent region)
        for (int k = 0; k < 3; ++k) {
            out->lo[k] = std::max(out->lo[k], rb.lo[k]);
            out->hi[k] = std::min(out->hi[k], rb.hi[k]);
        }
        return out->lo[0] <= out->hi[0] && out->lo[1] <= out->hi[1] && out->lo[2] <= out->hi[2];
    }

    static Box meet(const Box& a, const Box& b) {
        Box m;
        for (int k = 0; k < 3; ++k) { m.lo[k] = std::max(a.lo[k], b.lo[k]); m.hi[k] = std::min(a.hi[k], b.hi[k]); }
        for (int k = 0; k < 3; ++k)
            if (!(m.lo[k] <= m.hi[k])) return Box();
        return m;
    }

    int32_t make_leaf(int32_t me, const std::vector<int32_t>& refs) {
        nodes[me].first = (int64_t)order.size();
        nodes[me].count = (int32_t)refs.size();
        order.insert(order.end(), refs.begin(), refs.end());
        leaves++;
        return me;
    }

    int32_t build(std::vector<int32_t>& refs, int depth) {
        const int64_t count = (int64_t)refs.size();
        int32_t me = (int32_t)nodes.size();
        nodes.emplace_back();
        Box b, cb;
        for (int32_t r : refs) {
            b.grow(tb[(size_t)r]);
            cb.grow(&cen[3 * (size_t)r]);
        }
        nodes[me].box = b;
        max_depth = std::max(max_depth, depth);
        if (count <= max_leaf && (count <= leaf_min || depth > 32)) return make_leaf(me, refs);
        std::vector<int32_t> left, right;
        if (depth >= 32) {
            // depth guard (bounds the traversal stack): object median on the widest centroid axis
            int ax = 0;
            for (int k = 1; k < 3; ++k)
                if (cb.hi[k] - cb.lo[k] > cb.hi[ax] - cb.lo[ax]) ax = k;
            const int64_t mid = count / 2;
            std::nth_element(refs.begin(), refs.begin() + mid, refs.end(),
                             [&](int32_t a, int32_t c) { return cen[3 * (size_t)a + ax] < cen[3 * (size_t)c + ax]; });
            left.assign(refs.begin(), refs.begin() + mid);
            right.assign(refs.begin() + mid, refs.end());
            std::vector<int32_t>().swap(refs);
            nodes[me].left = build(left, depth + 1);
            nodes[me].right = build(right, depth + 1);
            return me;
        }
        // binned SAH object split over the three axes
        double best_cost = DBL_MAX;
        int best_axis = -1, best_split = -1;
        Box best_l, best_r;
        for (int ax = 0; ax < 3; ++ax) {
            float ext = cb.hi[ax] - cb.lo[ax];
            if (!(ext > 0.0f)) continue;
            const int kBins = bins;
            Box bb[kMaxBins];
            int64_t cnt[kMaxBins] = {0};
            double scale = kBins / (double)ext;
            for (int32_t r : refs) {
                int k = (int)(((double)cen[3 * (size_t)r + ax] - cb.lo[ax]) * scale);
                k = std::min(std::max(k, 0), kBins - 1);
                cnt[k]++;
                bb[k].grow(tb[(size_t)r]);
            }
            Box rbx[kMaxBins];
            int64_t rc[kMaxBins];
            Box acc;
            int64_t c = 0;
            for (int k = kBins - 1; k > 0; --k) {
                acc.grow(bb[k]); c += cnt[k];
                rbx[k] = acc; rc[k] = c;
            }
            Box lacc;
            int64_t lc = 0;
            for (int k = 0; k < kBins - 1; ++k) {
                lacc.grow(bb[k]); lc += cnt[k];
                if (lc == 0 || rc[k + 1] == 0) continue;
                double cost = lacc.area() * (double)lc + rbx[k + 1].area() * (double)rc[k + 1];
                if (cost < best_cost) {
                    best_cost = cost; best_axis = ax; best_split = k;
                    best_l = lacc; best_r = rbx[k + 1];
                }
            }
        }
        // spatial split: only where the object split's children overlap, within the reference budget
        double s_cost = DBL_MAX;
        int s_axis = -1, s_split = -1;
        if (sbvh && best_axis >= 0 && (int64_t)tb.size() < ref_budget && meet(best_l, best_r).area() > min_overlap) {
            for (int ax = 0; ax < 3; ++ax) {
                const double lo = b.lo[ax], ext = (double)b.hi[ax] - b.lo[ax];
                if (!(ext > 0.0)) continue;
                const int kBins = bins;
                const double w = ext / kBins;
                Box bb[kMaxBins];
                int64_t entry[kMaxBins] = {0}, exit_[kMaxBins] = {0};
                for (int32_t r : refs) {
                    const Box& rb = tb[(size_t)r];
                    int b0 = (int)(((double)rb.lo[ax] - lo) / w), b1 = (int)(((double)rb.hi[ax] - lo) / w);
                    b0 = std::min(std::max(b0, 0), kBins - 1);
                    b1 = std::min(std::max(b1, b0), kBins - 1);
                    entry[b0]++;
                    exit_[b1]++;
                    if (b0 == b1) {
                        bb[b0].grow(rb);
                        continue;
                    }
                    // the search bins the reference box cut by the bin's slab (an upper bound of the
                    // clipped triangle's bounds, exact for axis-aligned faces); the split itself clips
                    for (int k = b0; k <= b1; ++k) {
                        Box part = rb;
                        if (k > b0) part.lo[ax] = std::max(part.lo[ax], (float)(lo + w * k));
                        if (k < b1) part.hi[ax] = std::min(part.hi[ax], (float)(lo + w * (k + 1)));
                        bb[k].grow(part);
                    }
                }
                Box rbx[kMaxBins];
                int64_t rc[kMaxBins];
                Box acc;
                int64_t c = 0;
                for (int k = kBins - 1; k > 0; --k) {
                    acc.grow(bb[k]); c += exit_[k];
                    rbx[k] = acc; rc[k] = c;
                }
                Box lacc;
                int64_t lc = 0;
                for (int k = 0; k < kBins - 1; ++k) {
                    lacc.grow(bb[k]); lc += entry[k];
                    if (lc == 0 || rc[k + 1] == 0) continue;
                    double cost = lacc.area() * (double)lc + rbx[k + 1].area() * (double)rc[k + 1];
                    if (cost < s_cost) { s_cost = cost; s_axis = ax; s_split = k; }
                }
            }
        }
        const bool spatial = s_axis >= 0 && s_cost < best_cost;
        const double split_sah = spatial ? s_cost : best_cost;
        double parent_area = b.area();
        double leaf_cost = (double)count;
        double split_cost = parent_area > 0.0 ? ct + split_sah / parent_area : DBL_MAX;
        if (count <= max_leaf && !(split_cost < leaf_cost)) return make_leaf(me, refs);
        if (spatial) {
            spatial_splits++;
            const int ax = s_axis;
            const double lo = b.lo[ax], w = ((double)b.hi[ax] - b.lo[ax]) / bins;
            const double plane = lo + w * (s_split + 1);
            // classify by the same bins as the search; straddling references are split or moved whole
            std::vector<int32_t> straddle;
            Box lb, rb_;
            for (int32_t r : refs) {
                const Box& x = tb[(size_t)r];
                int b0 = (int)(((double)x.lo[ax] - lo) / w), b1 = (int)(((double)x.hi[ax] - lo) / w);
                b0 = std::min(std::max(b0, 0), bins - 1);
                b1 = std::min(std::max(b1, b0), bins - 1);
                if (b1 <= s_split) { left.push_back(r); lb.grow(x); }
                else if (b0 > s_split) { right.push_back(r); rb_.grow(x); }
                else straddle.push_back(r);
            }
            std::vector<int32_t>().swap(refs);
            for (int32_t r : straddle) {
                Box pl, pr;
                const bool hl = clip_ref(r, -INFINITY, plane, ax, &pl), hr = clip_ref(r, plane, INFINITY, ax, &pr);
                if (!hr || (!hl && !hr)) { left.push_back(r); lb.grow(tb[(size_t)r]); continue; }
                if (!hl) { right.push_back(r); rb_.grow(tb[(size_t)r]); continue; }
                // reference unsplitting (Stich et al. 2009 §4.3): whole to one side when cheaper
                const double nl = (double)left.size() + 1, nr = (double)right.size() + 1;
                Box lsplit = lb, rsplit = rb_, lwhole = lb, rwhole = rb_;
                lsplit.grow(pl); rsplit.grow(pr);
                lwhole.grow(tb[(size_t)r]); rwhole.grow(tb[(size_t)r]);
                const double c_split = lsplit.area() * nl + rsplit.area() * nr;
                const double c_left = lwhole.area() * nl + rb_.area() * (nr - 1);
                const double c_right = lb.area() * (nl - 1) + rwhole.area() * nr;
                if ((int64_t)tb.size() >= ref_budget || (c_left <= c_split && c_left <= c_right)) {
                    left.push_back(r); lb = lwhole;
                } else if (c_right <= c_split) {
                    right.push_back(r); rb_ = rwhole;
                } else {
                    const int32_t r2 = (int32_t)tb.size();
                    tb[(size_t)r] = pl;
                    set_centre(r);
                    tb.push_back(pr);
                    ref_tri.push_back(ref_tri[(size_t)r]);
                    cen.resize(cen.size() + 3);
                    set_centre(r2);
                    left.push_back(r); lb = lsplit;
                    right.push_back(r2); rb_ = rsplit;
                }
            }
            if (left.empty() || right.empty()) {
                // degenerate plane (everything on one side): object median instead
                std::vector<int32_t> all(left);
                all.insert(all.end(), right.begin(), right.end());
                left.clear(); right.clear();
                const int64_t mid = (int64_t)all.size() / 2;
                left.assign(all.begin(), all.begin() + mid);
                right.assign(all.begin() + mid, all.end());
            }
        } else if (best_axis < 0) {
            const int64_t mid = count / 2;  // all centroids coincide: split the range
            left.assign(refs.begin(), refs.begin() + mid);
            right.assign(refs.begin() + mid, refs.end());
            std::vector<int32_t>().swap(refs);
        } else {
            float ext = cb.hi[best_axis] - cb.lo[best_axis];
            const int kBins = bins;
            double scale = kBins / (double)ext;
            auto it = std::partition(refs.begin(), refs.end(), [&](int32_t t) {
                int k = (int)(((double)cen[3 * (size_t)t + best_axis] - cb.lo[best_axis]) * scale);
                k = std::min(std::max(k, 0), kBins - 1);
                return k <= best_split;
            });
            int64_t mid = it - refs.begin();
            if (mid == 0 || mid == count) mid = count / 2;
            left.assign(refs.begin(), refs.begin() + mid);
            right.assign(refs.begin() + mid, refs.end());
            std::vector<int32_t>().swap(refs);
        }
        int32_t l = build(left, depth + 1);
        int32_t r = build(right, depth + 1);
        nodes[me].left = l;
        nodes[me].right = r;
        return me;
    }
};

inline float bits_f(int32_t v) { float f; std::memcpy(&f, &v, 4); return f; }

// Treelet restructuring (Karras & Aila 2013, "Fast Parallel Construction of High-Quality Bounding
// Volume Hierarchies" §4): bottom-up, each inner node and its descendants down to 7 subtrees (the
// largest-area subtree expanded first) form a treelet whose binary topology over those 7 subtrees
// is replaced by the SAH-optimal one (a dynamic program over the 127 subsets), reusing the
// treelet's inner nodes.  Leaves and the references they hold are unchanged, so the leaf order
// and the triangle records stay valid; only inner boxes and child links move.  SAH cost of a
// subtree: leaf area x references, inner node ct x area + its children's costs.
void restructure_treelets(std::vector<TNode>& nodes, int32_t root, double ct, int passes) {
    constexpr int kT = 7;
    std::vector<double> cost(nodes.size(), 0.0);
    std::vector<int32_t> post;
    std::vector<std::pair<int32_t, bool>> st;
    double box_a[1 << kT];
    Box box_m[1 << kT];
    double copt[1 << kT];
    int part[1 << kT];
    for (int pass = 0; pass < passes; ++pass) {
        post.clear();
        st.assign(1, {root, false});
        while (!st.empty()) {
            const auto [t, done] = st.back();
            st.pop_back();
            if (done || nodes[t].count > 0) { post.push_back(t); continue; }
            st.push_back({t, true});
            st.push_back({nodes[t].right, false});
            st.push_back({nodes[t].left, false});
        }
        int64_t changed = 0;
        for (int32_t t : post) {
            TNode& nd = nodes[t];
            if (nd.count > 0) { cost[t] = nd.box.area() * nd.count; continue; }
            int32_t lv[kT] = {nd.left, nd.right};
            int32_t inner[kT];
            int nl = 2, ni = 0;
            double old = ct * nd.box.area();
            while (nl < kT) {
                int j = -1;
                double best_a = -1.0;
                for (int i = 0; i < nl; ++i)
                    if (nodes[lv[i]].count == 0 && nodes[lv[i]].box.area() > best_a) { best_a = nodes[lv[i]].box.area(); j = i; }
                if (j < 0) break;
                const int32_t x = lv[j];
                inner[ni++] = x;
                old += ct * best_a;
                lv[j] = nodes[x].left;
                lv[nl++] = nodes[x].right;
            }
            for (int i = 0; i < nl; ++i) old += cost[lv[i]];
            if (nl < 3) { cost[t] = old; continue; }
            const int full = (1 << nl) - 1;
            for (int m = 1; m <= full; ++m) {
                const int low = m & -m;
                if (m == low) {
                    const int i = __builtin_ctz((unsigned)m);
                    box_m[m] = nodes[lv[i]].box;
                    copt[m] = cost[lv[i]];
                    continue;
                }
                box_m[m] = box_m[m ^ low];
                box_m[m].grow(box_m[low]);
                box_a[m] = box_m[m].area();
                double best = DBL_MAX;
                int bp = 0;
                // partitions {sub, m ^ sub} with the lowest subtree in sub (each split once)
                for (int sub = (m - 1) & m; sub; sub = (sub - 1) & m) {
                    if (!(sub & low)) continue;
                    const double c = copt[sub] + copt[m ^ sub];
                    if (c < best) { best = c; bp = sub; }
                }
                copt[m] = ct * box_a[m] + best;
                part[m] = bp;
            }
            if (!(copt[full] < old * (1.0 - 1e-12))) { cost[t] = old; continue; }
            // rebuild the treelet below t with the optimal splits, reusing its inner nodes
            int used = 0;
            std::vector<std::pair<int32_t, int>> todo{{t, full}};
            while (!todo.empty()) {
                const auto [id, m] = todo.back();
                todo.pop_back();
                const int a = part[m], b = m ^ part[m];
                int32_t kids[2];
                const int ms[2] = {a, b};
                for (int s = 0; s < 2; ++s) {
                    if ((ms[s] & (ms[s] - 1)) == 0) {
                        kids[s] = lv[__builtin_ctz((unsigned)ms[s])];
                    } else {
                        const int32_t nid = inner[used++];
                        nodes[nid].box = box_m[ms[s]];
                        nodes[nid].count = 0;
                        cost[nid] = copt[ms[s]];
                        todo.push_back({nid, ms[s]});
                        kids[s] = nid;
                    }
                }
                nodes[id].left = kids[0];
                nodes[id].right = kids[1];
            }
            cost[t] = copt[full];
            ++changed;
        }
        if (std::getenv("PRT_BVH_VERBOSE"))
            std::fprintf(stderr, "prt_bvh: treelet pass %d: %lld treelets restructured, SAH %.3f\n", pass,
                         (long long)changed, nodes[root].box.area() > 0 ? cost[root] / nodes[root].box.area() : 0.0);
        if (!changed) break;
    }
}

// depth of the deepest node below `root` (root = 0), as Builder::build counts it
int32_t tree_depth(const std::vector<TNode>& nodes, int32_t root) {
    int32_t d = 0;
    std::vector<std::pair<int32_t, int32_t>> st{{root, 0}};
    while (!st.empty()) {
        const auto [t, k] = st.back();
        st.pop_back();
        d = std::max(d, k);
        if (nodes[t].count == 0) { st.push_back({nodes[t].left, k + 1}); st.push_back({nodes[t].right, k + 1}); }
    }
    return d;
}

}  // namespace

bool build_bvh(const float* tri_v, int64_t n_tri, int max_leaf, BvhHost* out, std::string* err) {
    if (max_leaf < 1 || max_leaf > kMaxLeaf) { *err = "max_leaf must be in [1, 8]"; return false; }
    if (n_tri < 0 || n_tri >= ((int64_t)1 << 27)) { *err = "triangle count out of range (< 2^27)"; return false; }
    Builder B;
    B.tv = tri_v; B.max_leaf = max_leaf;
    // scenes of >= 2^14 triangles (never LDS-resident) build finer: 64 SAH bins, early split clipping
    // above 128 x the mean box area, treelet restructuring (config 4: node visits 144.3 -> 138.1 per
    // sample against 32 bins / 64 x / no treelets, profiles/r05/treelet/); the small LDS scenes keep
    // the round-4 tree (the restructured Cornell tree collapses to a BVH4 that visits more nodes)
    const bool large = n_tri >= (1 << 14);
    if (large) B.bins = 64;
    if (const char* e = std::getenv("PRT_SAH_BINS")) B.bins = std::max(2, std::min(kMaxBins, std::atoi(e)));
    if (const char* e = std::getenv("PRT_SBVH")) B.sbvh = std::atoi(e) != 0;
    if (const char* e = std::getenv("PRT_SBVH_ALPHA")) B.alpha = std::max(0.0, std::atof(e));
    double budget = 1.3;
    if (const char* e = std::getenv("PRT_SBVH_BUDGET")) budget = std::max(1.0, std::atof(e));
    if (const char* e = std::getenv("PRT_SAH_CT")) B.ct = std::max(0.0, std::atof(e));
    if (const char* e = std::getenv("PRT_LEAF_MIN")) B.leaf_min = std::max(1, std::min(max_leaf, std::atoi(e)));
    std::vector<Box> tri_box((size_t)n_tri);
    Box scene;
    float max_abs = 0.0f;
    double mean_area = 0.0;
    for (int64_t i = 0; i < n_tri; ++i) {
        const float* t = tri_v + 9 * i;
        Box b;
        b.grow(t); b.grow(t + 3); b.grow(t + 6);
        for (int k = 0; k < 9; ++k) {
            if (!std::isfinite(t[k])) { *err = "non-finite vertex in triangle " + std::to_string(i); return false; }
            max_abs = std::max(max_abs, std::fabs(t[k]));
        }
        tri_box[(size_t)i] = b;
        mean_area += b.area();
        scene.grow(b);
    }
    mean_area /= (double)std::max<int64_t>(n_tri, 1);
    // references: one per triangle, several (early split clipping) for triangles whose box
    // area exceeds esc_beta x the mean (env PRT_ESC_BETA, 0 = off; at most 2 n_tri + 4096)
    double esc_beta = large ? 128.0 : 64.0;
    if (const char* e = std::getenv("PRT_ESC_BETA")) esc_beta = std::max(0.0, std::atof(e));
    std::vector<int32_t>& ref_tri = B.ref_tri;
    ref_tri.reserve((size_t)n_tri);
    // the cap stays below the 2^27 references the leaf encoding addresses: past it every further
    // triangle keeps one reference (a scene with < 2^27 triangles always builds)
    const int64_t ref_cap = std::min<int64_t>(2 * n_tri + 4096, ((int64_t)1 << 27) - 1);
    std::vector<RefBox> pieces;
    for (int64_t i = 0; i < n_tri; ++i) {
        const Box& b = tri_box[(size_t)i];
        pieces.clear();
        // mean_area > 0: a scene of degenerate boxes (area 0) would split every other triangle
        // to the maximum depth against a zero threshold
        if (esc_beta > 0.0 && mean_area > 0.0 && b.area() > esc_beta * mean_area && (int64_t)B.tb.size() < ref_cap) {
            const float* t = tri_v + 9 * i;
            double v[3][3];
            for (int a = 0; a < 3; ++a)
                for (int k = 0; k < 3; ++k) v[a][k] = (double)t[3 * a + k];
            RefBox cell;
            for (int k = 0; k < 3; ++k) { cell.lo[k] = b.lo[k]; cell.hi[k] = b.hi[k]; }
            split_refs(v, cell, esc_beta * mean_area, 0, &pieces);
        }
        // one triangle yields up to 2^12 pieces: past the remaining budget it keeps one reference
        if (pieces.size() <= 1 || (int64_t)(B.tb.size() + pieces.size() + (size_t)(n_tri - i - 1)) > ref_cap) {
            B.tb.push_back(b);
            ref_tri.push_back((int32_t)i);
        } else {
            for (const RefBox& r : pieces) {
                B.tb.push_back(outward_f32(r, b));
                ref_tri.push_back((int32_t)i);
            }
        }
    }
    const int64_t n_ref0 = (int64_t)B.tb.size();
    if (n_ref0 >= ((int64_t)1 << 27)) { *err = "too many BVH references (< 2^27)"; return false; }
    B.cen.resize((size_t)n_ref0 * 3);
    std::vector<int32_t> all((size_t)n_ref0);
    for (int64_t i = 0; i < n_ref0; ++i) {
        B.set_centre((int32_t)i);
        all[(size_t)i] = (int32_t)i;
    }
    // spatial splits add references up to the budget, below the 2^27 the leaf encoding addresses
    B.ref_budget = std::min<int64_t>((int64_t)((double)n_ref0 * budget), ((int64_t)1 << 27) - 1);
    float extent = scene.valid() ? std::max({scene.hi[0] - scene.lo[0], scene.hi[1] - scene.lo[1], scene.hi[2] - scene.lo[2]}) : 0.0f;
    // Padding: ~8 ulps of the largest coordinate magnitude / extent.  Keeps the
    // slab test conservative against Moller-Trumbore accepting hit points that
    // lie a rounding error outside the triangle (axis-aligned Cornell edges).
    float pad = std::max(max_abs, extent) * 1e-6f + 1e-30f;
    int32_t root = -1;
    if (n_ref0 > 0) {
        B.nodes.reserve((size_t)(2 * n_ref0 / std::max(1, max_leaf / 2) + 8));
        if (scene.valid()) B.min_overlap = B.alpha * scene.area();
        root = B.build(all, 0);
        // treelet restructuring passes (env PRT_TREELET, 0 = off): on by default for large scenes
        // (config 4: BVH2 SAH -3 %, node visits -2.1 %, 157.5 -> 154.6 ms per launch); the small
        // LDS-resident scenes keep the plain tree, whose BVH4 collapse visits fewer nodes there
        // (Cornell: 22.7 vs 26.3 node visits per sample with the restructured tree, profiles/r05/treelet/)
        int passes = large ? 3 : 0;
        if (const char* e = std::getenv("PRT_TREELET")) passes = std::max(0, std::min(8, std::atoi(e)));
        if (passes > 0 && B.nodes[root].count == 0) {
            restructure_treelets(B.nodes, root, B.ct, passes);
            B.max_depth = tree_depth(B.nodes, root);
        }
    }
    // every reference sits in exactly one leaf: the leaf order is the triangle records' order
    const int64_t n_ref = (int64_t)B.order.size();
    if (n_ref != (int64_t)B.tb.size()) { *err = "internal: BVH references lost in the build"; return false; }
    // flatten: inner nodes in DFS preorder; leaves become child references
    std::vector<int32_t> inner_id(B.nodes.size(), -1);
    std::vector<int32_t> stack;
    int32_t n_inner = 0;
    std::vector<int32_t> preorder;
    if (root >= 0 && B.nodes[root].count == 0) {
        stack.push_back(root);
        while (!stack.empty()) {
            int32_t t = stack.back(); stack.pop_back();
            inner_id[t] = n_inner++;
            preorder.push_back(t);
            const TNode& nd = B.nodes[t];
            if (B.nodes[nd.right].count == 0) stack.push_back(nd.right);
            if (B.nodes[nd.left].count == 0) stack.push_back(nd.left);
        }
    }
    auto child_ref = [&](int32_t t) -> int32_t {
        const TNode& c = B.nodes[t];
        if (c.count > 0) return leaf_ref(c.first, c.count);
        return inner_id[t];
    };
    auto put_box = [&](float* f, int side, const Box& bx, bool valid) {
        float lo[3], hi[3];
        for (int k = 0; k < 3; ++k) {
            lo[k] = valid ? bx.lo[k] - pad : INFINITY;
            hi[k] = valid ? bx.hi[k] + pad : -INFINITY;
        }
        if (side == 0) {
            f[0] = lo[0]; f[1] = hi[0]; f[2] = lo[1]; f[3] = hi[1]; f[4] = lo[2]; f[5] = hi[2];
        } else {
            f[6] = lo[0]; f[7] = hi[0]; f[8] = lo[1]; f[9] = hi[1]; f[10] = lo[2]; f[11] = hi[2];
        }
    };
    out->nodes.assign((size_t)std::max<int32_t>(n_inner, 1) * 16, 0.0f);
    if (n_inner == 0) {
        // empty scene or a single leaf: one inner node, left = leaf (if any), right = empty
        float* f = out->nodes.data();
        Box empty;
        if (root >= 0) put_box(f, 0, B.nodes[root].box, true); else put_box(f, 0, empty, false);
        put_box(f, 1, empty, false);
        int32_t lr = root >= 0 ? leaf_ref(0, (int)n_ref) : leaf_ref(0, 1);
        f[12] = bits_f(lr); f[13] = bits_f(lr); f[14] = 0.0f; f[15] = 0.0f;
        out->n_nodes = 1;
    } else {
        for (int32_t t : preorder) {
            float* f = out->nodes.data() + (size_t)inner_id[t] * 16;
            const TNode& nd = B.nodes[t];
            put_box(f, 0, B.nodes[nd.left].box, true);
            put_box(f, 1, B.nodes[nd.right].box, true);
            f[12] = bits_f(child_ref(nd.left));
            f[13] = bits_f(child_ref(nd.right));
            f[14] = 0.0f; f[15] = 0.0f;
        }
        out->n_nodes = n_inner;
    }
    out->order.resize((size_t)n_ref);
    for (int64_t s = 0; s < n_ref; ++s) out->order[(size_t)s] = ref_tri[(size_t)B.order[(size_t)s]];
    out->tris.assign((size_t)n_ref * 12, 0.0f);
    for (int64_t s = 0; s < n_ref; ++s) {
        int32_t o = out->order[(size_t)s];
        const float* t = tri_v + 9 * (int64_t)o;
        float* d = out->tris.data() + 12 * s;
        for (int k = 0; k < 3; ++k) {
            d[k] = t[k];
            d[4 + k] = t[3 + k] - t[k];   // e1 = v1 - v0 in f32 (bit-identical to on-the-fly)
            d[8 + k] = t[6 + k] - t[k];   // e2 = v2 - v0
        }
        d[3] = bits_f(o); d[7] = 0.0f; d[11] = 0.0f;
    }
    out->depth = n_ref > 0 ? std::max(1, B.max_depth) : 1;
    out->n_refs = n_ref;
    out->n_leaves = B.leaves;
    out->pad = pad;
    double sah = 0.0;
    if (root >= 0 && B.nodes[root].box.area() > 0.0) {
        double ra = B.nodes[root].box.area();
        for (const TNode& nd : B.nodes) sah += nd.box.area() / ra * (nd.count > 0 ? (double)nd.count : 1.0);
    }
    out->sah_cost = sah;
    out->n_spatial = B.spatial_splits;
    if (std::getenv("PRT_BVH_VERBOSE"))
        std::fprintf(stderr, "prt_bvh: %lld triangles, %lld references (%lld before spatial splits), %lld spatial "
                             "splits, %lld leaves, depth %d, SAH %.3f\n", (long long)n_tri, (long long)n_ref,
                     (long long)n_ref0, (long long)B.spatial_splits, (long long)B.leaves, (int)out->depth, sah);
    return true;
}

namespace {

struct Child {
    float lo[3], hi[3];
    int32_t ref;
    bool empty;
};

inline int32_t ref_of(const float* n2, int side) {
    int32_t r;
    std::memcpy(&r, n2 + 12 + side, 4);
    return r;
}

inline Child child_of(const float* n2, int side) {
    Child c;
    const float* b = n2 + 6 * side;
    c.lo[0] = b[0]; c.hi[0] = b[1]; c.lo[1] = b[2]; c.hi[1] = b[3]; c.lo[2] = b[4]; c.hi[2] = b[5];
    c.ref = ref_of(n2, side);
    c.empty = !(c.lo[0] <= c.hi[0]);
    return c;
}

inline double child_area(const Child& c) {
    double dx = (double)c.hi[0] - c.lo[0], dy = (double)c.hi[1] - c.lo[1], dz = (double)c.hi[2] - c.lo[2];
    return 2.0 * (dx * dy + dy * dz + dz * dx);
}

}  // namespace

// SAH-optimal collapse of the BVH2 into BVH4 nodes (Ylitie et al. 2017's dynamic program, for
// four-wide nodes).  Expected cost of a tree = sum over BVH4 nodes of area x 1 (one visit) + sum
// over leaf entries of area x ct x triangles.  cost[i][k] (k = 2..4) = least cost of representing
// inner BVH2 node i's subtree by exactly k entries of one BVH4 node, the subtrees below those
// entries included; cost[i][1] = least cost of i as one entry: its own BVH4 node, or (subtrees of
// <= leaf_cap triangles) one leaf of its whole triangle range.  split[i][k] = entries taken from
// the left child.
struct DpCollapse {
    std::vector<double> cost;     // n2 * 5
    std::vector<int8_t> split;    // n2 * 5
    std::vector<double> area;     // n2: surface area of inner node i
    std::vector<int64_t> first;   // n2: triangle range of i's subtree (BVH order)
    std::vector<int32_t> count;   //     (-1: not one contiguous range)
    std::vector<uint8_t> as_leaf; // n2: cost[i][1] is the merged leaf
    const BvhHost& b2;
    double ct;
    int leaf_cap;
    DpCollapse(const BvhHost& b, double ct_, int leaf_cap_) : b2(b), ct(ct_), leaf_cap(leaf_cap_) {
        const int64_t n2 = b2.n_nodes;
        cost.assign((size_t)n2 * 5, INFINITY);
        split.assign((size_t)n2 * 5, 0);
        area.assign((size_t)n2, 0.0);
        first.assign((size_t)n2, 0);
        count.assign((size_t)n2, -1);
        as_leaf.assign((size_t)n2, 0);
        for (int64_t i = 0; i < n2; ++i) {
            const float* n = b2.nodes.data() + (size_t)i * 16;
            for (int s = 0; s < 2; ++s) {
                Child c = child_of(n, s);
                if (c.ref >= 0 && !c.empty) area[(size_t)c.ref] = child_area(c);
            }
        }
        if (n2 > 0) {
            Child a = child_of(b2.nodes.data(), 0), b = child_of(b2.nodes.data(), 1);
            Child u = a;
            for (int k = 0; k < 3; ++k) {
                if (!b.empty) { u.lo[k] = std::min(u.lo[k], b.lo[k]); u.hi[k] = std::max(u.hi[k], b.hi[k]); }
            }
            area[0] = a.empty ? 0.0 : child_area(u);
        }
        // preorder ids: children follow their parent, so a reverse sweep is bottom-up
        for (int64_t i = n2 - 1; i >= 0; --i) {
            const float* n = b2.nodes.data() + (size_t)i * 16;
            Child c[2] = {child_of(n, 0), child_of(n, 1)};
            double* ci = &cost[(size_t)i * 5];
            for (int k = 2; k <= 4; ++k) {
                for (int a = c[0].empty ? 0 : 1; a <= k; ++a) {
                    int b = k - a;
                    if (c[1].empty ? b != 0 : b < 1) continue;
                    double v = side(c[0], a) + side(c[1], b);
                    if (v < ci[k]) { ci[k] = v; split[(size_t)i * 5 + k] = (int8_t)a; }
                }
            }
            // a single-leaf scene (one empty child) still gets a node of its one entry
            double best = std::min({ci[2], ci[3], ci[4], c[1].empty ? side(c[0], 1) : INFINITY});
            ci[1] = area[(size_t)i] + best;
            int64_t f[2];
            int32_t m[2];
            for (int s = 0; s < 2; ++s) range(c[s], &f[s], &m[s]);
            if (m[0] >= 0 && m[1] >= 0 && f[0] + m[0] == f[1]) {
                first[(size_t)i] = f[0];
                count[(size_t)i] = m[0] + m[1];
                double leaf = area[(size_t)i] * ct * (double)(m[0] + m[1]);
                if (i > 0 && m[0] + m[1] <= leaf_cap && leaf < ci[1]) { ci[1] = leaf; as_leaf[(size_t)i] = 1; }
            }
        }
    }
    void range(const Child& c, int64_t* f, int32_t* m) const {
        if (c.empty) { *f = 0; *m = -1; return; }
        if (c.ref < 0) { int32_t v = -c.ref - 1; *f = v >> 3; *m = (v & 7) + 1; return; }
        *f = first[(size_t)c.ref]; *m = count[(size_t)c.ref];
    }
    double side(const Child& c, int a) const {
        if (c.empty) return a == 0 ? 0.0 : INFINITY;
        if (a == 0) return INFINITY;
        if (c.ref < 0) return a == 1 ? child_area(c) * ct * (double)(((-c.ref - 1) & 7) + 1) : INFINITY;
        return cost[(size_t)c.ref * 5 + a];
    }
    // one entry: a BVH2 leaf, an inner node, or an inner node's subtree merged into one leaf
    Child entry(const Child& c) const {
        Child e = c;
        if (c.ref >= 0 && as_leaf[(size_t)c.ref]) e.ref = leaf_ref(first[(size_t)c.ref], count[(size_t)c.ref]);
        return e;
    }
    // entries of inner node i's k-entry cut (k >= 2)
    void expand(int32_t i, int k, std::vector<Child>* outc) const {
        const float* n = b2.nodes.data() + (size_t)i * 16;
        Child c[2] = {child_of(n, 0), child_of(n, 1)};
        int a = split[(size_t)i * 5 + k];
        int parts[2] = {a, k - a};
        for (int s = 0; s < 2; ++s) {
            if (parts[s] == 0) continue;
            if (parts[s] == 1) outc->push_back(entry(c[s]));
            else expand(c[s].ref, parts[s], outc);
        }
    }
    // children of the BVH4 node made from inner node i
    void children(int32_t i, std::vector<Child>* outc) const {
        const double* ci = &cost[(size_t)i * 5];
        const float* n = b2.nodes.data() + (size_t)i * 16;
        if (child_of(n, 1).empty) {
            Child c0 = child_of(n, 0);
            if (!c0.empty) outc->push_back(entry(c0));
            return;
        }
        int k = 2;
        for (int j = 3; j <= 4; ++j)
            if (ci[j] < ci[k]) k = j;
        expand(i, k, outc);
    }
};

void collapse_bvh4(const BvhHost& b2, Bvh4Host* out) {
    // Each BVH4 node takes a BVH2 node's two children and repeatedly opens the
    // inner child with the largest surface area until it holds four children (greedy, env
    // PRT_BVH4_DP=0), or takes the SAH-optimal cut of DpCollapse (default).
    // anc = entries the traversal can hold for the node's strict ancestors: a visit continues
    // with one hit child and pushes the others (<= children - 1), and LIFO order means the
    // stack below a node holds only siblings of its ancestors (traverse_ww4)
    struct Item { int32_t b2node; int32_t slot; int32_t depth; int32_t anc; };
    std::vector<Item> work;
    out->nodes.clear();
    out->nodes.resize(32, 0.0f);
    out->n_nodes = 1;
    out->depth = 0;
    int32_t max_anc = 0;
    work.push_back({0, 0, 0, 0});
    // env PRT_BVH4_DP=0: the greedy collapse (config 2: 24.8 node visits per sample against 22.7)
    const char* dp_env = std::getenv("PRT_BVH4_DP");
    std::unique_ptr<DpCollapse> dp;
    if (!dp_env || std::atoi(dp_env) != 0) {
        double ct = 0.5;
        int cap = 0;
        if (const char* e = std::getenv("PRT_DP_CT")) ct = std::max(0.0, std::atof(e));
        if (const char* e = std::getenv("PRT_DP_LEAF")) cap = std::max(0, std::min(kMaxLeaf, std::atoi(e)));
        dp.reset(new DpCollapse(b2, ct, cap));
    }
    while (!work.empty()) {
        Item it = work.back();
        work.pop_back();
        const float* n2 = b2.nodes.data() + (size_t)it.b2node * 16;
        std::vector<Child> ch;
        if (dp) {
            dp->children(it.b2node, &ch);
        } else {
            for (int side = 0; side < 2; ++side) {
                Child c = child_of(n2, side);
                if (!c.empty) ch.push_back(c);
            }
        }
        while (!dp && ch.size() < 4) {
            int best = -1;
            double ba = -1.0;
            for (size_t k = 0; k < ch.size(); ++k)
                if (ch[k].ref >= 0 && child_area(ch[k]) > ba) { ba = child_area(ch[k]); best = (int)k; }
            if (best < 0) break;
            const float* m = b2.nodes.data() + (size_t)ch[best].ref * 16;
            Child a = child_of(m, 0), b = child_of(m, 1);
            ch.erase(ch.begin() + best);
            if (!a.empty) ch.push_back(a);
            if (!b.empty) ch.push_back(b);
        }
        float* f = out->nodes.data() + (size_t)it.slot * 32;
        for (int k = 0; k < 4; ++k) {
            bool ok = k < (int)ch.size();
            for (int a = 0; a < 3; ++a) {
                // empty slot: inverted box (lo = +inf, hi = -inf) is missed by every ray
                // whose direction has one finite 1/d, whatever t_max (even NaN / inf)
                f[(2 * a) * 4 + k] = ok ? ch[k].lo[a] : INFINITY;
                f[(2 * a + 1) * 4 + k] = ok ? ch[k].hi[a] : -INFINITY;
            }
            // empty slot ref = the traversal sentinel: if a NaN ray ever "hits" it, the lane's
            // traversal ends instead of restarting at the root (a NaN ray hits nothing anyway)
            int32_t ref = 0x7FFFFFFF;
            if (ok) {
                if (ch[k].ref >= 0) {
                    ref = (int32_t)out->n_nodes++;
                    out->nodes.resize((size_t)out->n_nodes * 32, 0.0f);
                    f = out->nodes.data() + (size_t)it.slot * 32;   // storage may have moved
                    work.push_back({ch[k].ref, ref, it.depth + 1, it.anc + (int32_t)ch.size() - 1});
                } else {
                    ref = ch[k].ref;
                }
            }
            std::memcpy(f + 24 + k, &ref, 4);
        }
        out->depth = std::max(out->depth, it.depth);
        max_anc = std::max(max_anc, it.anc);
    }
    // the sentinel, the deepest node's ancestor entries, and the <= 3 slots a visit writes
    // above the top unconditionally (visit_node4); <= 3 (depth + 1) + 1, the per-level bound
    out->stack_need = 1 + max_anc + 3;
}

void quantize_bvh4(const Bvh4Host& b4, float pad, std::vector<float>* out) {
    out->assign((size_t)b4.n_nodes * 16, 0.0f);
    const double margin = 2.0 * (double)pad;
    for (int64_t n = 0; n < b4.n_nodes; ++n) {
        const float* f = b4.nodes.data() + (size_t)n * 32;
        float* q = out->data() + (size_t)n * 16;
        int32_t refs[4];
        std::memcpy(refs, f + 24, 16);
        bool ok[4];
        for (int k = 0; k < 4; ++k) ok[k] = std::isfinite(f[k]);   // empty slots hold +inf
        float origin[3], step[3];
        uint32_t ql[3] = {0, 0, 0}, qh[3] = {0, 0, 0};
        for (int a = 0; a < 3; ++a) {
            double lo = INFINITY, hi = -INFINITY;
            for (int k = 0; k < 4; ++k)
                if (ok[k]) {
                    lo = std::min(lo, (double)f[(2 * a) * 4 + k]);
                    hi = std::max(hi, (double)f[(2 * a + 1) * 4 + k]);
                }
            if (!(lo <= hi)) { lo = 0.0; hi = 0.0; }
            // origin rounded down to f32; grid step = the f32 at or above range / 254
            float o = (float)(lo - margin);
            if ((double)o > lo - margin) o = std::nextafter(o, -INFINITY);
            double ext = hi + margin - (double)o;
            float stf = (float)std::max(ext / 254.0, 1e-30);
            if ((double)stf < ext / 254.0) stf = std::nextafter(stf, INFINITY);
            double st = (double)stf;
            origin[a] = o;
            step[a] = (float)st;
            for (int k = 0; k < 4; ++k) {
                if (!ok[k]) continue;
                double l = (double)f[(2 * a) * 4 + k], h = (double)f[(2 * a + 1) * 4 + k];
                long ql_k = (long)std::floor((l - margin - (double)o) / st);
                long qh_k = (long)std::ceil((h + margin - (double)o) / st);
                ql_k = std::max(0L, std::min(255L, ql_k));
                qh_k = std::max(0L, std::min(255L, qh_k));
                ql[a] |= (uint32_t)ql_k << (8 * k);
                qh[a] |= (uint32_t)qh_k << (8 * k);
            }
        }
        q[0] = origin[0]; q[1] = origin[1]; q[2] = origin[2]; q[3] = step[0];
        q[4] = step[1]; q[5] = step[2];
        std::memcpy(q + 6, &ql[0], 4); std::memcpy(q + 7, &qh[0], 4);
        std::memcpy(q + 8, &ql[1], 4); std::memcpy(q + 9, &qh[1], 4);
        std::memcpy(q + 10, &ql[2], 4); std::memcpy(q + 11, &qh[2], 4);
        for (int k = 0; k < 4; ++k) {
            int32_t r = ok[k] ? refs[k] : 0x7FFFFFFF;
            std::memcpy(q + 12 + k, &r, 4);
        }
    }
}


}  // namespace prt
