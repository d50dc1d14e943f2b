// coherence_c4 — the config-4 coherence model of VERDICT r05 item 6, on the CPU.
//
// Config 4's global-scene kernel is bound by the vector-L1 pipeline (TA/TD busy 0.93 / 0.98,
// 27.4 L1 accesses per vector-memory instruction, profiles/r05/final/pmc_mem_c4/): a wave's node load
// costs one tag lookup per DISTINCT line its active lanes touch.  This model prices a ray-sorting
// stage on that metric before anything is built: it builds the library's BVH (pyrenderer_amd/csrc/
// prt_bvh.cpp: SBVH + treelets + 64 bins, BVH4 collapse, 64-B quantised nodes) of the 1,000,044-
// triangle scene, walks every ray of tools/c4_rays.py through the BVH4 in the kernel's visiting order
// (closest hit: nearest hit child first; shadow: farthest first, stop at the first hit; prune by the
// best t), and then forms waves of 64 rays under several schedules, advancing each lane through its
// visit sequence in lockstep (trip k: every lane's k-th node), to count per wave trip the distinct
// 64-B nodes (and 128-B lines) and the distinct 48-B triangle records of the leaf tests:
//   regen   (extension rays) the kernel's schedule: 64 lanes run pixels' paths bounce after bounce
//           and refill from the pixel-major queue, so a wave mixes bounces of neighbouring pixels
//   pixel   rays of one (bounce, kind) in pixel order — pixel-major chunks without that drift
//   random  64 random rays of the (bounce, kind) — fully incoherent
//   sortN   windows of N consecutive rays (pixel order) sorted by (direction octant, Morton code of
//           the origin in a 2^10-cell grid per axis) — a sorted extension-ray stage over N-ray windows
//
//   g++ -O2 -std=c++17 -I pyrenderer_amd/csrc tools/coherence_c4.cpp pyrenderer_amd/csrc/prt_bvh.cpp \
//       -o build/coherence_c4
//   build/coherence_c4 /tmp/c4_rays_soup.f32 /tmp/c4_rays.f32  > profiles/r06/coherence_c4/model.json
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <numeric>
#include <random>
#include <string>
#include <unordered_set>
#include <vector>

#include "prt_internal.h"

namespace {

struct Ray { double o[3], d[3], tmax; int kind, pixel; };
struct Visit { std::vector<int32_t> nodes, tris; };

std::vector<float> read_f32(const char* path) {
    FILE* f = std::fopen(path, "rb");
    if (!f) { std::perror(path); std::exit(2); }
    std::fseek(f, 0, SEEK_END);
    const long n = std::ftell(f) / 4;
    std::fseek(f, 0, SEEK_SET);
    std::vector<float> v((size_t)n);
    if (std::fread(v.data(), 4, v.size(), f) != v.size()) std::exit(2);
    std::fclose(f);
    return v;
}
int32_t ibits(float f) { int32_t v; std::memcpy(&v, &f, 4); return v; }
uint32_t ubits(float f) { uint32_t v; std::memcpy(&v, &f, 4); return v; }

struct Model {
    std::vector<float> q4, tris;   // quantised BVH4 (16 floats per node), triangle records (12 per ref)
    // child k's box of quantised node n (double, dequantised as the kernel's planes)
    void box(int64_t n, int k, double lo[3], double hi[3]) const {
        const float* q = q4.data() + 16 * n;
        const uint32_t ql[3] = {ubits(q[6]), ubits(q[8]), ubits(q[10])}, qh[3] = {ubits(q[7]), ubits(q[9]), ubits(q[11])};
        const double st[3] = {q[3], q[4], q[5]};
        for (int a = 0; a < 3; ++a) {
            lo[a] = q[a] + (double)((ql[a] >> (8 * k)) & 0xFFu) * st[a];
            hi[a] = q[a] + (double)((qh[a] >> (8 * k)) & 0xFFu) * st[a];
        }
    }
    bool tri_hit(int64_t r, const Ray& ray, double tmin, double tmax, double* t) const {
        const float* p = tris.data() + 12 * r;
        const double v0[3] = {p[0], p[1], p[2]}, e1[3] = {p[4], p[5], p[6]}, e2[3] = {p[8], p[9], p[10]};
        const double* d = ray.d;
        const double c[3] = {e1[1] * d[2] - e1[2] * d[1], e1[2] * d[0] - e1[0] * d[2], e1[0] * d[1] - e1[1] * d[0]};
        const double det = c[0] * e2[0] + c[1] * e2[1] + c[2] * e2[2];
        if (det == 0.0) return false;
        const double f = 1.0 / det;
        const double s[3] = {ray.o[0] - v0[0], ray.o[1] - v0[1], ray.o[2] - v0[2]};
        const double q[3] = {s[1] * e2[2] - s[2] * e2[1], s[2] * e2[0] - s[0] * e2[2], s[0] * e2[1] - s[1] * e2[0]};
        const double tt = -f * (q[0] * e1[0] + q[1] * e1[1] + q[2] * e1[2]);
        const double u = -f * (q[0] * d[0] + q[1] * d[1] + q[2] * d[2]);
        const double v = f * (c[0] * s[0] + c[1] * s[1] + c[2] * s[2]);
        if (!(tmin < tt && tt < tmax && u >= 0 && u <= 1 && v >= 0 && 1 - u - v >= 0)) return false;
        *t = tt;
        return true;
    }
    // the node and triangle-record sequence of one query in the kernel's order
    Visit walk(const Ray& ray) const {
        Visit out;
        const bool any = (ray.kind & 1) != 0;
        double inv[3];
        for (int a = 0; a < 3; ++a) inv[a] = 1.0 / (ray.d[a] == 0.0 ? 1e-30 : ray.d[a]);
        double best = ray.tmax;
        std::vector<int32_t> stack = {0};
        while (!stack.empty()) {
            const int32_t cur = stack.back();
            stack.pop_back();
            if (cur < 0) {
                const int64_t v = -(int64_t)cur - 1, first = v >> 3, cnt = (v & 7) + 1;
                for (int64_t r = first; r < first + cnt; ++r) {
                    out.tris.push_back((int32_t)r);
                    double t;
                    if (tri_hit(r, ray, 1e-5, best, &t)) {
                        best = t;
                        if (any) return out;
                    }
                }
                continue;
            }
            out.nodes.push_back(cur);
            const float* q = q4.data() + 16 * (int64_t)cur;
            std::pair<double, int32_t> hit[4];
            int nh = 0;
            for (int k = 0; k < 4; ++k) {
                const int32_t ref = ibits(q[12 + k]);
                if (ref == 0x7FFFFFFF) continue;
                double lo[3], hi[3];
                box(cur, k, lo, hi);
                double tn = 1e-5, tf = best;
                for (int a = 0; a < 3; ++a) {
                    double t0 = (lo[a] - ray.o[a]) * inv[a], t1 = (hi[a] - ray.o[a]) * inv[a];
                    if (t0 > t1) std::swap(t0, t1);
                    tn = std::max(tn, t0);
                    tf = std::min(tf, t1);
                }
                if (tn <= tf) hit[nh++] = {tn, ref};
            }
            // closest hit: nearest child on top of the stack (visited next); shadow: farthest
            std::sort(hit, hit + nh, [&](auto& a, auto& b) { return any ? a.first < b.first : a.first > b.first; });
            for (int k = 0; k < nh; ++k) stack.push_back(hit[k].second);
        }
        return out;
    }
};

struct Stats { double rays = 0, node_trips = 0, node_lanes = 0, node_lines64 = 0, node_lines128 = 0,
               tri_trips = 0, tri_lanes = 0, tri_lines = 0, node_quad_cost = 0; };

// The vector-L1 cost of one wave load by lane quads, as tools/micro/l1_lines.hip measured it on
// L1/L2-resident nodes (profiles/r06/micro/): a quad whose active lanes all read ONE node costs 0.26 of
// a quad whose lanes read two or more (lanes sharing nodes in pairs cost as much as all-distinct lanes);
// a quad without active lanes costs nothing
double quad_cost(const int32_t* node_of_lane, int n) {
    double c = 0.0;
    for (int q = 0; q < n; q += 4) {
        int32_t first = -1;
        bool any = false, uniform = true;
        for (int j = q; j < std::min(n, q + 4); ++j) {
            if (node_of_lane[j] < 0) continue;
            if (!any) { first = node_of_lane[j]; any = true; }
            else if (node_of_lane[j] != first) uniform = false;
        }
        c += !any ? 0.0 : uniform ? 0.26 : 1.0;
    }
    return c;
}

// lockstep waves: trip k of a wave holds every lane's k-th element
void wave(const std::vector<const Visit*>& lanes, Stats& s) {
    static const Visit kIdle;   // an idle lane (null entry): no visits, keeps its position in the quads
    std::vector<const Visit*> L(lanes.size());
    for (size_t j = 0; j < lanes.size(); ++j) { L[j] = lanes[j] ? lanes[j] : &kIdle; s.rays += lanes[j] ? 1.0 : 0.0; }
    size_t kn = 0, kt = 0;
    for (auto* v : L) { kn = std::max(kn, v->nodes.size()); kt = std::max(kt, v->tris.size()); }
    std::unordered_set<int64_t> a, b, c;
    int32_t nl[64];
    for (size_t k = 0; k < kn; ++k) {
        a.clear(); b.clear();
        int act = 0;
        for (size_t j = 0; j < L.size(); ++j) {
            const Visit* v = L[j];
            nl[j] = k < v->nodes.size() ? v->nodes[k] : -1;
            if (k < v->nodes.size()) { ++act; a.insert(v->nodes[k]); b.insert(v->nodes[k] >> 1); }
        }
        s.node_trips += 1; s.node_lanes += act; s.node_lines64 += (double)a.size(); s.node_lines128 += (double)b.size();
        s.node_quad_cost += quad_cost(nl, (int)L.size());
    }
    for (size_t k = 0; k < kt; ++k) {
        c.clear();
        int act = 0;
        // a 48-B record spans one or two 64-B lines
        for (auto* v : L)
            if (k < v->tris.size()) { ++act; c.insert((int64_t)v->tris[k] * 48 / 64); c.insert(((int64_t)v->tris[k] * 48 + 47) / 64); }
        s.tri_trips += 1; s.tri_lanes += act; s.tri_lines += (double)c.size();
    }
}

uint64_t morton10(uint32_t x, uint32_t y, uint32_t z) {
    auto spread = [](uint64_t v) {
        v &= 0x3FF;
        v = (v | (v << 16)) & 0x030000FF;
        v = (v | (v << 8)) & 0x0300F00F;
        v = (v | (v << 4)) & 0x030C30C3;
        v = (v | (v << 2)) & 0x09249249;
        return v;
    };
    return spread(x) | (spread(y) << 1) | (spread(z) << 2);
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 3) { std::fprintf(stderr, "usage: %s <soup.f32> <rays.f32>\n", argv[0]); return 2; }
    const std::vector<float> tv = read_f32(argv[1]);
    const std::vector<float> rv = read_f32(argv[2]);
    prt::BvhHost b2;
    std::string err;
    if (!prt::build_bvh(tv.data(), (int64_t)(tv.size() / 9), 4, &b2, &err)) { std::fprintf(stderr, "%s\n", err.c_str()); return 1; }
    prt::Bvh4Host b4;
    prt::collapse_bvh4(b2, &b4);
    Model m;
    prt::quantize_bvh4(b4, b2.pad, &m.q4);
    m.tris = b2.tris;
    std::vector<Ray> rays(rv.size() / 9);
    double lo[3] = {1e30, 1e30, 1e30}, hi[3] = {-1e30, -1e30, -1e30};
    for (size_t i = 0; i < rays.size(); ++i) {
        const float* r = rv.data() + 9 * i;
        for (int a = 0; a < 3; ++a) {
            rays[i].o[a] = r[a]; rays[i].d[a] = r[3 + a];
            lo[a] = std::min(lo[a], (double)r[a]); hi[a] = std::max(hi[a], (double)r[a]);
        }
        rays[i].tmax = r[6]; rays[i].kind = (int)r[7]; rays[i].pixel = (int)r[8];
    }
    std::vector<Visit> vis(rays.size());
#pragma omp parallel for schedule(dynamic, 64)
    for (size_t i = 0; i < rays.size(); ++i) vis[i] = m.walk(rays[i]);
    // groups: (bounce, kind), rays in file (pixel) order
    std::map<int, std::vector<size_t>> groups;
    for (size_t i = 0; i < rays.size(); ++i) groups[rays[i].kind].push_back(i);
    // sort keys: (direction octant, origin Morton code in a 2^10 grid) — VERDICT r05's proposal;
    // "dirbin": (cube-map face of d and an 8 x 8 cell of it, origin Morton in a 2^6 grid); "origin":
    // the origin's Morton code alone
    auto cell = [&](const Ray& r, double n) {
        uint32_t c[3];
        for (int a = 0; a < 3; ++a)
            c[a] = (uint32_t)std::min(n - 1, std::max(0.0, (r.o[a] - lo[a]) / (hi[a] - lo[a] + 1e-12) * n));
        return morton10(c[0], c[1], c[2]);
    };
    auto key = [&](size_t i, int kind) -> uint64_t {
        const Ray& r = rays[i];
        if (kind == 2) return cell(r, 1024.0);
        if (kind == 1) {
            const double ax = std::fabs(r.d[0]), ay = std::fabs(r.d[1]), az = std::fabs(r.d[2]);
            const int ma = ax >= ay && ax >= az ? 0 : ay >= az ? 1 : 2;
            const double m = std::max(ax, std::max(ay, az));
            const int u = (ma + 1) % 3, v = (ma + 2) % 3;
            const uint32_t face = 2 * ma + (r.d[ma] < 0), cu = (uint32_t)std::min(7.0, (r.d[u] / m + 1) * 4),
                           cv = (uint32_t)std::min(7.0, (r.d[v] / m + 1) * 4);
            return ((uint64_t)(face * 64 + cu * 8 + cv) << 32) | cell(r, 64.0);
        }
        const uint32_t oct = (r.d[0] < 0) | ((r.d[1] < 0) << 1) | ((r.d[2] < 0) << 2);
        return ((uint64_t)oct << 32) | cell(r, 1024.0);
    };
    const std::vector<std::string> scheds = {"pixel", "random", "sort4096", "sort65536", "sort_all", "dirbin4096",
                                             "dirbin65536", "origin256", "origin1024", "origin4096", "origin65536"};
    std::printf("{\"bvh4_nodes\": %lld, \"rays\": %zu, \"groups\": {", (long long)b4.n_nodes, rays.size());
    std::map<std::string, Stats> tot_ext, tot_sh;
    bool first_g = true;
    std::mt19937 g(7);
    for (auto& [kind, idx] : groups) {
        std::printf("%s\"%d\": {\"rays\": %zu", first_g ? "" : ", ", kind, idx.size());
        first_g = false;
        for (const auto& sc : scheds) {
            std::vector<size_t> order = idx;
            if (sc == "random") std::shuffle(order.begin(), order.end(), g);
            size_t win = 0;
            for (size_t w : {65536, 4096, 1024, 256})
                if (!win && sc.find(std::to_string(w)) != std::string::npos) win = w;
            if (sc == "sort_all") win = order.size();
            const int kk = sc.rfind("dirbin", 0) == 0 ? 1 : sc.rfind("origin", 0) == 0 ? 2 : 0;
            if (win)
                for (size_t a = 0; a < order.size(); a += win) {
                    const size_t b = std::min(order.size(), a + win);
                    std::stable_sort(order.begin() + a, order.begin() + b, [&](size_t x, size_t y) { return key(x, kk) < key(y, kk); });
                }
            Stats s;
            for (size_t a = 0; a < order.size(); a += 64) {
                std::vector<const Visit*> lanes;
                for (size_t j = a; j < std::min(order.size(), a + 64); ++j) lanes.push_back(&vis[order[j]]);
                wave(lanes, s);
            }
            auto& T = (kind & 1) ? tot_sh[sc] : tot_ext[sc];
            T.rays += s.rays; T.node_trips += s.node_trips; T.node_lanes += s.node_lanes; T.node_lines64 += s.node_lines64;
            T.node_lines128 += s.node_lines128; T.tri_trips += s.tri_trips; T.tri_lanes += s.tri_lanes; T.tri_lines += s.tri_lines;
            T.node_quad_cost += s.node_quad_cost;
            std::printf(", \"%s\": {\"node_lines_per_ray\": %.3f, \"node_lines_per_trip\": %.2f, \"tri_lines_per_ray\": %.3f}",
                        sc.c_str(), s.node_lines64 / s.rays, s.node_lines64 / std::max(1.0, s.node_trips), s.tri_lines / s.rays);
        }
        std::printf("}");
    }
    // regen: today's kernel with path regeneration — 64 lanes each run one pixel's path bounce after
    // bounce (its extension queries), a lane whose path ended takes the next pixel of the pixel-major
    // queue; each iteration's wave holds the lanes' current rays (different bounces, nearby pixels)
    {
        std::map<int, std::vector<size_t>> path;   // pixel -> extension rays by bounce
        std::vector<int> queue;
        for (size_t i = 0; i < rays.size(); ++i)
            if ((rays[i].kind & 1) == 0) {
                if ((rays[i].kind >> 3) == 0) queue.push_back(rays[i].pixel);
                path[rays[i].pixel].push_back(i);
            }
        // quad 1: a quad of lanes refills only when all four are idle, with four consecutive pixels;
        // quad 2: per-lane refills, then the wave's 64 rays permuted across its lanes by origin Morton
        // code before the traversal (an in-wave sort: bitonic over 64 keys + one ray permutation)
        for (int quad = 0; quad < 8; ++quad) {
            Stats s;
            size_t qn = 0;
            std::vector<int> lane_px(64, -1), lane_b(64, 0);
            while (true) {
                std::vector<const Visit*> lanes(64, nullptr);
                bool any = false;
                for (int j = 0; j < 64; ++j)
                    if (lane_px[j] >= 0 && lane_b[j] >= (int)path[lane_px[j]].size()) lane_px[j] = -1;
                for (int j = 0; j < 64; ++j) {
                    if (quad == 1) {
                        if ((j & 3) == 0 && lane_px[j] < 0 && lane_px[j + 1] < 0 && lane_px[j + 2] < 0 && lane_px[j + 3] < 0)
                            for (int t = 0; t < 4 && qn < queue.size(); ++t) { lane_px[j + t] = queue[qn++]; lane_b[j + t] = 0; }
                    } else if (lane_px[j] < 0 && qn < queue.size()) {
                        lane_px[j] = queue[qn++];
                        lane_b[j] = 0;
                    }
                    if (lane_px[j] >= 0) { lanes[(size_t)j] = &vis[path[lane_px[j]][(size_t)lane_b[j]++]]; any = true; }
                }
                if (!any) break;
                if (quad == 3) {   // compaction only: active lanes first, in lane order
                    std::stable_partition(lanes.begin(), lanes.end(), [](const Visit* v) { return v != nullptr; });
                }
                if (quad == 2 || quad >= 4) {
                    // quad 4..7: coarse keys, Morton code of a 2 / 4 / 8 / 256-cell grid per axis
                    const double n = quad == 4 ? 2.0 : quad == 5 ? 4.0 : quad == 6 ? 8.0 : quad == 7 ? 256.0 : 1024.0;
                    std::vector<std::pair<uint64_t, const Visit*>> kv;
                    for (int j = 0; j < 64; ++j)
                        kv.push_back({lanes[(size_t)j] ? cell(rays[(size_t)(lanes[(size_t)j] - vis.data())], n) : ~0ull, lanes[(size_t)j]});
                    std::stable_sort(kv.begin(), kv.end(), [](auto& a, auto& b) { return a.first < b.first; });
                    for (int j = 0; j < 64; ++j) lanes[(size_t)j] = kv[(size_t)j].second;
                }
                wave(lanes, s);
            }
            static const char* names[8] = {"regen", "quadregen", "regen_wavesort", "regen_compact", "wavesort_2",
                                           "wavesort_4", "wavesort_8", "wavesort_256"};
            tot_ext[names[quad]] = s;
        }
    }
    std::printf("}, \"totals\": {");
    bool fk = true;
    for (auto* T : {&tot_ext, &tot_sh}) {
        std::printf("%s\"%s\": {", fk ? "" : ", ", T == &tot_ext ? "extension" : "shadow");
        fk = false;
        bool fs = true;
        std::vector<std::string> all = scheds;
        if (T == &tot_ext)
            all.insert(all.begin(), {"regen", "quadregen", "regen_wavesort", "regen_compact", "wavesort_2", "wavesort_4",
                                     "wavesort_8", "wavesort_256"});
        for (const auto& sc : all) {
            const Stats& s = (*T)[sc];
            std::printf("%s\"%s\": {\"rays\": %.0f, \"node_visits_per_ray\": %.2f, \"node_trips_per_ray\": %.4f, "
                        "\"node_lanes\": %.3f, \"node_lines64_per_ray\": %.3f, \"node_lines128_per_ray\": %.3f, "
                        "\"node_lines64_per_trip\": %.2f, \"tri_tests_per_ray\": %.2f, \"tri_lines_per_ray\": %.3f, "
                        "\"tri_lines_per_trip\": %.2f, \"node_quad_cost_per_ray\": %.3f}",
                        fs ? "" : ", ", sc.c_str(), s.rays, s.node_lanes / s.rays, s.node_trips / s.rays,
                        s.node_lanes / (64.0 * s.node_trips), s.node_lines64 / s.rays, s.node_lines128 / s.rays,
                        s.node_lines64 / s.node_trips, s.tri_lanes / s.rays, s.tri_lines / s.rays,
                        s.tri_lines / std::max(1.0, s.tri_trips), s.node_quad_cost / s.rays);
            fs = false;
        }
        std::printf("}");
    }
    std::printf("}}\n");
    return 0;
}
