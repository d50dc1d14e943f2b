// lds_f16_model — what half-precision child planes in the LDS-resident BVH4 (configs 1, 2, 3, 5) would
// cost in extra node visits and triangle tests (round 6).
//
// The pooled kernel reads a node's octant copy from LDS as seven ds_read_b128 (six f32 plane vectors and
// the refs).  f16 planes, rounded outward (lo down, hi up) and consumed by v_fma_mix_f32 at no extra
// VALU, would make it four reads.  That pays only if the looser boxes add few visits.  This tool builds
// the library's tree for the scene soup (prt_bvh.cpp: build_bvh + collapse_bvh4), walks every ray of
// tools/c4_rays.py --scene cornell in the kernel's order (closest hit: nearest child first; shadow:
// first hit ends the query) through the f32 boxes and through the f16-rounded ones, and counts node
// visits and triangle tests per ray.
//
//   g++ -O2 -fopenmp -std=c++17 -I pyrenderer_amd/csrc tools/lds_f16_model.cpp pyrenderer_amd/csrc/prt_bvh.cpp \
//       -o build/lds_f16_model
//   python tools/c4_rays.py --scene cornell --x0 0 --y0 0 --w 512 --h 512 --out /tmp/cb_rays.f32
//   build/lds_f16_model /tmp/cb_rays_soup.f32 /tmp/cb_rays.f32
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "prt_internal.h"

namespace {

struct Ray { double o[3], d[3], tmax; int kind; };

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

// x rounded to an IEEE half, down (up = false) or up; beyond the half range: -inf / +inf
double half_round(double x, bool up) {
    if (!std::isfinite(x) || x == 0.0) return x;
    const double a = std::fabs(x);
    int e = (int)std::floor(std::log2(a));
    if (e < -14) e = -14;
    const double ulp = std::ldexp(1.0, e - 10);
    const double r = (up ? std::ceil(x / ulp) : std::floor(x / ulp)) * ulp;
    if (r > 65504.0) return up ? INFINITY : 65504.0;
    if (r < -65504.0) return up ? -65504.0 : -INFINITY;
    return r;
}

struct Box { double lo[3], hi[3]; };

struct Walker {
    const prt::Bvh4Host& b4;
    const std::vector<float>& tris;
    std::vector<Box> boxes;   // 4 per node
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
    void walk(const Ray& ray, long* nodes, long* ntris) const {
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
                    ++*ntris;
                    double t;
                    if (tri_hit(r, ray, 1e-5, best, &t)) {
                        best = t;
                        if (any) return;
                    }
                }
                continue;
            }
            ++*nodes;
            std::pair<double, int32_t> hit[4];
            int nh = 0;
            for (int k = 0; k < 4; ++k) {
                int32_t ref;
                std::memcpy(&ref, b4.nodes.data() + (size_t)cur * 32 + 24 + k, 4);
                if (ref == 0x7FFFFFFF) continue;
                const Box& b = boxes[(size_t)cur * 4 + k];
                double tn = 1e-5, tf = best;
                for (int a = 0; a < 3; ++a) {
                    double t0 = (b.lo[a] - ray.o[a]) * inv[a], t1 = (b.hi[a] - ray.o[a]) * inv[a];
                    if (t0 > t1) std::swap(t0, t1);
                    tn = std::max(tn, t0);
                    tf = std::min(tf, t1);
                }
                if (tn <= tf) hit[nh++] = {tn, ref};
            }
            std::sort(hit, hit + nh, [&](auto& a, auto& b) { return any ? a.first < b.first : a.first > b.first; });
            for (int k = 0; k < nh; ++k) stack.push_back(hit[k].second);
        }
    }
};

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
    std::vector<Ray> rays(rv.size() / 9);
    for (size_t i = 0; i < rays.size(); ++i) {
        const float* r = rv.data() + 9 * i;
        for (int a = 0; a < 3; ++a) { rays[i].o[a] = r[a]; rays[i].d[a] = r[3 + a]; }
        rays[i].tmax = r[6];
        rays[i].kind = (int)r[7];
    }
    std::printf("{\"triangles\": %zu, \"nodes4\": %lld, \"rays\": %zu, \"encodings\": [\n", tv.size() / 9,
                (long long)b4.n_nodes, rays.size());
    double base[4] = {0, 0, 0, 0};
    for (int enc = 0; enc < 2; ++enc) {
        Walker w{b4, b2.tris, {}};
        w.boxes.resize((size_t)b4.n_nodes * 4);
        for (int64_t n = 0; n < b4.n_nodes; ++n)
            for (int k = 0; k < 4; ++k) {
                Box& b = w.boxes[(size_t)n * 4 + k];
                const float* f = b4.nodes.data() + (size_t)n * 32;
                for (int a = 0; a < 3; ++a) {
                    b.lo[a] = f[(2 * a) * 4 + k];
                    b.hi[a] = f[(2 * a + 1) * 4 + k];
                    if (enc == 1) { b.lo[a] = half_round(b.lo[a], false); b.hi[a] = half_round(b.hi[a], true); }
                }
            }
        long n[2] = {0, 0}, t[2] = {0, 0}, c[2] = {0, 0};
#pragma omp parallel for schedule(dynamic, 1024) reduction(+ : n[:2], t[:2], c[:2])
        for (size_t i = 0; i < rays.size(); ++i) {
            const int s = rays[i].kind & 1;
            long a = 0, b = 0;
            w.walk(rays[i], &a, &b);
            n[s] += a; t[s] += b; c[s] += 1;
        }
        const double v[4] = {(double)n[0] / c[0], (double)t[0] / c[0], (double)n[1] / c[1], (double)t[1] / c[1]};
        if (enc == 0) std::copy(v, v + 4, base);
        std::printf("%s {\"planes\": \"%s\", \"ext_nodes\": %.4f, \"ext_tris\": %.4f, \"shadow_nodes\": %.4f, "
                    "\"shadow_tris\": %.4f, \"rel\": [%.4f, %.4f, %.4f, %.4f]}",
                    enc ? ",\n" : "", enc ? "f16, rounded outward" : "f32 (today)", v[0], v[1], v[2], v[3],
                    v[0] / base[0], v[1] / base[1], v[2] / base[2], v[3] / base[3]);
    }
    std::printf("\n]}\n");
    return 0;
}
