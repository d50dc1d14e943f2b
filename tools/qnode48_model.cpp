// qnode48_model — what a 48-B quantised BVH4 node would cost config 4 in extra node visits and
// triangle tests, before any kernel work (round 6).
//
// Measured (profiles/r06/micro/l1_width_*.json, profiles/r06/knobs/extra_node_load/): at config 4 one
// more 16-B load instruction per node visit costs +11.9 % kernel time, and on L1/L2-resident data a
// wave's load costs per instruction, not per byte.  A node of three dwordx4 loads instead of four
// therefore pays if the coarser encoding it needs does not add more visits than that saves.  The
// 64-B node holds origin (3 f32), steps (3 f32), 24 B of 8-bit child planes and 4 child refs; a 48-B
// node keeps the planes and the origin and has 96 bits for the steps and the refs: refs as two
// 25-bit bases (inner children, leaf triangles) plus 20 bits of per-slot leaf ends leave 26-30 bits
// for the steps, i.e. steps rounded up to 8 exponent + m mantissa bits, and possibly origins rounded
// down to k fewer mantissa bits.  This tool builds the library's config-4 tree (prt_bvh.cpp),
// re-quantises it per candidate encoding and walks every ray of tools/c4_rays.py in the kernel's
// visiting order, counting node visits and triangle tests per ray.
//
//   g++ -O2 -fopenmp -std=c++17 -I pyrenderer_amd/csrc tools/qnode48_model.cpp pyrenderer_amd/csrc/prt_bvh.cpp \
//       -o build/qnode48_model
//   build/qnode48_model /tmp/c4_rays_soup.f32 /tmp/c4_rays.f32 > profiles/r06/qnode48/model.json
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
uint32_t ubits(float f) { uint32_t v; std::memcpy(&v, &f, 4); return v; }
float fbits(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }

// f32 at or above x (> 0) with only `m` mantissa bits
float round_up_mant(float x, int m) {
    if (m >= 23) return x;
    const uint32_t low = (1u << (23 - m)) - 1u;
    uint32_t u = ubits(x);
    if (u & low) u = (u | low) + 1u;
    return fbits(u);
}
// f32 at or below x with its low k mantissa bits zero
float round_down_low(float x, int k) {
    if (k == 0) return x;
    const uint32_t low = (1u << k) - 1u;
    uint32_t u = ubits(x);
    if (!(u & low)) return x;
    if (x >= 0.0f) return fbits(u & ~low);          // smaller magnitude = below
    return fbits((u | low) + 1u);                    // larger magnitude = below
}

struct Enc { const char* name; int step_mant; int origin_drop; bool fit = false; };

struct QNode { float origin[3], step[3]; uint8_t lo[3][4], hi[3][4]; int32_t ref[4]; };

// prt_bvh.cpp quantize_bvh4 with the step / origin rounding of `e`
std::vector<QNode> quantize(const prt::Bvh4Host& b4, float pad, const Enc& e) {
    std::vector<QNode> out((size_t)b4.n_nodes);
    const double margin = 2.0 * (double)pad;
    for (int64_t n = 0; n < b4.n_nodes; ++n) {
        const float* f = b4.nodes.data() + (size_t)n * 32;
        QNode& q = out[(size_t)n];
        int32_t refs[4];
        std::memcpy(refs, f + 24, 16);
        bool ok[4];
        for (int k = 0; k < 4; ++k) ok[k] = std::isfinite(f[k]);
        for (int a = 0; a < 3; ++a) {
            double lo = INFINITY, hi = -INFINITY;
            for (int k = 0; k < 4; ++k)
                if (ok[k]) { lo = std::min(lo, (double)f[(2 * a) * 4 + k]); hi = std::max(hi, (double)f[(2 * a + 1) * 4 + k]); }
            if (!(lo <= hi)) { lo = 0.0; hi = 0.0; }
            // grid: origin at or below lo - margin, step covering the range in <= 254 (fit: 255) steps
            auto grid = [&](double div, double shift, float* po, float* pst) {
                float o = (float)(lo - margin);
                if ((double)o > lo - margin) o = std::nextafter(o, -INFINITY);
                o = round_down_low(o, e.origin_drop);
                const double ext0 = hi + margin - (double)o;
                float stf = (float)std::max(ext0 / div, 1e-30);
                if ((double)stf < ext0 / div) stf = std::nextafter(stf, INFINITY);
                stf = round_up_mant(stf, e.step_mant);
                if (shift > 0.0) {
                    float o2 = (float)((double)o - shift * (double)stf);
                    if ((double)o2 > (double)o - shift * (double)stf) o2 = std::nextafter(o2, -INFINITY);
                    o = round_down_low(o2, e.origin_drop);
                }
                *po = o;
                *pst = stf;
                return (hi + margin - (double)o) / (double)stf <= 255.0;
            };
            // the children's total quantised extent along this axis for a grid
            auto cost = [&](float o, float stf) {
                double c = 0.0;
                for (int k = 0; k < 4; ++k) {
                    if (!ok[k]) continue;
                    const double l = f[(2 * a) * 4 + k], h = f[(2 * a + 1) * 4 + k];
                    long ql = (long)std::floor((l - margin - (double)o) / stf), qh = (long)std::ceil((h + margin - (double)o) / stf);
                    c += (double)(std::min(255L, qh) - std::max(0L, ql)) * (double)stf;
                }
                return c;
            };
            float o, stf;
            grid(254.0, 0.0, &o, &stf);
            if (e.fit) {
                // every grid of N <= 254 steps over the range (the reduced-precision step rounded up from
                // range / N): the node's own far plane lands just below a grid line for some N
                double best = cost(o, stf);
                for (int div = 254; div >= 128; --div) {
                    float o2, st2;
                    if (!grid((double)div, 0.0, &o2, &st2)) continue;
                    const double c = cost(o2, st2);
                    if (c < best) { best = c; o = o2; stf = st2; }
                }
            }
            const double st = stf;
            q.origin[a] = o;
            q.step[a] = stf;
            for (int k = 0; k < 4; ++k) {
                q.lo[a][k] = 255; q.hi[a][k] = 0;
                if (!ok[k]) continue;
                const double l = f[(2 * a) * 4 + k], h = f[(2 * a + 1) * 4 + k];
                long ql = (long)std::floor((l - margin - (double)o) / st), qh = (long)std::ceil((h + margin - (double)o) / st);
                q.lo[a][k] = (uint8_t)std::max(0L, std::min(255L, ql));
                q.hi[a][k] = (uint8_t)std::max(0L, std::min(255L, qh));
            }
        }
        for (int k = 0; k < 4; ++k) q.ref[k] = ok[k] ? refs[k] : 0x7FFFFFFF;
    }
    return out;
}

struct Walker {
    const std::vector<QNode>& q;
    const std::vector<float>& tris;
    bool tri_hit(int64_t r, const Ray& ray, double tmin, double tmax, double* t) const {
        const float* p = tris.data() + 12 * r;
        const double v0[3] = {p[0], p[1], p[2]}, e1[3] = {p[4], p[5], p[6]}, e2[3] = {p[8], p[9], p[10]};
        const double* d = ray.d;
        const double c[3] = {e1[1] * d[2] - e1[2] * d[1], e1[2] * d[0] - e1[0] * d[2], e1[0] * d[1] - e1[1] * d[0]};
        const double det = c[0] * e2[0] + c[1] * e2[1] + c[2] * e2[2];
        if (det == 0.0) return false;
        const double f = 1.0 / det;
        const double s[3] = {ray.o[0] - v0[0], ray.o[1] - v0[1], ray.o[2] - v0[2]};
        const double qq[3] = {s[1] * e2[2] - s[2] * e2[1], s[2] * e2[0] - s[0] * e2[2], s[0] * e2[1] - s[1] * e2[0]};
        const double tt = -f * (qq[0] * e1[0] + qq[1] * e1[1] + qq[2] * e1[2]);
        const double u = -f * (qq[0] * d[0] + qq[1] * d[1] + qq[2] * d[2]);
        const double v = f * (c[0] * s[0] + c[1] * s[1] + c[2] * s[2]);
        if (!(tmin < tt && tt < tmax && u >= 0 && u <= 1 && v >= 0 && 1 - u - v >= 0)) return false;
        *t = tt;
        return true;
    }
    // node visits and triangle tests of one query in the kernel's order (coherence_c4.cpp's walk)
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
            const QNode& nd = q[(size_t)cur];
            std::pair<double, int32_t> hit[4];
            int nh = 0;
            for (int k = 0; k < 4; ++k) {
                if (nd.ref[k] == 0x7FFFFFFF) continue;
                double tn = 1e-5, tf = best;
                for (int a = 0; a < 3; ++a) {
                    const double lo = nd.origin[a] + nd.lo[a][k] * (double)nd.step[a];
                    const double hi = nd.origin[a] + nd.hi[a][k] * (double)nd.step[a];
                    double t0 = (lo - ray.o[a]) * inv[a], t1 = (hi - ray.o[a]) * inv[a];
                    if (t0 > t1) std::swap(t0, t1);
                    tn = std::max(tn, t0);
                    tf = std::min(tf, t1);
                }
                if (tn <= tf) hit[nh++] = {tn, nd.ref[k]};
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
    const Enc encs[] = {{"f32 steps (today)", 23, 0}, {"f32 steps, best-fit grid", 23, 0, true},
                        {"8e+2m steps, best-fit grid", 2, 0, true}, {"8e+3m steps, best-fit grid", 3, 0, true},
                        {"8e+5m steps, best-fit grid", 5, 0, true}, {"8e+2m steps, origin -4 bits, best-fit grid", 2, 4, true},
                        {"8e+20m steps", 20, 0}, {"8e+12m steps", 12, 0},
                        {"8e+7m steps", 7, 0}, {"8e+5m steps", 5, 0}, {"8e+3m steps", 3, 0}, {"8e+2m steps", 2, 0},
                        {"8e+1m steps", 1, 0}, {"power-of-two steps", 0, 0}, {"8e+2m steps, origin -4 bits", 2, 4},
                        {"8e+2m steps, origin -8 bits", 2, 8}};
    std::printf("{\"nodes4\": %lld, \"rays\": %zu, \"encodings\": [\n", (long long)b4.n_nodes, rays.size());
    double base_n[2] = {0, 0}, base_t[2] = {0, 0};
    bool first = true;
    for (const Enc& e : encs) {
        const std::vector<QNode> q = quantize(b4, b2.pad, e);
        Walker w{q, b2.tris};
        long n[2] = {0, 0}, t[2] = {0, 0}, c[2] = {0, 0};
#pragma omp parallel for schedule(dynamic, 256) reduction(+ : n[:2], t[:2], c[:2])
        for (size_t i = 0; i < rays.size(); ++i) {
            const int s = rays[i].kind & 1;
            long a = 0, b = 0;
            w.walk(rays[i], &a, &b);
            n[s] += a; t[s] += b; c[s] += 1;
        }
        double nv[2], tt[2];
        for (int s = 0; s < 2; ++s) { nv[s] = (double)n[s] / (double)c[s]; tt[s] = (double)t[s] / (double)c[s]; }
        if (first) for (int s = 0; s < 2; ++s) { base_n[s] = nv[s]; base_t[s] = tt[s]; }
        std::printf("%s {\"encoding\": \"%s\", \"ext_nodes\": %.4f, \"ext_tris\": %.4f, \"shadow_nodes\": %.4f, "
                    "\"shadow_tris\": %.4f, \"ext_nodes_rel\": %.4f, \"ext_tris_rel\": %.4f, \"shadow_nodes_rel\": %.4f, "
                    "\"shadow_tris_rel\": %.4f}",
                    first ? "" : ",\n", e.name, nv[0], tt[0], nv[1], tt[1], nv[0] / base_n[0], tt[0] / base_t[0],
                    nv[1] / base_n[1], tt[1] / base_t[1]);
        std::fflush(stdout);
        first = false;
    }
    std::printf("\n]}\n");
    return 0;
}
