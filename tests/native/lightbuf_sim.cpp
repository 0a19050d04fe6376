// lightbuf_sim.cpp — CPU check that the shadow-ray light buffers
// (raingun_amd/csrc/rg_lightbuf.cpp) never leave out a sphere the exact
// reference test would accept: for every shadow ray, the any-hit answer from
// the ray's cell list (cell lookup: the kernel's own rg_lightbuf_ray.h) must
// equal the brute-force scan over all spheres.  Built and run by
// tests/test_lightbuf_cpu.py.
//
// usage: lightbuf_sim [rays_per_kind] < scene.txt
//   scene.txt: n, n lines "cx cy cz r", then m, m lines "kind x y z"
//   (kind 0 = directional with direction xyz, 1 = spherical at position xyz)
// Prints one JSON line; exit 1 on any mismatch.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <vector>

#include "../../raingun_amd/csrc/rg_bvh.h"
#include "../../include/raingun.h"
#include "../../raingun_amd/csrc/rg_lightbuf.h"

// bodies.rs:92-119 (f64, unfused; compiled with -ffp-contract=off)
static bool sphere_exact(const double *s, const double o[3], const double d[3], double &t) {
    const double hx = s[0] - o[0], hy = s[1] - o[1], hz = s[2] - o[2];
    const double adj = (hx * d[0] + hy * d[1]) + hz * d[2];
    const double opp = ((hx * hx + hy * hy) + hz * hz) - adj * adj;
    const double r2 = s[3] * s[3];
    if (opp > r2) return false;
    const double th = std::sqrt(r2 - opp);
    const double d0 = adj - th, d1 = adj + th;
    if (d0 < 0.0 && d1 < 0.0) return false;
    t = d0 < 0.0 ? d1 : (d1 < 0.0 ? d0 : std::fmin(d0, d1));
    return true;
}

static uint64_t rng_state = 0x5EEDULL;
static double urand() {  // SplitMix64 -> [0, 1)
    uint64_t z = (rng_state += 0x9E3779B97F4A7C15ULL);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    z ^= z >> 31;
    return (double)(z >> 11) * (1.0 / 9007199254740992.0);
}
static void unit(double v[3]) {
    const double inv = 1.0 / std::sqrt((v[0] * v[0] + v[1] * v[1]) + v[2] * v[2]);
    v[0] *= inv; v[1] *= inv; v[2] *= inv;
}
static void rand_dir(double v[3]) {
    do { for (int k = 0; k < 3; ++k) v[k] = 2.0 * urand() - 1.0; } while ((v[0] * v[0] + v[1] * v[1]) + v[2] * v[2] < 1e-6);
    unit(v);
}
static void cross(const double a[3], const double b[3], double c[3]) {
    c[0] = a[1] * b[2] - a[2] * b[1];
    c[1] = a[2] * b[0] - a[0] * b[2];
    c[2] = a[0] * b[1] - a[1] * b[0];
}

struct Light {
    int kind;            // RG_LIGHT_DIRECTIONAL / RG_LIGHT_SPHERICAL
    double v[3];         // direction / position
    double dn[3];        // normalize(-direction), as rg_capi.hip computes it
    RgLightBufBuild lb;
    bool has = false;
};

static std::vector<double> sp;  // BVH order, 4 per sphere
static int n_sph = 0;
static long g_rays = 0, g_occl = 0, g_mismatch = 0, g_skip = 0, g_empty = 0, g_tests = 0, g_near = 0;

// shadow ray towards light l from o: direction and distance as the kernel's light_dir_dist
static void shadow_ray(const Light &l, const double o[3], double d[3], double &ld) {
    if (l.kind == RG_LIGHT_DIRECTIONAL) {
        d[0] = l.dn[0]; d[1] = l.dn[1]; d[2] = l.dn[2];
        ld = HUGE_VAL;
        return;
    }
    const double v[3] = {l.v[0] - o[0], l.v[1] - o[1], l.v[2] - o[2]};
    const double m = std::sqrt((v[0] * v[0] + v[1] * v[1]) + v[2] * v[2]);
    const double inv = 1.0 / m;
    d[0] = v[0] * inv; d[1] = v[1] * inv; d[2] = v[2] * inv;
    ld = m;
}

static void check(const Light &l, const double o[3], float obound) {
    double d[3], ld;
    shadow_ray(l, o, d, ld);
    bool brute = false;
    double tmin = HUGE_VAL;
    for (int i = 0; i < n_sph; ++i) {
        double t;
        if (sphere_exact(&sp[4 * i], o, d, t) && !(t > ld)) { brute = true; tmin = std::min(tmin, t); }
    }
    ++g_rays;
    g_occl += brute;
    const int cell = rg_lb_cell(l.lb.dev, l.v[0], l.v[1], l.v[2], o[0], o[1], o[2], obound);
    if (cell == RG_LB_SKIP) { ++g_skip; return; }
    bool lbv = false;
    auto test = [&](uint32_t j) {
        double t;
        ++g_tests;
        if (sphere_exact(&sp[4 * j], o, d, t) && !(t > ld)) lbv = true;
    };
    for (uint32_t k = l.lb.dev.always0; k < l.lb.dev.always1; ++k) test(l.lb.ent[k]);
    if (cell == RG_LB_EMPTY) ++g_empty;
    else
        for (uint32_t k = l.lb.start[cell]; k < l.lb.start[cell + 1]; ++k) test(l.lb.ent[k]);
    if (lbv != brute) {
        if (g_mismatch < 5)
            std::fprintf(stderr, "mismatch: light kind %d o=(%.17g %.17g %.17g) brute %d lb %d cell %d\n", l.kind, o[0],
                         o[1], o[2], (int)brute, (int)lbv, cell);
        ++g_mismatch;
    }
}

// camera buffer (a spherical buffer at the origin): a primary ray from the origin along d; the
// closest hit over the direction's list must equal the brute-force closest hit (t bits, index)
static long g_cam_rays = 0, g_cam_hits = 0, g_cam_mismatch = 0, g_cam_tests = 0;
static void check_primary(const RgLightBufBuild &cam, const double d[3], float obound) {
    const double o[3] = {0.0, 0.0, 0.0};
    double bt = 0.0, lt = 0.0;
    int bi = -1, li = -1;
    auto add = [](double &ct, int &ci, double t, int i) {
        if (ci < 0 || t < ct || (t == ct && i < ci)) { ct = t; ci = i; }
    };
    for (int i = 0; i < n_sph; ++i) {
        double t;
        if (sphere_exact(&sp[4 * i], o, d, t)) add(bt, bi, t, i);
    }
    ++g_cam_rays;
    g_cam_hits += bi >= 0;
    const int cell = rg_lb_cell(cam.dev, 0.0, 0.0, 0.0, d[0], d[1], d[2], obound);
    if (cell == RG_LB_SKIP) { ++g_skip; return; }
    auto test = [&](uint32_t j) {
        double t;
        ++g_cam_tests;
        if (sphere_exact(&sp[4 * j], o, d, t)) add(lt, li, t, (int)j);
    };
    for (uint32_t k = cam.dev.always0; k < cam.dev.always1; ++k) test(cam.ent[k]);
    if (cell >= 0)
        for (uint32_t k = cam.start[cell]; k < cam.start[cell + 1]; ++k) test(cam.ent[k]);
    if (li != bi || (bi >= 0 && std::memcmp(&lt, &bt, sizeof bt) != 0)) {
        if (g_cam_mismatch < 5)
            std::fprintf(stderr, "camera mismatch: d=(%.17g %.17g %.17g) brute %d lb %d\n", d[0], d[1], d[2], bi, li);
        ++g_cam_mismatch;
    }
}

int main(int argc, char **argv) {
    const int R = argc > 1 ? std::atoi(argv[1]) : 4000;
    int n;
    if (std::scanf("%d", &n) != 1 || n < 2) return 2;
    std::vector<double> raw(4 * (size_t)n);
    for (int i = 0; i < 4 * n; ++i)
        if (std::scanf("%lf", &raw[i]) != 1) return 2;
    int m;
    if (std::scanf("%d", &m) != 1) return 2;
    std::vector<Light> lights(m);
    for (auto &l : lights) {
        int k;
        if (std::scanf("%d %lf %lf %lf", &k, &l.v[0], &l.v[1], &l.v[2]) != 4) return 2;
        l.kind = k == 0 ? RG_LIGHT_DIRECTIONAL : RG_LIGHT_SPHERICAL;
        const double nx = -l.v[0], ny = -l.v[1], nz = -l.v[2];
        const double inv = 1.0 / std::sqrt((nx * nx + ny * ny) + nz * nz);
        l.dn[0] = nx * inv; l.dn[1] = ny * inv; l.dn[2] = nz * inv;
    }
    RgBvhBuild bvh;
    if (!rg_build_bvh(raw.data(), n, bvh)) return 2;
    sp.resize(raw.size());
    for (int j = 0; j < n; ++j) std::memcpy(&sp[4 * j], &raw[4 * (size_t)bvh.order[j]], 4 * sizeof(double));
    n_sph = n;
    const float O = bvh.obound;
    double mean_c = 0.0;
    uint32_t max_c = 0;
    int built = 0;
    for (auto &l : lights) {
        l.has = rg_build_lightbuf(sp.data(), n, l.kind, l.dn, l.v, bvh.extent, (double)O, l.lb);
        if (l.has) {
            ++built;
            mean_c = std::max(mean_c, l.lb.mean_candidates);
            max_c = std::max(max_c, l.lb.max_candidates);
        }
    }
    double lo[3] = {HUGE_VAL, HUGE_VAL, HUGE_VAL}, hi[3] = {-HUGE_VAL, -HUGE_VAL, -HUGE_VAL};
    for (int i = 0; i < n; ++i)
        for (int k = 0; k < 3; ++k) {
            lo[k] = std::min(lo[k], sp[4 * i + k] - std::fabs(sp[4 * i + 3]));
            hi[k] = std::max(hi[k], sp[4 * i + k] + std::fabs(sp[4 * i + 3]));
        }
    for (const auto &l : lights) {
        if (!l.has) continue;
        for (int r = 0; r < R; ++r) {
            double o[3];
            // 1. points on sphere surfaces, pushed out along the normal by the shadow bias (rendering.rs:148)
            {
                const double *s = &sp[4 * (int)(urand() * n)];
                double nrm[3];
                rand_dir(nrm);
                for (int k = 0; k < 3; ++k) o[k] = (s[k] + nrm[k] * std::fabs(s[3])) + nrm[k] * 1e-13;
                check(l, o, O);
            }
            // 2. points in the scene's box, and in a box 3x its size
            for (int k = 0; k < 3; ++k) o[k] = lo[k] + (hi[k] - lo[k]) * urand();
            check(l, o, O);
            for (int k = 0; k < 3; ++k) o[k] = lo[k] - (hi[k] - lo[k]) + 3.0 * (hi[k] - lo[k]) * urand();
            check(l, o, O);
            // 3. grazing: the shadow ray passes at r (1 +- eps) from a sphere's centre
            {
                const double *s = &sp[4 * (int)(urand() * n)];
                const double rr = std::fabs(s[3]) * (1.0 + (urand() < 0.5 ? -1.0 : 1.0) * (urand() < 0.5 ? 1e-9 : 1e-13));
                if (l.kind == RG_LIGHT_DIRECTIONAL) {
                    double u[3], w[3];
                    rand_dir(w);
                    cross(l.dn, w, u);
                    unit(u);
                    const double back = std::fabs(s[3]) + 50.0 * urand();  // the sphere ahead of o along dn
                    for (int k = 0; k < 3; ++k) o[k] = s[k] + rr * u[k] - back * l.dn[k];
                } else {
                    double c_l[3] = {s[0] - l.v[0], s[1] - l.v[1], s[2] - l.v[2]};
                    const double D = std::sqrt(c_l[0] * c_l[0] + c_l[1] * c_l[1] + c_l[2] * c_l[2]);
                    if (!(D > rr * 1.01)) continue;
                    unit(c_l);
                    double w[3], u[3];
                    rand_dir(w);
                    cross(c_l, w, u);
                    unit(u);
                    const double th = std::asin(rr / D);  // a ray from L tangent to the (r(1 +- eps)) sphere
                    double dir[3];
                    for (int k = 0; k < 3; ++k) dir[k] = std::cos(th) * c_l[k] + std::sin(th) * u[k];
                    const double reach = D * std::cos(th) * (1.0 + 2.0 * urand()) + std::fabs(s[3]);
                    for (int k = 0; k < 3; ++k) o[k] = l.v[k] + reach * dir[k];
                }
                ++g_near;
                check(l, o, O);
            }
        }
    }
    // the camera buffer: frustum directions (normalize(sx, sy, -1), ray.rs:46-53), random directions,
    // and directions grazing a sphere at r (1 +- eps) as seen from the origin
    RgLightBufBuild cam;
    const double zero[3] = {0.0, 0.0, 0.0};
    const bool cam_built = rg_build_lightbuf(sp.data(), n, RG_LIGHT_SPHERICAL, zero, zero, bvh.extent, (double)O, cam);
    if (cam_built) {
        for (int r = 0; r < 4 * R; ++r) {
            double d[3] = {(2.0 * urand() - 1.0) * 1.7778, 2.0 * urand() - 1.0, -1.0};
            unit(d);
            check_primary(cam, d, O);
            rand_dir(d);
            check_primary(cam, d, O);
            const double *s = &sp[4 * (int)(urand() * n)];
            double c[3] = {s[0], s[1], s[2]};
            const double D = std::sqrt(c[0] * c[0] + c[1] * c[1] + c[2] * c[2]);
            const double rr = std::fabs(s[3]) * (1.0 + (urand() < 0.5 ? -1.0 : 1.0) * (urand() < 0.5 ? 1e-9 : 1e-13));
            if (D > rr * 1.01) {
                unit(c);
                double w[3], u[3];
                rand_dir(w);
                cross(c, w, u);
                unit(u);
                const double th = std::asin(rr / D);
                for (int k = 0; k < 3; ++k) d[k] = std::cos(th) * c[k] + std::sin(th) * u[k];
                unit(d);
                ++g_near;
                check_primary(cam, d, O);
            }
        }
    }
    std::printf("{\"camera_built\": %d, \"camera_rays\": %ld, \"camera_hits\": %ld, \"camera_mismatches\": %ld, "
                "\"camera_tests_per_ray\": %.3f, ", (int)cam_built, g_cam_rays, g_cam_hits, g_cam_mismatch,
                g_cam_rays ? (double)g_cam_tests / g_cam_rays : 0.0);
    std::printf("\"rays\": %ld, \"occluded\": %ld, \"mismatches\": %ld, \"skipped\": %ld, \"empty_cells\": %ld, "
                "\"grazing\": %ld, \"tests_per_ray\": %.3f, \"lights_built\": %d, \"mean_candidates_max\": %.3f, "
                "\"max_candidates\": %u, \"brute_tests_per_ray\": %d}\n",
                g_rays, g_occl, g_mismatch, g_skip, g_empty, g_near, g_rays ? (double)g_tests / g_rays : 0.0, built,
                mean_c, max_c, n);
    return (g_mismatch || g_cam_mismatch) ? 1 : 0;
}
