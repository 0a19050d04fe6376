// bvh_sim.cpp — CPU check that the sphere BVH (raingun_amd/csrc/rg_bvh.cpp)
// never culls a sphere the exact reference test would accept: every ray's
// closest hit (t, YAML index) and any-hit shadow answer via BVH traversal must
// equal the brute-force scan.  The traversal uses the kernel's own slab test
// (rg_bvh_ray.h).  Built and run by tests/test_bvh_cpu.py.
//
// usage: bvh_sim [n_rays_per_kind] < spheres.txt   (n, then n lines "cx cy cz r")
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <vector>

#include "../../raingun_amd/csrc/rg_bvh.h"
#include "../../raingun_amd/csrc/rg_bvh_ray.h"

struct Hit { double t; int id; };

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
static void add(Hit &h, double t, int id) {
    if (h.id < 0 || t < h.t || (t == h.t && id < h.id)) { h.t = t; h.id = id; }
}

struct Scene {
    std::vector<double> sp;      // input order, 4 per sphere
    RgBvhBuild bvh;
    std::vector<double> sp_bvh;  // BVH order
};

static Hit brute(const Scene &S, const double o[3], const double d[3]) {
    Hit h{0.0, -1};
    const int n = (int)S.sp.size() / 4;
    for (int i = 0; i < n; ++i) {
        double t;
        if (sphere_exact(&S.sp[4 * i], o, d, t)) add(h, t, i);
    }
    return h;
}
static bool brute_any(const Scene &S, const double o[3], const double d[3], double ld) {
    const int n = (int)S.sp.size() / 4;
    for (int i = 0; i < n; ++i) {
        double t;
        if (sphere_exact(&S.sp[4 * i], o, d, t) && !(t > ld)) return true;
    }
    return false;
}

static long g_tests = 0, g_nodes = 0;

// shadow: ld >= 0 -> any-hit within ld; ld < 0 -> closest hit
static float bound(double v) { return v <= 0.0 ? 0.0f : rg_f32_up(v); }

static Hit bvh_trace(const Scene &S, const double o[3], const double d[3], double ld, double t0s, bool &any,
                     float grow = 0.0f) {
    const double ob[3] = {o[0] + d[0] * t0s, o[1] + d[1] * t0s, o[2] + d[2] * t0s};
    const RayB rb = t0s > 0.0 ? rg_make_rayb(ob[0], ob[1], ob[2], d[0], d[1], d[2])
                              : rg_make_rayb(o[0], o[1], o[2], d[0], d[1], d[2]);
    Hit h{0.0, -1};
    any = false;
    const bool shadow = ld >= 0.0;
    int stack[64], sp = 0, node = 0;
    for (;;) {
        const RgBvhNode &N = S.bvh.nodes[node];
        ++g_nodes;
        const float tb = shadow ? bound(ld - t0s) : (h.id >= 0 ? bound(h.t - t0s) : HUGE_VALF);
        int kids[4], nk = 0;
        float keys[4];
        for (int k = 0; k < N.nchild; ++k) {
            float tn;
            if (grow > 0.0f ? !rg_child_hit<true>(N, k, rb, tb, tn, grow) : !rg_child_hit(N, k, rb, tb, tn)) continue;
            if (N.child[k] < 0) {
                const int v = ~N.child[k], first = v >> 3, count = (v & 7) + 1;
                for (int j = first; j < first + count; ++j) {
                    double t;
                    ++g_tests;
                    if (sphere_exact(&S.sp_bvh[4 * j], o, d, t)) {
                        if (shadow) { if (!(t > ld)) { any = true; return h; } }
                        else add(h, t, (int)S.bvh.order[j]);
                    }
                }
            } else {
                kids[nk] = N.child[k];
                keys[nk++] = tn;
            }
        }
        if (nk == 0) {
            if (sp == 0) break;
            node = stack[--sp];
            continue;
        }
        for (int i = 1; i < nk; ++i)  // ascending entry distance
            for (int j = i; j > 0 && keys[j] < keys[j - 1]; --j) {
                std::swap(keys[j], keys[j - 1]);
                std::swap(kids[j], kids[j - 1]);
            }
        for (int i = nk - 1; i >= 1; --i) {
            if (sp >= 64) { std::fprintf(stderr, "stack overflow\n"); std::exit(3); }
            stack[sp++] = kids[i];
        }
        node = kids[0];
    }
    return h;
}

// per-lane nearest-first walk with a bounded stack, as bvh_lane in the kernel:
// entries = f32 bits of the entry distance with the low RG_LANE_NODE_BITS
// cleared | node; a popped entry is skipped when its (lower-bound) distance
// exceeds the current bound.  Stack overflow is a failure (the host sizes the
// stack to lane_stack_need, so it must never happen).
static long g_lane_steps = 0;
static int g_lane_max_sp = 0;
static uint32_t lane_key(float tn, int node) {
    uint32_t b;
    std::memcpy(&b, &tn, 4);
    return (b & ~((1u << RG_LANE_NODE_BITS) - 1u)) | (uint32_t)node;
}
static float lane_key_t(uint32_t e) {
    const uint32_t b = e & ~((1u << RG_LANE_NODE_BITS) - 1u);
    float f;
    std::memcpy(&f, &b, 4);
    return f;
}
static Hit lane_trace(const Scene &S, const double o[3], const double d[3], double ld, double t0s, bool &any) {
    const double ob[3] = {o[0] + d[0] * t0s, o[1] + d[1] * t0s, o[2] + d[2] * t0s};
    const RayB rb = t0s > 0.0 ? rg_make_rayb(ob[0], ob[1], ob[2], d[0], d[1], d[2])
                              : rg_make_rayb(o[0], o[1], o[2], d[0], d[1], d[2]);
    Hit h{0.0, -1};
    any = false;
    const bool shadow = ld >= 0.0;
    const int cap = S.bvh.lane_stack;
    uint32_t stack[RG_LANE_STACK_MAX];
    int sp = 0, node = 0;
    const uint32_t mask = (1u << RG_LANE_NODE_BITS) - 1u;
    while (node >= 0) {
        ++g_lane_steps;
        const RgBvhNode &N = S.bvh.nodes[node];
        const float tb = shadow ? bound(ld - t0s) : (h.id >= 0 ? bound(h.t - t0s) : HUGE_VALF);
        uint32_t e[4] = {~0u, ~0u, ~0u, ~0u};
        for (int k = 0; k < N.nchild; ++k) {
            float tn;
            if (!rg_child_hit(N, k, rb, tb, tn)) continue;
            if (N.child[k] < 0) {
                const int v = ~N.child[k], first = v >> 3, count = (v & 7) + 1;
                for (int j = first; j < first + count; ++j) {
                    double t;
                    if (sphere_exact(&S.sp_bvh[4 * j], o, d, t)) {
                        if (shadow) { if (!(t > ld)) { any = true; return h; } }
                        else add(h, t, (int)S.bvh.order[j]);
                    }
                }
            } else {
                e[k] = lane_key(tn, N.child[k]);
            }
        }
        std::sort(e, e + 4);
        for (int i = 3; i >= 1; --i) {
            if (e[i] == ~0u) continue;
            if (sp >= cap) { std::fprintf(stderr, "lane stack overflow (cap %d)\n", cap); std::exit(3); }
            stack[sp++] = e[i];
            g_lane_max_sp = std::max(g_lane_max_sp, sp);
        }
        const float tbn = shadow ? bound(ld - t0s) : (h.id >= 0 ? bound(h.t - t0s) : HUGE_VALF);
        if (e[0] != ~0u && (shadow || !(lane_key_t(e[0]) > tbn))) { node = (int)(e[0] & mask); continue; }
        node = -1;
        while (sp > 0) {
            const uint32_t x = stack[--sp];
            if (shadow || !(lane_key_t(x) > tbn)) { node = (int)(x & mask); break; }
        }
    }
    return h;
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

int main(int argc, char **argv) {
    const long per_kind = argc > 1 ? std::atol(argv[1]) : 20000;
    int n = 0;
    if (std::scanf("%d", &n) != 1 || n < 2) { std::fprintf(stderr, "bad input\n"); return 2; }
    Scene S;
    S.sp.resize(4 * (size_t)n);
    for (int i = 0; i < 4 * n; ++i)
        if (std::scanf("%lf", &S.sp[i]) != 1) { std::fprintf(stderr, "bad sphere\n"); return 2; }
    if (!rg_build_bvh(S.sp.data(), n, S.bvh)) { std::fprintf(stderr, "build failed\n"); return 2; }
    S.sp_bvh.resize(S.sp.size());
    for (int j = 0; j < n; ++j) std::memcpy(&S.sp_bvh[4 * j], &S.sp[4 * S.bvh.order[j]], 32);
    // structural checks: every sphere in exactly one leaf, leaf boxes contain it
    if (!std::getenv("BVH_SIM_SKIP_STRUCT")) {
    std::vector<int> seen(n, 0);
    for (const RgBvhNode &N : S.bvh.nodes)
        for (int k = 0; k < N.nchild; ++k)
            if (N.child[k] < 0) {
                const int v = ~N.child[k], first = v >> 3, count = (v & 7) + 1;
                for (int j = first; j < first + count; ++j) {
                    ++seen[j];
                    const double *s = &S.sp_bvh[4 * j];
                    const double r = std::fabs(s[3]);
                    if (!(N.lox[k] <= s[0] - r && N.hix[k] >= s[0] + r && N.loy[k] <= s[1] - r && N.hiy[k] >= s[1] + r &&
                          N.loz[k] <= s[2] - r && N.hiz[k] >= s[2] + r)) { std::fprintf(stderr, "leaf box\n"); return 1; }
                }
            }
    for (int j = 0; j < n; ++j) if (seen[j] != 1) { std::fprintf(stderr, "leaf cover\n"); return 1; }
    if (S.bvh.nodes.size() > (1u << RG_LANE_NODE_BITS) || S.bvh.lane_stack > RG_LANE_STACK_MAX) {
        std::fprintf(stderr, "tree too large for the per-lane walk\n");
        return 1;
    }
    }

    long rays = 0, fallback = 0, mism = 0, hits = 0, shadow_rays = 0, occluded = 0, shifted = 0, nosphere = 0, grown = 0;
    const double O = S.bvh.obound;
    auto check = [&](const double o[3], const double d[3]) {
        ++rays;
        double t0s = 0.0;
        float grow = 0.0f;
        const int cls = rg_bvh_classify(S.bvh.obound, S.bvh.rbound, S.bvh.margin, S.bvh.extent, o[0], o[1], o[2], d[0],
                                        d[1], d[2], t0s, grow);
        grown += grow > 0.0f;
        if (cls == RG_BVH_SCAN) { ++fallback; return; }
        shifted += t0s > 0.0;
        nosphere += cls == RG_BVH_NO_SPHERE;
        bool any = false;
        const Hit b = brute(S, o, d);
        const Hit v = cls == RG_BVH_NO_SPHERE ? Hit{0.0, -1} : bvh_trace(S, o, d, -1.0, t0s, any, grow);
        const Hit w = (cls == RG_BVH_NO_SPHERE || grow > 0.0f) ? v : lane_trace(S, o, d, -1.0, t0s, any);
        if (w.id != b.id || (b.id >= 0 && std::memcmp(&b.t, &w.t, 8) != 0)) {
            if (++mism <= 5) std::fprintf(stderr, "lane closest mismatch brute %d bvh %d\n", b.id, w.id);
        }
        if (b.id != v.id || (b.id >= 0 && std::memcmp(&b.t, &v.t, 8) != 0)) {
            if (++mism <= 5)
                std::fprintf(stderr, "closest mismatch o=(%.17g %.17g %.17g) d=(%.17g %.17g %.17g) brute %d %.17g bvh %d %.17g\n",
                             o[0], o[1], o[2], d[0], d[1], d[2], b.id, b.t, v.id, v.t);
        }
        hits += b.id >= 0;
        const double lds[3] = {b.id >= 0 ? b.t : 10.0, urand() * 60.0, HUGE_VAL};
        for (double ld : lds) {
            ++shadow_rays;
            const bool ba = brute_any(S, o, d, ld);
            any = false;
            if (cls != RG_BVH_NO_SPHERE) bvh_trace(S, o, d, ld, t0s, any, grow);
            bool any2 = any;
            if (cls != RG_BVH_NO_SPHERE && grow == 0.0f) lane_trace(S, o, d, ld, t0s, any2);
            if (ba != any2 && ++mism <= 5) std::fprintf(stderr, "lane shadow mismatch ld=%.17g\n", ld);
            occluded += ba;
            if (ba != any && ++mism <= 5) std::fprintf(stderr, "shadow mismatch ld=%.17g\n", ld);
        }
    };
    double o[3], d[3];
    // 1. primary rays (ray.rs:37-54 at 3840x2160, fov 90, sampled pixels)
    for (long i = 0; i < per_kind; ++i) {
        const double x = std::floor(urand() * 3840), y = std::floor(urand() * 2160);
        const double sx = (((x + 0.5) / 3840.0) * 2.0 - 1.0) * (3840.0 / 2160.0) * std::tan(90.0 * (M_PI / 180.0) / 2.0);
        const double sy = (1.0 - ((y + 0.5) / 2160.0) * 2.0) * std::tan(90.0 * (M_PI / 180.0) / 2.0);
        o[0] = o[1] = o[2] = 0.0;
        d[0] = sx; d[1] = sy; d[2] = -1.0;
        unit(d);
        check(o, d);
    }
    // 2. secondary/shadow-like rays from sphere surfaces (hit + n * 1e-13)
    for (long i = 0; i < per_kind; ++i) {
        const double *s = &S.sp[4 * (size_t)(urand() * n)];
        double nrm[3];
        rand_dir(nrm);
        for (int k = 0; k < 3; ++k) o[k] = s[k] + nrm[k] * std::fabs(s[3]) + nrm[k] * 1e-13;
        rand_dir(d);
        check(o, d);
    }
    // 3. grazing rays: offset r(1 +- eps) from a sphere centre, perpendicular to d
    const double eps[4] = {1e-9, -1e-9, 1e-13, -1e-13};
    for (long i = 0; i < per_kind; ++i) {
        const double *s = &S.sp[4 * (size_t)(urand() * n)];
        rand_dir(d);
        double p[3];
        rand_dir(p);
        const double pd = (p[0] * d[0] + p[1] * d[1]) + p[2] * d[2];
        for (int k = 0; k < 3; ++k) p[k] -= pd * d[k];
        unit(p);
        const double L = 2.0 + urand() * 60.0, off = std::fabs(s[3]) * (1.0 + eps[i & 3]);
        for (int k = 0; k < 3; ++k) o[k] = s[k] - d[k] * L + p[k] * off;
        check(o, d);
    }
    // 4. arbitrary origins, up to 1.2x the origin bound (some take the fallback)
    for (long i = 0; i < per_kind; ++i) {
        for (int k = 0; k < 3; ++k) o[k] = (2.0 * urand() - 1.0) * 1.2 * O * (urand() < 0.7 ? 0.1 : 1.0);
        rand_dir(d);
        check(o, d);
    }
    // 5. far origins (floor points seen at grazing angles): |o| from 1.5 O to 3e4 and beyond 1e7,
    //    directions towards a random sphere or random
    for (long i = 0; i < per_kind; ++i) {
        const double R = O * (1.5 + urand() * (i % 3 == 0 ? 80.0 : 10.0)) * (i % 13 == 0 ? 1e5 : (i % 7 == 0 ? 300.0 : 1.0));
        rand_dir(o);
        for (int k = 0; k < 3; ++k) o[k] *= R;
        if (i & 1) {
            const double *s = &S.sp[4 * (size_t)(urand() * n)];
            for (int k = 0; k < 3; ++k) d[k] = s[k] + (urand() - 0.5) * 2.5 * std::fabs(s[3]) - o[k];
            unit(d);
        } else {
            rand_dir(d);
        }
        check(o, d);
    }
    std::printf("{\"spheres\": %d, \"nodes\": %zu, \"leaves\": %d, \"depth\": %d, \"margin\": %.6g, \"obound\": %.6g, "
                "\"rays\": %ld, \"fallback\": %ld, \"hits\": %ld, \"shadow_rays\": %ld, \"occluded\": %ld, "
                "\"shifted\": %ld, \"no_sphere\": %ld, \"grown\": %ld, "
                "\"exact_tests_per_ray\": %.3f, \"nodes_per_ray\": %.3f, \"lane_steps_per_ray\": %.3f, "
                "\"lane_stack\": %d, \"lane_stack_used\": %d, \"mismatches\": %ld}\n",
                n, S.bvh.nodes.size(), S.bvh.leaves, S.bvh.depth, S.bvh.margin, (double)S.bvh.obound, rays, fallback,
                hits, shadow_rays, occluded, shifted, nosphere, grown, (double)g_tests / (double)(4 * (rays - fallback)),
                (double)g_nodes / (double)(4 * (rays - fallback)), (double)g_lane_steps / (double)(4 * (rays - fallback)),
                S.bvh.lane_stack, g_lane_max_sp, mism);
    return mism ? 1 : 0;
}
