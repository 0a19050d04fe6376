// bvh_width_sim.cpp — what a wider sphere BVH would change for the heavy path's walks (CPU model).
//
// The product tree is 4-wide (rg_bvh.cpp: binned-SAH binary tree collapsed by opening the child of
// largest area).  This model collapses the SAME binary tree (rg_bvh.cpp's Builder, included below)
// to W-wide nodes for W = 2, 4, 8, with the product's margin and f32 rounding, and walks it the way
// the kernel's per-lane walk does (nearest-first, one node per iteration, every child box tested,
// internal children pushed by entry distance; rg_kernels.hip bvh_lane): per ray kind it counts
// walk iterations (node visits: the dependent loads of the walk), child box tests (the f32 VALU of
// the walk) and exact sphere tests (the f64 VALU), and the worst-case per-lane stack the tree needs
// (rg_bvh.cpp lane_stack_need).  Every BVH answer is checked against the brute-force scan.
//
// Rays: 4K camera rays (every `stride`-th pixel in x and y), and from each primary sphere hit one
// shadow ray per light and the mirror-reflected secondary ray -- the ray kinds of the north star.
//
// usage: bvh_width_sim W H stride < scene.txt
//   scene.txt: fov_deg; n; n lines "cx cy cz r"; m; m lines "kind x y z" (0 directional: x y z =
//   direction, 1 spherical: position)
#include "../raingun_amd/csrc/rg_bvh_ray.h"
#include "../raingun_amd/csrc/rg_bvh.cpp"  // Builder, f32_down/up (anonymous namespace, same TU)

#include <cstdio>
#include <cstdlib>
#include <functional>

namespace {

struct WNode {
    std::vector<float> lo[3], hi[3];
    std::vector<int> child;  // >= 0 internal node, < 0: ~(first << 8 | count)
};

struct Wide {
    int W;
    double margin;
    const std::vector<BNode> &bn;
    std::vector<WNode> out;

    int emit(int b) {
        std::vector<int> kids = {bn[b].left, bn[b].right};
        for (;;) {
            if ((int)kids.size() >= W) break;
            int open = -1;
            double area = -1.0;
            for (int i = 0; i < (int)kids.size(); ++i) {
                const BNode &k = bn[kids[i]];
                if (k.count == 0 && k.box.area() > area) { area = k.box.area(); open = i; }
            }
            if (open < 0) break;
            const int c = kids[open];
            kids[open] = bn[c].left;
            kids.insert(kids.begin() + open + 1, bn[c].right);
        }
        const int me = (int)out.size();
        out.emplace_back();
        WNode node;
        for (int k = 0; k < (int)kids.size(); ++k) {
            const BNode &c = bn[kids[k]];
            for (int a = 0; a < 3; ++a) {
                node.lo[a].push_back(f32_down(c.box.lo[a] - margin));
                node.hi[a].push_back(f32_up(c.box.hi[a] + margin));
            }
            node.child.push_back(c.count > 0 ? ~((c.first << 8) | c.count) : emit(kids[k]));
        }
        out[me] = node;
        return me;
    }
    int lane_stack(int i) const {
        int m = 0, below = 0;
        for (int c : out[i].child)
            if (c >= 0) { ++m; below = std::max(below, lane_stack(c)); }
        return m == 0 ? 0 : (m - 1) + below;
    }
    int depth(int i) const {
        int d = 0;
        for (int c : out[i].child) if (c >= 0) d = std::max(d, depth(c));
        return d + 1;
    }
};

bool sphere_exact(const double *s, const double o[3], const double d[3], double &t) {  // bodies.rs:92-119
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

struct Count { long rays = 0, iters = 0, boxes = 0, spheres = 0, max_stack = 0; };

struct Hit { double t; int id; };

// per-lane nearest-first walk; ld >= 0: any hit within ld (shadow), else closest hit
Hit walk(const Wide &T, const std::vector<double> &sp, const std::vector<uint32_t> &order, const double o[3],
         const double d[3], double ld, Count &c) {
    float ix[3], oi[3];
    for (int a = 0; a < 3; ++a) {
        ix[a] = 1.0f / rg_bvh_clamp_dir((float)d[a]);
        oi[a] = (float)o[a] * ix[a];
    }
    Hit h{0.0, -1};
    std::vector<std::pair<float, int>> st;
    st.push_back({0.0f, 0});
    c.rays++;
    while (!st.empty()) {
        const auto [key, ni] = st.back();
        st.pop_back();
        const float tb = ld >= 0.0 ? rg_f32_up(ld) : (h.id >= 0 ? rg_f32_up(h.t) : HUGE_VALF);
        if (key > tb) continue;  // pruned at pop (no iteration in the kernel either)
        c.iters++;
        const WNode &N = T.out[ni];
        std::vector<std::pair<float, int>> kids;
        for (int k = 0; k < (int)N.child.size(); ++k) {
            c.boxes++;
            float t1[3], t2[3];
            for (int a = 0; a < 3; ++a) {
                t1[a] = std::fmaf(N.lo[a][k], ix[a], -oi[a]);
                t2[a] = std::fmaf(N.hi[a][k], ix[a], -oi[a]);
            }
            const float tmin = std::fmax(std::fmax(std::fmin(t1[0], t2[0]), std::fmin(t1[1], t2[1])),
                                         std::fmax(std::fmin(t1[2], t2[2]), 0.0f));
            const float tmax = std::fmin(std::fmin(std::fmax(t1[0], t2[0]), std::fmax(t1[1], t2[1])),
                                         std::fmin(std::fmax(t1[2], t2[2]), tb));
            if (!(tmin <= tmax)) continue;
            const int ch = N.child[k];
            if (ch < 0) {
                const int v = ~ch, first = v >> 8, count = v & 255;
                for (int j = first; j < first + count; ++j) {
                    double t;
                    c.spheres++;
                    if (!sphere_exact(&sp[4 * order[j]], o, d, t)) continue;
                    const int id = (int)order[j];
                    if (ld >= 0.0) {
                        if (!(t > ld)) return Hit{t, id};
                    } else if (h.id < 0 || t < h.t || (t == h.t && id < h.id)) {
                        h = Hit{t, id};
                    }
                }
            } else {
                kids.push_back({tmin, ch});
            }
        }
        std::sort(kids.begin(), kids.end(), [](auto &a, auto &b) { return a.first > b.first; });
        for (auto &k : kids) st.push_back(k);  // nearest on top
        c.max_stack = std::max(c.max_stack, (long)st.size());
    }
    return h;
}

Hit brute(const std::vector<double> &sp, const double o[3], const double d[3], double ld) {
    Hit h{0.0, -1};
    for (int i = 0; i < (int)sp.size() / 4; ++i) {
        double t;
        if (!sphere_exact(&sp[4 * i], o, d, t)) continue;
        if (ld >= 0.0) {
            if (!(t > ld)) return Hit{t, i};
        } else if (h.id < 0 || t < h.t || (t == h.t && i < h.id)) {
            h = Hit{t, i};
        }
    }
    return h;
}

}  // namespace

int main(int argc, char **argv) {
    if (argc < 4) { std::fprintf(stderr, "usage: bvh_width_sim W H stride < scene\n"); return 2; }
    const int IW = std::atoi(argv[1]), IH = std::atoi(argv[2]), stride = std::atoi(argv[3]);
    double fov;
    int n, m;
    if (std::scanf("%lf %d", &fov, &n) != 2 || n < 2) return 2;
    std::vector<double> sp(4 * (size_t)n);
    for (auto &v : sp) if (std::scanf("%lf", &v) != 1) return 2;
    if (std::scanf("%d", &m) != 1) return 2;
    std::vector<int> lk(m);
    std::vector<double> lv(3 * (size_t)m);
    for (int i = 0; i < m; ++i)
        if (std::scanf("%d %lf %lf %lf", &lk[i], &lv[3 * i], &lv[3 * i + 1], &lv[3 * i + 2]) != 4) return 2;

    // rg_build_bvh's binary tree and margin
    Builder b;
    b.prim.resize(n);
    b.cen.resize(3 * (size_t)n);
    double S = 0.0;
    for (int i = 0; i < n; ++i) {
        const double r = std::fabs(sp[4 * i + 3]);
        for (int k = 0; k < 3; ++k) {
            b.prim[i].lo[k] = sp[4 * i + k] - r;
            b.prim[i].hi[k] = sp[4 * i + k] + r;
            b.cen[3 * i + k] = sp[4 * i + k];
            S = std::max(S, std::max(std::fabs(b.prim[i].lo[k]), std::fabs(b.prim[i].hi[k])));
        }
    }
    const double margin = RG_BVH_MARGIN_ULPS * 5.9604644775390625e-08 * (S + 4.0 * S + 1.0);
    b.idx.resize(n);
    std::iota(b.idx.begin(), b.idx.end(), 0u);
    const int root = b.build(0, n);

    const double aspect = (double)IW / IH, fadj = std::tan(fov * M_PI / 180.0 / 2.0);
    long mismatches = 0;
    for (int W : {2, 4, 8}) {
        Wide T{W, margin, b.bn, {}};
        T.emit(root);
        Count prim, shad, sec;
        for (int y = stride / 2; y < IH; y += stride)
            for (int x = stride / 2; x < IW; x += stride) {
                const double sx = ((((double)x + 0.5) / IW) * 2.0 - 1.0) * aspect * fadj;
                const double sy = (1.0 - (((double)y + 0.5) / IH) * 2.0) * fadj;
                const double l = std::sqrt((sx * sx + sy * sy) + 1.0);
                const double o[3] = {0, 0, 0}, d[3] = {sx / l, sy / l, -1.0 / l};
                const Hit h = walk(T, sp, b.idx, o, d, -1.0, prim);
                if (W == 4 && (x / stride) % 7 == 0) {
                    const Hit g = brute(sp, o, d, -1.0);
                    mismatches += g.id != h.id || (g.id >= 0 && g.t != h.t);
                }
                if (h.id < 0) continue;
                const double *s = &sp[4 * h.id];
                double p[3], nn[3];
                for (int a = 0; a < 3; ++a) p[a] = o[a] + d[a] * h.t;
                for (int a = 0; a < 3; ++a) nn[a] = (p[a] - s[a]) / std::fabs(s[3]);
                double q[3];
                for (int a = 0; a < 3; ++a) q[a] = p[a] + nn[a] * 1e-13;  // shadow bias (rendering.rs)
                for (int li = 0; li < m; ++li) {
                    double ld[3], dist;
                    if (lk[li] == 0) {
                        for (int a = 0; a < 3; ++a) ld[a] = -lv[3 * li + a];
                        dist = HUGE_VAL;
                    } else {
                        for (int a = 0; a < 3; ++a) ld[a] = lv[3 * li + a] - q[a];
                        dist = std::sqrt((ld[0] * ld[0] + ld[1] * ld[1]) + ld[2] * ld[2]);
                    }
                    const double ll = std::sqrt((ld[0] * ld[0] + ld[1] * ld[1]) + ld[2] * ld[2]);
                    for (double &v : ld) v /= ll;
                    walk(T, sp, b.idx, q, ld, dist, shad);
                }
                const double dn = (d[0] * nn[0] + d[1] * nn[1]) + d[2] * nn[2];
                double r[3];
                for (int a = 0; a < 3; ++a) r[a] = d[a] - 2.0 * dn * nn[a];
                const Hit hs = walk(T, sp, b.idx, q, r, -1.0, sec);
                if (W == 8 && (x / stride) % 5 == 0) {
                    const Hit g = brute(sp, q, r, -1.0);
                    mismatches += g.id != hs.id || (g.id >= 0 && g.t != hs.t);
                }
            }
        auto pr = [&](const char *k, const Count &c) {
            std::printf("{\"width\": %d, \"nodes\": %zu, \"depth\": %d, \"lane_stack_need\": %d, \"kind\": \"%s\", "
                        "\"rays\": %ld, \"iterations_per_ray\": %.3f, \"box_tests_per_ray\": %.3f, "
                        "\"sphere_tests_per_ray\": %.3f, \"max_stack_seen\": %ld}\n",
                        W, T.out.size(), T.depth(0), T.lane_stack(0), k, c.rays, (double)c.iters / c.rays,
                        (double)c.boxes / c.rays, (double)c.spheres / c.rays, c.max_stack);
        };
        pr("primary", prim);
        pr("shadow", shad);
        pr("secondary", sec);
    }
    std::printf("{\"brute_force_mismatches\": %ld}\n", mismatches);
    return mismatches ? 1 : 0;
}
