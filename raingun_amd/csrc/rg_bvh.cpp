// rg_bvh.cpp — 4-wide sphere BVH for the heavy render path (host code).
//
// Build: binary tree by binned SAH (16 bins, largest centroid axis; median
// split when the centroids coincide or a side would be empty), leaves of at
// most RG_BVH_LEAF_MAX spheres, then collapsed to 4-wide nodes by repeatedly
// opening the child with the largest surface area.  Leaves are contiguous
// ranges of the reordered sphere tables.
//
// Conservative boxes.  A box must contain every point at which the exact
// reference test (bodies.rs:92-119, evaluated in f64 by the kernel) can report
// a hit for a ray the traversal accepts, with room for the f32 slab test's
// rounding.  With S = max |coordinate| of any sphere bound and O = 4 S + 1 the
// origin bound (|o_k| <= O, and ||d|^2 - 1| <= 1e-13, checked per ray in the
// kernel; other rays take the brute-force loop):
//   * f64 "hit by rounding" slack of the exact test: < 1e-8 (S + O);
//   * |d|^2 = 1 + eta moves the accepted perpendicular distance by <= sqrt(eta) |h|
//     <= 3.2e-7 (S + O), and the hit parameter by the same amount;
//   * f32 slab test (o, 1/d rounded to f32, one fma per slab): per-axis error in
//     t of <= 8u (|lo_k| + |o_k|) / |d_k| with u = 2^-24, i.e. <= 8u (S + m + O) / |d_k|.
// Inflating every sphere box by m = 256 u (S + O) (~1.5e-5 (S + O)) covers the
// sum with a margin > 2x, so for every sphere the exact test could accept with
// t <= best, the computed slab interval of every box on its path is non-empty,
// has tmax >= 0 and tmin <= best.  Boxes are then rounded outward to f32.
//
// The exact test's slack, precisely: with H = c - o, eta = |d|^2 - 1 and
// gamma ~ 9e-16 (relative error of the few f64 ops in opp), the computed opp is
// >= p^2 - (eta + 2 gamma)|H|^2 (p = true distance of c from the ray line), so
// an accepted sphere has p <= r + sqrt(eta + 1.8e-15)|H|, and the computed hit
// point lies within 3 sqrt(eta + 1.8e-15)|H| of the true (slack-inflated)
// sphere.  Near rays: |H| <= sqrt(3) O + S and eta <= 1e-13 give <= m/5.  Far
// origins (rg_bvh_classify) are admitted while that term is <= m/4, and their
// box tests start at the f64 entry point into [-(S + 2m), S + 2m]^3 so the f32
// slab bound above still applies.
#if defined(__HIP__)
#include <hip/hip_runtime.h>  // hipcc builds this file as HIP (host code only)
#endif
#include "rg_bvh.h"

#include <algorithm>
#include <cmath>
#include <numeric>

namespace {

struct Box {
    double lo[3] = {HUGE_VAL, HUGE_VAL, HUGE_VAL};
    double hi[3] = {-HUGE_VAL, -HUGE_VAL, -HUGE_VAL};
    void grow(const Box &b) {
        for (int k = 0; k < 3; ++k) {
            lo[k] = std::min(lo[k], b.lo[k]);
            hi[k] = std::max(hi[k], b.hi[k]);
        }
    }
    void grow(const double *p) {
        for (int k = 0; k < 3; ++k) {
            lo[k] = std::min(lo[k], p[k]);
            hi[k] = std::max(hi[k], p[k]);
        }
    }
    double area() const {
        double e[3];
        for (int k = 0; k < 3; ++k) e[k] = std::max(0.0, hi[k] - lo[k]);
        return 2.0 * (e[0] * e[1] + e[1] * e[2] + e[2] * e[0]);
    }
};

struct BNode {
    Box box;
    int left = -1, right = -1;  // internal
    int first = 0, count = 0;   // leaf when count > 0
};

struct Builder {
    std::vector<Box> prim;            // per input sphere
    std::vector<double> cen;          // 3 per input sphere
    std::vector<uint32_t> idx;        // permutation being partitioned
    std::vector<BNode> bn;

    int build(int first, int count) {
        BNode node;
        for (int i = 0; i < count; ++i) node.box.grow(prim[idx[first + i]]);
        const int me = (int)bn.size();
        bn.push_back(node);
        if (count <= RG_BVH_LEAF_MAX) {
            bn[me].first = first;
            bn[me].count = count;
            return me;
        }
        Box cb;
        for (int i = 0; i < count; ++i) cb.grow(&cen[3 * idx[first + i]]);
        int axis = 0;
        for (int k = 1; k < 3; ++k)
            if (cb.hi[k] - cb.lo[k] > cb.hi[axis] - cb.lo[axis]) axis = k;
        const double ext = cb.hi[axis] - cb.lo[axis];
        int mid = first + count / 2;
        auto key = [&](uint32_t i) { return cen[3 * i + axis]; };
        if (ext > 0.0) {
            constexpr int B = 16;
            Box bb[B];
            int bc[B] = {0};
            auto bin = [&](uint32_t i) {
                int b = (int)((key(i) - cb.lo[axis]) / ext * B);
                return std::min(std::max(b, 0), B - 1);
            };
            for (int i = 0; i < count; ++i) {
                const uint32_t p = idx[first + i];
                const int b = bin(p);
                bb[b].grow(prim[p]);
                ++bc[b];
            }
            double best = HUGE_VAL;
            int best_split = -1;
            for (int s = 1; s < B; ++s) {
                Box l, r;
                int nl = 0, nr = 0;
                for (int b = 0; b < s; ++b) if (bc[b]) { l.grow(bb[b]); nl += bc[b]; }
                for (int b = s; b < B; ++b) if (bc[b]) { r.grow(bb[b]); nr += bc[b]; }
                if (!nl || !nr) continue;
                const double cost = l.area() * nl + r.area() * nr;
                if (cost < best) { best = cost; best_split = s; }
            }
            if (best_split > 0) {
                auto it = std::partition(idx.begin() + first, idx.begin() + first + count,
                                         [&](uint32_t i) { return bin(i) < best_split; });
                mid = (int)(it - idx.begin());
            }
        }
        if (mid <= first || mid >= first + count) {  // degenerate: median by centroid, then by index
            mid = first + count / 2;
            std::nth_element(idx.begin() + first, idx.begin() + mid, idx.begin() + first + count,
                             [&](uint32_t a, uint32_t b) { return key(a) < key(b) || (key(a) == key(b) && a < b); });
        }
        const int l = build(first, mid - first);
        const int r = build(mid, first + count - mid);
        bn[me].left = l;
        bn[me].right = r;
        return me;
    }
};

float f32_down(double v) {
    float f = (float)v;
    if ((double)f > v) f = std::nextafter(f, -HUGE_VALF);
    return f;
}
float f32_up(double v) {
    float f = (float)v;
    if ((double)f < v) f = std::nextafter(f, HUGE_VALF);
    return f;
}

struct Collapser {
    const std::vector<BNode> &bn;
    double margin;
    std::vector<RgBvhNode> out;
    int depth = 0, leaves = 0;

    int emit(int b, int level) {
        depth = std::max(depth, level + 1);
        std::vector<int> kids = {bn[b].left, bn[b].right};
        for (;;) {
            if ((int)kids.size() >= 4) break;
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
        RgBvhNode node;
        for (int k = 0; k < 4; ++k) {
            node.lox[k] = node.loy[k] = node.loz[k] = HUGE_VALF;
            node.hix[k] = node.hiy[k] = node.hiz[k] = -HUGE_VALF;
            node.child[k] = 0;
        }
        node.nchild = (int)kids.size();
        node.pad[0] = node.pad[1] = node.pad[2] = 0;
        for (int k = 0; k < (int)kids.size(); ++k) {
            const BNode &c = bn[kids[k]];
            node.lox[k] = f32_down(c.box.lo[0] - margin);
            node.loy[k] = f32_down(c.box.lo[1] - margin);
            node.loz[k] = f32_down(c.box.lo[2] - margin);
            node.hix[k] = f32_up(c.box.hi[0] + margin);
            node.hiy[k] = f32_up(c.box.hi[1] + margin);
            node.hiz[k] = f32_up(c.box.hi[2] + margin);
            if (c.count > 0) {
                node.child[k] = ~((c.first << 3) | (c.count - 1));
                ++leaves;
            } else {
                node.child[k] = emit(kids[k], level + 1);
            }
        }
        out[me] = node;
        return me;
    }
};

// Per-lane nearest-first walk: visiting a node pushes all but one of its
// internal children and descends into one, and a popped node is a sibling of an
// ancestor, so the stack never exceeds max over root paths of sum (m - 1),
// m = internal children of each node on the path.
int lane_stack_need(const std::vector<RgBvhNode> &nodes, int i) {
    const RgBvhNode &N = nodes[i];
    int m = 0, below = 0;
    for (int k = 0; k < N.nchild; ++k)
        if (N.child[k] >= 0) {
            ++m;
            below = std::max(below, lane_stack_need(nodes, N.child[k]));
        }
    return m == 0 ? 0 : (m - 1) + below;
}

}  // namespace

bool rg_build_bvh(const double *sp, int n, RgBvhBuild &out) {
    out = RgBvhBuild();
    if (n < 2 || n > (1 << 27)) return false;
    Builder b;
    b.prim.resize(n);
    b.cen.resize(3 * (size_t)n);
    double S = 0.0;
    for (int i = 0; i < n; ++i) {
        const double *p = sp + 4 * (size_t)i;
        const double r = std::fabs(p[3]);
        for (int k = 0; k < 4; ++k)
            if (!std::isfinite(p[k])) return false;
        for (int k = 0; k < 3; ++k) {
            b.prim[i].lo[k] = p[k] - r;
            b.prim[i].hi[k] = p[k] + r;
            b.cen[3 * (size_t)i + k] = p[k];
            S = std::max(S, std::max(std::fabs(b.prim[i].lo[k]), std::fabs(b.prim[i].hi[k])));
        }
    }
    const double u = 5.9604644775390625e-08;  // 2^-24
    const double O = 4.0 * S + 1.0;
#ifndef RG_BVH_MARGIN_ULPS
#define RG_BVH_MARGIN_ULPS 256.0
#endif
    const double margin = RG_BVH_MARGIN_ULPS * u * (S + O);
    if (!(O < 1e30)) return false;
    b.idx.resize(n);
    std::iota(b.idx.begin(), b.idx.end(), 0u);
    b.bn.reserve(2 * (size_t)n);
    const int root = b.build(0, n);
    if (b.bn[root].count > 0) return false;  // a single leaf: nothing to cull
    Collapser c{b.bn, margin, {}, 0, 0};
    c.out.reserve((size_t)n);
    c.emit(root, 0);
    out.nodes = std::move(c.out);
    out.order = std::move(b.idx);
    out.obound = f32_down(O);
    out.margin = margin;
    out.extent = S;
    out.rbound = S + 2.0 * margin;
    out.depth = c.depth;
    out.leaves = c.leaves;
    out.max_stack = 3 * c.depth;
    out.lane_stack = lane_stack_need(out.nodes, 0);
    if (out.max_stack > 64) {
        out = RgBvhBuild();
        return false;
    }
    return true;
}
