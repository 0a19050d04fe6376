// rg_lightbuf.cpp — shadow-ray light buffers for the heavy render path (host code).
//
// Per light, a 2-D grid whose cell lists hold every sphere a shadow ray from a
// point of the cell could hit (cell lookup: rg_lightbuf_ray.h).  The shadow
// query of the reference (rendering.rs:141-155: trace the ray, in light iff no
// hit or the closest hit is beyond the light) is an any-hit question on this
// path (rg_kernels.hip "shadow rays are any-hit"), so a ray that tests its
// cell's spheres -- each with the exact reference test, f32 pre-filter first --
// gets the answer of the brute-force scan as long as no sphere the exact test
// could accept is missing from its cell.  The lists are built so it cannot be.
//
// Bounds (S = max |coordinate| of any sphere bound, O = 4 S + 1 the near-ray
// origin bound of the BVH, rg_bvh.cpp; rays with |o_k| > O do not use the
// buffer).  The exact test accepts a sphere only if the true distance p of its
// centre from the ray's line satisfies p <= r + sqrt(eta + 1.8e-15) |c - o|
// (rg_bvh.cpp: eta = |d|^2 - 1 <= 1e-15 for the normalized shadow direction),
// i.e. within r + 2^-23.6 (S + O).
//  * Directional lights.  The device projects o on the f32 basis (e1, e2) of
//    the plane normal to dn: o rounded to f32 and an fma chain, error
//    <= 12 u Sum|o_k| <= 2^-20.4 O (u = 2^-24); the f32 basis is orthonormal and
//    normal to dn within 2^-22, which moves projected distances by
//    <= 2^-20.2 (S + O); the cell coordinate (p - g0) * inv carries two more
//    roundings, <= 2^-19.2 (S + O) in distance.  The sum is below 2^-18.2 (S + O):
//    every disk of radius r + m, m = 2^-16 (S + O), about the projected centre
//    (projected on the host with the same f32 basis, in f64) covers every cell
//    the device can compute for a ray that can hit the sphere (> 4x margin).
//  * Spherical lights.  A sphere at D = |c - L| > r + m from the light that meets
//    the segment from o to L (plus the exact test's slack, < m) subtends from L
//    a cone of half-angle asin((r + m) / D) containing the direction of o - L
//    (the angle at L of the triangle L, c, hit point is acute because the hit
//    point is within r + m < D of c).  The device's direction (o - L in f64,
//    rounded to f32) is off by < 2^-22 rad and its face coordinates
//    a = v_i / |v_k| (v_rcp_f32, <= 1 ulp) by < 2^-21: the cone is widened by
//    2^-16 rad and every face interval by 2^-12 (the device may also pick a face
//    whose axis is 2^-22 short of the largest; faces are therefore taken from
//    x_k >= 1/sqrt(3) - 2^-12).  Spheres within r + m of L go on the "always"
//    list.  The face intervals are interval arithmetic over a box containing
//    the cone's cap of unit directions (per axis m: the angle to the axis lies
//    in [alpha_m - theta, alpha_m + theta]).
// tests/native/lightbuf_sim.cpp checks the lists against the brute-force scan
// on millions of shadow rays (tests/test_lightbuf_cpu.py).
#if defined(__HIP__)
#include <hip/hip_runtime.h>  // hipcc builds this file as HIP (host code only)
#endif
#include "rg_lightbuf.h"

#include <algorithm>
#include <cmath>

#include "../../include/raingun.h"

// negative control of tests/test_lightbuf_cpu.py only: footprints 1 % smaller than the spheres, no margins
#ifdef RG_LB_TEST_NO_MARGIN
#define RG_LB_RSCALE 0.99
#define RG_LB_MARGINS 0.0
#else
#define RG_LB_RSCALE (1.0 + 1e-9)
#define RG_LB_MARGINS 1.0
#endif

namespace {

bool finite3(const double *v) { return std::isfinite(v[0]) && std::isfinite(v[1]) && std::isfinite(v[2]); }

// cells (lists per cell) -> CSR arrays; false if too many entries or too long on average
bool finish(std::vector<std::vector<uint32_t>> &cells, RgLightBufBuild &out) {
    size_t total = 0, nonempty = 0;
    uint32_t mx = 0;
    for (const auto &c : cells) {
        total += c.size();
        nonempty += !c.empty();
        mx = std::max<uint32_t>(mx, (uint32_t)c.size());
    }
    total += out.ent.size();  // the always list (spherical), already in ent
    if (total > RG_LB_MAX_ENTRIES) return false;
    out.mean_candidates = nonempty ? (double)(total - out.ent.size()) / (double)nonempty : 0.0;
    out.max_candidates = mx;
    if (out.mean_candidates > RG_LB_MAX_MEAN) return false;
    out.start.resize(cells.size() + 1);
    out.ent.reserve(total);
    for (size_t i = 0; i < cells.size(); ++i) {
        out.start[i] = (uint32_t)out.ent.size();
        out.ent.insert(out.ent.end(), cells[i].begin(), cells[i].end());
    }
    out.start[cells.size()] = (uint32_t)out.ent.size();
    return true;
}

bool build_directional(const double *sp, int n, const double dn[3], double m, RgLightBufBuild &out) {
    const double d2 = (dn[0] * dn[0] + dn[1] * dn[1]) + dn[2] * dn[2];
    if (!finite3(dn) || std::fabs(d2 - 1.0) > 1e-12) return false;
    // basis of the plane normal to dn: e1 = normalize(dn x axis of dn's smallest component), e2 = dn x e1
    int k = 0;
    for (int j = 1; j < 3; ++j)
        if (std::fabs(dn[j]) < std::fabs(dn[k])) k = j;
    double ax[3] = {0.0, 0.0, 0.0};
    ax[k] = 1.0;
    double e1[3] = {dn[1] * ax[2] - dn[2] * ax[1], dn[2] * ax[0] - dn[0] * ax[2], dn[0] * ax[1] - dn[1] * ax[0]};
    const double l1 = std::sqrt(e1[0] * e1[0] + e1[1] * e1[1] + e1[2] * e1[2]);
    for (double &v : e1) v /= l1;
    const double e2[3] = {dn[1] * e1[2] - dn[2] * e1[1], dn[2] * e1[0] - dn[0] * e1[2], dn[0] * e1[1] - dn[1] * e1[0]};
    float f1[3], f2[3];
    for (int j = 0; j < 3; ++j) {
        f1[j] = (float)e1[j];
        f2[j] = (float)e2[j];
    }
    // projected centres (the device's f32 basis, evaluated in f64) and footprint half-widths
    std::vector<double> px(n), py(n), R(n);
    double lox = HUGE_VAL, loy = HUGE_VAL, hix = -HUGE_VAL, hiy = -HUGE_VAL, rsum = 0.0;
    for (int i = 0; i < n; ++i) {
        const double *s = sp + 4 * i;
        px[i] = s[0] * (double)f1[0] + s[1] * (double)f1[1] + s[2] * (double)f1[2];
        py[i] = s[0] * (double)f2[0] + s[1] * (double)f2[1] + s[2] * (double)f2[2];
        R[i] = std::fabs(s[3]) * RG_LB_RSCALE + m;
        rsum += std::fabs(s[3]);
        lox = std::min(lox, px[i] - R[i]);
        hix = std::max(hix, px[i] + R[i]);
        loy = std::min(loy, py[i] - R[i]);
        hiy = std::max(hiy, py[i] + R[i]);
    }
    if (!(std::isfinite(lox) && std::isfinite(hix) && std::isfinite(loy) && std::isfinite(hiy))) return false;
    const double ext = std::max(hix - lox, hiy - loy);
    const double cs = std::max(RG_LB_DIR_CELL * rsum / n, ext / RG_LB_DIR_MAX_G);
    if (!(cs > 0.0)) return false;
    const float inv = (float)(1.0 / cs);
    // grid origin rounded down to f32; the cells are [g0 + k / inv, g0 + (k + 1) / inv) exactly
    float g0x = (float)lox, g0y = (float)loy;
    if ((double)g0x > lox) g0x = std::nextafter(g0x, -HUGE_VALF);
    if ((double)g0y > loy) g0y = std::nextafter(g0y, -HUGE_VALF);
    const double fgx = std::floor((hix - g0x) * inv) + 1, fgy = std::floor((hiy - g0y) * inv) + 1;
    if (!(fgx <= RG_LB_DIR_MAX_G + 2 && fgy <= RG_LB_DIR_MAX_G + 2)) return false;  // every footprint on the grid
    const int gx = (int)fgx, gy = (int)fgy;
    std::vector<std::vector<uint32_t>> cells((size_t)gx * gy);
    for (int i = 0; i < n; ++i) {
        const int x0 = std::max(0, (int)std::floor((px[i] - R[i] - g0x) * inv));
        const int x1 = std::min(gx - 1, (int)std::floor((px[i] + R[i] - g0x) * inv));
        const int y0 = std::max(0, (int)std::floor((py[i] - R[i] - g0y) * inv));
        const int y1 = std::min(gy - 1, (int)std::floor((py[i] + R[i] - g0y) * inv));
        const double cw = 1.0 / (double)inv;
        for (int y = y0; y <= y1; ++y)
            for (int x = x0; x <= x1; ++x) {
                // keep the cell only if it meets the disk (nearest point of the cell to the centre)
                const double cx0 = g0x + x * cw, cy0 = g0y + y * cw;
                const double qx = std::min(std::max(px[i], cx0), cx0 + cw), qy = std::min(std::max(py[i], cy0), cy0 + cw);
                const double dx = px[i] - qx, dy = py[i] - qy;
                if (dx * dx + dy * dy <= R[i] * R[i] * (1.0 + 1e-9)) cells[(size_t)y * gx + x].push_back((uint32_t)i);
            }
    }
    RgLightBufDev &B = out.dev;
    B.kind = RG_LB_DIRECTIONAL;
    B.gx = gx;
    B.gy = gy;
    for (int j = 0; j < 3; ++j) {
        B.e1[j] = f1[j];
        B.e2[j] = f2[j];
    }
    B.g0x = g0x;
    B.g0y = g0y;
    B.inv = inv;
    return finish(cells, out);
}

bool build_spherical(const double *sp, int n, const double L[3], double m, RgLightBufBuild &out) {
    if (!finite3(L)) return false;
    const int G = RG_LB_CUBE_G;
    const double wid = RG_LB_MARGINS * std::ldexp(1.0, -12), ang = RG_LB_MARGINS * std::ldexp(1.0, -16),
                 face_min = 1.0 / std::sqrt(3.0) - wid;
    std::vector<std::vector<uint32_t>> cells((size_t)6 * G * G);
    for (int i = 0; i < n; ++i) {
        const double *s = sp + 4 * i;
        const double v[3] = {s[0] - L[0], s[1] - L[1], s[2] - L[2]};
        const double D = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
        const double R = std::fabs(s[3]) * RG_LB_RSCALE + m;
        if (!(D > R * (1.0 + 1e-6) + m)) {  // the light is inside or at the sphere: test it for every ray
            out.ent.push_back((uint32_t)i);
            continue;
        }
        const double th = std::asin(std::min(1.0, R / D)) * (1.0 + 1e-9) + ang;
        double lo[3], hi[3];  // component ranges of the unit directions in the cone's cap
        for (int k = 0; k < 3; ++k) {
            const double al = std::acos(std::min(1.0, std::max(-1.0, v[k] / D)));
            lo[k] = std::cos(std::min(M_PI, al + th)) - RG_LB_MARGINS * 1e-12;
            hi[k] = std::cos(std::max(0.0, al - th)) + RG_LB_MARGINS * 1e-12;
        }
        for (int k = 0; k < 3; ++k) {
            const int i1 = k == 0 ? 1 : 0, i2 = k == 2 ? 1 : 2;  // face coordinates a = x_i1 / |x_k|, b = x_i2 / |x_k|
            for (int sgn = 0; sgn < 2; ++sgn) {
                // s x_k over the cap, limited to the face's region (s x_k >= 1/sqrt(3), less the margin)
                const double xlo = sgn ? -hi[k] : lo[k], xhi = sgn ? -lo[k] : hi[k];
                if (xhi < face_min) continue;
                const double k0 = std::max(xlo, face_min), k1 = xhi;
                auto range = [&](int c, double &rlo, double &rhi) {
                    rlo = std::min(lo[c] / k0, lo[c] / k1) - wid;
                    rhi = std::max(hi[c] / k0, hi[c] / k1) + wid;
                };
                double alo, ahi, blo, bhi;
                range(i1, alo, ahi);
                range(i2, blo, bhi);
                auto cell = [&](double x) { return std::min(G - 1, std::max(0, (int)std::floor((x + 1.0) * (0.5 * G)))); };
                const int a0 = cell(alo), a1 = cell(ahi), b0 = cell(blo), b1 = cell(bhi);
                const int face = 2 * k + sgn;
                for (int b = b0; b <= b1; ++b)
                    for (int a = a0; a <= a1; ++a) cells[((size_t)face * G + b) * G + a].push_back((uint32_t)i);
            }
        }
    }
    RgLightBufDev &B = out.dev;
    B.kind = RG_LB_SPHERICAL;
    B.gx = B.gy = G;
    B.inv = 0.5f * (float)G;
    B.always0 = 0;
    B.always1 = (uint32_t)out.ent.size();  // the always list leads ent
    return finish(cells, out);
}

}  // namespace

bool rg_build_lightbuf(const double *spheres, int n, int kind, const double dn[3], const double pos[3], double extent,
                       double obound, RgLightBufBuild &out) {
    out = RgLightBufBuild{};
    if (n < 1 || !(extent >= 0.0) || !(obound > 0.0) || !std::isfinite(extent + obound)) return false;
    for (int i = 0; i < 4 * n; ++i)
        if (!std::isfinite(spheres[i])) return false;
    const double m = RG_LB_MARGINS * std::ldexp(extent + obound, -16);
    const bool ok = kind == RG_LIGHT_DIRECTIONAL ? build_directional(spheres, n, dn, m, out)
                                                 : build_spherical(spheres, n, pos, m, out);
    if (!ok) out = RgLightBufBuild{};
    return ok;
}
