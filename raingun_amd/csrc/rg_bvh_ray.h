// rg_bvh_ray.h — the f32 ray/box slab test of the BVH traversal, shared by the
// kernel (rg_kernels.hip) and the CPU simulation test (tests/native/bvh_sim.cpp)
// so the host check exercises the very expressions the GPU runs.
//
// Conservativeness (rg_bvh.cpp header): for a ray with |o_k| <= bvh_obound and
// ||d|^2 - 1| <= 1e-13, every child box containing a sphere the exact test can
// accept at t <= tb passes child_hit().  Directions are clamped to
// |d_k| >= 1e-20 so 1/d is finite (no inf*0 NaNs); for a relevant ray that
// only widens the slab interval of a near-parallel axis.
#pragma once
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "rg_device.h"

#if defined(__HIP_DEVICE_COMPILE__)
#define RG_RCPF(x) __builtin_amdgcn_rcpf(x)  // v_rcp_f32: <= 1 ulp, covered by the margin
#define RG_FMAF(a, b, c) __builtin_fmaf(a, b, c)
#else
#define RG_RCPF(x) (1.0f / (x))
#define RG_FMAF(a, b, c) fmaf(a, b, c)
#endif

struct RayB {
    float ix, iy, iz;     // 1 / d (f32)
    float oix, oiy, oiz;  // o * (1 / d)
};

__device__ __forceinline__ float rg_bvh_clamp_dir(float v) {
    const float lim = 1e-20f;
    return fabsf(v) >= lim ? v : (v < 0.0f ? -lim : lim);
}

__device__ __forceinline__ RayB rg_make_rayb(double ox, double oy, double oz, double dx, double dy, double dz) {
    RayB r;
    r.ix = RG_RCPF(rg_bvh_clamp_dir((float)dx));
    r.iy = RG_RCPF(rg_bvh_clamp_dir((float)dy));
    r.iz = RG_RCPF(rg_bvh_clamp_dir((float)dz));
    r.oix = (float)ox * r.ix;
    r.oiy = (float)oy * r.iy;
    r.oiz = (float)oz * r.iz;
    return r;
}

// Smallest float >= t for t >= 0 (t = +inf stays inf).
__device__ __forceinline__ float rg_f32_up(double t) {
    float f = (float)t;
    if ((double)f < t) {
        uint32_t b;
        memcpy(&b, &f, 4);
        ++b;
        memcpy(&f, &b, 4);
    }
    return f;
}

// Slab test of child k of N against [0, tb]; tn = entry distance (f32).
// GROW: the box is grown by g on every side first (far rays, rg_bvh_classify).
template <bool GROW = false>
__device__ __forceinline__ bool rg_child_hit(const RgBvhNode &N, int k, const RayB &r, float tb, float &tn,
                                             float g = 0.0f) {
    const float lx = GROW ? N.lox[k] - g : N.lox[k], hx = GROW ? N.hix[k] + g : N.hix[k];
    const float ly = GROW ? N.loy[k] - g : N.loy[k], hy = GROW ? N.hiy[k] + g : N.hiy[k];
    const float lz = GROW ? N.loz[k] - g : N.loz[k], hz = GROW ? N.hiz[k] + g : N.hiz[k];
    const float tx1 = RG_FMAF(lx, r.ix, -r.oix), tx2 = RG_FMAF(hx, r.ix, -r.oix);
    const float ty1 = RG_FMAF(ly, r.iy, -r.oiy), ty2 = RG_FMAF(hy, r.iy, -r.oiy);
    const float tz1 = RG_FMAF(lz, r.iz, -r.oiz), tz2 = RG_FMAF(hz, r.iz, -r.oiz);
    const float tmin = fmaxf(fmaxf(fminf(tx1, tx2), fminf(ty1, ty2)), fmaxf(fminf(tz1, tz2), 0.0f));
    const float tmax = fminf(fminf(fmaxf(tx1, tx2), fmaxf(ty1, ty2)), fminf(fmaxf(tz1, tz2), tb));
    tn = tmin;
    return tmin <= tmax;
}

// Slab test of one box (threaded layout), same expressions as rg_child_hit.
__device__ __forceinline__ bool rg_box_hit(const float lo[3], const float hi[3], const RayB &r, float tb) {
    const float tx1 = RG_FMAF(lo[0], r.ix, -r.oix), tx2 = RG_FMAF(hi[0], r.ix, -r.oix);
    const float ty1 = RG_FMAF(lo[1], r.iy, -r.oiy), ty2 = RG_FMAF(hi[1], r.iy, -r.oiy);
    const float tz1 = RG_FMAF(lo[2], r.iz, -r.oiz), tz2 = RG_FMAF(hi[2], r.iz, -r.oiz);
    const float tmin = fmaxf(fmaxf(fminf(tx1, tx2), fminf(ty1, ty2)), fmaxf(fminf(tz1, tz2), 0.0f));
    const float tmax = fminf(fminf(fmaxf(tx1, tx2), fmaxf(ty1, ty2)), fminf(fmaxf(tz1, tz2), tb));
    return tmin <= tmax;
}

// Rays the boxes are conservative for as they are (NaN anywhere -> false).
__device__ __forceinline__ bool rg_bvh_ray_ok(float obound, double ox, double oy, double oz, double dx, double dy,
                                              double dz) {
    const double dd = (dx * dx + dy * dy) + dz * dz;
    const double ob = (double)obound;
    return fabs(ox) <= ob && fabs(oy) <= ob && fabs(oz) <= ob && fabs(dd - 1.0) <= 1e-13;
}

enum { RG_BVH_SCAN = 0, RG_BVH_TRAVERSE = 1, RG_BVH_NO_SPHERE = 2 };

// How a ray meets the sphere BVH.  Near rays (rg_bvh_ray_ok) traverse from o
// with grow = 0.  A far origin (|o_k| > obound) is first clipped, in f64,
// against the region R = [-(rbound + grow), rbound + grow]^3 that holds every
// (grown) inflated sphere box: a ray missing R cannot be accepted by any
// sphere's exact test (NO_SPHERE); otherwise the box tests run from
// o' = o + t0s d (|o'_k| <= rbound + grow + m, so the f32 slab bound holds)
// with distances shifted by t0s.  The exact test's rounding slack for this ray,
// s = 3 sqrt(||d|^2 - 1| + 1.8e-15) |c - o| (derivation: rg_bvh.cpp), is
// covered by the stored margin while s <= m/4; beyond that every box is grown
// by grow = s in the slab test (allowed while s <= S, the scene extent, which
// keeps the f32 slab error inside the margin's budget).  NaN/inf, |o| > 1e9 or
// s > S: SCAN.
__device__ __forceinline__ int rg_bvh_classify(float obound, double rbound, double margin, double extent, double ox,
                                               double oy, double oz, double dx, double dy, double dz, double &t0s,
                                               float &grow) {
    t0s = 0.0;
    grow = 0.0f;
    if (rg_bvh_ray_ok(obound, ox, oy, oz, dx, dy, dz)) return RG_BVH_TRAVERSE;
    const double dd = (dx * dx + dy * dy) + dz * dz;
    const double on = sqrt((ox * ox + oy * oy) + oz * oz);
    const double slack = 3.0 * sqrt(fabs(dd - 1.0) + 1.8e-15) * (on + 1.7321 * extent);
    if (!(on <= 1e9) || !(slack <= extent)) return RG_BVH_SCAN;  // also NaN / inf
    double g = 0.0;
    if (slack > 0.25 * margin) {
        g = slack * (1.0 + 1e-6);
        grow = (float)g;
        if ((double)grow < g) grow = nextafterf(grow, __builtin_huge_valf());
        g = (double)grow;
    }
    const double rb = rbound + g;
    double lo = -HUGE_VAL, hi = HUGE_VAL;
    const double o3[3] = {ox, oy, oz}, d3[3] = {dx, dy, dz};
    for (int k = 0; k < 3; ++k) {
        if (d3[k] == 0.0) {
            if (fabs(o3[k]) > rb) return RG_BVH_NO_SPHERE;
            continue;
        }
        const double t1 = (-rb - o3[k]) / d3[k], t2 = (rb - o3[k]) / d3[k];
        lo = fmax(lo, fmin(t1, t2));
        hi = fmin(hi, fmax(t1, t2));
    }
    if (!(hi >= lo) || !(hi >= -margin)) return RG_BVH_NO_SPHERE;
    t0s = fmax(lo - margin, 0.0);
    return RG_BVH_TRAVERSE;
}
