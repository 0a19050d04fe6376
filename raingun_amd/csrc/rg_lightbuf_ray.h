// rg_lightbuf_ray.h — the cell lookup of the shadow-ray light buffers, shared by
// the kernel (rg_kernels.hip) and the CPU check (tests/native/lightbuf_sim.cpp),
// so the host test exercises the very expressions the GPU runs.
//
// A light buffer (rg_lightbuf.cpp, built per light at rg_scene_create) lists,
// per cell of a 2-D grid, every sphere that a shadow ray towards that light
// starting in the cell could hit -- a conservative superset (margins in
// rg_lightbuf.cpp), so testing only the cell's spheres with the reference's
// exact test (bodies.rs:92-119) answers the any-hit query exactly as testing
// all of them (rendering.rs:141-155 -> scene.rs:34-39 on the shadow ray).
//  * Directional light: the shadow ray is o + t dn (dn = normalize(-direction),
//    lights.rs:48, one vector for every ray).  A sphere can be hit only if the
//    ray's line passes within r of its centre, i.e. if the projection of o onto
//    the plane normal to dn lies within r of the projection of c: the grid lives
//    in that plane (basis e1, e2), cell of o = floor((o.e - g0) / cell).
//  * Spherical light at L: the ray runs from o towards L (lights.rs:50-52).  A
//    sphere that meets the segment subtends, seen from L, a cone of half-angle
//    asin(r / |c - L|) that contains the direction of o - L: the grid is a cube
//    map around L, G x G cells per face, indexed by the direction of o - L.
//    Spheres within the margin of L are on an "always" list.
// Rays outside the near-ray bound (|o_k| > bvh_obound) or with non-finite
// values do not use the buffer (rg_lb_cell returns RG_LB_SKIP); the caller then
// takes the BVH walk.
#pragma once
#include <math.h>
#include <stdint.h>

#include "rg_device.h"

#define RG_LB_NONE 0
#define RG_LB_DIRECTIONAL 1
#define RG_LB_SPHERICAL 2
#define RG_LB_SKIP (-2)   // rg_lb_cell: use the BVH instead
#define RG_LB_EMPTY (-1)  // rg_lb_cell: no sphere can occlude this ray

#ifndef RG_LB_MAX_LIGHTS
#define RG_LB_MAX_LIGHTS 8  // lights (in scene order) that get a buffer
#endif

// Per light, 64 B (device array RgKernelArgs::lbuf[n_lbuf]).
struct alignas(16) RgLightBufDev {
    int32_t kind;          // RG_LB_*
    int32_t gx, gy;        // directional: grid cells per axis; spherical: G cells per face edge (gx = gy)
    uint32_t cell_off;     // first of this light's (cells + 1) words in RgKernelArgs::lb_start
    uint32_t always0, always1;  // spherical: lb_ent[always0, always1) are tested for every ray
    float e1[3], e2[3];    // directional: the plane's f32 basis
    float g0x, g0y;        // directional: grid origin in (e1, e2) coordinates
    float inv;             // directional: 1 / cell; spherical: G / 2
    float pad;
};
static_assert(sizeof(RgLightBufDev) == 64, "64-B descriptor");

#if defined(__HIP_DEVICE_COMPILE__)
#define RG_LB_RCPF(x) __builtin_amdgcn_rcpf(x)  // v_rcp_f32 (<= 1 ulp): inside the cube-map margin
#define RG_LB_FMAF(a, b, c) __builtin_fmaf(a, b, c)
#else
#define RG_LB_RCPF(x) (1.0f / (x))
#define RG_LB_FMAF(a, b, c) fmaf(a, b, c)
#endif

__device__ __forceinline__ int rg_lb_clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// Cell of a shadow ray from o towards light L (spherical) or along dn
// (directional): a cell index >= 0 into the light's lb_start words,
// RG_LB_EMPTY when no sphere can occlude it, RG_LB_SKIP when the buffer does not
// cover this ray.  obound: the BVH's near-ray origin bound (the margins assume it).
__device__ __forceinline__ int rg_lb_cell(const RgLightBufDev &B, double lx, double ly, double lz, double ox,
                                          double oy, double oz, float obound) {
    if (!(fabs(ox) <= (double)obound && fabs(oy) <= (double)obound && fabs(oz) <= (double)obound)) return RG_LB_SKIP;
    if (B.kind == RG_LB_DIRECTIONAL) {
        const float fx = (float)ox, fy = (float)oy, fz = (float)oz;
        const float px = RG_LB_FMAF(fz, B.e1[2], RG_LB_FMAF(fy, B.e1[1], fx * B.e1[0]));
        const float py = RG_LB_FMAF(fz, B.e2[2], RG_LB_FMAF(fy, B.e2[1], fx * B.e2[0]));
        const float ux = (px - B.g0x) * B.inv, uy = (py - B.g0y) * B.inv;
        if (!(ux >= 0.0f && uy >= 0.0f && ux < (float)B.gx && uy < (float)B.gy)) return RG_LB_EMPTY;  // NaN: empty too
        const int ix = rg_lb_clampi((int)ux, 0, B.gx - 1), iy = rg_lb_clampi((int)uy, 0, B.gy - 1);
        return iy * B.gx + ix;
    }
    if (B.kind == RG_LB_SPHERICAL) {
        const float vx = (float)(ox - lx), vy = (float)(oy - ly), vz = (float)(oz - lz);
        const float ax = fabsf(vx), ay = fabsf(vy), az = fabsf(vz);
        int face;
        float a, b, m;
        if (ax >= ay && ax >= az) { face = vx < 0.0f ? 1 : 0; m = ax; a = vy; b = vz; }
        else if (ay >= az) { face = vy < 0.0f ? 3 : 2; m = ay; a = vx; b = vz; }
        else { face = vz < 0.0f ? 5 : 4; m = az; a = vx; b = vy; }
        if (!(m >= 1e-30f)) return RG_LB_SKIP;  // o at the light (or NaN): no direction
        const float im = RG_LB_RCPF(m);
        const float ua = RG_LB_FMAF(a * im, B.inv, B.inv), ub = RG_LB_FMAF(b * im, B.inv, B.inv);  // (x + 1) G / 2
        const int G = B.gx;
        const int ia = rg_lb_clampi((int)floorf(ua), 0, G - 1), ib = rg_lb_clampi((int)floorf(ub), 0, G - 1);
        return (face * G + ib) * G + ia;
    }
    return RG_LB_SKIP;
}
