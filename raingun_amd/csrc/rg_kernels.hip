// rg_kernels.hip — the render megakernel for gfx950 (MI355X).
//
// One lane = one pixel.  A wave renders 8x8 pixel tiles (ray coherence) taken
// from a sharded atomic queue.  The reference's recursion
//   render_pixel -> get_color -> {shade_diffuse | cast_ray -> get_color ...}
// (raingun-lib/src/rendering.rs:71-172) becomes a per-lane state machine:
// every loop iteration each live lane owns exactly ONE query ray (closest-hit
// or shadow) and all lanes of the wave walk the body tables together, with a
// wave-uniform body index, so body parameters come in through the scalar
// cache as SGPR operands and the only divergence is in shading.
//
// Post-order evaluation with an explicit frame stack reproduces the
// reference's f32 colour composition bit for bit (same operations, same
// order), so the RGBA8 output is byte-identical to the CPU restatement.
//
// Numerics: -ffp-contract=off (and the pragma below): every f64/f32 multiply
// and add is rounded separately, exactly as the reference's unfused Rust.
// Division and sqrt are the correctly-rounded hipcc expansions.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstddef>
#include <mutex>
#include <type_traits>
#include <utility>
#include <vector>

#include "../../include/raingun.h"
#include "rg_bvh_ray.h"
#include "rg_device.h"
#include "rg_lightbuf_ray.h"

#pragma clang fp contract(off)

namespace rgk {

constexpr double SHADOW_BIAS = 1e-13;                 // lib.rs:11
constexpr float PI_F = 3.14159265358979323846f;       // std::f32::consts::PI

// MODE_WAIT: the lane's top frame awaits a subtree another lane is tracing (task splitting)
enum : int { MODE_CLOSEST = 0, MODE_SHADOW = 1, MODE_DONE = 2, MODE_WAIT = 3, MODE_SHADOW_H = 4 };
// MODE_SHADOW_H: an idle lane tracing one shadow ray for another lane of its wave (shadow fan-out)
// FR_REFR_TASK / FR_REFR_WAIT carry their pool slot in bits 8+ of Frame::type
enum : int { FR_REFL = 0, FR_REFR_T = 1, FR_REFR_R = 2, FR_REFR_TASK = 4, FR_REFR_WAIT = 5 };

struct V3 { double x, y, z; };
struct C3 { float r, g, b; };

__device__ __forceinline__ V3 v3(double x, double y, double z) { return V3{x, y, z}; }
__device__ __forceinline__ V3 add(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ V3 sub(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ V3 scl(V3 a, double s) { return v3(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ V3 neg(V3 a) { return v3(-a.x, -a.y, -a.z); }
__device__ __forceinline__ double dot(V3 a, V3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
__device__ __forceinline__ V3 normalize(V3 a) { return scl(a, 1.0 / sqrt(dot(a, a))); }
__device__ __forceinline__ V3 cross(V3 a, V3 b) {
    return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}

__device__ __forceinline__ C3 c3(float r, float g, float b) { return C3{r, g, b}; }
__device__ __forceinline__ C3 cadd(C3 a, C3 b) { return c3(a.r + b.r, a.g + b.g, a.b + b.b); }
__device__ __forceinline__ C3 cmul(C3 a, C3 b) { return c3(a.r * b.r, a.g * b.g, a.b * b.b); }
__device__ __forceinline__ C3 cscl(C3 a, float s) { return c3(a.r * s, a.g * s, a.b * s); }
__device__ __forceinline__ C3 cclamp(C3 a) {  // color.rs:39-43 (f32::min/max ignore NaN)
    return c3(fmaxf(fminf(a.r, 1.0f), 0.0f), fmaxf(fminf(a.g, 1.0f), 0.0f), fmaxf(fminf(a.b, 1.0f), 0.0f));
}

// Rust `f32 as u8` / `f32 as i32`: truncate, saturate, NaN -> 0.
__device__ __forceinline__ uint32_t f32_to_u8(float v) {
    if (!(v > 0.0f)) return 0u;
    if (v >= 255.0f) return 255u;
    return (uint32_t)v;
}
__device__ __forceinline__ int32_t f32_to_i32(float v) {
    if (v != v) return 0;
    if (v >= 2147483648.0f) return 2147483647;
    if (v < -2147483648.0f) return (-2147483647 - 1);
    return (int32_t)v;
}

// Region visit counts (diagnostic build -DRG_REGION_STATS; scripts/region_stats.py): every time a
// wave enters region k, its first active lane adds 1 to counters[RG_REGION_BASE + 2k] and the
// active lanes to [+ 2k + 1] -- the dynamic weights of the static ISA budget (scripts/isa_budget.py).
// Words 144.. lie in the lines of tile-queue heads 8-15, unused with RG_NQ = 8.
#define RG_REGION_BASE 144
enum : int {
    RGR_LOOP = 0, RGR_PRIM, RGR_PRIM_SPH_TAIL, RGR_PRIM_PLANE_DIV, RGR_GETCOLOR, RGR_NORMAL_SPHERE,
    RGR_BATCH, RGR_TEXEL, RGR_UV_SPHERE, RGR_UV_PLANE, RGR_LIGHT_SPH, RGR_REFRACT, RGR_SHADE, RGR_UNWIND,
    RGR_UNWIND_STEP, RGR_TILE_FETCH, RGR_Q_CLOSEST, RGR_Q_SHADOW, RGR_SH_GROUP, RGR_SH_TAIL, RGR_SH_PLANE,
    RGR_SH_PLANE_DIV, RGR_QC_GROUP, RGR_QC_TAIL, RGR_QC_PLANE, RGR_PRIM_GROUP, RGR_PRIM_PLANE, RGR_DISK, RGR_BOX,
    RGR_PUSH_REFL, RGR_PUSH_REFR, RGR_UNWIND_REFRT, RGR_ERROR, RGR_SH_PAIR, RGR_PRIM_PAIR, RGR_QC_PAIR,
    RGR_WALK, RGR_WALK_LEAF, RGR_LB_SHADOW, RGR_COUNT
};
static_assert(RG_REGION_BASE + 2 * RGR_COUNT <= 16 + 16 * 15, "region counters stay below tile-queue head 15");
#ifdef RG_REGION_STATS
#define RG_REGION(k)                                                                                  \
    do {                                                                                              \
        const unsigned long long m_ = __ballot(1);                                                    \
        if ((int)(threadIdx.x & 63u) == __builtin_ffsll((long long)m_) - 1) {                         \
            atomicAdd(&a.counters[RG_REGION_BASE + 2 * (k)], 1ull);                                   \
            atomicAdd(&a.counters[RG_REGION_BASE + 2 * (k) + 1], (unsigned long long)__builtin_popcountll(m_)); \
        }                                                                                             \
    } while (0)
#else
#define RG_REGION(k) do { } while (0)
#endif

__device__ __forceinline__ void raise_error(const RgKernelArgs &a, uint32_t pixel, int status) {
    RG_REGION(RGR_ERROR);
    // lowest pixel wins: max of the complemented key; 0 (memset) = no error
    unsigned long long key = ((unsigned long long)pixel << 8) | (unsigned long long)(-status);
    atomicMax(&a.counters[3], ~key);
    if (a.err_sticky) atomicMax(a.err_sticky, ~key);  // survives the next launch's counter reset
}

// ---------------------------------------------------------------- closest hit
// Scene::trace (scene.rs:34-39): first minimum in list order.  The body tables
// are grouped by kind, so ties across groups are broken by the YAML index.
struct Closest {
    double t;
    int id;
    int nhit;
    bool nan;
};
__device__ __forceinline__ void closest_init(Closest &c) { c.t = 0.0; c.id = -1; c.nhit = 0; c.nan = false; }
__device__ __forceinline__ void closest_add(Closest &c, double t, int id) {
    c.nhit++;
    if (t != t) c.nan = true;
    if (c.id < 0 || t < c.t || (t == c.t && id < c.id)) { c.t = t; c.id = id; }
}

// Sphere tail after the opp <= r2 test (bodies.rs:105-119).
__device__ __forceinline__ bool sphere_tail(double r2, double opp, double adj, double &t) {
    double th = sqrt(r2 - opp);
    double d0 = adj - th, d1 = adj + th;
    if (d0 < 0.0 && d1 < 0.0) return false;
    t = d0 < 0.0 ? d1 : (d1 < 0.0 ? d0 : fmin(d0, d1));
    return true;
}

struct Ray {
    V3 o, d;
};

// AABB slab test (bodies.rs:242-282).  inv = 1/d, sg = (inv < 0).
__device__ __forceinline__ bool aabb_hit(const RgBox &b, V3 o, V3 inv, int sx, int sy, int sz, double &t) {
    double tmin = ((sx ? b.hi[0] : b.lo[0]) - o.x) * inv.x;
    double tmax = ((sx ? b.lo[0] : b.hi[0]) - o.x) * inv.x;
    double tymin = ((sy ? b.hi[1] : b.lo[1]) - o.y) * inv.y;
    double tymax = ((sy ? b.lo[1] : b.hi[1]) - o.y) * inv.y;
    if (tmin > tymax || tymin > tmax) return false;
    if (tymin > tmin) tmin = tymin;
    if (tymax < tmax) tmax = tymax;
    double tzmin = ((sz ? b.hi[2] : b.lo[2]) - o.z) * inv.z;
    double tzmax = ((sz ? b.lo[2] : b.hi[2]) - o.z) * inv.z;
    if (tmin > tzmax || tzmin > tmax) return false;
    if (tzmin > tmin) tmin = tzmin;
    if (tzmax < tmax) tmax = tzmax;
    if (tmin >= 0.0) { t = tmin; return true; }
    if (tmax >= 0.0) { t = tmax; return true; }
    return false;
}

// Disk (bodies.rs:173-192).
__device__ __forceinline__ bool disk_hit(const RgDsk &k, V3 o, V3 d, double &t) {
    double den = (k.nx * d.x + k.ny * d.y) + k.nz * d.z;
    if (!(den > 1e-6)) return false;
    V3 v = v3(k.ox - o.x, k.oy - o.y, k.oz - o.z);
    double dist = ((v.x * k.nx + v.y * k.ny) + v.z * k.nz) / den;
    if (!(dist >= 0.0)) return false;
    V3 h = add(o, scl(d, dist));
    V3 w = v3(h.x - k.ox, h.y - k.oy, h.z - k.oz);
    if (!(sqrt(dot(w, w)) < k.r)) return false;
    t = dist;
    return true;
}

// ---------------------------------------------------------------- sphere sources
// The sphere tables are read with a wave-uniform index.  Three sources:
//  * SphLds: the persistent block stages the tables into LDS once and every
//    test reads them with broadcast ds_read_b128 (always a hit);
//  * SphScalar: scalar loads through the constant address space (s_load,
//    SGPR operands) for scenes whose tables exceed the LDS budget;
//  * SphNodesLds: the same, but the BVH nodes (read per lane by the per-lane
//    walk: vector loads from global memory otherwise) staged in LDS when the
//    sphere tables do not fit and the nodes do (BASELINE configs[4]: 4,096 spheres).
template <bool NODES_LDS>
struct SphGlobal {
    static constexpr bool in_lds = false;
    const RG_CONST RgSph *s;
    const RG_CONST double *cc;
    const RG_CONST RgSphF *f;
    const RG_CONST RgSphF2 *f2;
    const RG_CONST RgPln *pl;
    const RG_CONST RgDsk *dk;
    const RG_CONST RgBox *bx;
    typename std::conditional<NODES_LDS, const RgBvhNode *, const RG_CONST RgBvhNode *>::type nd;
    const RgLightBufDev *lb = nullptr;  // light-buffer descriptors (global)
    const RgLightDev *lt = nullptr;     // lights (global)
    __device__ __forceinline__ RgBvhNode getn(int i) const { return nd[i]; }
    __device__ __forceinline__ RgBvhNode getn_uniform(int i) const { return nd[i]; }
    __device__ __forceinline__ RgSph getv(int i) const { return ((const RgSph *)s)[i]; }
    __device__ __forceinline__ RgPln getp(int i) const { return pl[i]; }
    __device__ __forceinline__ RgDsk getd(int i) const { return dk[i]; }
    __device__ __forceinline__ RgBox getb(int i) const { return bx[i]; }
    __device__ __forceinline__ RgSph get(int i) const { return s[i]; }
    __device__ __forceinline__ double getcc(int i) const { return cc[i]; }
    __device__ __forceinline__ RgSphF getf(int i) const { return f[i]; }
    __device__ __forceinline__ RgSphF2 getf2(int i) const { return f2[i]; }
};
using SphScalar = SphGlobal<false>;
using SphNodesLds = SphGlobal<true>;
struct SphLds {
    static constexpr bool in_lds = true;
    const RgSph *s;
    const double *cc;
    const RgSphF *f;
    const RgSphF2 *f2;
    const RgPln *pl;
    const RgDsk *dk;
    const RgBox *bx;
    const RgBvhNode *nd;
    const RgLightBufDev *lb = nullptr;  // light-buffer descriptors (LDS copy, hot tables)
    const RgLightDev *lt = nullptr;     // lights (LDS copy)
    __device__ __forceinline__ RgBvhNode getn_uniform(int i) const { return nd[i]; }
    __device__ __forceinline__ RgBvhNode getn(int i) const { return nd[i]; }
    __device__ __forceinline__ RgSph getv(int i) const { return s[i]; }
    __device__ __forceinline__ RgPln getp(int i) const { return pl[i]; }
    __device__ __forceinline__ RgDsk getd(int i) const { return dk[i]; }
    __device__ __forceinline__ RgBox getb(int i) const { return bx[i]; }
    __device__ __forceinline__ RgSph get(int i) const { return s[i]; }
    __device__ __forceinline__ double getcc(int i) const { return cc[i]; }
    __device__ __forceinline__ RgSphF getf(int i) const { return f[i]; }
    __device__ __forceinline__ RgSphF2 getf2(int i) const { return f2[i]; }
};

// ---------------------------------------------------------------- f32 pre-filter
// Heavy scenes first test every sphere in f32 (FMA allowed, 2 cycles per wave
// instruction vs 4 for f64) against an INFLATED threshold, and run the exact
// reference test (f64, unfused, bodies.rs:92-119) only for candidates, so the
// accepted set and every distance are bit-identical to the reference.
//
// Bound (u = 2^-24, P_k = |c_k| + |o_k|, S_pp = sum P_k^2, S_p = sum P_k |d_k|):
// with c, o, d rounded to f32, h = c - o, adj = h.d and hh = h.h as FMA chains
// and opp = fma(-adj, adj, hh):
//   |opp32 - OPP| <= u (8.002 S_pp + 13.004 S_p^2)   (f32 path, vs exact reals)
//   |opp64 - OPP| <= 2^-53 (6.02 S_pp + 10.04 S_p^2) (the reference's f64 path)
// and S_pp <= 2(|c|^2 + |o|^2), S_p^2 <= S_pp |d|^2, hence
//   |opp32 - opp64| <= Kd (|c|^2 + |o|^2),  Kd = u (16.2 + 26.2 |d|^2) (rounded up, +1%).
// "miss" is declared only if opp32 > r2hi + Kd(|c|^2 + |o|^2) with r2hi >= r2
// (rounded up on the host with 4u slack, which also covers the two f32
// roundings of the threshold), so opp64 > r2 there: the exact test would
// reject too.  NaN/inf anywhere makes the comparison false -> candidate.
struct RayF {
    float ox, oy, oz, dx, dy, dz;
    float kd;    // Kd for this ray
    float kdo2;  // Kd * |o|^2 (rounded up)
};
__device__ __forceinline__ RayF make_rayf(V3 o, V3 d) {
    RayF r;
    r.ox = (float)o.x; r.oy = (float)o.y; r.oz = (float)o.z;
    r.dx = (float)d.x; r.dy = (float)d.y; r.dz = (float)d.z;
    const float d2 = (float)dot(d, d) * 1.000001f;   // >= |d|^2
    const float o2 = (float)dot(o, o) * 1.000001f;   // >= |o|^2
    r.kd = 5.9604645e-08f * (16.2f + 26.2f * d2) * 1.01f;
    r.kdo2 = r.kd * o2 * 1.000001f;
    return r;
}
// true: the exact test may accept this sphere (run it); false: certain miss
__device__ __forceinline__ bool filter_general(const RgSphF &f, const RgSphF2 &f2, const RayF &r) {
    const float hx = f.cx - r.ox, hy = f.cy - r.oy, hz = f.cz - r.oz;
    const float adj = __builtin_fmaf(hz, r.dz, __builtin_fmaf(hy, r.dy, hx * r.dx));
    const float hh = __builtin_fmaf(hz, hz, __builtin_fmaf(hy, hy, hx * hx));
    const float opp = __builtin_fmaf(-adj, adj, hh);
    const float thr = __builtin_fmaf(r.kd, f2.cchi, f.r2hi + r.kdo2);
    return !(opp > thr);
}
// primary rays: o = 0 and |d|^2 <= 1.00001, so the threshold is a per-sphere
// constant (thrp, host-precomputed) and h.h = fl32(c.c) (cc32)
__device__ __forceinline__ bool filter_primary(const RgSphF &f, const RgSphF2 &f2, float dx, float dy, float dz) {
    const float adj = __builtin_fmaf(f.cz, dz, __builtin_fmaf(f.cy, dy, f.cx * dx));
    const float opp = __builtin_fmaf(-adj, adj, f2.cc32);
    return !(opp > f2.thrp);
}

#ifndef RG_SPH_GROUP
#define RG_SPH_GROUP 2     // spheres per exact miss-test group (one divergent branch per group)
#endif
#define RG_FILTER_GROUP 4  // spheres per f32-filter group (2 and 8 measured slower)

// Primary rays start at the origin (ray.rs:53): h = c - 0 = c exactly, so
// h.h = c.c is a per-sphere constant (bit-identical): 8 FP64 ops per sphere.
template <int G, class Src>
__device__ __forceinline__ void sph_primary_group(const RgKernelArgs &a, const Src &src, int i, V3 d, Closest &c) {
    RgSph s[G];
    double cc[G], adj[G], opp[G];
    bool cand[G];
    bool any = false;
    RG_REGION(RGR_PRIM_GROUP);
#pragma unroll
    for (int k = 0; k < G; ++k) { s[k] = src.get(i + k); cc[k] = src.getcc(i + k); }
#pragma unroll
    for (int k = 0; k < G; ++k) {
        adj[k] = (s[k].cx * d.x + s[k].cy * d.y) + s[k].cz * d.z;
        opp[k] = cc[k] - adj[k] * adj[k];
        cand[k] = !(opp[k] > s[k].r2);   // bodies.rs:99
        any |= cand[k];
    }
    if (any) {
        RG_REGION(RGR_PRIM_SPH_TAIL);
#pragma unroll
        for (int k = 0; k < G; ++k) {
            double t;
#ifdef RG_REGION_STATS
            if (cand[k]) RG_REGION(RGR_PRIM_PAIR);
#endif
            if (cand[k] && sphere_tail(s[k].r2, opp[k], adj[k], t)) closest_add(c, t, rg_cptr(a.sph_id)[i + k]);
        }
    }
}

// f32-filtered primary group: exact f64 work only for candidate spheres
template <int G, class Src>
__device__ __forceinline__ void sph_primary_group_f(const RgKernelArgs &a, const Src &src, int i, V3 d, float dx,
                                                    float dy, float dz, Closest &c) {
    // the group's filter results are OR-ed into one lane predicate (lane masks
    // stay in SGPRs); the rare candidate branch re-evaluates the filter per
    // sphere instead of keeping G per-lane flags alive
    bool any = false;
#pragma unroll
    for (int k = 0; k < G; ++k) any |= filter_primary(src.getf(i + k), src.getf2(i + k), dx, dy, dz);
    if (any) {
#pragma unroll
        for (int k = 0; k < G; ++k) {
            if (filter_primary(src.getf(i + k), src.getf2(i + k), dx, dy, dz)) {
                const RgSph s = src.get(i + k);
                const double cc = src.getcc(i + k);
                const double adj = (s.cx * d.x + s.cy * d.y) + s.cz * d.z;
                const double opp = cc - adj * adj;
                double t;
                if (!(opp > s.r2) && sphere_tail(s.r2, opp, adj, t)) closest_add(c, t, rg_cptr(a.sph_id)[i + k]);
            }
        }
    }
}

template <bool F32F, class Src>
__device__ __forceinline__ void sph_primary(const RgKernelArgs &a, const Src &src, V3 d, Closest &c) {
    if constexpr (F32F) {
        constexpr int G = RG_FILTER_GROUP;
        const float dx = (float)d.x, dy = (float)d.y, dz = (float)d.z;
        const int n = a.n_sph, nfull = n - n % G;
        int i = 0;
        for (; i < nfull; i += G) sph_primary_group_f<G>(a, src, i, d, dx, dy, dz, c);
        for (; i < n; ++i) sph_primary_group_f<1>(a, src, i, d, dx, dy, dz, c);
        return;
    }
    constexpr int G = RG_SPH_GROUP;
    const int n = a.n_sph, nfull = n - n % G;
    int i = 0;
    for (; i < nfull; i += G) sph_primary_group<G>(a, src, i, d, c);
    for (; i < n; ++i) sph_primary_group<1>(a, src, i, d, c);
}

// General rays: closest-hit (secondary) or any-hit (shadow; see trace_query).
template <int G, class Src>
__device__ __forceinline__ void sph_query_group(const RgKernelArgs &a, const Src &src, int i, V3 o, V3 d,
                                                bool shadow, double ld, Closest &c, bool &occl, bool &need) {
    RgSph s[G];
    double adj[G], opp[G];
    bool cand[G];
    bool any = false;
    RG_REGION(RGR_QC_GROUP);
#pragma unroll
    for (int k = 0; k < G; ++k) s[k] = src.get(i + k);
#pragma unroll
    for (int k = 0; k < G; ++k) {
        double hx = s[k].cx - o.x, hy = s[k].cy - o.y, hz = s[k].cz - o.z;     // bodies.rs:92
        adj[k] = (hx * d.x + hy * d.y) + hz * d.z;                              // :93
        opp[k] = ((hx * hx + hy * hy) + hz * hz) - adj[k] * adj[k];             // :95
        cand[k] = !(opp[k] > s[k].r2);                                          // :97-101
        any |= cand[k];
    }
    if (any && need) {
        RG_REGION(RGR_QC_TAIL);
#pragma unroll
        for (int k = 0; k < G; ++k) {
            double t;
#ifdef RG_REGION_STATS
            if (cand[k]) RG_REGION(RGR_QC_PAIR);
#endif
            if (cand[k] && sphere_tail(s[k].r2, opp[k], adj[k], t)) {
                if (shadow) {
                    if (!(t > ld)) { occl = true; need = false; }
                } else {
                    closest_add(c, t, rg_cptr(a.sph_id)[i + k]);
                }
            }
        }
    }
}

template <int G, class Src>
__device__ __forceinline__ void sph_query_group_f(const RgKernelArgs &a, const Src &src, int i, V3 o, V3 d,
                                                  const RayF &rf, bool shadow, double ld, Closest &c, bool &occl,
                                                  bool &need) {
    bool any = false;
#pragma unroll
    for (int k = 0; k < G; ++k) any |= filter_general(src.getf(i + k), src.getf2(i + k), rf);
    if (any && need) {
#pragma unroll
        for (int k = 0; k < G; ++k) {
            if (need && filter_general(src.getf(i + k), src.getf2(i + k), rf)) {
                const RgSph s = src.get(i + k);
                const double hx = s.cx - o.x, hy = s.cy - o.y, hz = s.cz - o.z;
                const double adj = (hx * d.x + hy * d.y) + hz * d.z;
                const double opp = ((hx * hx + hy * hy) + hz * hz) - adj * adj;
                double t;
                if (!(opp > s.r2) && sphere_tail(s.r2, opp, adj, t)) {
                    if (shadow) {
                        if (!(t > ld)) { occl = true; need = false; }
                    } else {
                        closest_add(c, t, rg_cptr(a.sph_id)[i + k]);
                    }
                }
            }
        }
    }
}

template <bool F32F, class Src>
__device__ __forceinline__ bool sph_query(const RgKernelArgs &a, const Src &src, V3 o, V3 d, bool shadow, double ld,
                                          Closest &c, bool &occl, bool &need) {
    if constexpr (F32F) {
        constexpr int G = RG_FILTER_GROUP;
        const RayF rf = make_rayf(o, d);
        const int n = a.n_sph, nfull = n - n % G;
        int i = 0;
        for (; i < nfull; i += G) {
            sph_query_group_f<G>(a, src, i, o, d, rf, shadow, ld, c, occl, need);
            if (((i / G) & 3) == 3 && !__any(need)) return false;
        }
        for (; i < n; ++i) sph_query_group_f<1>(a, src, i, o, d, rf, shadow, ld, c, occl, need);
        return __any(need);
    }
    constexpr int G = RG_SPH_GROUP;
    const int n = a.n_sph, nfull = n - n % G;
    int i = 0;
    for (; i < nfull; i += G) {
        sph_query_group<G>(a, src, i, o, d, shadow, ld, c, occl, need);
        if (((i / G) & 1) && !__any(need)) return false;
    }
    for (; i < n; ++i) sph_query_group<1>(a, src, i, o, d, shadow, ld, c, occl, need);
    return __any(need);
}

// ---------------------------------------------------------------- BVH traversal
// (the tree is built on the host by rg_bvh.cpp.)  The wave
// walks ONE node at a time: every lane tests the node's child boxes against
// its own ray (f32 slab test, rg_bvh_ray.h), the wave ballots, a leaf hit by
// any lane is tested at once by the lanes whose box test passed (f32 sphere
// pre-filter, then the reference's f64 test), and the internal children hit by
// any lane are visited depth-first, nearest first by the first active lane's
// entry distance, through a wave-uniform stack in LDS (one 64-entry stack per
// wave, written by the first active lane).  Boxes only cull spheres the exact
// test would reject or whose hit cannot be <= the lane's current best (closest
// hit) or light distance (shadow), and closest_add is order-independent, so the
// result and every distance equal the brute-force scan.  Lanes whose ray is
// outside the boxes' error analysis (rg_bvh_ray_ok) or whose closest-hit query
// already saw a NaN distance (AABB; nhit must stay exact) use the brute-force
// loop instead.
#define RG_BVH_STACK 64
#define RG_BVH_MAX_WAVES 16   // waves per block on the BVH path (256 * RG_HEAVY_WPS threads)
__shared__ int rg_bvh_stack[RG_BVH_MAX_WAVES][RG_BVH_STACK];  // allocated only by kernels that traverse

__device__ __forceinline__ int wave_uniform(int v) { return __builtin_amdgcn_readfirstlane(v); }

// Diagnostic build (-DRG_BVH_STATS): counters[4..15] = traversals, node visits,
// leaf visits (per wave), lanes traversing, lanes scanning all spheres (any
// reason), ... by reason (origin out of bound, |d| not unit, NaN), wave clock
// cycles in traversals, in full scans, in the whole kernel, waves.
#ifdef RG_BVH_STATS
// accumulated per wave in LDS (cheap), flushed to counters[] once per wave
__shared__ unsigned long long rg_stat_lds[RG_BVH_MAX_WAVES][16];
#define RG_STAT(word, v)                                                                        \
    do {                                                                                        \
        const unsigned long long rg_stat_v = (unsigned long long)(v);                           \
        if ((threadIdx.x & 63u) == (unsigned)__builtin_amdgcn_readfirstlane(threadIdx.x & 63u)) \
            rg_stat_lds[(threadIdx.x >> 6) % RG_BVH_MAX_WAVES][word] += rg_stat_v;              \
    } while (0)
#define RG_LANES(pred) __builtin_popcountll(__ballot(pred))
#define RG_CLOCK() ((unsigned long long)wall_clock64())
#else
#define RG_STAT(word, v) do { } while (0)
#define RG_LANES(pred) 0
#define RG_CLOCK() 0ull
#endif
__device__ __forceinline__ float wave_uniform_f(float v) {
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}

template <class Src>
__device__ __forceinline__ void leaf_primary(const RgKernelArgs &a, const Src &src, int first, int count, V3 d,
                                             float dx, float dy, float dz, Closest &c) {
    for (int j = first; j < first + count; ++j) {
        const RgSphF2 f2 = src.getf2(j);
        if (filter_primary(src.getf(j), f2, dx, dy, dz)) {
            const RgSph s = src.get(j);
            const double cc = src.getcc(j);
            const double adj = (s.cx * d.x + s.cy * d.y) + s.cz * d.z;
            const double opp = cc - adj * adj;
            double t;
            if (!(opp > s.r2) && sphere_tail(s.r2, opp, adj, t)) closest_add(c, t, f2.id);
        }
    }
}

template <class Src>
__device__ __forceinline__ void leaf_query(const RgKernelArgs &a, const Src &src, int first, int count, V3 o, V3 d,
                                           const RayF &rf, bool shadow, double ld, Closest &c, bool &occl,
                                           bool &need) {
    for (int j = first; j < first + count; ++j) {
        // the id comes with the filter record (RgSphF2::id): a per-lane j (bvh_lane) would
        // otherwise make sph_id[j] a vector global load whose latency the hit waits for
        const RgSphF f = src.getf(j);
        const RgSphF2 f2 = src.getf2(j);
        if (need && filter_general(f, f2, rf)) {
            const RgSph s = src.get(j);
            const double hx = s.cx - o.x, hy = s.cy - o.y, hz = s.cz - o.z;
            const double adj = (hx * d.x + hy * d.y) + hz * d.z;
            const double opp = ((hx * hx + hy * hy) + hz * hz) - adj * adj;
            double t;
            if (!(opp > s.r2) && sphere_tail(s.r2, opp, adj, t)) {
                if (shadow) {
                    if (!(t > ld)) { occl = true; need = false; }
                } else {
                    closest_add(c, t, f2.id);
                }
            }
        }
    }
}

// KIND 0: primary ray (o = 0); 1: a query, per lane closest hit or (`shadow`)
// any hit with t <= ld -- closest-hit and shadow lanes of a wave share ONE walk
// instead of running one walk per kind one after the other.
// Called by the lanes that take the BVH (exec mask); `need` drops for a
// shadow lane at its first occluder.  The box tests start at o + t0s d
// (t0s > 0 only for far origins, rg_bvh_classify) and prune against
// distances shifted by t0s; the exact sphere tests use the ray as given.
__device__ __forceinline__ float bvh_bound(double v) { return v <= 0.0 ? 0.0f : rg_f32_up(v); }

template <int KIND, bool GROW = false, class Src>
__device__ __forceinline__ void bvh_spheres(const RgKernelArgs &a, const Src &src, V3 o, V3 d, bool shadow, double ld,
                                            double t0s, Closest &c, bool &occl, bool &need, float grow = 0.0f) {
    int *stack = rg_bvh_stack[threadIdx.x >> 6];
    const V3 ob = t0s > 0.0 ? add(o, scl(d, t0s)) : o;
    const RayB rb = rg_make_rayb(ob.x, ob.y, ob.z, d.x, d.y, d.z);
    RayF rf;
    const float dx = (float)d.x, dy = (float)d.y, dz = (float)d.z;
    if constexpr (KIND != 0) rf = make_rayf(o, d);
    const float tld = shadow ? bvh_bound(ld - t0s) : 0.0f;
    const int lane = (int)(threadIdx.x & 63u);
    const bool writer = lane == wave_uniform(lane);
    int sp = 0;
    int node = 0;
    RG_STAT(4, 1);
    RG_STAT(7, RG_LANES(1));
    [[maybe_unused]] const unsigned long long t_in = RG_CLOCK();
    for (;;) {
        RG_STAT(5, 1);
        const RgBvhNode N = src.getn_uniform(node);
        const int nch = wave_uniform(N.nchild);
        const float tb = shadow ? tld : (c.id >= 0 ? bvh_bound(c.t - t0s) : __builtin_huge_valf());
        int next = -1;
        float next_key = 0.0f;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (k < nch) {
                float tn = 0.0f;
                const bool h = need && rg_child_hit<GROW>(N, k, rb, tb, tn, grow);
                if (__any(h)) {
                    const int ch = wave_uniform(N.child[k]);
                    if (ch < 0) {
                        const int v = ~ch, first = v >> 3, count = (v & 7) + 1;
                        RG_STAT(6, 1);
                        if (h) {
                            if constexpr (KIND == 0) leaf_primary(a, src, first, count, d, dx, dy, dz, c);
                            else leaf_query(a, src, first, count, o, d, rf, shadow, ld, c, occl, need);
                        }
                    } else {
                        const float key = wave_uniform_f(h ? tn : __builtin_huge_valf());
                        int push = ch;
                        if (next < 0 || key < next_key) {
                            push = next;
                            next = ch;
                            next_key = key;
                        }
                        if (push >= 0 && sp < RG_BVH_STACK) {
                            if (writer) stack[sp] = push;
                            ++sp;
                        }
                    }
                }
            }
        }
        if constexpr (KIND != 0) {
            if (!__any(need)) break;  // every shadow lane occluded (closest-hit lanes keep `need`)
        }
        if (next >= 0) {
            node = next;
        } else {
            if (sp == 0) break;
            --sp;
            node = wave_uniform(stack[sp]);
        }
    }
    RG_STAT(12, RG_CLOCK() - t_in);
}

// Per-lane traversal for incoherent rays (secondary rays and the shadow rays
// of their hits).  The wave-coherent walk above visits the UNION of its lanes'
// paths; for 64 rays in 64 directions that is most of the tree, so every lane
// here walks its own path: nearest-first over the same 4-wide nodes (per-lane
// LDS gathers), the other hit children on a per-lane stack in LDS
// (RG_LANE_NODE_BITS entry format, rg_device.h), each popped entry skipped when
// its stored entry distance -- a lower bound -- already exceeds the current
// bound, exactly as a fresh slab test against that bound would skip it.  Same
// boxes, bounds and leaf tests (f32 pre-filter, then the exact f64 test) as
// bvh_spheres, so the accepted set and every distance are identical.  The host
// sizes the stack to the tree's worst case (rg_bvh.cpp lane_stack_need).
extern __shared__ __attribute__((aligned(16))) unsigned char rg_dyn_smem[];

__device__ __forceinline__ uint32_t lane_key(float tn, int node) {
    return (__float_as_uint(tn) & ~((1u << RG_LANE_NODE_BITS) - 1u)) | (uint32_t)node;
}
__device__ __forceinline__ float lane_key_t(uint32_t e) {
    return __uint_as_float(e & ~((1u << RG_LANE_NODE_BITS) - 1u));
}
__device__ __forceinline__ void cswap(uint32_t &x, uint32_t &y) {
    const uint32_t lo = min(x, y), hi = max(x, y);
    x = lo;
    y = hi;
}

template <class Src>
__device__ __forceinline__ void bvh_lane(const RgKernelArgs &a, const Src &src, V3 o, V3 d, bool shadow, double ld,
                                         double t0s, Closest &c, bool &occl, bool &need) {
    uint32_t *stk = reinterpret_cast<uint32_t *>(rg_dyn_smem) + threadIdx.x;  // entry e at stk[e * blockDim.x]
    const uint32_t stride = blockDim.x;
    const uint32_t mask = (1u << RG_LANE_NODE_BITS) - 1u;
    const V3 ob = t0s > 0.0 ? add(o, scl(d, t0s)) : o;
    const RayB rb = rg_make_rayb(ob.x, ob.y, ob.z, d.x, d.y, d.z);
    const RayF rf = make_rayf(o, d);
    const float tld = shadow ? bvh_bound(ld - t0s) : 0.0f;
    int node = 0;
    RG_STAT(4, 1);
    RG_STAT(7, RG_LANES(1));
    [[maybe_unused]] const unsigned long long t_in = RG_CLOCK();
    // slot `cap` is a spare: a write that is not a push may land there, never on an entry;
    // the stack pointer is kept scaled by the stride (spo = sp * stride: no multiplies)
    const uint32_t capo = (uint32_t)a.lane_stack * stride;
    uint32_t spo = 0u;
    for (;;) {
        const bool act = need && node >= 0;
        if (!__any(act)) break;
        RG_STAT(5, 1);
#ifdef RG_ITER_STATS  // per-lane walk: iterations, active lanes (counters[12..13])
        {
            const unsigned long long m = __ballot(act);
            if ((int)(threadIdx.x & 63u) == __builtin_ffsll((long long)__ballot(1)) - 1) {
                atomicAdd(&a.counters[12], 1ull);
                atomicAdd(&a.counters[13], (unsigned long long)__builtin_popcountll(m));
            }
        }
#endif
        if (act) {
            RG_REGION(RGR_WALK);  // per-lane walk iteration (heavy path)
            // the node's children without divergent branches: every slot's slab test,
            // hit leaves as a bit mask (tested below in child order), hit internal
            // children as sort keys (~0: none), pushes written unconditionally
            const RgBvhNode N = src.getn(node);
            const float tb = shadow ? tld : (c.id >= 0 ? bvh_bound(c.t - t0s) : __builtin_huge_valf());
            uint32_t e[4], leaves = 0u;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                float tn = 0.0f;
                const bool h = (k < N.nchild) & rg_child_hit(N, k, rb, tb, tn);
                const int ch = N.child[k];
                leaves |= (h & (ch < 0)) ? (1u << k) : 0u;
                e[k] = (h & (ch >= 0)) ? lane_key(tn, ch) : ~0u;
            }
            // leaves first (they tighten a closest-hit bound), in child order
            while (leaves != 0u && need) {
                RG_REGION(RGR_WALK_LEAF);
                const uint32_t k = (uint32_t)__builtin_ctz(leaves);
                leaves &= leaves - 1u;
                const int v = ~(k == 0u ? N.child[0] : k == 1u ? N.child[1] : k == 2u ? N.child[2] : N.child[3]);
                leaf_query(a, src, v >> 3, (v & 7) + 1, o, d, rf, shadow, ld, c, occl, need);
            }
            uint32_t e0 = e[0], e1 = e[1], e2 = e[2], e3 = e[3];
            // ascending (entry distance, node); empty slots (~0) last
            cswap(e0, e1); cswap(e2, e3); cswap(e0, e2); cswap(e1, e3); cswap(e1, e2);
            stk[min(spo, capo)] = e3;
            spo += ((e3 != ~0u) & (spo < capo)) ? stride : 0u;
            stk[min(spo, capo)] = e2;
            spo += ((e2 != ~0u) & (spo < capo)) ? stride : 0u;
            stk[min(spo, capo)] = e1;
            spo += ((e1 != ~0u) & (spo < capo)) ? stride : 0u;
            const float tbn = shadow ? tld : (c.id >= 0 ? bvh_bound(c.t - t0s) : __builtin_huge_valf());
            if (e0 != ~0u && (shadow || !(lane_key_t(e0) > tbn))) {
                node = (int)(e0 & mask);
            } else {
                node = -1;
                while (spo > 0u && need) {
                    spo -= stride;
                    const uint32_t e = stk[spo];
                    if (shadow || !(lane_key_t(e) > tbn)) {
                        node = (int)(e & mask);
                        break;
                    }
                }
            }
        }
    }
    RG_STAT(13, RG_CLOCK() - t_in);  // per-lane walk: word 13 (with the rare full scans)
}

// Light buffers (rg_lightbuf_ray.h, rg_lightbuf.cpp) in two steps, so the list bounds' load is in
// flight while the plane/disk/box tests run: lbuf_begin finds the ray's cell and loads its list
// bounds, lbuf_finish tests the list's spheres (and the always list), each with the leaf tests' f32
// pre-filter and exact test.  The lists hold every sphere the exact test could accept for the ray,
// so the answer is the BVH walk's; use == false: the buffer does not cover this ray (origin beyond
// the near-ray bound, no direction) and the caller walks the BVH.
struct LbRange {
    uint32_t k0, k1;  // the cell's entries (k0 == k1: an empty cell)
    bool use;
};
template <class Src>
__device__ __forceinline__ LbRange lbuf_begin(const RgKernelArgs &a, const Src &src, int buf, V3 o, double lx,
                                              double ly, double lz) {
    LbRange r{0u, 0u, false};
    const RgLightBufDev &B = src.lb[buf];
    if (B.kind == RG_LB_NONE) return r;
    const int cell = rg_lb_cell(B, lx, ly, lz, o.x, o.y, o.z, a.bvh_obound);
    if (cell == RG_LB_SKIP) return r;
    r.use = true;
    if (cell >= 0) {
        const uint32_t *st = a.lb_start + B.cell_off + (uint32_t)cell;
        r.k0 = st[0];
        r.k1 = st[1];
    }
    return r;
}
// the light's position for a spherical light's buffer (directional: unused)
template <class Src>
__device__ __forceinline__ V3 lbuf_light_pos(const Src &src, int light) {
    const RgLightDev &L = src.lt[light];
    return v3(L.v[0], L.v[1], L.v[2]);
}

// Shadow ray of `light`: any hit with t <= ld among the listed spheres
template <class Src>
__device__ __forceinline__ void lbuf_shadow(const RgKernelArgs &a, const Src &src, int light, const LbRange &r, V3 o,
                                            V3 d, double ld, bool &occl, bool &need) {
    const RgLightBufDev &B = src.lb[light];
    RG_REGION(RGR_LB_SHADOW);
    const RayF rf = make_rayf(o, d);
    Closest unused;
    closest_init(unused);
    for (uint32_t k = B.always0; k < B.always1 && need; ++k)
        leaf_query(a, src, (int)a.lb_ent[k], 1, o, d, rf, true, ld, unused, occl, need);
    // the list's entries four at a time: their loads in flight together, not one round trip per sphere
    for (uint32_t k = r.k0; k < r.k1 && need; k += 4) {
        uint32_t j[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) j[i] = a.lb_ent[min(k + (uint32_t)i, r.k1 - 1u)];
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (k + (uint32_t)i < r.k1 && need) leaf_query(a, src, (int)j[i], 1, o, d, rf, true, ld, unused, occl, need);
    }
}

// Primary ray through the camera buffer (a light buffer around the camera at the origin, ray.rs:53:
// every primary ray starts there; closest hit, order-independent rule)
template <class Src>
__device__ __forceinline__ void cambuf_primary(const RgKernelArgs &a, const Src &src, const LbRange &r, V3 d, float dx,
                                               float dy, float dz, Closest &c) {
    const RgLightBufDev &B = src.lb[a.lb_cam];
    for (uint32_t k = B.always0; k < B.always1; ++k) leaf_primary(a, src, (int)a.lb_ent[k], 1, d, dx, dy, dz, c);
    for (uint32_t k = r.k0; k < r.k1; k += 4) {
        uint32_t j[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) j[i] = a.lb_ent[min(k + (uint32_t)i, r.k1 - 1u)];
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (k + (uint32_t)i < r.k1) leaf_primary(a, src, (int)j[i], 1, d, dx, dy, dz, c);
    }
}

template <bool F32F, bool BVH, class Src>
__device__ __forceinline__ void trace_primary(const RgKernelArgs &a, const Src &src, V3 d, Closest &c) {
    if constexpr (!BVH) sph_primary<F32F>(a, src, d, c);
    // the camera buffer's list bounds, loaded while the other bodies are tested
    [[maybe_unused]] LbRange cam{0u, 0u, false};
    if constexpr (BVH) {
        if (a.lb_cam >= 0) cam = lbuf_begin(a, src, a.lb_cam, d, 0.0, 0.0, 0.0);
    }
    for (int i = 0; i < a.n_pln; ++i) {
        RG_REGION(RGR_PRIM_PLANE);
        const RgPln p = src.getp(i);
        double den = (p.nx * d.x + p.ny * d.y) + p.nz * d.z;   // bodies.rs:137
        if (den > 1e-6) {
            RG_REGION(RGR_PRIM_PLANE_DIV);
            double dist = p.on / den;                           // v = o_p - 0 = o_p: v.n = o.n
            if (dist >= 0.0) closest_add(c, dist, rg_cptr(a.pln_id)[i]);
        }
    }
    const V3 o = v3(0.0, 0.0, 0.0);
    for (int i = 0; i < a.n_dsk; ++i) {
        RG_REGION(RGR_DISK);
        const RgDsk k = src.getd(i);
        double t;
        if (disk_hit(k, o, d, t)) closest_add(c, t, rg_cptr(a.dsk_id)[i]);
    }
    if (a.n_box > 0) {
        RG_REGION(RGR_BOX);
        V3 inv = v3(1.0 / d.x, 1.0 / d.y, 1.0 / d.z);           // ray.rs:24
        int sx = inv.x < 0.0, sy = inv.y < 0.0, sz = inv.z < 0.0;
        for (int i = 0; i < a.n_box; ++i) {
            RG_REGION(RGR_BOX);
            const RgBox b = src.getb(i);
            double t;
            if (aabb_hit(b, o, inv, sx, sy, sz, t)) closest_add(c, t, rg_cptr(a.box_id)[i]);
        }
    }
    if constexpr (BVH) {  // spheres last: the other bodies' hits already bound the search
        const bool ok = !c.nan && rg_bvh_ray_ok(a.bvh_obound, 0.0, 0.0, 0.0, d.x, d.y, d.z);
        RG_STAT(8, RG_LANES(!ok));
        if (!ok) {
            [[maybe_unused]] const unsigned long long t0 = RG_CLOCK();
            sph_primary<F32F>(a, src, d, c);
            RG_STAT(13, RG_CLOCK() - t0);
        }
        const bool walk = ok && !cam.use;
        if (ok && cam.use) cambuf_primary(a, src, cam, d, (float)d.x, (float)d.y, (float)d.z, c);
        if (walk) {
            bool need = true, unused = false;
            bvh_spheres<0>(a, src, o, d, false, 0.0, 0.0, c, unused, need);
        }
    }
}

// General query: closest-hit for secondary rays, any-hit for shadow rays.
// A shadow ray is occluded iff some body has a hit distance t with
// !(t > light_distance)  <=>  !(min t > light_distance)  (rendering.rs:152-155),
// so a lane stops testing at its first such hit and the wave leaves the body
// loops as soon as every lane that is still testing is a finished shadow ray.
template <bool F32F, bool BVH, class Src>
__device__ __forceinline__ void trace_query(const RgKernelArgs &a, const Src &src, const Ray &r, bool shadow, double ld,
                                            Closest &c, bool &occl, bool lane_walk = false, int light = -1) {
    const V3 o = r.o, d = r.d;
    bool need = true;
    if constexpr (!BVH) {
        if (!sph_query<F32F>(a, src, o, d, shadow, ld, c, occl, need)) return;
    }
    // shadow rays of a light with a buffer: the ray's list bounds, loaded while the planes,
    // disks and boxes are tested
    [[maybe_unused]] LbRange lbr{0u, 0u, false};
    if constexpr (BVH) {
        if (shadow && light >= 0 && light < a.n_lbuf) {
            const V3 lp = lbuf_light_pos(src, light);
            lbr = lbuf_begin(a, src, light, o, lp.x, lp.y, lp.z);
        }
    }
    for (int i = 0; i < a.n_pln; ++i) {
        const RgPln p = src.getp(i);
        double den = (p.nx * d.x + p.ny * d.y) + p.nz * d.z;   // bodies.rs:137-148
        RG_REGION(RGR_QC_PLANE);
        if (den > 1e-6 && need) {
            double vx = p.ox - o.x, vy = p.oy - o.y, vz = p.oz - o.z;
            double dist = ((vx * p.nx + vy * p.ny) + vz * p.nz) / den;
            if (dist >= 0.0) {
                if (shadow) {
                    if (!(dist > ld)) { occl = true; need = false; }
                } else {
                    closest_add(c, dist, rg_cptr(a.pln_id)[i]);
                }
            }
        }
    }
    if (!__any(need)) return;
    for (int i = 0; i < a.n_dsk; ++i) {
        RG_REGION(RGR_DISK);
        const RgDsk k = src.getd(i);
        double t;
        if (need && disk_hit(k, o, d, t)) {
            if (shadow) {
                if (!(t > ld)) { occl = true; need = false; }
            } else {
                closest_add(c, t, rg_cptr(a.dsk_id)[i]);
            }
        }
    }
    if (a.n_box > 0 && __any(need)) {
        RG_REGION(RGR_BOX);
        V3 inv = v3(1.0 / d.x, 1.0 / d.y, 1.0 / d.z);
        int sx = inv.x < 0.0, sy = inv.y < 0.0, sz = inv.z < 0.0;
        for (int i = 0; i < a.n_box; ++i) {
            RG_REGION(RGR_BOX);
            const RgBox b = src.getb(i);
            double t;
            if (need && aabb_hit(b, o, inv, sx, sy, sz, t)) {
                if (shadow) {
                    if (!(t > ld)) { occl = true; need = false; }
                } else {
                    closest_add(c, t, rg_cptr(a.box_id)[i]);
                }
            }
        }
    }
    if constexpr (BVH) {  // spheres last: plane/disk/box hits already bound the search
        if (!__any(need)) return;
        double t0s = 0.0;
        float grow = 0.0f;
        const int cls = (need && !c.nan) ? rg_bvh_classify(a.bvh_obound, a.bvh_rbound, a.bvh_margin, a.bvh_extent,
                                                           o.x, o.y, o.z, d.x, d.y, d.z, t0s, grow)
                                         : RG_BVH_SCAN;
        // shadow rays of a light with a light buffer: their cell's spheres instead of the walk (near rays)
        const bool lb = shadow && need && cls == RG_BVH_TRAVERSE && grow == 0.0f && lbr.use;
        if (lb) lbuf_shadow(a, src, light, lbr, o, d, ld, occl, need);
        const bool ok = need && cls == RG_BVH_TRAVERSE && !lb;
#ifdef RG_BVH_STATS
        {
            RG_STAT(8, RG_LANES(need && cls == RG_BVH_SCAN));
            RG_STAT(9, RG_LANES(need && cls == RG_BVH_TRAVERSE && grow > 0.0f));
            RG_STAT(10, RG_LANES(need && cls == RG_BVH_NO_SPHERE));
            RG_STAT(11, RG_LANES(need && c.nan));
        }
#endif
        if (need && cls == RG_BVH_SCAN) {
            [[maybe_unused]] const unsigned long long t0 = RG_CLOCK();
            bool nd = true;
            sph_query<F32F>(a, src, o, d, shadow, ld, c, occl, nd);
            RG_STAT(13, RG_CLOCK() - t0);
        }
        const bool grown = ok && grow > 0.0f;  // far rays: boxes grown in the slab test
        // one walk kind per wave: if any lane's ray is incoherent, every near lane walks per lane
        // (a mixed wave would otherwise run the per-lane walk and then the wave walk)
        const bool per_lane = ok && !grown && a.lane_stack > 0 && __any(ok && !grown && lane_walk);
        if (per_lane) bvh_lane(a, src, o, d, shadow, ld, t0s, c, occl, need);
        if (ok && !grown && !per_lane) {
            bvh_spheres<1>(a, src, o, d, shadow, ld, t0s, c, occl, need);
        }
        if (grown) {
            bvh_spheres<1, true>(a, src, o, d, shadow, ld, t0s, c, occl, need, grow);
        }
    }
}

// A query ray whose arithmetic may overflow.  With every scene coordinate
// below 1e100 in magnitude (the host's `nan_scene` test, rg_capi.hip), a ray
// with |o_k| < 1e100 and |d_k| < 1e50 keeps every intermediate of the body
// tests (bodies.rs:92-119, 136-148, 173-192, 242-282) finite, so no hit
// distance can be NaN and Scene::trace's `partial_cmp().unwrap()`
// (scene.rs:38) cannot panic.  Anything else (NaN/inf included: the
// comparisons are false) is exotic and takes the exact, fully counted query.
__device__ __forceinline__ bool ray_exotic(V3 o, V3 d) {
    const bool ok = fabs(o.x) < 1e100 && fabs(o.y) < 1e100 && fabs(o.z) < 1e100 && fabs(d.x) < 1e50 &&
                    fabs(d.y) < 1e50 && fabs(d.z) < 1e50;
    return !ok;
}

// ---------------------------------------------------------------- shadow batches
// shade_diffuse traces one shadow ray per light from the SAME origin
// hit + n*bias (rendering.rs:141-150).  A lane traces up to RG_LB of them in
// one pass: per sphere the origin-dependent part (h = c - o, h.h) is computed
// once and only adj/opp/compare are per light, so a 3-light batch costs
// 8 + 3*8 FP64 ops per sphere instead of 3*16, with bit-identical per-ray
// arithmetic.  Bit l of `occl` = light l of the batch is occluded.
// RG_LB (lights per shadow batch on the light path) lives in rg_device.h
#ifndef RG_SHADOW_GROUP
#define RG_SHADOW_GROUP 2  // spheres per miss-test group in the shadow pass
#endif

template <int LB>
struct ShadowBatch {
    V3 d[LB];           // direction_from(light) (lights.rs:46-51)
    double ld[LB];      // light.distance(hit) (lights.rs:53-58), +inf for directional
};

template <int LB, class Src>
__device__ __forceinline__ void trace_shadow(const RgKernelArgs &a, const Src &src, V3 o, const ShadowBatch<LB> &sb,
                                             uint32_t full, uint32_t &occl) {
    constexpr int G = RG_SHADOW_GROUP;
    const int n = a.n_sph, nfull = n - n % G;
    for (int i = 0; i < n;) {
        const int g = i < nfull ? G : 1;  // wave-uniform
        RG_REGION(RGR_SH_GROUP);
        RgSph s[G];
        double hx[G], hy[G], hz[G], hh[G], adj[G][LB], opp[G][LB];
        bool cand[G][LB];
        bool any = false;
#pragma unroll
        for (int k = 0; k < G; ++k) {
            if (k < g) {
                s[k] = src.get(i + k);
                hx[k] = s[k].cx - o.x; hy[k] = s[k].cy - o.y; hz[k] = s[k].cz - o.z;   // bodies.rs:92
                hh[k] = (hx[k] * hx[k] + hy[k] * hy[k]) + hz[k] * hz[k];                // :95 (first term)
#pragma unroll
                for (int l = 0; l < LB; ++l) {
                    adj[k][l] = (hx[k] * sb.d[l].x + hy[k] * sb.d[l].y) + hz[k] * sb.d[l].z;   // :93
                    opp[k][l] = hh[k] - adj[k][l] * adj[k][l];                               // :95
                    cand[k][l] = !(opp[k][l] > s[k].r2) && !((occl >> l) & 1u);              // :99
                    any |= cand[k][l];
                }
            }
        }
        if (any) {
            RG_REGION(RGR_SH_TAIL);
#pragma unroll
            for (int k = 0; k < G; ++k) {
#pragma unroll
                for (int l = 0; l < LB; ++l) {
                    double t;
#ifdef RG_REGION_STATS
                    if (k < g && cand[k][l]) RG_REGION(RGR_SH_PAIR);
#endif
                    if (k < g && cand[k][l] && sphere_tail(s[k].r2, opp[k][l], adj[k][l], t) && !(t > sb.ld[l]))
                        occl |= 1u << l;
                }
            }
        }
        i += g;
        if ((i & 7) == 0 && !__any(occl != full)) return;
    }
    if (!__any(occl != full)) return;
    for (int i = 0; i < a.n_pln; ++i) {
        const RgPln p = src.getp(i);
        const double vx = p.ox - o.x, vy = p.oy - o.y, vz = p.oz - o.z;     // bodies.rs:139
        const double num = (vx * p.nx + vy * p.ny) + vz * p.nz;             // :140 numerator
        RG_REGION(RGR_SH_PLANE);
#pragma unroll
        for (int l = 0; l < LB; ++l) {
            const double den = (p.nx * sb.d[l].x + p.ny * sb.d[l].y) + p.nz * sb.d[l].z;  // :137
            if (den > 1e-6 && !((occl >> l) & 1u)) {
                bool hit;
                if (sb.ld[l] == __builtin_inf() && num >= 0.0) {
                    hit = true;  // fl(num/den) >= 0 and !(fl(num/den) > inf): no division needed
                } else {
                    RG_REGION(RGR_SH_PLANE_DIV);
                    const double dist = num / den;
                    hit = dist >= 0.0 && !(dist > sb.ld[l]);
                }
                if (hit) occl |= 1u << l;
            }
        }
    }
    if (!__any(occl != full)) return;
    for (int i = 0; i < a.n_dsk; ++i) {
        RG_REGION(RGR_DISK);
        const RgDsk k = src.getd(i);
#pragma unroll
        for (int l = 0; l < LB; ++l) {
            double t;
            if (!((occl >> l) & 1u) && disk_hit(k, o, sb.d[l], t) && !(t > sb.ld[l])) occl |= 1u << l;
        }
    }
    if (a.n_box > 0 && __any(occl != full)) {
        RG_REGION(RGR_BOX);
#pragma unroll
        for (int l = 0; l < LB; ++l) {
            const V3 d = sb.d[l];
            const V3 inv = v3(1.0 / d.x, 1.0 / d.y, 1.0 / d.z);
            const int sx = inv.x < 0.0, sy = inv.y < 0.0, sz = inv.z < 0.0;
            for (int i = 0; i < a.n_box; ++i) {
                RG_REGION(RGR_BOX);
                const RgBox b = src.getb(i);
                double t;
                if (!((occl >> l) & 1u) && aabb_hit(b, o, inv, sx, sy, sz, t) && !(t > sb.ld[l])) occl |= 1u << l;
            }
        }
    }
}

// ---------------------------------------------------------------- shading
__device__ __forceinline__ V3 bp3(const RgBodyDev &b, int k) { return v3(b.p[k], b.p[k + 1], b.p[k + 2]); }

// bodies.rs:122-124, 151-153, 194-196, 284-328.  false = the AABB assert.
__device__ __forceinline__ bool surface_normal(const RgBodyDev &b, V3 h, V3 &n) {
    if (b.kind == RG_BODY_SPHERE) { n = normalize(sub(h, bp3(b, 0))); return true; }
    if (b.kind != RG_BODY_AABB) { n = neg(bp3(b, 3)); return true; }
    if (fabs(h.x - b.p[0]) < 1e-8) n = v3(-1.0, 0.0, 0.0);
    else if (fabs(h.x - b.p[3]) < 1e-8) n = v3(1.0, 0.0, 0.0);
    else if (fabs(h.y - b.p[1]) < 1e-8) n = v3(0.0, -1.0, 0.0);
    else if (fabs(h.y - b.p[4]) < 1e-8) n = v3(0.0, 1.0, 0.0);
    else if (fabs(h.z - b.p[2]) < 1e-8) n = v3(0.0, 0.0, -1.0);
    else if (fabs(h.z - b.p[5]) < 1e-8) n = v3(0.0, 0.0, 1.0);
    else { n = v3(1.0, 0.0, 0.0); return false; }
    return true;
}

// Sphere texture coordinates (bodies.rs:126-132).  Kept out of line: the
// f64 atan2/acos expansions need ~70 VGPRs, and inlined into the megakernel
// they set its register peak (247 VGPRs) while every other live value waits.
__device__ __attribute__((noinline))
float2 sphere_uv(double hx, double hy, double hz, double r) {  // returned in VGPRs (no scratch round trip)
    return make_float2((1.0f + ((float)atan2(hz, hx)) / PI_F) * 0.5f, ((float)acos(hy / r)) / PI_F);
}

// bodies.rs:126-132, 155-169, 198-212, 330-333
__device__ __forceinline__ void texture_coords(const RgBodyDev &b, V3 h, float &tx, float &ty) {
    if (b.kind == RG_BODY_SPHERE) {
        V3 hv = sub(h, bp3(b, 0));
        const float2 uv = sphere_uv(hv.x, hv.y, hv.z, b.p[3]);
        tx = uv.x;
        ty = uv.y;
    } else if (b.kind == RG_BODY_AABB) {
        tx = 0.0f;
        ty = 0.0f;
    } else {
        V3 n = bp3(b, 3);
        V3 xa = cross(n, v3(0.0, 0.0, 1.0));
        if (dot(xa, xa) == 0.0) xa = cross(n, v3(0.0, 1.0, 0.0));
        V3 ya = cross(n, xa);
        V3 hv = sub(h, bp3(b, 0));
        tx = (float)dot(hv, xa);
        ty = (float)dot(hv, ya);
    }
}

// material.rs:70-79
__device__ __forceinline__ uint32_t wrap(float v, int32_t max) {
    int32_t w = f32_to_i32(v * (float)max) % max;
    return w < 0 ? (uint32_t)(w + max) : (uint32_t)w;
}

// material.rs:62-68, 82-89 + color.rs:26-30
// (float)b / 255.0f for a byte b (material.rs Texture::color, color.rs from_rgba), correctly
// rounded: one multiply and a residual correction instead of the IEEE division expansion.  Equal to
// the division for every one of the 256 inputs (checked exhaustively: tests/test_primitives_kat.py).
__device__ __forceinline__ float u8_div255(uint32_t b) {
    const float x = (float)b, inv = 1.0f / 255.0f;
    const float q0 = x * inv;
    return __builtin_fmaf(__builtin_fmaf(-q0, 255.0f, x), inv, q0);
}

__device__ __forceinline__ C3 material_color(const RgTexDev *texs, const RgMatDev &m, float tx, float ty) {
    if (m.coloration == RG_COLORATION_COLOR) return c3(m.color[0], m.color[1], m.color[2]);
    const RgTexDev t = texs[m.tex];
    uint32_t x = wrap(tx + m.xoff, t.w);
    uint32_t y = wrap(ty + m.yoff, t.h);
    // texels live in global memory: a global (not flat) load, so its wait does not also drain LDS
    const __attribute__((address_space(1))) uint32_t *tg = (const __attribute__((address_space(1))) uint32_t *)t.texels;
    uint32_t px = tg[(size_t)y * (uint32_t)t.w + x];
    return c3(u8_div255(px & 0xffu), u8_div255((px >> 8) & 0xffu), u8_div255((px >> 16) & 0xffu));
}

// material_color in two halves (light path): the texel load
// is issued at the hit and its conversion runs after the shadow batch's setup, so
// the load's latency overlaps the per-light work instead of stalling the wave.
__device__ __forceinline__ uint32_t texel_fetch(const RgTexDev *texs, const RgMatDev &m, const RgBodyDev &b, V3 h) {
    float tx, ty;
    texture_coords(b, h, tx, ty);
    const RgTexDev t = texs[m.tex];
    uint32_t x = wrap(tx + m.xoff, t.w);
    uint32_t y = wrap(ty + m.yoff, t.h);
    const __attribute__((address_space(1))) uint32_t *tg = (const __attribute__((address_space(1))) uint32_t *)t.texels;
    return tg[(size_t)y * (uint32_t)t.w + x];
}
__device__ __forceinline__ C3 texel_color(uint32_t px) {
    return c3(u8_div255(px & 0xffu), u8_div255((px >> 8) & 0xffu), u8_div255((px >> 16) & 0xffu));
}

// body.color(&body.texture_coords(hit)) (rendering.rs:134-135, 103).  The
// texture coordinates are pure functions of the hit and only a Texture
// coloration reads them, so they are computed for textured materials only:
// a Color material yields the same colour without the atan2/acos/cross work.
__device__ __forceinline__ C3 surface_color(const RgTexDev *texs, const RgMatDev &m, const RgBodyDev &b, V3 h) {
    if (m.coloration == RG_COLORATION_COLOR) return c3(m.color[0], m.color[1], m.color[2]);
    float tx, ty;
    texture_coords(b, h, tx, ty);
    return material_color(texs, m, tx, ty);
}

// rendering.rs:174-200, `cos_i = cos_t.abs()` (:194) kept as written.
__device__ __forceinline__ double fresnel(V3 inc, V3 n, float index) {
    double i_dot_n = dot(inc, n);
    double eta_i, eta_t;
    if (i_dot_n > 0.0) { eta_i = (double)index; eta_t = 1.0; }
    else { eta_i = 1.0; eta_t = (double)index; }
    double sin_t = eta_i / eta_t * sqrt(fmax(1.0 - i_dot_n * i_dot_n, 0.0));
    if (sin_t > 1.0) return 1.0;
    double cos_t = sqrt(fmax(1.0 - sin_t * sin_t, 0.0));
    double cos_i = fabs(cos_t);
    double r_s = ((eta_t * cos_i) - (eta_i * cos_t)) / ((eta_t * cos_i) + (eta_i * cos_t));
    double r_p = ((eta_i * cos_i) - (eta_t * cos_t)) / ((eta_i * cos_i) + (eta_t * cos_t));
    return (r_s * r_s + r_p * r_p) / 2.0;
}

// ray.rs:56-60
__device__ __forceinline__ Ray reflection(V3 n, V3 inc, V3 h) {
    Ray r;
    r.o = add(h, scl(n, SHADOW_BIAS));
    r.d = sub(inc, scl(n, 2.0 * dot(inc, n)));
    return r;
}

// ray.rs:62-94
__device__ __forceinline__ bool transmission(V3 n, V3 inc, V3 h, float index, Ray &r) {
    V3 ref_n = n;
    double eta_t = (double)index, eta_i = 1.0;
    double i_dot_n = dot(inc, n);
    if (i_dot_n < 0.0) i_dot_n = -i_dot_n;
    else { ref_n = neg(n); eta_t = 1.0; eta_i = (double)index; }
    double eta = eta_i / eta_t;
    double k = 1.0 - (eta * eta) * (1.0 - i_dot_n * i_dot_n);
    if (k < 0.0) return false;
    r.o = add(h, scl(ref_n, -SHADOW_BIAS));
    r.d = sub(scl(add(inc, scl(ref_n, i_dot_n)), eta), scl(ref_n, sqrt(k)));
    return true;
}

// direction_from + distance for one light (lights.rs:46-58).  For a spherical
// light both use |pos - p| = sqrt(dot(v, v)): computed once, same bits.
__device__ __forceinline__ void light_dir_dist(const RgLightDev &l, V3 p, V3 &dir, double &dist) {
    if (l.kind == RG_LIGHT_DIRECTIONAL) {
        dir = v3(l.dn[0], l.dn[1], l.dn[2]);  // normalize(-direction), precomputed
        dist = __builtin_inf();
        return;
    }
    V3 v = sub(v3(l.v[0], l.v[1], l.v[2]), p);
    double m = sqrt(dot(v, v));
    dir = scl(v, 1.0 / m);
    dist = m;
}

// lights.rs:46-58
__device__ __forceinline__ V3 light_dir(const RgLightDev &l, V3 p) {
    if (l.kind == RG_LIGHT_DIRECTIONAL) return v3(l.dn[0], l.dn[1], l.dn[2]);  // normalize(-dir), precomputed
    return normalize(sub(v3(l.v[0], l.v[1], l.v[2]), p));
}
__device__ __forceinline__ double light_distance(const RgLightDev &l, V3 p) {
    if (l.kind == RG_LIGHT_DIRECTIONAL) return __builtin_inf();
    V3 d = sub(v3(l.v[0], l.v[1], l.v[2]), p);
    return sqrt(dot(d, d));
}
__device__ __forceinline__ float light_intensity(const RgLightDev &l, V3 p) {  // lights.rs:36-44
    if (l.kind == RG_LIGHT_DIRECTIONAL) return l.intensity;
    V3 d = sub(v3(l.v[0], l.v[1], l.v[2]), p);
    float r2 = (float)dot(d, d);
    return l.intensity / (4.0f * PI_F * r2);
}

// One open node of the shading tree.
struct Frame {
    float f[8];   // REFL: D.rgb, r.  REFR: kr, tau, surf.rgb, Tc.rgb
    double rr[6]; // REFR_T: pending reflection ray (origin, direction)
    int type;
    int cdepth;   // depth of this node's children (task-splitting kernels only: elsewhere a lane's
                  // stack index IS its recursion depth, so frame sp-1's children are at depth sp)
};

// The lane's stack of open frames: at most max_recursion_depth - 1 deep
// (rendering.rs:122-130 stops at depth >= max).  MAXD > 0: a per-lane array
// (scratch).  MAXD == 0 (depths above the largest compiled array,
// scene.rs:16 is a u32): frames live in a global buffer owned by the launch
// context, frame i of the grid's thread g at base[i * stride + g], so frame
// i of a wave is one contiguous run; that launch is persistent, so the grid
// (and the buffer) stays bounded whatever the frame size.
static_assert(sizeof(Frame) == RG_FRAME_BYTES, "host sizes the deep frame buffer with RG_FRAME_BYTES");

template <int MAXD>
struct FrameStack {
    Frame f[MAXD];
    __device__ __forceinline__ void init(const RgKernelArgs &) {}
    __device__ __forceinline__ Frame &operator[](int i) { return f[i]; }
};
// Global frames are stored field-major, like scratch: dword k of frame i of grid
// thread g at plane (i * RG_FRAME_DWORDS + k), element g, so each field access
// of a wave is one coalesced 256-B run (a Frame-struct array would make every
// field a 64-line gather at an 88-B stride).  FrameRefG mirrors Frame's fields.
constexpr int RG_FRAME_DWORDS = (int)(sizeof(Frame) / 4);
static_assert(offsetof(Frame, f) == 0 && offsetof(Frame, rr) == 32 && offsetof(Frame, type) == 80 &&
                  offsetof(Frame, cdepth) == 84 && RG_FRAME_DWORDS == 22,
              "FrameRefG plane numbers");
struct FrameRefG {
    uint32_t *p;      // plane 0 of this frame, this thread
    uint32_t stride;  // dwords between planes (grid threads)
    struct F {        // a float field
        uint32_t *q;
        __device__ __forceinline__ void operator=(float v) const { *q = __float_as_uint(v); }
        __device__ __forceinline__ operator float() const { return __uint_as_float(*q); }
    };
    struct D {        // a double field: two planes
        uint32_t *q;
        uint32_t stride;
        __device__ __forceinline__ void operator=(double v) const {
            const unsigned long long b = (unsigned long long)__double_as_longlong(v);
            q[0] = (uint32_t)b;
            q[stride] = (uint32_t)(b >> 32);
        }
        __device__ __forceinline__ operator double() const {
            return __longlong_as_double((long long)(((unsigned long long)q[stride] << 32) | q[0]));
        }
    };
    struct I {        // an int field
        uint32_t *q;
        __device__ __forceinline__ void operator=(int v) const { *q = (uint32_t)v; }
        __device__ __forceinline__ operator int() const { return (int)*q; }
    };
    struct FA {
        uint32_t *q;
        uint32_t stride;
        __device__ __forceinline__ F operator[](int k) const { return F{q + (size_t)k * stride}; }
    };
    struct DA {
        uint32_t *q;
        uint32_t stride;
        __device__ __forceinline__ D operator[](int k) const { return D{q + (size_t)(2 * k) * stride, stride}; }
    };
    FA f;
    DA rr;
    I type, cdepth;
    __device__ __forceinline__ FrameRefG(uint32_t *p0, uint32_t s)
        : p(p0), stride(s), f{p0, s}, rr{p0 + (size_t)8 * s, s}, type{p0 + (size_t)20 * s},
          cdepth{p0 + (size_t)21 * s} {}
};
template <>
struct FrameStack<0> {
    uint32_t *base;   // plane 0 of frame 0, this thread
    uint32_t stride;  // grid threads
    __device__ __forceinline__ void init(const RgKernelArgs &a) {
        stride = a.deep_stride;
        base = static_cast<uint32_t *>(a.deep_stack) + (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    }
    __device__ __forceinline__ FrameRefG operator[](int i) {
        return FrameRefG(base + (size_t)i * RG_FRAME_DWORDS * stride, stride);
    }
};


__device__ __forceinline__ uint32_t out_row_to_y(const RgKernelArgs &a, uint32_t orow) {
    uint32_t tl = orow / a.tile_rows, r = orow - tl * a.tile_rows;
    const unsigned long long i = (unsigned long long)(tl + a.tile_base);
    const unsigned long long ti = a.tile_group > 1u ? (i / a.tile_group) * a.tile_stride + a.tile_offset + i % a.tile_group
                                                    : i * a.tile_stride + a.tile_offset;
    unsigned long long y = ti * a.tile_rows + r;
    return y >= a.height ? 0xFFFFFFFFu : (uint32_t)y;
}

// Output row of the launch's dense row `orow`: itself, or -- one launch of a call split over
// several (RgKernelArgs::out_tile_mul > 1) -- the row of the CALL's selected tile
// (orow / tile_rows) * mul + add that this launch's tile is.
__device__ __forceinline__ uint32_t out_row_of(const RgKernelArgs &a, uint32_t orow) {
    if (a.out_tile_mul <= 1u) return orow;
    const uint32_t tl = orow / a.tile_rows;
    return (tl * a.out_tile_mul + a.out_tile_add) * a.tile_rows + (orow - tl * a.tile_rows);
}

constexpr size_t RG_NO_PIXEL = ~(size_t)0;  // a lane of a tile that lies outside the output

// A wave finished tile `tile`: store its pixels (one coalesced store), then,
// for a consumer on the host (RgKernelArgs::tile_flags), make them visible
// (system-scope release, all lanes) and publish the tile.
__device__ __forceinline__ void flush_tile(const RgKernelArgs &a, size_t oidx, uint32_t px, uint32_t tile, int lane) {
    if (a.defer_px && oidx != RG_NO_PIXEL) a.rgba[oidx] = px;
    if (a.tile_flags) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        if (lane == 0) __hip_atomic_store(&a.tile_flags[tile], a.frame_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

__device__ __forceinline__ unsigned long long wave_sum(uint32_t v32) {
    unsigned long long v = v32;
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// ---------------------------------------------------------------- task splitting
// A refractive hit opens two independent subtrees (transmission, then
// reflection: rendering.rs:100-113); the lane traces the transmission ray and
// PUBLISHES the reflection ray in a block-local pool in LDS.  Any idle lane of
// the block (its pixel finished, or its wave out of tiles) may take it, trace
// the subtree with the same state machine and hand the colour back; if nobody
// took it by the time the owner needs it, the owner reclaims it and traces it
// itself.  A subtree's colour is a function of its ray only, and the owner
// combines it with exactly the expression of FR_REFR_R, so results are
// identical whoever traces it.  This splits the long ray trees of
// refractive pixels (the slowest tiles, which bound a frame's makespan)
// across the waves of a CU.  Waits only ever point down a tree, so there is
// no cycle: every awaited subtree is held by a live lane.
#ifndef RG_PIPE_TILES_PER_WAVE
#define RG_PIPE_TILES_PER_WAVE 64  // heavy launches with frames in flight (launch_one, RgKernelArgs::pipelined;
                                   // 32 -> 64: configs[4] scene at 1080p 2.50 -> 2.33 ms, profiles/r05/s21)
#endif
#ifndef RG_PIPE_MIN_CU_DIV
#define RG_PIPE_MIN_CU_DIV 4  // ... and at least 1/this of the CUs' blocks (3 -> 4: north-star 1/8 share 0.349 -> 0.327 ms)
#endif
// Light path, non-persistent waves: a wave renders at most this many 8x8 tiles
// and exits, and the grid holds one wave per that many tiles, so the hardware
// dispatcher hands out CU slots wave by wave -- across the kernels of frames in
// flight too -- instead of 3072 persistent waves pinning their slots until the
// frame's queue is empty.  16 measured best for the whole 4K frame and for
// 1/2 .. 1/8 shares (profiles/r01/variants_light_tiles_per_wave.txt; 12 / 20 / 32
// re-measured in rounds 3-4: profiles/r04/s29, profiles/r04/s13).
#ifndef RG_LIGHT_TILES_PER_WAVE
#define RG_LIGHT_TILES_PER_WAVE 16
#endif
#ifndef RG_HEAVY_TILES_PER_WAVE
#define RG_HEAVY_TILES_PER_WAVE 0  // heavy path: 0 = persistent blocks (one per CU)
#endif
#ifndef RG_SHADOW_FAN
// heavy path, single small launches (TASKS): up to this many more lights of a hit traced by idle
// lanes per iteration.  Off for frames in flight and whole frames since the light buffers made
// shadow rays cheap: north star 1.594 -> 1.497 ms (8K 5.38 -> 5.06), while a 1/8 share as one
// launch keeps it (slowest share 0.648 vs 0.712 ms without; profiles/r05/s20, s21)
#define RG_SHADOW_FAN 3
#endif
__device__ __forceinline__ double readlane_d(double v, int l) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), l);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
#ifndef RG_HEAVY_TASKS
#define RG_HEAVY_TASKS 1   // task splitting on the heavy path, for launches of fewer than RG_HEAVY_TASK_TILES tiles
#endif
#ifndef RG_HEAVY_TASK_TILES
// Task splitting shortens the slowest pixels' ray trees, which bound a small
// launch; on a large one (and with frames in flight, whose next frame fills
// the tail) its bookkeeping costs more than it saves: with 4 frames in flight
// synth1024 4K 3.10 -> 2.88 ms and 8K 11.18 -> 9.94 ms without it, but a 1/8
// share (16k tiles) 0.538 -> 0.561 ms (profiles/r01/variants_heavy_tasks.txt)
#define RG_HEAVY_TASK_TILES 24576
#endif
#ifndef RG_TASK_SLOTS
#define RG_TASK_SLOTS 128
#endif
struct TaskPool {
    static constexpr int S = RG_TASK_SLOTS;
    static_assert(S % 32 == 0, "whole bitmap words");
    double ray[S][6];  // published ray (origin, direction)
    float col[S][4];   // the subtree's colour once done
    int depth[S];      // recursion depth of the published ray
    uint32_t pix[S];   // owner's pixel (error reports)
    int done[S];       // 1: col holds the result
    uint32_t free_m[S / 32];  // 1 = slot free
    uint32_t pend_m[S / 32];  // 1 = published, not taken
    int busy;                 // waves of the block that hold work
};
// one pool per block (heavy path: a CU's 12 waves); allocated only by the kernels that split tasks
__shared__ TaskPool rg_pool;
__device__ __forceinline__ TaskPool &pool_of() { return rg_pool; }
constexpr int pool_slots() { return RG_TASK_SLOTS; }

#define RG_WG __HIP_MEMORY_SCOPE_WORKGROUP
__device__ __forceinline__ void pool_init() {
    auto &P = pool_of();
    constexpr int S = pool_slots();
    if (threadIdx.x < S / 32) {
        P.free_m[threadIdx.x] = ~0u;
        P.pend_m[threadIdx.x] = 0u;
    }
    for (uint32_t k = threadIdx.x; k < (uint32_t)S; k += blockDim.x) P.done[k] = 0;
    if (threadIdx.x == 0) P.busy = 0;
}
// Claim a free slot (-1: pool full).  Lanes start at different words/bits.
__device__ __forceinline__ int pool_alloc(int lane) {
    auto &P = pool_of();
    constexpr int S = pool_slots();
    const int rot = (lane >> 2) & 31;
    for (int i = 0; i < S / 32; ++i) {
        const int w = (lane + i) & (S / 32 - 1);
        uint32_t m = __hip_atomic_load(&P.free_m[w], __ATOMIC_RELAXED, RG_WG);
        while (m != 0u) {
            const uint32_t r = rot ? ((m >> rot) | (m << (32 - rot))) : m;
            const int b = (__builtin_ctz(r) + rot) & 31;
            const uint32_t bit = 1u << b;
            const uint32_t old = __hip_atomic_fetch_and(&P.free_m[w], ~bit, __ATOMIC_ACQUIRE, RG_WG);
            if (old & bit) return w * 32 + b;
            m = old & ~bit;
        }
    }
    return -1;
}
__device__ __forceinline__ void pool_publish(int slot) {  // ray/depth/pix written before
    __hip_atomic_fetch_or(&pool_of().pend_m[slot >> 5], 1u << (slot & 31), __ATOMIC_RELEASE, RG_WG);
}
__device__ __forceinline__ bool pool_any_pending() {
    uint32_t m = 0u;
#pragma unroll
    for (int w = 0; w < pool_slots() / 32; ++w) m |= __hip_atomic_load(&pool_of().pend_m[w], __ATOMIC_RELAXED, RG_WG);
    return m != 0u;
}
// Take the k-th pending task of a snapshot (k = rank among the wave's idle lanes).
__device__ __forceinline__ int pool_take(int k) {
    auto &P = pool_of();
    for (int w = 0; w < pool_slots() / 32; ++w) {
        uint32_t m = __hip_atomic_load(&P.pend_m[w], __ATOMIC_RELAXED, RG_WG);
        const int n = __builtin_popcount(m);
        if (k >= n) {
            k -= n;
            continue;
        }
        for (int j = 0; j < k; ++j) m &= m - 1u;
        const uint32_t bit = m & (~m + 1u);
        const uint32_t old = __hip_atomic_fetch_and(&P.pend_m[w], ~bit, __ATOMIC_ACQUIRE, RG_WG);
        return (old & bit) ? w * 32 + __builtin_ctz(bit) : -1;
    }
    return -1;
}
__device__ __forceinline__ bool pool_reclaim(int slot) {  // owner: un-publish if still pending
    const uint32_t bit = 1u << (slot & 31);
    return (__hip_atomic_fetch_and(&pool_of().pend_m[slot >> 5], ~bit, __ATOMIC_ACQ_REL, RG_WG) & bit) != 0u;
}
__device__ __forceinline__ void pool_finish(int slot, C3 c) {  // taker: result, then done
    auto &P = pool_of();
    P.col[slot][0] = c.r;
    P.col[slot][1] = c.g;
    P.col[slot][2] = c.b;
    __hip_atomic_store(&P.done[slot], 1, __ATOMIC_RELEASE, RG_WG);
}
__device__ __forceinline__ bool pool_done(int slot) {
    return __hip_atomic_load(&pool_of().done[slot], __ATOMIC_ACQUIRE, RG_WG) != 0;
}
__device__ __forceinline__ void pool_release(int slot) {  // owner: slot free again
    auto &P = pool_of();
    __hip_atomic_store(&P.done[slot], 0, __ATOMIC_RELAXED, RG_WG);
    __hip_atomic_fetch_or(&P.free_m[slot >> 5], 1u << (slot & 31), __ATOMIC_RELEASE, RG_WG);
}

}  // namespace rgk

using namespace rgk;

#ifndef RG_HOST_RING
#define RG_HOST_RING 16  // light path into pinned host memory: tiles per queue group and ring flush (0: one store per tile)
#endif
#ifndef RG_LIGHT_BLOCK_WAVES
#define RG_LIGHT_BLOCK_WAVES 1  // light path: waves per block (blocks retire wave by wave)
#endif
#ifndef RG_NQ
#define RG_NQ 8   // tile-queue heads (see the kernel's tile loop)
#endif
#define RG_QUEUE_BASE 16   // counters[16 + 16*q]: head q, one 128-B line each
#define RG_QUEUE_STRIDE 16

// Per-launch view of the cold (shading) tables: LDS copies or global.
struct Cold {
    const RgBodyDev *bodies;
    const RgMatDev *mats;
    const RgLightDev *lights;
    const RgTexDev *texs;
};

// Stage [src, src+bytes) into LDS at dst (both 16-B aligned, bytes % 16 == 0).
__device__ __forceinline__ void stage16(unsigned char *dst, const void *src, uint32_t bytes) {
    uint4 *d = reinterpret_cast<uint4 *>(dst);
    const uint4 *g = reinterpret_cast<const uint4 *>(src);
    for (uint32_t k = threadIdx.x; k < bytes / 16u; k += blockDim.x) d[k] = g[k];
}

// Render kernel.  Heavy path: ONE persistent block of 256*WPS threads per CU
// (WPS waves per SIMD).  Light path: one-wave blocks, each rendering at most
// RG_LIGHT_TILES_PER_WAVE tiles (launcher: launch_one).  A block stages the
// scene into LDS (LSPH: sphere, plane, disk and box tables, lights, texture
// descriptors; LCOLD: bodies, materials; LCOLD without LSPH: only the BVH nodes, after the per-lane
// walk stacks -- scenes whose sphere tables exceed the budget), then every wave repeatedly takes the next 8x8 pixel
// tile from an atomic queue (counters[16..], sharded) and runs the per-lane
// state machine until its 64 lanes have written their pixels.
template <int MAXD, bool LSPH, bool LCOLD, int WPS, int LBT, bool F32F, bool BVH, bool TASKS, int TPW = 0,
          bool HF = false>
// LBT: lights per shadow batch on the light path (2, 3; -1: one light), 1: the heavy path.
// HF: the host-frame features (HOSTF below) with MAXD array frames.  TPW: light path, tiles per wave (0: RG_LIGHT_TILES_PER_WAVE; < 0: persistent waves that take tiles
// until the queue is empty -- single launches, whose makespan is their slowest wave's tile sum).  Light path (LBT != 1): blocks of RG_LIGHT_BLOCK_WAVES waves, at least WPS waves
// per SIMD (the second bound is waves per execution unit on AMD); heavy path:
// one block of 4*WPS waves per CU.  Both cap the VGPRs at 512 / WPS.
__global__ __launch_bounds__(LBT != 1 ? 64 * RG_LIGHT_BLOCK_WAVES : 256 * WPS, LBT != 1 ? WPS : 1)
void rg_render_kernel(RgKernelArgs a) {
    constexpr int LB = LBT < 0 ? -LBT : LBT;  // lights per shadow batch (1 on the heavy path)
    constexpr bool LIGHTP = LBT != 1;         // the light path
    static_assert(!BVH || 4 * WPS <= RG_BVH_MAX_WAVES, "one BVH stack per wave");
#ifdef RG_WAVE_TIMES  // diagnostic: per-wave start (before staging), staged, end (100 MHz ticks), tiles
    const unsigned long long t_wave0 = wall_clock64();
    uint32_t wt_tiles = 0;
#endif
    constexpr bool GFRAMES = MAXD == 0;
    // the launch context's other counter set (the previous launch's, read back
    // already: same stream) starts the next launch at zero -- no memset per frame
    if (blockIdx.x == 0 && a.counters_next)
        for (uint32_t k = threadIdx.x; k < RG_COUNTER_WORDS; k += blockDim.x) a.counters_next[k] = 0ull;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr bool LNODES = !LSPH && LCOLD && BVH;  // only the BVH nodes in LDS (SphNodesLds)
    typename std::conditional<LSPH, SphLds, typename std::conditional<LNODES, SphNodesLds, SphScalar>::type>::type src;
    Cold T;
    // light path: every one-wave block stages its own copy of the (few-KB) scene; with the
    // arena's device image that is one loop with all its loads in flight at once
    const bool blob = LIGHTP && LSPH && LCOLD && a.lds_blob != nullptr;
    if (blob) {
        const uint4 *g = reinterpret_cast<const uint4 *>(a.lds_blob);
        uint4 *d = reinterpret_cast<uint4 *>(smem);
        const uint32_t n16 = a.lds_total_bytes / 16u;
        // four loads in flight per lane: unconditional (indices clamped into the image), then
        // the guarded LDS stores -- no per-lane array, which hipcc placed in scratch
        const uint32_t last = n16 - 1u;
        for (uint32_t k0 = threadIdx.x; k0 < n16; k0 += 4u * blockDim.x) {
            const uint32_t k1 = k0 + blockDim.x, k2 = k1 + blockDim.x, k3 = k2 + blockDim.x;
            const uint4 v0 = g[k0], v1 = g[min(k1, last)], v2 = g[min(k2, last)], v3 = g[min(k3, last)];
            d[k0] = v0;
            if (k1 < n16) d[k1] = v1;
            if (k2 < n16) d[k2] = v2;
            if (k3 < n16) d[k3] = v3;
        }
    }
    if constexpr (LSPH) {
        if (!blob) {
        stage16(smem + a.lds_sphf, a.sphf, (uint32_t)a.n_sph * (uint32_t)sizeof(RgSphF));
        stage16(smem + a.lds_sphf + (size_t)a.n_sph * sizeof(RgSphF), a.sphf2, (uint32_t)a.n_sph * (uint32_t)sizeof(RgSphF2));
        stage16(smem + a.lds_sph, a.sph, (uint32_t)a.n_sph * (uint32_t)sizeof(RgSph));
        stage16(smem + a.lds_cc, a.sph_cc, a.lds_nodes - a.lds_cc);
        if constexpr (BVH) {
            stage16(smem + a.lds_nodes, a.nodes, (uint32_t)a.n_nodes * (uint32_t)sizeof(RgBvhNode));
        }
        stage16(smem + a.lds_pln, a.pln, (uint32_t)a.n_pln * (uint32_t)sizeof(RgPln));
        stage16(smem + a.lds_dsk, a.dsk, (uint32_t)a.n_dsk * (uint32_t)sizeof(RgDsk));
        stage16(smem + a.lds_box, a.box, a.lds_lights - a.lds_box);
        stage16(smem + a.lds_lights, a.lights, (uint32_t)a.n_lights * (uint32_t)sizeof(RgLightDev));
        stage16(smem + a.lds_texs, a.texs, a.lds_lbuf - a.lds_texs);
        if (a.lbuf) stage16(smem + a.lds_lbuf, a.lbuf, a.lds_bodies - a.lds_lbuf);
        }
        src.f = reinterpret_cast<const RgSphF *>(smem + a.lds_sphf);
        src.f2 = reinterpret_cast<const RgSphF2 *>(smem + a.lds_sphf + (size_t)a.n_sph * sizeof(RgSphF));
        src.s = reinterpret_cast<const RgSph *>(smem + a.lds_sph);
        src.cc = reinterpret_cast<const double *>(smem + a.lds_cc);
        src.pl = reinterpret_cast<const RgPln *>(smem + a.lds_pln);
        src.dk = reinterpret_cast<const RgDsk *>(smem + a.lds_dsk);
        src.bx = reinterpret_cast<const RgBox *>(smem + a.lds_box);
        src.nd = reinterpret_cast<const RgBvhNode *>(smem + a.lds_nodes);
        src.lb = reinterpret_cast<const RgLightBufDev *>(smem + a.lds_lbuf);
        src.lt = reinterpret_cast<const RgLightDev *>(smem + a.lds_lights);
    } else {
        src.s = rg_cptr(a.sph);
        src.cc = rg_cptr(a.sph_cc);
        src.f = rg_cptr(a.sphf);
        src.f2 = rg_cptr(a.sphf2);
        src.pl = rg_cptr(a.pln);
        src.dk = rg_cptr(a.dsk);
        src.bx = rg_cptr(a.box);
        if constexpr (LNODES) {  // the nodes after the per-lane walk stacks
            stage16(smem + a.lds_lstack_bytes, a.nodes, (uint32_t)a.n_nodes * (uint32_t)sizeof(RgBvhNode));
            src.nd = reinterpret_cast<const RgBvhNode *>(smem + a.lds_lstack_bytes);
        } else {
            src.nd = rg_cptr(a.nodes);
        }
        src.lb = a.lbuf;
        src.lt = a.lights;
    }
    if constexpr (LSPH && LCOLD) {
        if (!blob) {
            stage16(smem + a.lds_bodies, a.bodies, (uint32_t)a.n_bodies * (uint32_t)sizeof(RgBodyDev));
            stage16(smem + a.lds_mats, a.mats, (uint32_t)a.n_bodies * (uint32_t)sizeof(RgMatDev));
        }
        T.bodies = reinterpret_cast<const RgBodyDev *>(smem + a.lds_bodies);
        T.mats = reinterpret_cast<const RgMatDev *>(smem + a.lds_mats);
    } else {
        T.bodies = a.bodies;
        T.mats = a.mats;
    }
    if constexpr (LSPH) {  // lights and texture descriptors: part of the hot tables
        T.lights = reinterpret_cast<const RgLightDev *>(smem + a.lds_lights);
        T.texs = reinterpret_cast<const RgTexDev *>(smem + a.lds_texs);
    } else {
        T.lights = a.lights;
        T.texs = a.texs;
    }
    if (TASKS || LSPH || LCOLD) {
        if constexpr (TASKS) pool_init();
        __syncthreads();
    }

    const int lane = threadIdx.x & 63;
    // With the frame in host memory (a.defer_px) the wave's finished pixels
    // wait here until its whole tile is done, then go out as ONE coalesced
    // store per tile (flush_tile): every store is a PCIe write whose
    // acknowledgement the wave's next vmcnt wait would otherwise sit out once
    // per finishing lane.
    // Host-frame features (deferred tile stores, tile publication, streaming
    // cancellation, tile shapes other than 8x8) exist only in the MAXD == 0
    // instantiations, which host-visible one-launch renders use: the array
    // instantiations of device-resident renders stay as lean as before (the
    // runtime checks alone cost test1 3 %, profiles/r02/ab_hostf.txt).
    constexpr bool HOSTF = MAXD == 0 || HF;
    __shared__ uint32_t tile_px[HOSTF ? (LIGHTP ? RG_LIGHT_BLOCK_WAVES : 4 * WPS) : 1][64];
    uint32_t *my_px = &tile_px[HOSTF ? threadIdx.x >> 6 : 0][lane];
    // Light path into page-locked host memory without tile publication: the
    // finished tiles of a wave collect in an LDS ring and go out RING at a time.
    // A store to host memory completes only after its PCIe round trip, and on
    // gfx9 every later `s_waitcnt vmcnt` (a texel load, a frame pop from the
    // global frame buffer) waits for it too: one flush per RING tiles instead of
    // one per tile.
    constexpr int RING = (HOSTF && LIGHTP) ? RG_HOST_RING : 0;
    __shared__ uint32_t ring_px[RING > 0 ? RG_LIGHT_BLOCK_WAVES : 1][RING > 0 ? RING : 1][64];
    __shared__ uint32_t ring_tile[RING > 0 ? RG_LIGHT_BLOCK_WAVES : 1][RING > 0 ? RING : 1];
    [[maybe_unused]] const uint32_t rw = RING > 0 ? (threadIdx.x >> 6) % RG_LIGHT_BLOCK_WAVES : 0u;
    [[maybe_unused]] uint32_t nring = 0;  // tiles waiting in the ring (wave-uniform)
    [[maybe_unused]] uint32_t grp_next = 0, grp_end = 0;  // the wave's group of consecutive tiles (ring mode)
    // Light path: a diffuse hit's shading factors wait in LDS while its shadow
    // batch is traced (field k of the lane at park[k][lane], conflict-free), so
    // that only the query's own state is held in VGPRs across the trace.
    constexpr int PK_PP = 0, PK_LIN = LB, PK_REFL = 2 * LB, PK_COL = 2 * LB + 1, PK_KIND = 2 * LB + 4,
                  PK_R = 2 * LB + 5, PK_N = 2 * LB + 6;
    __shared__ float park_lds[LIGHTP ? RG_LIGHT_BLOCK_WAVES : 1][LIGHTP ? PK_N : 1][64];
    float *park = &park_lds[LIGHTP ? (threadIdx.x >> 6) % RG_LIGHT_BLOCK_WAVES : 0][0][lane];  // field k at park[64 k]
#ifdef RG_BVH_STATS
    if (lane < 16) rg_stat_lds[(threadIdx.x >> 6) % RG_BVH_MAX_WAVES][lane] = 0ull;
#endif
    [[maybe_unused]] const unsigned long long t_kernel = RG_CLOCK();
#ifdef RG_WAVE_TIMES
    const unsigned long long t_staged = wall_clock64();
#endif
    const uint32_t twlog = HOSTF ? a.tile_wlog : 3u, twmask = (1u << twlog) - 1u, th = 64u >> twlog;
    const uint32_t tiles_x = (a.width + twmask) >> twlog;
    const uint32_t ntiles = tiles_x * ((a.out_rows + th - 1u) / th);
    const C3 def = c3(a.def[0], a.def[1], a.def[2]);
    const int max_depth = (int)a.max_depth;
    [[maybe_unused]] const bool use_ring = RING > 0 && a.defer_px;
    // the launch's ring flush size and queue group (RgKernelArgs::ring_flush / ring_group)
    [[maybe_unused]] const uint32_t ring_n = RING > 0 ? (a.ring_flush ? min(a.ring_flush, (uint32_t)(RING > 0 ? RING : 1)) : (uint32_t)RING) : 1u;
    [[maybe_unused]] const uint32_t ring_g = RING > 0 ? (a.ring_group ? min(a.ring_group, ring_n) : ring_n) : 1u;
    // store the ring's tiles: each lane its pixel of every tile (same index rule as the tile start)
    [[maybe_unused]] auto flush_ring = [&]() {
        for (uint32_t k = 0; k < nring; ++k) {
            const uint32_t tile = ring_tile[rw][k];
            const uint32_t ty = tile / tiles_x, tx = tile - ty * tiles_x;
            const uint32_t x = (tx << twlog) + ((uint32_t)lane & twmask);
            const uint32_t orow = ty * th + ((uint32_t)lane >> twlog);
            if (x < a.width && orow < a.out_rows) {
                const uint32_t row = a.image_rows ? out_row_to_y(a, orow) : out_row_of(a, orow);
                if (row != 0xFFFFFFFFu) a.rgba[(size_t)row * a.width + x] = ring_px[rw][k][lane];
            }
        }
        if (a.tile_flags) {  // a consumer on the host: ONE system-scope release publishes the ring's tiles
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            if ((uint32_t)lane < nring)
                __hip_atomic_store(&a.tile_flags[ring_tile[rw][lane]], a.frame_seq, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
        }
        nring = 0;
    };
    uint32_t n_prim = 0, n_shadow = 0, n_sec = 0;
    FrameStack<GFRAMES ? 0 : MAXD> stk;  // GFRAMES: field-major frames in a global buffer, no scratch array
    stk.init(a);

    // Sharded tile queue: RG_NQ heads, head q serving tiles q, q + RG_NQ, ... (one
    // 128-B line per head).  A single head saturates at ~88 dequeues/us
    // (MI355X_MICROARCH.md "dequeue"), i.e. ~1.5 ms for a 4K frame of 8x8 tiles.
    // The waves of a block start on head (block % RG_NQ) -- adjacent tiles per CU --
    // and move to the next head when theirs is drained (work stealing for the tail).
    uint32_t qi = blockIdx.x % RG_NQ, qtried = 0;
    // Lane state.  A lane holds one pixel of the wave's 8x8 tile, or (task
    // splitting, TASKS) one published subtree of another lane of the block;
    // the wave takes the next tile when none of its lanes has work.
    int mode = MODE_DONE;
    Ray q;                 // current query (shadow: q.o = shared origin)
    ShadowBatch<LB> sb;        // shadow: the batch's directions and light distances
    uint32_t occl_full = 0u;
    int qdepth = 0;        // closest: depth of the ray
    // hit being shaded
    V3 hp = v3(0, 0, 0), hn = v3(0, 0, 0);
    int hb = 0, hdepth = 0, li = 0;
    int nfan = 0;              // shadow fan-out: lights li+1 .. li+nfan of this hit traced by helper lanes
    uint32_t fan_lanes = 0u;   // ... their lanes, 6 bits each
    uint32_t fan_bits = 0u;    // ... their occlusion results, bit k
    C3 fin = c3(0, 0, 0), bcol = c3(0, 0, 0), ret = def;
    int sp = 0;
    Closest c;
    closest_init(c);
    bool have_result = false;  // c / occl hold a fresh result for the lane's query
    uint32_t occl = 0u;
    size_t oidx = 0;           // output index of the lane's pixel
    uint32_t pixel = 0;        // image pixel index (error reports) of the lane's pixel or task
    int task = -1;             // pool slot whose subtree this lane computes (-1: its own pixel)
    bool tiles_left = true;    // the tile queue has not been found empty
    [[maybe_unused]] uint32_t pf_k = 0u;       // lane 0: the prefetched slot of head qi (tile-slot prefetch)
    [[maybe_unused]] bool pf_valid = false;    // (wave-uniform) a slot is claimed
    uint32_t my_tile = 0xFFFFFFFFu;  // the wave's current tile (published when done: a.tile_flags)
    [[maybe_unused]] uint32_t tiles_taken = 0;
    [[maybe_unused]] bool counted = false;  // this wave is counted in pool_of().busy
#ifdef RG_TILE_TIMES
    uint32_t cur_tile = 0xFFFFFFFFu;  // diagnostic: per-tile time into rgb[tile] (us), wave iterations
    unsigned long long t_tile = 0, t_query = 0;  // into rgb[ntiles + tile], start, query time
    uint32_t tile_iters = 0;
#endif
    for (;;) {
        RG_REGION(RGR_LOOP);
        if constexpr (!LIGHTP && TASKS && RG_SHADOW_FAN > 0) {
            // shadow fan-out, collect: the helpers' occlusion bits (every lane active here)
            if (__any(nfan > 0)) {
                fan_bits = 0u;
#pragma unroll
                for (int k = 0; k < RG_SHADOW_FAN; ++k) {
                    const uint32_t b = (uint32_t)__shfl((int)occl, (int)((fan_lanes >> (6 * k)) & 63u), 64);
                    if (k < nfan) fan_bits |= (b & 1u) << k;
                }
            }
            if (mode == MODE_SHADOW_H) {  // a helper is idle again
                mode = MODE_DONE;
                have_result = false;
            }
        }
        if (have_result) {
            bool unwind = false;
            bool shade = false;           // run a shade_diffuse step this iteration
            const int rmode = mode;       // kind of result the lane holds
            if (TASKS && rmode == MODE_WAIT) {
                unwind = true;  // poll the awaited subtree (top frame FR_REFR_WAIT)
            } else if (rmode == MODE_CLOSEST) {
                if (c.nan && c.nhit >= 2) raise_error(a, pixel, RG_ERR_NAN_DISTANCE);
                if (c.id < 0) {
                    ret = def;  // rendering.rs:76-77, 128-129
                    unwind = true;
                } else {
                    // get_color (rendering.rs:80-120)
                    const RgBodyDev b = T.bodies[c.id];
                    const RgMatDev m = T.mats[c.id];
                    RG_REGION(RGR_GETCOLOR);
                    if (b.kind == RG_BODY_SPHERE) RG_REGION(RGR_NORMAL_SPHERE);
                    V3 h = add(q.o, scl(q.d, c.t));
                    V3 n;
                    if (!surface_normal(b, h, n)) raise_error(a, pixel, RG_ERR_AABB_NORMAL);
                    if (m.surface != RG_SURFACE_REFRACTIVE) {
                        if constexpr (LIGHTP) {
                            // ONE batch covers every light (n_lights <= LB on this path): set it
                            // up now, with the per-light shading factors (parked in LDS), so that
                            // no hit-point state (h, n, incident) has to survive the shadow pass
                            // a textured hit's texel load goes out now and is converted after the
                            // lights' setup below (its latency overlaps that work: test1 0.2979 ->
                            // 0.2955 ms over 200 frames, profiles/r04/s15/session.txt)
                            const bool textured = m.coloration != RG_COLORATION_COLOR;
                            uint32_t texel = 0u;
                            RG_REGION(RGR_BATCH);
#ifdef RG_REGION_STATS
                            if (textured) {
                                RG_REGION(RGR_TEXEL);
                                if (b.kind == RG_BODY_SPHERE) RG_REGION(RGR_UV_SPHERE);
                                else if (b.kind != RG_BODY_AABB) RG_REGION(RGR_UV_PLANE);
                            }
#endif
                            if (textured) texel = texel_fetch(T.texs, m, b, h);
                            else { park[64 * PK_COL] = m.color[0]; park[64 * (PK_COL + 1)] = m.color[1]; park[64 * (PK_COL + 2)] = m.color[2]; }
                            park[64 * PK_REFL] = m.albedo_pi;                       // rendering.rs:164
                            // how the batch's colour is used: 0 diffuse, 1 reflecting at the depth
                            // limit (mix with the default colour), 2 reflecting with a frame
                            const int kind = m.surface == RG_SURFACE_DIFFUSE ? 0 : qdepth + 1 < max_depth ? 2 : 1;
                            park[64 * PK_KIND] = __int_as_float(kind);
                            park[64 * PK_R] = m.reflectivity;
                            // the shadow rays' origin hit + n*bias (rendering.rs:148) is also the
                            // reflection ray's origin (ray.rs:57): q.o serves both, and q.d (unused
                            // by the shadow pass) carries the reflection direction until the
                            // batch is shaded -- the frame holds only colour state
                            q.o = add(h, scl(n, SHADOW_BIAS));
                            // (rendering.rs:88: its frame is pushed once the batch is shaded)
                            if (kind == 2) q.d = sub(q.d, scl(n, 2.0 * dot(q.d, n)));  // ray.rs:58
                            occl_full = 0u;
#pragma unroll
                            for (int l = 0; l < LB; ++l) {
                                if (l < a.n_lights) {
                                    const RgLightDev L = T.lights[l];
                                    if (L.kind != RG_LIGHT_DIRECTIONAL) RG_REGION(RGR_LIGHT_SPH);
                                    light_dir_dist(L, h, sb.d[l], sb.ld[l]);
                                    park[64 * (PK_PP + l)] = fmaxf((float)dot(n, sb.d[l]), 0.0f);  // rendering.rs:161-162
                                    park[64 * (PK_LIN + l)] = light_intensity(L, h);               // pure; used if lit
                                    occl_full |= 1u << l;
                                    n_shadow++;
                                } else {
                                    sb.d[l] = v3(0.0, 0.0, 1.0);
                                    sb.ld[l] = 0.0;
                                }
                            }
                            if (textured) {
                                const C3 col = texel_color(texel);
                                park[64 * PK_COL] = col.r; park[64 * (PK_COL + 1)] = col.g; park[64 * (PK_COL + 2)] = col.b;
                            }
                            if (a.n_lights > 0) mode = MODE_SHADOW;
                            else shade = true;  // no lights: finish with black (rendering.rs:138)
                        } else {
                            bcol = surface_color(T.texs, m, b, h);
                            hb = c.id; hdepth = qdepth;
                            fin = c3(0.0f, 0.0f, 0.0f);
                            hp = h; hn = n; li = 0;
                            // a reflecting hit's reflection direction (ray.rs:58) goes into q.d
                            // now -- the shadow queries use q.o and sb only -- so the incident
                            // direction does not stay live across the light loop
                            if (m.surface == RG_SURFACE_REFLECTING && qdepth + 1 < max_depth)
                                q.d = sub(q.d, scl(n, 2.0 * dot(q.d, n)));
                            shade = true;
                        }
                    } else {
                        RG_REGION(RGR_REFRACT);
                        float kr = (float)fresnel(q.d, n, m.index);
                        C3 surf = surface_color(T.texs, m, b, h);
                        int cd = qdepth + 1;
                        if (cd >= max_depth) {
                            // the transmission ray's unwrap (rendering.rs:106) precedes cast_ray's depth test
                            Ray tr;
                            if (kr < 1.0f && !transmission(n, q.d, h, m.index, tr)) raise_error(a, pixel, RG_ERR_TRANSMISSION);
                            C3 col = cadd(cscl(def, kr), cscl(def, 1.0f - kr));
                            ret = cmul(cscl(col, m.transparency), surf);
                            unwind = true;
                        } else {
                            RG_REGION(RGR_PUSH_REFR);  // frame writes: 18 dwords per lane (kr .. surf, pending ray, type)
                            auto &&f = stk[sp++];
                            f.f[0] = kr; f.f[1] = m.transparency;
                            f.f[2] = surf.r; f.f[3] = surf.g; f.f[4] = surf.b;
                            if constexpr (TASKS) f.cdepth = cd;
                            // rendering.rs:100-113: the transmission subtree is traced first while
                            // the reflection ray (ray.rs:56-60) waits in the frame or, with task
                            // splitting, is published so an idle lane of the block can trace it now
                            bool trace_t = false;
                            if (kr < 1.0f) {
                                if constexpr (TASKS) {
                                    Ray tr;
                                    if (transmission(n, q.d, h, m.index, tr)) {
                                        trace_t = true;
                                        const Ray rr = reflection(n, q.d, h);
                                        const int slot = pool_alloc(lane);
                                        if (slot >= 0) {
                                            double *pr = pool_of().ray[slot];
                                            pr[0] = rr.o.x; pr[1] = rr.o.y; pr[2] = rr.o.z;
                                            pr[3] = rr.d.x; pr[4] = rr.d.y; pr[5] = rr.d.z;
                                            pool_of().depth[slot] = cd;
                                            pool_of().pix[slot] = pixel;
                                            pool_publish(slot);
                                            f.type = FR_REFR_TASK | (slot << 8);
                                        } else {
                                            f.type = FR_REFR_T;
                                            f.rr[0] = rr.o.x; f.rr[1] = rr.o.y; f.rr[2] = rr.o.z;
                                            f.rr[3] = rr.d.x; f.rr[4] = rr.d.y; f.rr[5] = rr.d.z;
                                        }
                                        q = tr;
                                    }
                                } else {
                                    // the reflection ray goes to the frame BEFORE the transmission ray
                                    // is built (into q, written only on success): fewer live values
                                    const Ray rr = reflection(n, q.d, h);
                                    f.rr[0] = rr.o.x; f.rr[1] = rr.o.y; f.rr[2] = rr.o.z;
                                    f.rr[3] = rr.d.x; f.rr[4] = rr.d.y; f.rr[5] = rr.d.z;
                                    f.type = FR_REFR_T;
                                    trace_t = transmission(n, q.d, h, m.index, q);
                                }
                                if (!trace_t) raise_error(a, pixel, RG_ERR_TRANSMISSION);
                            }
                            if (!trace_t) {  // kr >= 1 (or the transmission panic): refraction colour = default
                                f.type = FR_REFR_R;
                                f.f[5] = def.r; f.f[6] = def.g; f.f[7] = def.b;
                                q = reflection(n, q.d, h);
                            }
                            qdepth = cd;
                            mode = MODE_CLOSEST;
                            n_sec++;
                        }
                    }
                }
            } else if (rmode == MODE_SHADOW) {
                shade = true;  // a shadow result for light li
            }
            if constexpr (LIGHTP) {
              if (shade) {
                RG_REGION(RGR_SHADE);
                // shade_diffuse accumulation over the batch (rendering.rs:141-170), in light order
                const C3 bc = c3(park[64 * PK_COL], park[64 * (PK_COL + 1)], park[64 * (PK_COL + 2)]);
                const float refl = park[64 * PK_REFL];
                C3 acc = c3(0.0f, 0.0f, 0.0f);
#pragma unroll
                for (int l = 0; l < LB; ++l) {
                    if (l < a.n_lights) {
                        const RgLightDev L = T.lights[l];
                        const float inten = !((occl >> l) & 1u) ? park[64 * (PK_LIN + l)] : 0.0f;
                        const float power = park[64 * (PK_PP + l)] * inten;
                        C3 lc = cscl(cscl(c3(L.color[0], L.color[1], L.color[2]), power), refl);
                        acc = cadd(acc, cmul(bc, lc));
                    }
                }
                C3 dcol = cclamp(acc);
                const int kind = __float_as_int(park[64 * PK_KIND]);
                if (kind == 0) {  // Diffuse
                    ret = dcol;
                    unwind = true;
                } else {  // Reflecting (rendering.rs:86-91)
                    if (kind == 1) {  // the reflection ray would be at depth >= max (rendering.rs:123-124)
                        const float r = park[64 * PK_R];
                        ret = cadd(cscl(dcol, 1.0f - r), cscl(def, r));
                        unwind = true;
                    } else {
                        RG_REGION(RGR_PUSH_REFL);  // frame writes: 5 dwords per lane (D.rgb, r, type)
                        auto &&f = stk[sp++];  // rendering.rs:88
                        f.type = FR_REFL;
                        f.f[0] = dcol.r; f.f[1] = dcol.g; f.f[2] = dcol.b; f.f[3] = park[64 * PK_R];
                        // q = the reflection ray (origin = the shadow origin, direction set at the hit)
                        // without task splitting the stack index is the depth; a lane tracing a pooled
                        // subtree starts at sp = 0 with a non-zero depth, so TASKS keeps the hit's depth
                        qdepth = TASKS ? qdepth + 1 : sp;
                        mode = MODE_CLOSEST;
                        n_sec++;
                    }
                }
              }
            } else if (shade) {
                // shade_diffuse loop body (rendering.rs:141-170), one light per iteration
                const RgMatDev m = T.mats[hb];
                if (rmode == MODE_SHADOW) {
                    const float refl = m.albedo_pi;  // albedo / PI (rendering.rs:164)
#pragma unroll
                    for (int l = 0; l < LB; ++l) {
                        if (li + l < a.n_lights) {
                            const RgLightDev L = T.lights[li + l];
                            float inten = !((occl >> l) & 1u) ? light_intensity(L, hp) : 0.0f;
                            float power = fmaxf((float)dot(hn, sb.d[l]), 0.0f) * inten;
                            C3 lc = cscl(cscl(c3(L.color[0], L.color[1], L.color[2]), power), refl);
                            fin = cadd(fin, cmul(bcol, lc));
                        }
                    }
                    if constexpr (!LIGHTP && TASKS && RG_SHADOW_FAN > 0) {
                        // the lights helper lanes traced, in light order (rendering.rs:141-170)
                        for (int k = 0; k < nfan; ++k) {
                            const RgLightDev L = T.lights[li + 1 + k];
                            V3 ldir;
                            double ldist;
                            light_dir_dist(L, hp, ldir, ldist);  // as at setup: same bits
                            float inten = !((fan_bits >> k) & 1u) ? light_intensity(L, hp) : 0.0f;
                            float power = fmaxf((float)dot(hn, ldir), 0.0f) * inten;
                            C3 lc = cscl(cscl(c3(L.color[0], L.color[1], L.color[2]), power), refl);
                            fin = cadd(fin, cmul(bcol, lc));
                        }
                        li += nfan;
                        nfan = 0;
                    }
                    li += LB;
                }
                if (li < a.n_lights) {
                    q.o = add(hp, scl(hn, SHADOW_BIAS));  // rendering.rs:148
                    occl_full = 0u;
#pragma unroll
                    for (int l = 0; l < LB; ++l) {
                        if (li + l < a.n_lights) {
                            light_dir_dist(T.lights[li + l], hp, sb.d[l], sb.ld[l]);
                            occl_full |= 1u << l;
                            n_shadow++;
                        } else {
                            sb.d[l] = v3(0.0, 0.0, 1.0);
                            sb.ld[l] = 0.0;
                        }
                    }
                    mode = MODE_SHADOW;
                } else {
                    C3 dcol = cclamp(fin);
                    if (m.surface == RG_SURFACE_DIFFUSE) {
                        ret = dcol;
                        unwind = true;
                    } else {  // Reflecting (rendering.rs:86-91)
                        float r = m.reflectivity;
                        int cd = hdepth + 1;
                        if (cd >= max_depth) {
                            ret = cadd(cscl(dcol, 1.0f - r), cscl(def, r));
                            unwind = true;
                        } else {
                            RG_REGION(RGR_PUSH_REFL);  // frame writes: 5 dwords per lane (D.rgb, r, type)
                            auto &&f = stk[sp++];
                            f.type = FR_REFL;
                            f.f[0] = dcol.r; f.f[1] = dcol.g; f.f[2] = dcol.b; f.f[3] = r;
                            q.o = add(hp, scl(hn, SHADOW_BIAS));  // ray.rs:57; q.d set at the hit
                            qdepth = cd;
                            mode = MODE_CLOSEST;
                            n_sec++;
                        }
                    }
                }
            }
            if (unwind) {
                RG_REGION(RGR_UNWIND);
                for (;;) {
                    RG_REGION(RGR_UNWIND_STEP);
                    if (sp == 0) {
                        bool handed = false;
                        if constexpr (TASKS) {
                            if (task >= 0) {  // a published subtree: hand its colour back
                                pool_finish(task, ret);
                                task = -1;
                                handed = true;
                            }
                        }
                        if (!handed) {
                            const uint32_t px = f32_to_u8(ret.r * 255.0f) | (f32_to_u8(ret.g * 255.0f) << 8) |
                                                (f32_to_u8(ret.b * 255.0f) << 16) | 0xFF000000u;
                            if (HOSTF && a.defer_px) *my_px = px;
                            else a.rgba[oidx] = px;
#if !defined(RG_TILE_TIMES) && !defined(RG_WAVE_TIMES)
                            if (a.rgb) { a.rgb[3 * oidx] = ret.r; a.rgb[3 * oidx + 1] = ret.g; a.rgb[3 * oidx + 2] = ret.b; }
#endif
                        }
                        mode = MODE_DONE;
                        break;
                    }
                    auto &&f = stk[sp - 1];
                    if constexpr (TASKS) {
                        const int ftype = f.type & 0xFF;
                        if (ftype == FR_REFR_TASK || ftype == FR_REFR_WAIT) {
                            const int slot = f.type >> 8;
                            if (ftype == FR_REFR_TASK) {  // ret = the transmission subtree's colour
                                f.f[5] = ret.r; f.f[6] = ret.g; f.f[7] = ret.b;
                                if (pool_reclaim(slot)) {  // nobody took the reflection ray: trace it here
                                    const double *r = pool_of().ray[slot];
                                    q.o = v3(r[0], r[1], r[2]);
                                    q.d = v3(r[3], r[4], r[5]);
                                    pool_release(slot);
                                    f.type = FR_REFR_R;
                                    qdepth = f.cdepth;
                                    mode = MODE_CLOSEST;
                                    n_sec++;
                                    break;
                                }
                                f.type = FR_REFR_WAIT | (slot << 8);
                            }
                            if (!pool_done(slot)) {  // another lane is still tracing it
                                mode = MODE_WAIT;
                                break;
                            }
                            const C3 rc = c3(pool_of().col[slot][0], pool_of().col[slot][1], pool_of().col[slot][2]);
                            pool_release(slot);
                            const float kr = f.f[0];  // as FR_REFR_R below (rendering.rs:115-117)
                            C3 col = cadd(cscl(rc, kr), cscl(c3(f.f[5], f.f[6], f.f[7]), 1.0f - kr));
                            ret = cmul(cscl(col, f.f[1]), c3(f.f[2], f.f[3], f.f[4]));
                            sp--;
                            continue;
                        }
                    }
                    if (f.type == FR_REFL) {
                        ret = cadd(cscl(c3(f.f[0], f.f[1], f.f[2]), 1.0f - f.f[3]), cscl(ret, f.f[3]));
                        sp--;
                    } else if (f.type == FR_REFR_T) {
                        RG_REGION(RGR_UNWIND_REFRT);  // frame writes: 4 dwords per lane (Tc.rgb, type)
                        f.f[5] = ret.r; f.f[6] = ret.g; f.f[7] = ret.b;
                        f.type = FR_REFR_R;
                        q.o = v3(f.rr[0], f.rr[1], f.rr[2]);
                        q.d = v3(f.rr[3], f.rr[4], f.rr[5]);
                        qdepth = TASKS ? f.cdepth : sp;  // without tasks the stack index is the depth
                        mode = MODE_CLOSEST;
                        n_sec++;
                        break;
                    } else {  // FR_REFR_R (rendering.rs:115-117)
                        float kr = f.f[0];
                        C3 col = cadd(cscl(ret, kr), cscl(c3(f.f[5], f.f[6], f.f[7]), 1.0f - kr));
                        ret = cmul(cscl(col, f.f[1]), c3(f.f[2], f.f[3], f.f[4]));
                        sp--;
                    }
                }
            }
        }
        have_result = false;
        // every lane of the wave is done: its tile is complete (owners hold their pixels)
        if (HOSTF && my_tile != 0xFFFFFFFFu && (a.defer_px || a.tile_flags) && !__any(mode != MODE_DONE)) {
            bool ringed = false;
            if constexpr (RING > 0) {
                if (use_ring) {
                    ring_px[rw][nring][lane] = *my_px;
                    if (lane == 0) ring_tile[rw][nring] = my_tile;
                    if (++nring == ring_n) flush_ring();
                    ringed = true;
                }
            }
            if (!ringed) flush_tile(a, oidx, *my_px, my_tile, lane);
            my_tile = 0xFFFFFFFFu;
        }
        // a wave with no live lane takes the next tile
        if (tiles_left && !__any(mode != MODE_DONE)) {
            RG_REGION(RGR_TILE_FETCH);
#ifdef RG_TILE_TIMES
            if (cur_tile != 0xFFFFFFFFu && lane == 0 && a.rgb) {
                a.rgb[cur_tile] = (float)(wall_clock64() - t_tile) * 0.01f;  // 100 MHz clock
                a.rgb[ntiles + cur_tile] = (float)tile_iters;
                a.rgb[2 * ntiles + cur_tile] = (float)(t_tile & 0xFFFFFFull);  // start, 24-bit ticks (exact in f32)
                a.rgb[3 * ntiles + cur_tile] = (float)t_query * 0.01f;
            }
            cur_tile = 0xFFFFFFFFu;
#endif
            uint32_t tile = 0xFFFFFFFFu;
            if constexpr (RING > 0) {  // the rest of the wave's group of consecutive tiles
                if (use_ring && grp_next < grp_end) tile = grp_next++;
            }
            if (HOSTF && a.cancel) {  // streaming: the consumer stopped (rendering.rs:53-67 `.all` short-circuits)
                uint32_t cv = 0u;
                if (lane == 0) cv = __hip_atomic_load(a.cancel, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                if (__builtin_amdgcn_readfirstlane(__shfl((int)cv, 0, 64)) != 0) qtried = RG_NQ;
            }
            // ring mode: the queue hands out groups of RING consecutive tiles (one contiguous
            // run of host memory per ring flush: 4 KB with 64x1 tiles)
            const uint32_t qlimit = (RING > 0 && use_ring) ? (ntiles + ring_g - 1) / ring_g : ntiles;
            // Tile-slot prefetch (light path, device-resident launches): the slot claimed at the
            // previous tile's start, so the atomic's round trip overlaps that tile (round 4, same
            // box, interleaved: test1 0.2972 -> 0.2939 ms over 200 frames, test3 0.2656 -> 0.2631:
            // profiles/r04/s21/session.txt, s22).  Not on the heavy path: a claimed tile waits
            // behind the wave's current (long) one, which lengthens the tail (north star +0.6 %);
            // nor in the light path's persistent single launches (TPW < 0), for the same reason:
            // rg_render_multi's shares, whose waves ended by 84 us (p50) while claimed tiles still
            // started at 145 us (profiles/r05/s18, s26)
            if constexpr (!HOSTF && LIGHTP && TPW >= 0) {
                if (pf_valid) {  // the slot claimed at the previous tile's start
                    const uint32_t k = (uint32_t)__builtin_amdgcn_readfirstlane(__shfl((int)pf_k, 0, 64));
                    const unsigned long long t = (unsigned long long)k * RG_NQ + qi;
                    if (t < qlimit) tile = (uint32_t)t;
                    else { qi = (qi + 1) % RG_NQ; ++qtried; }  // that head is drained
                    pf_valid = false;
                }
            }
            while (tile == 0xFFFFFFFFu && qtried < RG_NQ) {
                uint32_t k = 0;
                if (lane == 0) k = atomicAdd(reinterpret_cast<unsigned int *>(&a.counters[RG_QUEUE_BASE + RG_QUEUE_STRIDE * qi]), 1u);
                k = __builtin_amdgcn_readfirstlane(__shfl(k, 0, 64));
                // head q serves tiles q, q+NQ, q+2NQ, ...: the tiles in flight stay a
                // compact raster-order band of the frame, as with a single head (the slot
                // prefetch above uses the same slot -> tile rule)
                const unsigned long long t = (unsigned long long)k * RG_NQ + qi;
                if (t < qlimit) {
                    tile = (uint32_t)t;
                    if constexpr (RING > 0) {
                        if (use_ring) {
                            tile = (uint32_t)t * ring_g;
                            grp_next = tile + 1u;
                            grp_end = min(tile + ring_g, ntiles);
                        }
                    }
                    break;
                }
                qi = (qi + 1) % RG_NQ;
                ++qtried;
            }
            if (tile == 0xFFFFFFFFu) {
                tiles_left = false;
            } else {
                constexpr uint32_t kmax = MAXD == 0 || HF || TPW < 0 ? 0u
                                          : LIGHTP ? (TPW > 0 ? (uint32_t)TPW : RG_LIGHT_TILES_PER_WAVE)
                                                   : RG_HEAVY_TILES_PER_WAVE;
                if constexpr (kmax > 0) {
                    // non-persistent: a wave renders at most kmax tiles, so the grid
                    // drains through the hardware dispatcher wave (block) by wave
                    if (++tiles_taken >= kmax) tiles_left = false;
                }
                if constexpr (!HOSTF && LIGHTP && TPW >= 0) {
                    // claim the wave's NEXT queue slot now: the atomic's round trip overlaps this
                    // tile's work instead of stalling the wave between tiles (the wave renders
                    // the claimed tile, or finds the head drained, at its next tile start)
                    if (tiles_left) {
                        if (lane == 0)
                            pf_k = atomicAdd(reinterpret_cast<unsigned int *>(&a.counters[RG_QUEUE_BASE + RG_QUEUE_STRIDE * qi]), 1u);
                        pf_valid = true;
                    }
                }
                if (a.tile_perm) tile = a.tile_perm[tile];  // scheduling order only; every tile is rendered once
#ifdef RG_WAVE_TIMES
                ++wt_tiles;
#endif
                if constexpr (HOSTF) my_tile = tile;
                const uint32_t ty = tile / tiles_x, tx = tile - ty * tiles_x;
#ifdef RG_TILE_TIMES
                cur_tile = tile;
                t_tile = wall_clock64();
                t_query = 0;
                tile_iters = 0;
#endif
                const uint32_t x = (tx << twlog) + ((uint32_t)lane & twmask);
                const uint32_t orow = ty * th + ((uint32_t)lane >> twlog);
                bool alive = x < a.width && orow < a.out_rows;
                const uint32_t y = alive ? out_row_to_y(a, orow) : 0u;
                oidx = (HOSTF && !alive) ? RG_NO_PIXEL : (size_t)out_row_of(a, orow) * a.width + x;
                if (HOSTF && a.image_rows && alive)  // the whole image: the pixel's own row (padding: no store)
                    oidx = y == 0xFFFFFFFFu ? RG_NO_PIXEL : (size_t)y * a.width + x;
                if (alive && y == 0xFFFFFFFFu) {  // padding row of a partial last tile
                    if (HOSTF && a.defer_px) *my_px = 0u;
                    else if (!HOSTF || oidx != RG_NO_PIXEL) a.rgba[oidx] = 0u;
#if !defined(RG_TILE_TIMES) && !defined(RG_WAVE_TIMES)
                    if (a.rgb) { a.rgb[3 * oidx] = 0.0f; a.rgb[3 * oidx + 1] = 0.0f; a.rgb[3 * oidx + 2] = 0.0f; }
#endif
                    alive = false;
                }
                pixel = y * a.width + x;
                if (alive) {
                    RG_REGION(RGR_PRIM);
                    // ray.rs:37-54 (aspect and fov_adjustment are per-frame constants)
                    double sx, sy;
                    // heavy path: the host's per-column / per-row table of the same expressions
                    // (north star -1 %); the light path keeps the divisions (the loads at the
                    // tile's start cost it more than they save: test1 +0.5 %, test3 +1.5 %)
                    if (!LIGHTP && a.prim_sx) {
                        sx = a.prim_sx[x];
                        sy = a.prim_sy[y];
                    } else {
                        sx = ((((double)x + 0.5) / a.width_d) * 2.0 - 1.0) * a.aspect * a.fov_adjustment;
                        sy = (1.0 - (((double)y + 0.5) / a.height_d) * 2.0) * a.fov_adjustment;
                    }
                    q.o = v3(0.0, 0.0, 0.0);
                    q.d = normalize(v3(sx, sy, -1.0));
                    n_prim++;
                    closest_init(c);
                    trace_primary<F32F, BVH>(a, src, q.d, c);
                    mode = MODE_CLOSEST;
                    qdepth = 0;
                    task = -1;
                    have_result = true;
                }
                continue;
            }
        }
        if constexpr (!LIGHTP && TASKS && RG_SHADOW_FAN > 0) {
            // shadow fan-out, assign: a lane about to trace the shadow ray of light li
            // hands lights li+1.. of the same hit to idle lanes of its wave, so up to
            // 1 + RG_SHADOW_FAN shadow rays of a hit are traced in one iteration instead
            // of one per iteration (the slowest pixels' ray trees are chains of such
            // iterations).  Each helper traces exactly the ray the lane would have.
            const int want = mode == MODE_SHADOW ? min(a.n_lights - li - 1, RG_SHADOW_FAN) : 0;
            unsigned long long owners = __ballot(want > 0);
            if (owners != 0ull) {
                unsigned long long idle = __ballot(mode == MODE_DONE);
                while (owners != 0ull && idle != 0ull) {
                    const int o = __builtin_ctzll(owners);
                    owners &= owners - 1ull;
                    const int w = __builtin_amdgcn_readlane(want, o);
                    const int oli = __builtin_amdgcn_readlane(li, o);
                    const int ohd = __builtin_amdgcn_readlane(hdepth, o);
                    const uint32_t opix = (uint32_t)__builtin_amdgcn_readlane((int)pixel, o);
                    const V3 ohp = v3(readlane_d(hp.x, o), readlane_d(hp.y, o), readlane_d(hp.z, o));
                    const V3 oso = v3(readlane_d(q.o.x, o), readlane_d(q.o.y, o), readlane_d(q.o.z, o));
                    uint32_t packed = 0u;
                    int k = 0;
                    for (; k < w && idle != 0ull; ++k) {
                        const int hl = __builtin_ctzll(idle);
                        idle &= idle - 1ull;
                        packed |= (uint32_t)hl << (6 * k);
                        if (lane == hl) {
                            hp = ohp;
                            q.o = oso;  // hit + n * bias (rendering.rs:148)
                            hdepth = ohd;
                            pixel = opix;  // error reports name the owner's pixel
                            light_dir_dist(T.lights[oli + 1 + k], hp, sb.d[0], sb.ld[0]);
                            li = oli + 1 + k;  // the light this helper traces (its li is unused otherwise)
                            mode = MODE_SHADOW_H;
                        }
                    }
                    if (lane == o) {
                        nfan = k;
                        fan_lanes = packed;
                        n_shadow += (uint32_t)k;
                    }
                }
            }
        }
        if constexpr (TASKS) {
            // idle lanes take subtrees other lanes of the block published
            const bool idle = mode == MODE_DONE;
            const unsigned long long want = __ballot(idle);
            if (want != 0ull && pool_any_pending()) {
                if (idle) {
                    const int slot = pool_take((int)__builtin_amdgcn_mbcnt_hi((uint32_t)(want >> 32),
                                                   __builtin_amdgcn_mbcnt_lo((uint32_t)want, 0u)));
                    if (slot >= 0) {
                        const double *r = pool_of().ray[slot];
                        q.o = v3(r[0], r[1], r[2]);
                        q.d = v3(r[3], r[4], r[5]);
                        qdepth = pool_of().depth[slot];
                        pixel = pool_of().pix[slot];
                        task = slot;
                        mode = MODE_CLOSEST;
                        n_sec++;  // the published reflection ray is traced here
                    }
                }
            }
        }
        const bool live = mode != MODE_DONE;
        const bool wave_live = __any(live);
        if constexpr (TASKS) {
            if (wave_live != counted) {  // the block's count of waves holding work (helpers' exit test)
                if (lane == 0) atomicAdd(&pool_of().busy, wave_live ? 1 : -1);
                counted = wave_live;
            }
        }
        if (!wave_live) {
            if (tiles_left) continue;
            if constexpr (!TASKS) break;
            // tiles exhausted: serve the block's tasks until no wave holds work
            if (!pool_any_pending() && __hip_atomic_load(&pool_of().busy, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0)
                break;
            __builtin_amdgcn_s_sleep(4);
            continue;
        }
        const bool querying = mode == MODE_CLOSEST || mode == MODE_SHADOW || mode == MODE_SHADOW_H;  // WAIT lanes only poll
        if (!__any(querying)) {
            __builtin_amdgcn_s_sleep(2);
            have_result = mode == MODE_WAIT;
            continue;
        }
#ifdef RG_ITER_STATS
        {  // SIMD use of the query iterations (diagnostic build), counters[4..11]: query
           // iterations, their querying lanes; iterations with a ray of depth >= 1, their
           // querying lanes, their depth >= 1 lanes; iterations with <= 16 querying lanes;
           // iterations with shadow lanes, shadow lanes
            const int qd = mode == MODE_CLOSEST ? qdepth : hdepth;
            const unsigned long long all = __ballot(querying), sec = __ballot(querying && qd >= 1);
            const unsigned long long shl = __ballot(querying && mode != MODE_CLOSEST);
            const unsigned n = (unsigned)__builtin_popcountll(all);
            if (lane == __builtin_ffsll((long long)__ballot(1)) - 1) {  // one atomic set per wave iteration
                atomicAdd(&a.counters[4], 1ull);
                atomicAdd(&a.counters[5], (unsigned long long)n);
                if (sec) {
                    atomicAdd(&a.counters[6], 1ull);
                    atomicAdd(&a.counters[7], (unsigned long long)n);
                    atomicAdd(&a.counters[8], (unsigned long long)__builtin_popcountll(sec));
                }
                if (n <= 16) atomicAdd(&a.counters[9], 1ull);
                if (shl) {
                    atomicAdd(&a.counters[10], 1ull);
                    atomicAdd(&a.counters[11], (unsigned long long)__builtin_popcountll(shl));
                }
                // light path (no BVH walk words): iterations with closest-hit lanes, those lanes
                if (LIGHTP && (all & ~shl)) {
                    atomicAdd(&a.counters[14], 1ull);
                    atomicAdd(&a.counters[15], (unsigned long long)__builtin_popcountll(all & ~shl));
                }
            }
        }
#endif
#ifdef RG_TILE_TIMES
        ++tile_iters;
        const unsigned long long t_q0 = wall_clock64();
#endif
        if (querying) {
            closest_init(c);
            occl = 0u;
        }
        if constexpr (!LIGHTP) {
            // one ray per lane, one pass: closest-hit and shadow lanes share the
            // body loop (best when a wave mixes ray kinds over many bodies)
            if (querying) {
                bool o1 = false;
                Ray r1;
                r1.o = q.o;
                const bool shadow = mode == MODE_SHADOW || mode == MODE_SHADOW_H;
                r1.d = shadow ? sb.d[0] : q.d;
                const bool lane_walk = (shadow ? hdepth : qdepth) >= (int)a.lane_min_depth;
                // a shadow ray that could see a NaN distance (ray_exotic) runs as a
                // fully counted closest-hit query: in_light = none || dist > light
                // distance (rendering.rs:150-155), the scene.rs:38 panic iff >= 2 hits, one NaN
                const bool exact = shadow && (a.nan_scene || ray_exotic(r1.o, r1.d));
                // li: the light of a shadow ray (owner lanes; fan-out helpers carry the light they trace)
                trace_query<F32F, BVH>(a, src, r1, shadow && !exact, sb.ld[0], c, o1, lane_walk, shadow ? li : -1);
                if (exact) {
                    o1 = c.id >= 0 && !(c.t > sb.ld[0]);
                    if (c.nan && c.nhit >= 2) raise_error(a, pixel, RG_ERR_NAN_DISTANCE);
                }
                occl = o1 ? 1u : 0u;
            }
        } else {
            // closest-hit lanes and shadow-batch lanes walk the body tables in two
            // passes; each pass is skipped when no lane of the wave needs it.  A
            // batch that could see a NaN distance (ray_exotic) instead runs its
            // lights one by one through the closest-hit pass, fully counted
            // (rendering.rs:150-155; the scene.rs:38 panic iff >= 2 hits, one NaN).
            bool exact = false;
            if (mode == MODE_SHADOW) {
                exact = a.nan_scene != 0;
#pragma unroll
                for (int l = 0; l < LB; ++l) exact |= ((occl_full >> l) & 1u) && ray_exotic(q.o, sb.d[l]);
            }
            const int passes = mode == MODE_CLOSEST ? 1 : exact ? LB : 0;
            if (exact) occl = ~occl_full & ((1u << LB) - 1u);
            for (int l = 0; __any(l < passes); ++l) {
                if (l < passes && (mode == MODE_CLOSEST || ((occl_full >> l) & 1u))) {
                    RG_REGION(RGR_Q_CLOSEST);
                    Ray rq;
                    rq.o = q.o;
                    rq.d = q.d;
                    double ld = 0.0;
                    if (exact) {
#pragma unroll
                        for (int k = 0; k < LB; ++k)
                            if (k == l) { rq.d = sb.d[k]; ld = sb.ld[k]; }
                        closest_init(c);
                    }
                    bool unused = false;
                    trace_query<F32F, BVH>(a, src, rq, false, 0.0, c, unused);
                    if (exact) {
                        if (c.id >= 0 && !(c.t > ld)) occl |= 1u << l;
                        if (c.nan && c.nhit >= 2) raise_error(a, pixel, RG_ERR_NAN_DISTANCE);
                    }
                }
            }
            if (mode == MODE_SHADOW && !exact) {
                RG_REGION(RGR_Q_SHADOW);
                occl = ~occl_full & ((1u << LB) - 1u);  // absent slots count as done
                trace_shadow<LB>(a, src, q.o, sb, (1u << LB) - 1u, occl);
            }
        }
#ifdef RG_TILE_TIMES
        t_query += wall_clock64() - t_q0;
#endif
        have_result = querying || mode == MODE_WAIT;
    }
    if (HOSTF && my_tile != 0xFFFFFFFFu && (a.defer_px || a.tile_flags)) {
        bool ringed = false;
        if constexpr (RING > 0) {
            if (use_ring) {
                ring_px[rw][nring][lane] = *my_px;
                if (lane == 0) ring_tile[rw][nring] = my_tile;
                ++nring;
                ringed = true;
            }
        }
        if (!ringed) flush_tile(a, oidx, *my_px, my_tile, lane);
    }
    if constexpr (RING > 0) {
        if (use_ring) flush_ring();
    }
#ifdef RG_TILE_TIMES
    if (cur_tile != 0xFFFFFFFFu && lane == 0 && a.rgb) {
        a.rgb[cur_tile] = (float)(wall_clock64() - t_tile) * 0.01f;
        a.rgb[ntiles + cur_tile] = (float)tile_iters;
        a.rgb[2 * ntiles + cur_tile] = (float)(t_tile & 0xFFFFFFull);
        a.rgb[3 * ntiles + cur_tile] = (float)t_query * 0.01f;
    }
#endif

    RG_STAT(14, RG_CLOCK() - t_kernel);
    RG_STAT(15, 1);
#ifdef RG_WAVE_TIMES
    if (lane == 0 && a.rgb) {  // wave w of the grid: 4 words at rgb[4 w]
        const unsigned long long t_end = wall_clock64();
        uint32_t *wt = reinterpret_cast<uint32_t *>(a.rgb) + 4u * (blockIdx.x * (blockDim.x / 64u) + (threadIdx.x >> 6));
        wt[0] = (uint32_t)t_wave0;
        wt[1] = (uint32_t)(t_staged - t_wave0);
        wt[2] = (uint32_t)(t_end - t_wave0);
        wt[3] = wt_tiles;
    }
#endif
#ifdef RG_BVH_STATS
    if (lane >= 4 && lane < 16) atomicAdd(&a.counters[lane], rg_stat_lds[(threadIdx.x >> 6) % RG_BVH_MAX_WAVES][lane]);
#endif
    // ray counters: wave reduction, one atomic per wave per class
    unsigned long long p64 = wave_sum(n_prim), s64 = wave_sum(n_shadow), q64 = wave_sum(n_sec);
    if (lane == 0) {
        if (p64) atomicAdd(&a.counters[0], p64);
        if (s64) atomicAdd(&a.counters[1], s64);
        if (q64) atomicAdd(&a.counters[2], q64);
        if (a.snap_out) {
            // the last wave to finish hands the statistics words to the host itself (the copy
            // after the kernel would be a blit kernel of its own on the stream): this wave's
            // counter atomics are complete before it is counted
            __builtin_amdgcn_s_waitcnt(0);
            const unsigned long long waves = (unsigned long long)gridDim.x * (blockDim.x >> 6);
            if (atomicAdd(&a.counters[RG_DONE_WORD], 1ull) == waves - 1ull) {
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    a.snap_out[k] = __hip_atomic_load(&a.counters[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
}

// Scene::trace for a batch of rays (rg_trace): one lane per ray.
__global__ __launch_bounds__(256) void rg_trace_kernel(RgKernelArgs a, const double *rays, uint32_t n,
                                                       double *dist, int32_t *body) {
    uint32_t i = blockIdx.x * 256u + threadIdx.x;
    bool alive = i < n;
    Ray r;
    r.o = v3(0, 0, 0);
    r.d = v3(0, 0, 1);
    if (alive) {
        r.o = v3(rays[6 * i], rays[6 * i + 1], rays[6 * i + 2]);
        r.d = v3(rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5]);
    }
    Closest c;
    closest_init(c);
    bool occl = false;
    if (alive) {
        SphScalar src{rg_cptr(a.sph), rg_cptr(a.sph_cc), rg_cptr(a.sphf), rg_cptr(a.sphf2),
                      rg_cptr(a.pln), rg_cptr(a.dsk), rg_cptr(a.box), rg_cptr(a.nodes), a.lbuf, a.lights};
        if (a.n_nodes > 0) trace_query<true, true>(a, src, r, false, 0.0, c, occl, a.lane_min_depth <= 1);
        else if (a.path == RG_PATH_HEAVY) trace_query<true, false>(a, src, r, false, 0.0, c, occl);
        else trace_query<false, false>(a, src, r, false, 0.0, c, occl);
        if (c.nan && c.nhit >= 2) raise_error(a, i, RG_ERR_NAN_DISTANCE);
        dist[i] = c.id >= 0 ? c.t : 0.0;
        body[i] = c.id;
    }
}

// ---------------------------------------------------------------- tile ordering
// A frame's makespan is max(average work per wave, slowest tile) only if the
// slowest tiles START early; in raster order an expensive band (refractive or
// reflective surfaces: ray trees of up to 2^depth rays per pixel) can start
// late and end the frame alone.  A probe traces 8 primary rays per 8x8 tile
// (NOT counted as rays of the frame), weights each by the material it hits,
// and a counting sort (wave-aggregated histogram, scan, scatter) orders the
// tile queue by descending weight (longest-processing-time-first).  This changes only the
// order in which tiles are dequeued: every pixel is still computed once, by
// the same code, so the output is identical.
#define RG_PROBE_SAMPLES 8   // per tile: 4 corners + 4 inner points; 8 tiles per wave
#define RG_ORDER_BUCKETS 16

__device__ __forceinline__ uint32_t probe_weight(const RgKernelArgs &a, const Closest &c) {
    if (c.id < 0) return 1u;                                        // sky: one ray
    const int s = a.mats[c.id].surface;
    const uint32_t diffuse = 2u + (uint32_t)a.n_lights;              // primary + shadow rays
    if (a.max_depth <= 1) return diffuse;
    if (s == RG_SURFACE_REFRACTIVE) return 8u * diffuse;            // a ray tree below the hit
    if (s == RG_SURFACE_REFLECTING) return 3u * diffuse;            // a reflection chain
    return diffuse;
}
// bucket 0 = heaviest; a tile's weight is the sum of its 8 samples
__device__ __forceinline__ uint32_t order_bucket(uint32_t w) {
    return (RG_ORDER_BUCKETS - 1u) - min(w >> 4, RG_ORDER_BUCKETS - 1u);
}

#define RG_ORDER_CHUNK 1024  // tiles per counting/scatter chunk (one wave each)

// 1) probe: 8 consecutive lanes per tile; writes the tile's bucket
template <bool BVH>
__global__ __launch_bounds__(256) void rg_tile_probe_kernel(RgKernelArgs a, uint32_t *bucket_of, uint32_t ntiles) {
    const uint32_t gid = blockIdx.x * 256u + threadIdx.x;
    const uint32_t tile = gid / RG_PROBE_SAMPLES, smp = gid % RG_PROBE_SAMPLES;
    const uint32_t tiles_x = rg_tiles_x(a), tw = rg_tile_w(a), th = rg_tile_h(a);
    bool alive = tile < ntiles;
    const uint32_t ty = alive ? tile / tiles_x : 0u, tx = alive ? tile - ty * tiles_x : 0u;
    // corners and inner points of an 8x8 tile, scaled to the tile's shape
    const uint32_t ox8 = (smp & 3u) == 0u ? 0u : (smp & 3u) == 1u ? 7u : (smp & 3u) == 2u ? 2u : 5u;
    const uint32_t oy8 = smp < 4u ? ((smp & 1u) ? 7u : 0u) : ((smp & 1u) ? 5u : 2u);
    const uint32_t x = min(tx * tw + ox8 * (tw - 1u) / 7u, a.width - 1u);
    const uint32_t orow = min(ty * th + oy8 * (th - 1u) / 7u, a.out_rows - 1u);
    const uint32_t y = alive ? out_row_to_y(a, orow) : 0u;
    uint32_t w = 0u;
    if (alive && y != 0xFFFFFFFFu) {
        Closest c;
        closest_init(c);
        SphScalar src{rg_cptr(a.sph), rg_cptr(a.sph_cc), rg_cptr(a.sphf), rg_cptr(a.sphf2),
                      rg_cptr(a.pln), rg_cptr(a.dsk), rg_cptr(a.box), rg_cptr(a.nodes), a.lbuf, a.lights};
        const double sx = a.prim_sx ? a.prim_sx[x]
                                    : ((((double)x + 0.5) / (double)a.width) * 2.0 - 1.0) * a.aspect * a.fov_adjustment;
        const double sy = a.prim_sy ? a.prim_sy[y] : (1.0 - (((double)y + 0.5) / (double)a.height) * 2.0) * a.fov_adjustment;
        trace_primary<true, BVH>(a, src, normalize(v3(sx, sy, -1.0)), c);
        w = probe_weight(a, c);
    }
    w += (uint32_t)__shfl_xor((int)w, 1, 64);
    w += (uint32_t)__shfl_xor((int)w, 2, 64);
    w += (uint32_t)__shfl_xor((int)w, 4, 64);
    if (alive && smp == 0u) bucket_of[tile] = order_bucket(w);
}

// 2) per-chunk bucket histograms (one wave per chunk; no global atomics)
__global__ __launch_bounds__(64) void rg_tile_count_kernel(const uint32_t *bucket_of, uint32_t *chunk_hist,
                                                           uint32_t ntiles) {
    __shared__ uint32_t hist[RG_ORDER_BUCKETS];
    const uint32_t lane = threadIdx.x;
    if (lane < RG_ORDER_BUCKETS) hist[lane] = 0u;
    __syncthreads();
    const uint32_t c0 = blockIdx.x * RG_ORDER_CHUNK, c1 = min(c0 + RG_ORDER_CHUNK, ntiles);
    for (uint32_t t = c0 + lane; t < c1; t += 64u) atomicAdd(&hist[bucket_of[t]], 1u);
    __syncthreads();
    if (lane < RG_ORDER_BUCKETS) chunk_hist[lane * gridDim.x + blockIdx.x] = hist[lane];  // bucket-major: the scan order
}

// 3) exclusive scan in (bucket, chunk) order -> each chunk's first slot per bucket
//    (one block: per-thread serial sums over contiguous ranges, shuffle scans)
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
    const int lane = (int)(threadIdx.x & 63u);
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, o, 64);
        if (lane >= o) x += y;
    }
    return x;
}
__global__ __launch_bounds__(1024) void rg_tile_scan_kernel(uint32_t *chunk_hist, uint32_t nchunks) {
    __shared__ uint32_t wave_tot[16];
    const uint32_t n = nchunks * RG_ORDER_BUCKETS;
    const uint32_t per = (n + 1023u) / 1024u;
    const uint32_t i0 = threadIdx.x * per, i1 = min(i0 + per, n);
    // chunk_hist is bucket-major (element k = bucket k / nchunks, chunk k % nchunks)
    auto at = [&](uint32_t k) -> uint32_t & { return chunk_hist[k]; };
    uint32_t sum = 0u;
    for (uint32_t k = i0; k < i1; ++k) sum += at(k);
    const uint32_t incl = wave_incl_scan(sum);
    const uint32_t w = threadIdx.x >> 6;
    if ((threadIdx.x & 63u) == 63u) wave_tot[w] = incl;
    __syncthreads();
    if (w == 0) {
        const uint32_t t = (threadIdx.x < 16u) ? wave_tot[threadIdx.x] : 0u;
        const uint32_t ti = wave_incl_scan(t);
        if (threadIdx.x < 16u) wave_tot[threadIdx.x] = ti - t;  // exclusive wave offsets
    }
    __syncthreads();
    uint32_t run = wave_tot[w] + incl - sum;
    for (uint32_t k = i0; k < i1; ++k) { const uint32_t v = at(k); at(k) = run; run += v; }
}

// 4) stable scatter: one wave walks its chunk in raster order
__global__ __launch_bounds__(64) void rg_tile_scatter_kernel(const uint32_t *bucket_of, const uint32_t *chunk_base,
                                                             uint32_t *perm, uint32_t ntiles) {
    __shared__ uint32_t cur[RG_ORDER_BUCKETS];
    const uint32_t lane = threadIdx.x;
    if (lane < RG_ORDER_BUCKETS) cur[lane] = chunk_base[lane * gridDim.x + blockIdx.x];
    __syncthreads();
    const uint32_t c0 = blockIdx.x * RG_ORDER_CHUNK, c1 = min(c0 + RG_ORDER_CHUNK, ntiles);
    for (uint32_t t0 = c0; t0 < c1; t0 += 64u) {
        const uint32_t t = t0 + lane;
        const bool act = t < c1;
        const uint32_t b = act ? bucket_of[t] : 0u;
        unsigned long long todo = __ballot(act);
        while (todo) {  // one pass per distinct bucket in this group of 64 tiles
            const uint32_t leader = (uint32_t)__builtin_ctzll(todo);
            const uint32_t k = (uint32_t)__shfl((int)b, (int)leader, 64);
            const unsigned long long grp = __ballot(act && b == k);
            if (act && b == k) perm[cur[k] + (uint32_t)__builtin_popcountll(grp & ((1ull << lane) - 1ull))] = t;
            __syncthreads();
            if (lane == leader) cur[k] += (uint32_t)__builtin_popcountll(grp);
            __syncthreads();
            todo &= ~grp;
        }
    }
}

// scratch: [bucket_of ntiles | chunk_hist 64 * nchunks (bucket-major)]
extern "C" size_t rg_tile_order_scratch_words(uint32_t ntiles) {
    const size_t nchunks = (ntiles + RG_ORDER_CHUNK - 1u) / RG_ORDER_CHUNK;
    return (size_t)ntiles + nchunks * RG_ORDER_BUCKETS;
}

extern "C" hipError_t rg_launch_tile_order(const RgKernelArgs *a, uint32_t *scratch, uint32_t *perm, hipStream_t stream) {
    const uint32_t ntiles = (uint32_t)rg_tile_count(*a);
    const uint32_t nchunks = (ntiles + RG_ORDER_CHUNK - 1u) / RG_ORDER_CHUNK;
    uint32_t *bucket_of = scratch, *chunk_hist = scratch + ntiles;
    const uint32_t lanes = ntiles * RG_PROBE_SAMPLES;
    if (a->n_nodes > 0)
        hipLaunchKernelGGL(rg_tile_probe_kernel<true>, dim3((lanes + 255u) / 256u), dim3(256), 0, stream, *a, bucket_of,
                           ntiles);
    else
        hipLaunchKernelGGL(rg_tile_probe_kernel<false>, dim3((lanes + 255u) / 256u), dim3(256), 0, stream, *a,
                           bucket_of, ntiles);
    hipLaunchKernelGGL(rg_tile_count_kernel, dim3(nchunks), dim3(64), 0, stream, bucket_of, chunk_hist, ntiles);
    hipLaunchKernelGGL(rg_tile_scan_kernel, dim3(1), dim3(1024), 0, stream, chunk_hist, nchunks);
    hipLaunchKernelGGL(rg_tile_scatter_kernel, dim3(nchunks), dim3(64), 0, stream, bucket_of, chunk_hist, perm, ntiles);
    return hipGetLastError();
}

// ---------------------------------------------------------------- launchers
// One persistent block per CU slot: grid = CUs x (blocks per CU the register
// and LDS budgets admit), capped by the tiles the frame has.
#ifndef RG_LIGHT_PERSIST_BLOCKS_PER_CU
// light persistent launches: one-wave blocks per CU (8 -> 6 once they stopped prefetching tile slots:
// test1 slowest 1/8 share 0.162-0.166 -> 0.153-0.156 ms, test3 0.139 -> 0.133; 4: 0.159, 12/16: slower;
// profiles/r05/s34, s35)
#define RG_LIGHT_PERSIST_BLOCKS_PER_CU 6
#endif
#ifndef RG_DEEP_BLOCKS_PER_CU
#define RG_DEEP_BLOCKS_PER_CU 8  // deep-stack light launches: resident one-wave blocks per CU (bounds the frame buffer)
#endif

// Occupancy of one kernel instantiation on the CURRENT device, cached per
// (device, kernel, dynamic LDS): hipFuncSetAttribute and the occupancy query
// are per device, and scenes on different devices (rg_render_multi) or host
// threads may launch the same instantiation.
struct OccKey {
    int dev;
    const void *kern;
    size_t lds;
};
static std::mutex occ_mu;
static std::vector<std::pair<OccKey, std::pair<int, int>>> occ_cache;  // -> (CUs, blocks per CU)

static hipError_t occupancy(const void *kern, int threads, size_t lds, int &cus, int &per_cu) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return hipErrorInvalidDevice;
    std::lock_guard<std::mutex> g(occ_mu);
    for (const auto &e : occ_cache)
        if (e.first.dev == dev && e.first.kern == kern && e.first.lds == lds) {
            cus = e.second.first;
            per_cu = e.second.second;
            return hipSuccess;
        }
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return hipErrorInvalidValue;
    if (lds > 64 * 1024 && hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
        return hipErrorInvalidValue;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, threads, lds) != hipSuccess)
        return hipErrorInvalidValue;
    if (per_cu < 1) return hipErrorInvalidConfiguration;
    occ_cache.push_back({OccKey{dev, kern, lds}, {cus, per_cu}});
    return hipSuccess;
}

// Launch (or, with grid_threads != nullptr, only size: the threads of the
// grid, which a MAXD == 0 launch needs for its frame buffer) one instantiation.
template <int MAXD, bool LSPH, bool LCOLD, int WPS, int LB, bool F32F, bool BVH, bool TASKS, int TPW = 0, bool HF = false>
static hipError_t launch_one(const RgKernelArgs *a, size_t lds, hipStream_t stream, size_t *grid_threads) {
    // Block size.  The heavy path shares one LDS copy of the scene (and the
    // BVH stacks / task pool) among the CU's 4*WPS waves: one block per CU.
    // The light path's scene is a few KB, so it runs small blocks, each with
    // its own copy: a block then holds its CU slot only while ITS waves work,
    // and with frames in flight the next frame's blocks take the slots of
    // waves that finished (a 4*WPS-wave block would keep the CU until its
    // slowest wave -- one refractive tile -- is done).
    constexpr int threads = LB != 1 ? 64 * RG_LIGHT_BLOCK_WAVES : 256 * WPS;  // LB != 1: the light path
    auto kern = rg_render_kernel<MAXD, LSPH, LCOLD, WPS, LB, F32F, BVH, TASKS, TPW, HF>;
    int cus = 0, per_cu = 0;
    const hipError_t oe = occupancy(reinterpret_cast<const void *>(kern), threads, lds, cus, per_cu);
    if (oe != hipSuccess) return oe;
    if ((MAXD == 0 || HF) && LB != 1 && per_cu > RG_DEEP_BLOCKS_PER_CU) per_cu = RG_DEEP_BLOCKS_PER_CU;
    // light single launches, persistent waves (TPW < 0): RG_LIGHT_PERSIST_BLOCKS_PER_CU one-wave
    // blocks per CU (2 per SIMD), never more than the occupancy query admits (a scene whose LDS
    // copy allows fewer would otherwise start the extra blocks only after the queue drained)
    if (MAXD != 0 && LB != 1 && TPW < 0) per_cu = std::min(per_cu, RG_LIGHT_PERSIST_BLOCKS_PER_CU);
    const unsigned long long tiles = rg_tile_count(*a);
    const unsigned long long waves = (unsigned long long)threads / 64u;
    unsigned long long blocks = (unsigned long long)cus * per_cu;
    const unsigned long long need = (tiles + waves - 1) / waves;
    if (blocks > need) blocks = need;
    if (LB == 1 && MAXD != 0 && a->pipelined) {
        // Heavy path, frames in flight: each persistent block takes >= RG_PIPE_TILES_PER_WAVE
        // tiles per wave, so its lifetime dwarfs its start (LDS staging) and its slowest
        // wave's tail, while every launch keeps >= 1/RG_PIPE_MIN_CU_DIV of the CUs; the other frames in
        // flight fill the rest.  North-star 1/8 share 0.440 -> 0.399 ms, 1/4 0.753 ->
        // 0.713, 8K 1/8 1.250 -> 1.220; whole frames unchanged (profiles/r02/ab_pipe_blocks.txt)
        const unsigned long long per = waves * RG_PIPE_TILES_PER_WAVE;
        unsigned long long cap = (tiles + per - 1) / per;
        const unsigned long long floor_blocks = ((unsigned long long)cus * per_cu + RG_PIPE_MIN_CU_DIV - 1) / RG_PIPE_MIN_CU_DIV;
        if (cap < floor_blocks) cap = floor_blocks;
        if (blocks > cap) blocks = cap;
    }
    constexpr unsigned long long kmax = MAXD == 0 || HF || TPW < 0 ? 0 : LB != 1 ? (TPW > 0 ? TPW : RG_LIGHT_TILES_PER_WAVE) : RG_HEAVY_TILES_PER_WAVE;
    if constexpr (kmax > 0)  // non-persistent: one wave per kmax tiles
        blocks = (tiles + waves * kmax - 1) / (waves * kmax);
    if (a->max_grid_threads && blocks * threads > a->max_grid_threads) blocks = a->max_grid_threads / threads;
    if (blocks < 1) blocks = 1;
    if (grid_threads) {
        *grid_threads = (size_t)blocks * threads;
        return hipSuccess;
    }
    if (MAXD == 0 && (a->deep_stack == nullptr || (unsigned long long)a->deep_stride < blocks * threads))
        return hipErrorInvalidValue;  // the caller sized the frame buffer for another grid
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(threads), lds, stream, *a);
    return hipGetLastError();
}

#ifndef RG_LDS_BUDGET
#define RG_LDS_BUDGET (160 * 1024)       // one block per CU owns the CU's LDS
#endif
#ifndef RG_HEAVY_F32_FILTER
#define RG_HEAVY_F32_FILTER true  // heavy path: f32 pre-filter in front of the exact sphere tests
#endif
// RG_HEAVY_SCENE_BODIES and the path decision (rg_heavy_path) live in rg_device.h

template <int MAXD, int WPS, int LB, bool F32F, bool BVH, bool TASKS, int TPW = 0, bool HF = false>
static hipError_t launch_waves(const RgKernelArgs *a, hipStream_t stream, size_t *gt) {
    // the BVH kernels also hold the static per-wave traversal stacks
    constexpr uint32_t budget = RG_LDS_BUDGET - (BVH ? (uint32_t)sizeof(rg_bvh_stack) : 0u) -
                                (uint32_t)(MAXD != 0 && !HF ? 0 : (LB != 1 ? RG_LIGHT_BLOCK_WAVES : 4 * WPS) * 64 * 4) -  // tile_px
                                (TASKS ? (uint32_t)sizeof(TaskPool) : 0u);
    if (a->lds_total_bytes <= budget)  // whole scene (empty sphere part if n_sph == 0)
        return launch_one<MAXD, true, true, WPS, LB, F32F, BVH, TASKS, TPW, HF>(a, a->lds_total_bytes, stream, gt);
    if (a->n_sph > 0 && a->lds_hot_bytes <= budget)
        return launch_one<MAXD, true, false, WPS, LB, F32F, BVH, TASKS, TPW, HF>(a, a->lds_hot_bytes, stream, gt);
    if constexpr (BVH) {  // the sphere tables do not fit: the BVH nodes alone, after the per-lane walk stacks
        const uint32_t nodes_lds = a->lds_lstack_bytes + (uint32_t)a->n_nodes * (uint32_t)sizeof(RgBvhNode);
        if (a->n_nodes > 0 && nodes_lds <= budget)
            return launch_one<MAXD, false, true, WPS, LB, F32F, BVH, TASKS, TPW, HF>(a, nodes_lds, stream, gt);
    }
    return launch_one<MAXD, false, false, WPS, LB, F32F, BVH, TASKS, TPW, HF>(a, a->lds_lstack_bytes, stream, gt);
}

#ifndef RG_LIGHT_BIG_TILES
#define RG_LIGHT_BIG_TILES 50000ull  // whole 4K frames and 1/2 shares (test1 1/2 share 0.1504 -> 0.1490 ms)
#endif
#ifndef RG_LIGHT_SINGLE_PERSISTENT
// light path: single launches run persistent waves (TPW < 0); 2: only launches below
// RG_LIGHT_BIG_TILES (rg_render_multi's shares and bands), at 2 waves per SIMD -- test1 1/8
// share 0.183 -> 0.166 ms, its 8-device rehearsal 0.3175 -> 0.297 ms (2.8x -> 3.0x); test3
// equal; 3 waves per SIMD: no gain (profiles/r04/s27/session.txt)
#define RG_LIGHT_SINGLE_PERSISTENT 2
#endif
#ifndef RG_LIGHT_WPS
#define RG_LIGHT_WPS 4            // light path: waves per SIMD (128 VGPRs; 3 -> 4: test1 -3 %, test3 -8 %, profiles/r02/ab_light_wps.txt)
#endif
#ifndef RG_LIGHT_TPW_BIG
// light path, 3-light batch: tiles per wave of whole-frame launches (0: off).  32: test1 0.2938 ->
// 0.2923 ms over 3 x 200 frames (-m gpu 284 passed, profiles/r06/s45), but 0.304 -> 0.319 ms in
// the driver's 20-frame configuration (longer waves, longer drain at the end of a short burst:
// s46), so off
#define RG_LIGHT_TPW_BIG 0
#endif
#ifndef RG_LIGHT_WPS_ONE
#define RG_LIGHT_WPS_ONE RG_LIGHT_WPS  // the one-light batch (118 VGPRs at 4 waves per SIMD)
#endif

template <int MAXD, bool HF = false>
static hipError_t launch_depth(const RgKernelArgs *a, hipStream_t stream, size_t *gt) {
    // Light scenes (few bodies): per-iteration overhead dominates -> fewer,
    // fatter iterations (RG_LB shadow rays per pass) at 2 waves/SIMD.  Heavy
    // scenes: the body loop dominates and waves mix ray kinds -> one ray per
    // lane in ONE shared loop, 4 waves/SIMD to hide LDS/FP64 latency.
    const bool heavy = rg_heavy_path(*a);
#ifndef RG_DEV_HEAVY_ONLY  // development builds: resource reports of the heavy kernels only
    if (!heavy) {
        if constexpr (HF) {
            // light host frames run the MAXD == 0 kernels: array-frame HF light kernels (9 spilled
            // VGPRs) measured slower into pinned memory, 0.768 -> 0.826 ms (profiles/r06/s5)
            return hipErrorInvalidValue;
        } else {
            // a launch on its own (not one of several frames in flight): persistent waves at full
            // occupancy balance the tiles dynamically, where a fixed tiles-per-wave grid makes every
            // wave render exactly that many tiles and the slowest wave's sum the makespan
            // (2: launches below RG_LIGHT_BIG_TILES tiles only -- rg_render_multi's shares and bands)
            const bool persistent = MAXD != 0 && RG_LIGHT_SINGLE_PERSISTENT && !a->pipelined &&
                                    (RG_LIGHT_SINGLE_PERSISTENT != 2 || rg_tile_count(*a) < RG_LIGHT_BIG_TILES);
#if RG_LB_ONE
            // one-light scenes: a batch of one (template LBT -1: 1 is the heavy path)
            if (a->n_lights <= 1) {
                if constexpr (MAXD != 0 && RG_LIGHT_SINGLE_PERSISTENT)
                    if (persistent) return launch_waves<MAXD, RG_LIGHT_WPS_ONE, -1, false, false, false, -1>(a, stream, gt);
                return launch_waves<MAXD, RG_LIGHT_WPS_ONE, -1, false, false, false>(a, stream, gt);
            }
#endif
#if RG_LB_SMALL > 1
            // scenes with at most RG_LB_SMALL lights: a batch that wide, not RG_LB (the per-light
            // loops of the shadow batch are unrolled over LB; test3's one light: 0.2525 -> 0.2293 ms
            // at LB 2, profiles/r06/s24)
            if (a->n_lights <= RG_LB_SMALL) {
                if constexpr (MAXD != 0 && RG_LIGHT_SINGLE_PERSISTENT)
                    if (persistent) return launch_waves<MAXD, RG_LIGHT_WPS, RG_LB_SMALL, false, false, false, -1>(a, stream, gt);
                return launch_waves<MAXD, RG_LIGHT_WPS, RG_LB_SMALL, false, false, false>(a, stream, gt);
            }
#endif
            if constexpr (MAXD != 0 && RG_LIGHT_SINGLE_PERSISTENT)
                if (persistent) return launch_waves<MAXD, RG_LIGHT_WPS, RG_LB, false, false, false, -1>(a, stream, gt);
#if RG_LIGHT_TPW_BIG > 0
            // whole frames (frames in flight): RG_LIGHT_TPW_BIG tiles per wave, half the waves of
            // RG_LIGHT_TILES_PER_WAVE (as a compile-time variant: test1 0.2968 -> 0.2943 ms over 200
            // frames, profiles/r06/s43); smaller launches (the 1/N shares) keep 16
            if constexpr (MAXD != 0)
                if (rg_tile_count(*a) >= RG_LIGHT_BIG_TILES)
                    return launch_waves<MAXD, RG_LIGHT_WPS, RG_LB, false, false, false, RG_LIGHT_TPW_BIG>(a, stream, gt);
#endif
            return launch_waves<MAXD, RG_LIGHT_WPS, RG_LB, false, false, false>(a, stream, gt);
        }
    }
#endif
#ifdef RG_DEV_LIGHT_ONLY  // development builds: resource reports of the light kernels only
    return hipErrorNotSupported;
#else
    const unsigned long long tiles = rg_tile_count(*a);
    // frames in flight (pipelined): the throughput-sized grid already keeps blocks long;
    // task splitting then costs more than it saves (1/8 share 0.400 -> 0.384 ms without:
    // profiles/r02/ab_task_split.txt); a single small launch keeps it (its latency)
    const bool tasks = RG_HEAVY_TASKS && tiles < RG_HEAVY_TASK_TILES && !a->pipelined;
    if (a->n_nodes > 0)
        return tasks ? launch_waves<MAXD, RG_HEAVY_WPS, 1, true, true, true, 0, HF>(a, stream, gt)
                     : launch_waves<MAXD, RG_HEAVY_WPS, 1, true, true, false, 0, HF>(a, stream, gt);
    return tasks ? launch_waves<MAXD, RG_HEAVY_WPS, 1, RG_HEAVY_F32_FILTER, false, true, 0, HF>(a, stream, gt)
                 : launch_waves<MAXD, RG_HEAVY_WPS, 1, RG_HEAVY_F32_FILTER, false, false, 0, HF>(a, stream, gt);
#endif
}

// Frame-stack capacity of each compiled array instantiation; deeper scenes use
// the global frame buffer (MAXD == 0).
extern "C" int rg_max_array_frames(void) { return 64; }

// Host-frame launches (pixels into page-locked host memory, tile publication,
// cancellation, other tile shapes) of heavy-path scenes needing at most this
// many frames run array-frame kernels with the host-frame features (HF:
// north star into pinned memory 2.59 -> 2.53 ms, profiles/r05/s15); deeper
// ones and light-path scenes the MAXD == 0 kernels (light HF measured slower:
// test1 0.878 -> 0.895 ms, 9 spills).
#ifndef RG_HOST_ARRAY_FRAMES
#define RG_HOST_ARRAY_FRAMES 8
#endif
extern "C" int rg_host_array_frames(void) { return RG_HOST_ARRAY_FRAMES; }

static bool host_frame_launch(const RgKernelArgs *a) {
    return a->defer_px || a->tile_flags || a->cancel || a->image_rows || a->tile_wlog != 3u;
}

// Does this launch keep its frames in the launch context's global buffer (the
// host sizes it with rg_render_grid_threads)?  Depths above the arrays.
extern "C" int rg_launch_global_frames(const RgKernelArgs *a, int maxd) {
    (void)a;
    return maxd > rg_max_array_frames();
}

static hipError_t dispatch_depth(const RgKernelArgs *a, int maxd, hipStream_t stream, size_t *gt) {
    if (host_frame_launch(a)) {
        if (RG_HOST_ARRAY_FRAMES > 0 && maxd <= RG_HOST_ARRAY_FRAMES && rg_heavy_path(*a))
            return launch_depth<8, true>(a, stream, gt);
#ifdef RG_DEV_ONE_DEPTH
        return hipErrorNotSupported;
#else
        return launch_depth<0>(a, stream, gt);
#endif
    }
#ifdef RG_DEV_ONE_DEPTH  // development builds: the MAXD = 8 instantiations only
    return maxd <= 8 ? launch_depth<8>(a, stream, gt) : hipErrorNotSupported;
#else
    if (maxd <= 8) return launch_depth<8>(a, stream, gt);
    if (maxd <= 16) return launch_depth<16>(a, stream, gt);
    if (maxd <= 64) return launch_depth<64>(a, stream, gt);
    return launch_depth<0>(a, stream, gt);
#endif
}

extern "C" hipError_t rg_launch_render(const RgKernelArgs *a, int maxd, hipStream_t stream) {
    return dispatch_depth(a, maxd, stream, nullptr);
}

// Threads of the grid rg_launch_render would use (frame-buffer sizing for maxd > 64).
extern "C" hipError_t rg_render_grid_threads(const RgKernelArgs *a, int maxd, size_t *threads) {
    return dispatch_depth(a, maxd, nullptr, threads);
}

extern "C" hipError_t rg_launch_trace(const RgKernelArgs *a, const double *rays, uint32_t n, double *dist,
                                      int32_t *body, hipStream_t stream) {
    dim3 grid((n + 255) / 256);
    // per-lane walk stacks (stride = block size): lane_stack entries + the spare slot
    const size_t lds = a->lane_stack > 0 ? ((size_t)(a->lane_stack + 1) * 4u) * 256u : 0u;
    hipLaunchKernelGGL(rg_trace_kernel, grid, dim3(256), lds, stream, *a, rays, n, dist, body);
    return hipGetLastError();
}
