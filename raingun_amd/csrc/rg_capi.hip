// rg_capi.hip — host side of libraingun_hip.so: the C ABI declared in
// include/raingun.h.  Scene upload (SoA hot tables + cold shading tables),
// tiled launches, ray counters, device error word, streaming bands and the
// batch closest-hit query.  No exception or abort crosses the ABI.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/raingun.h"
#include "../../include/raingun_debug.h"
#include "rg_bvh.h"
#include "rg_device.h"

#pragma clang fp contract(off)

#ifndef RG_BVH_MIN_SPHERES
#define RG_BVH_MIN_SPHERES 16  // below this a scan of the sphere table is as cheap as a traversal
#endif

extern "C" hipError_t rg_launch_render(const RgKernelArgs *a, int maxd, hipStream_t stream);
extern "C" hipError_t rg_launch_tile_order(const RgKernelArgs *a, uint32_t *scratch, uint32_t *perm, hipStream_t stream);
extern "C" size_t rg_tile_order_scratch_words(uint32_t ntiles);
extern "C" hipError_t rg_launch_trace(const RgKernelArgs *a, const double *rays, uint32_t n, double *dist,
                                      int32_t *body, hipStream_t stream);

// Per-stream launch state (ray counters, tile-queue heads, error word, tile
// ordering scratch, timing events).  Launches on distinct streams may run
// concurrently (frames in flight), so they must not share it; launches on one
// stream are ordered by the stream and reuse it.
struct rg_launch_ctx {
    hipStream_t stream = nullptr;
    unsigned long long *counters = nullptr;  // RG_COUNTER_WORDS words (rg_device.h)
    uint32_t *tile_cost = nullptr, *tile_perm = nullptr;  // probe/sort scratch (rg_launch_tile_order), order
    size_t tile_cap = 0;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
};

struct rg_scene {
    int device = 0;
    double fov = 90.0;
    float def[3] = {0, 0, 0};
    uint32_t max_depth = 10;
    int32_t n_sph = 0, n_pln = 0, n_dsk = 0, n_box = 0, n_bodies = 0, n_lights = 0, n_textures = 0;
    std::vector<void *> allocations;
    RgSph *sph = nullptr;
    double *sph_cc = nullptr;
    RgSphF *sphf = nullptr;
    RgSphF2 *sphf2 = nullptr;
    int32_t path = RG_PATH_AUTO;
    int32_t *sph_id = nullptr, *pln_id = nullptr, *dsk_id = nullptr, *box_id = nullptr;
    RgPln *pln = nullptr;
    RgDsk *dsk = nullptr;
    RgBox *box = nullptr;
    RgBodyDev *bodies = nullptr;
    RgMatDev *mats = nullptr;
    RgLightDev *lights = nullptr;
    RgTexDev *texs = nullptr;
    RgBvhNode *nodes = nullptr;  // sphere BVH (sphere tables are in its leaf order)
    int32_t n_nodes = 0;
    int32_t lane_stack = 0;      // per-lane walk stack entries the tree needs (0: per-lane walk unavailable)
#ifndef RG_LANE_MIN_DEPTH
#define RG_LANE_MIN_DEPTH 1
#endif
    int32_t lane_min_depth = RG_LANE_MIN_DEPTH;  // rays of this depth and deeper walk the BVH per lane
    bool bvh_enabled = true;
    float bvh_obound = 0.0f;
    double bvh_rbound = 0.0, bvh_margin = 0.0, bvh_extent = 0.0;
    rg_bvh_info bvh_info{};
    mutable std::vector<rg_launch_ctx *> ctxs;  // one per stream used
    mutable rg_launch_ctx *last = nullptr;       // the context of the latest launch (rg_debug_counters)
#ifndef RG_TILE_ORDER
#define RG_TILE_ORDER -1
#endif
    int tile_order = RG_TILE_ORDER;  // expensive tiles first (rg_kernels.hip "tile ordering"): -1 auto (heavy path), 0, 1
};

namespace {

constexpr int kMaxFrames = 64;  // largest compiled frame stack (rg_launch_render)

bool ok(hipError_t e) { return e == hipSuccess; }

template <class T>
rg_status upload(rg_scene *s, T **dst, const T *src, size_t n) {
    *dst = nullptr;
    if (n == 0) return RG_OK;
    void *p = nullptr;
    if (!ok(hipMalloc(&p, n * sizeof(T)))) return RG_ERR_OUT_OF_MEMORY;
    s->allocations.push_back(p);
    if (!ok(hipMemcpy(p, src, n * sizeof(T), hipMemcpyHostToDevice))) return RG_ERR_DEVICE;
    *dst = static_cast<T *>(p);
    return RG_OK;
}

double dot3(const double *a, const double *b) { return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]; }

// smallest float >= v (v finite, >= 0)
float f32_up(double v) {
    float f = (float)v;
    if ((double)f < v) f = std::nextafter(f, HUGE_VALF);
    return f;
}

// f32 pre-filter records of one sphere (bound derivation: rg_kernels.hip, "f32 pre-filter").
void make_filter_records(const double *p, RgSphF &f, RgSphF2 &f2) {
    const double u = 5.9604644775390625e-08;  // 2^-24
    const double r2 = p[3] * p[3];            // the reference's radius * radius (bodies.rs:97)
    const double cc = dot3(p, p);
    f.cx = (float)p[0];
    f.cy = (float)p[1];
    f.cz = (float)p[2];
    f.r2hi = std::max(f32_up(r2 * (1.0 + 4.0 * u)), 1e-30f);
    f2.cchi = f32_up(cc * (1.0 + 1e-6));
    f2.cc32 = (float)cc;
    const double kd1 = u * (16.2 + 26.2 * 1.00001) * 1.01;  // primary rays: |o| = 0, |d|^2 <= 1.00001
    f2.thrp = f32_up(((double)f.r2hi + kd1 * (double)f2.cchi) * (1.0 + 1e-6));
    f2.pad = 0.0f;
}

// f64::to_radians (2017 std: self * (PI / 180)), then libm tan (ray.rs:45).
double fov_adjustment(double fov) { return std::tan(fov * (3.14159265358979323846 / 180.0) / 2.0); }

void release(rg_scene *s) {
    if (!s) return;
    (void)hipSetDevice(s->device);
    for (void *p : s->allocations) (void)hipFree(p);
    s->allocations.clear();
    for (rg_launch_ctx *c : s->ctxs) {
        if (c->counters) (void)hipFree(c->counters);
        if (c->tile_cost) (void)hipFree(c->tile_cost);
        if (c->tile_perm) (void)hipFree(c->tile_perm);
        if (c->ev0) (void)hipEventDestroy(c->ev0);
        if (c->ev1) (void)hipEventDestroy(c->ev1);
        delete c;
    }
    delete s;
}

// The launch context of `stream`, created on first use (nullptr: out of memory / device error).
rg_launch_ctx *ctx_for(const rg_scene *s, hipStream_t stream) {
    for (rg_launch_ctx *c : s->ctxs)
        if (c->stream == stream) return c;
    rg_launch_ctx *c = new (std::nothrow) rg_launch_ctx();
    if (!c) return nullptr;
    c->stream = stream;
    void *p = nullptr;
    if (!ok(hipMalloc(&p, RG_COUNTER_WORDS * sizeof(unsigned long long)))) { delete c; return nullptr; }
    c->counters = static_cast<unsigned long long *>(p);
    if (!ok(hipEventCreate(&c->ev0)) || !ok(hipEventCreate(&c->ev1))) {
        (void)hipFree(c->counters);
        if (c->ev0) (void)hipEventDestroy(c->ev0);
        delete c;
        return nullptr;
    }
    s->ctxs.push_back(c);
    return c;
}

RgKernelArgs make_args(const rg_scene *s) {
    RgKernelArgs a;
    std::memset(&a, 0, sizeof a);
    a.sph = s->sph;
    a.sph_cc = s->sph_cc;
    a.sphf = s->sphf;
    a.sphf2 = s->sphf2;
    a.path = s->path;
    a.sph_id = s->sph_id;
    a.pln = s->pln;
    a.pln_id = s->pln_id;
    a.dsk = s->dsk;
    a.dsk_id = s->dsk_id;
    a.box = s->box;
    a.box_id = s->box_id;
    a.n_sph = s->n_sph;
    a.n_pln = s->n_pln;
    a.n_dsk = s->n_dsk;
    a.n_box = s->n_box;
    const bool bvh = s->bvh_enabled && s->n_nodes > 0;
    a.nodes = bvh ? s->nodes : nullptr;
    a.n_nodes = bvh ? s->n_nodes : 0;
    a.bvh_obound = s->bvh_obound;
    a.bvh_rbound = s->bvh_rbound;
    a.bvh_margin = s->bvh_margin;
    a.bvh_extent = s->bvh_extent;
#ifdef RG_BVH_DEBUG_OBOUND  // timing-only ablation builds (unsafe: skips the origin bound)
    a.bvh_obound = RG_BVH_DEBUG_OBOUND;
#endif
    a.bodies = s->bodies;
    a.mats = s->mats;
    a.lights = s->lights;
    a.texs = s->texs;
    a.n_bodies = s->n_bodies;
    a.n_lights = s->n_lights;
    a.n_textures = s->n_textures;
    // per-lane BVH walk (heavy path only): stacks of lane_stack entries per thread at LDS offset 0
    const bool lane = bvh && rg_heavy_path(a) && s->lane_stack > 0 && s->lane_min_depth < 1 << 20;
    a.lane_stack = lane ? s->lane_stack : 0;
    a.lane_min_depth = lane ? s->lane_min_depth : 1 << 30;
    a.lds_lstack_bytes = (uint32_t)a.lane_stack * 256u * RG_HEAVY_WPS * 4u;
    // LDS arena: [lane stacks | sphf | sphf2 | sph | cc (padded to 16 B) | nodes | pln | dsk | box (padded) |
    //             bodies | mats | lights | texs]
    auto al16 = [](uint32_t v) { return (v + 15u) & ~15u; };
    a.lds_sphf = a.lds_lstack_bytes;
    a.lds_sph = a.lds_sphf + (uint32_t)s->n_sph * (uint32_t)(sizeof(RgSphF) + sizeof(RgSphF2));
    a.lds_cc = a.lds_sph + (uint32_t)s->n_sph * (uint32_t)sizeof(RgSph);
    a.lds_nodes = al16(a.lds_cc + (uint32_t)s->n_sph * 8u);
    a.lds_pln = a.lds_nodes + (uint32_t)a.n_nodes * (uint32_t)sizeof(RgBvhNode);
    a.lds_dsk = a.lds_pln + (uint32_t)s->n_pln * (uint32_t)sizeof(RgPln);
    a.lds_box = a.lds_dsk + (uint32_t)s->n_dsk * (uint32_t)sizeof(RgDsk);
    a.lds_bodies = al16(a.lds_box + (uint32_t)s->n_box * (uint32_t)sizeof(RgBox));
    a.lds_hot_bytes = a.lds_bodies;
    a.lds_mats = a.lds_bodies + (uint32_t)s->n_bodies * (uint32_t)sizeof(RgBodyDev);
    a.lds_lights = al16(a.lds_mats + (uint32_t)s->n_bodies * (uint32_t)sizeof(RgMatDev));
    a.lds_texs = a.lds_lights + (uint32_t)s->n_lights * (uint32_t)sizeof(RgLightDev);
    a.lds_total_bytes = a.lds_texs + (uint32_t)s->n_textures * (uint32_t)sizeof(RgTexDev);
    a.def[0] = s->def[0];
    a.def[1] = s->def[1];
    a.def[2] = s->def[2];
    a.max_depth = s->max_depth;
    a.fov_adjustment = fov_adjustment(s->fov);
    return a;
}

bool tiling_valid(const rg_tiling *t) {
    return t && t->tile_rows > 0 && t->tile_stride > 0 && t->tile_offset < t->tile_stride;
}

int frames_needed(uint32_t max_depth) { return max_depth > 1 ? (int)max_depth - 1 : 1; }

}  // namespace

extern "C" {

int32_t rg_abi_version(void) { return RG_ABI_VERSION; }

const char *rg_status_string(int32_t st) {
    switch (st) {
    case RG_OK: return "ok";
    case RG_ERR_INVALID_ARGUMENT: return "invalid argument";
    case RG_ERR_PORTRAIT: return "width must be >= height (ray.rs:42)";
    case RG_ERR_AABB_NORMAL: return "could not determine normal of point (bodies.rs:324)";
    case RG_ERR_NAN_DISTANCE: return "NaN intersection distance compared (scene.rs:38)";
    case RG_ERR_TRANSMISSION: return "transmission ray is None while kr < 1 (rendering.rs:106)";
    case RG_ERR_TEXTURE: return "texture index out of range or empty texture";
    case RG_ERR_DEVICE: return "HIP runtime error";
    case RG_ERR_OUT_OF_MEMORY: return "out of device memory";
    case RG_ERR_CANCELLED: return "cancelled by the tile callback";
    default: return "unknown status";
    }
}

int32_t rg_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

uint32_t rg_tiling_rows(uint32_t height, const rg_tiling *t) {
    if (!tiling_valid(t) || height == 0) return 0;
    uint32_t tiles = (height + t->tile_rows - 1) / t->tile_rows;
    uint32_t mine = tiles > t->tile_offset ? (tiles - t->tile_offset + t->tile_stride - 1) / t->tile_stride : 0;
    return mine * t->tile_rows;
}

rg_status rg_scene_create(const rg_scene_desc *d, int32_t device, rg_scene **out) {
    if (!d || !out) return RG_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    if ((d->n_bodies && !d->bodies) || (d->n_lights && !d->lights) || (d->n_textures && !d->textures))
        return RG_ERR_INVALID_ARGUMENT;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return RG_ERR_DEVICE;
    // validate enums and textures on the host first
    for (uint32_t i = 0; i < d->n_bodies; ++i) {
        const rg_body &b = d->bodies[i];
        if (b.kind > RG_BODY_AABB || b.material.coloration > RG_COLORATION_TEXTURE ||
            b.material.surface > RG_SURFACE_REFRACTIVE)
            return RG_ERR_INVALID_ARGUMENT;
        if (b.material.coloration == RG_COLORATION_TEXTURE) {
            int32_t t = b.material.texture;
            if (t < 0 || (uint32_t)t >= d->n_textures || !d->textures[t].rgba || d->textures[t].width == 0 ||
                d->textures[t].height == 0 || d->textures[t].width > 0x7fffffffu || d->textures[t].height > 0x7fffffffu)
                return RG_ERR_TEXTURE;
        }
    }
    for (uint32_t i = 0; i < d->n_lights; ++i)
        if (d->lights[i].kind > RG_LIGHT_SPHERICAL) return RG_ERR_INVALID_ARGUMENT;

    rg_scene *s = new (std::nothrow) rg_scene();
    if (!s) return RG_ERR_OUT_OF_MEMORY;
    s->device = device;
    s->fov = d->fov;
    std::memcpy(s->def, d->default_color, sizeof s->def);
    s->max_depth = d->max_recursion_depth;
    if (!ok(hipSetDevice(device))) { release(s); return RG_ERR_DEVICE; }

    std::vector<RgSph> sph;
    std::vector<double> sph_raw;  // center xyz, radius (BVH build input)
    std::vector<RgSphF> sphf;
    std::vector<RgSphF2> sphf2;
    std::vector<double> sph_cc;
    std::vector<int32_t> sph_id, pln_id, dsk_id, box_id;
    std::vector<RgPln> pln;
    std::vector<RgDsk> dsk;
    std::vector<RgBox> box;
    std::vector<RgBodyDev> bodies(d->n_bodies);
    std::vector<RgMatDev> mats(d->n_bodies);
    for (uint32_t i = 0; i < d->n_bodies; ++i) {
        const rg_body &b = d->bodies[i];
        const double *p = b.p;
        bodies[i].kind = (int32_t)b.kind;
        bodies[i].pad = 0;
        std::memcpy(bodies[i].p, b.p, sizeof bodies[i].p);
        const rg_material &m = b.material;
        RgMatDev &md = mats[i];
        md.coloration = (int32_t)m.coloration;
        std::memcpy(md.color, m.color, sizeof md.color);
        md.tex = m.texture;
        md.xoff = m.x_offset;
        md.yoff = m.y_offset;
        md.albedo = m.albedo;
        md.surface = (int32_t)m.surface;
        md.reflectivity = m.reflectivity;
        md.index = m.index;
        md.transparency = m.transparency;
        switch (b.kind) {
        case RG_BODY_SPHERE:
            // r2 = radius * radius and cc = (c.c) evaluated exactly as the per-ray
            // reference expressions (bodies.rs:95,97) -> bit-identical.
            sph.push_back(RgSph{p[0], p[1], p[2], p[3] * p[3]});
            sphf.emplace_back();
            sphf2.emplace_back();
            make_filter_records(p, sphf.back(), sphf2.back());
            sph_cc.push_back(dot3(p, p));  // padded to an even count after the loop
            sph_id.push_back((int32_t)i);
            sph_raw.insert(sph_raw.end(), p, p + 4);
            break;
        case RG_BODY_PLANE:
            pln.push_back(RgPln{p[0], p[1], p[2], p[3], p[4], p[5], dot3(p, p + 3), 0.0});
            pln_id.push_back((int32_t)i);
            break;
        case RG_BODY_DISK:
            dsk.push_back(RgDsk{p[0], p[1], p[2], p[3], p[4], p[5], p[6], dot3(p, p + 3)});
            dsk_id.push_back((int32_t)i);
            break;
        default:
            box.push_back(RgBox{{p[0], p[1], p[2]}, {p[3], p[4], p[5]}});
            box_id.push_back((int32_t)i);
            break;
        }
    }
    // Sphere BVH: reorder the sphere tables into leaf order (sph_id keeps the
    // YAML index, so the closest-hit tie-break is unaffected).
    RgBvhBuild bvh;
    if ((int)sph.size() >= RG_BVH_MIN_SPHERES && rg_build_bvh(sph_raw.data(), (int)sph.size(), bvh)) {
        auto permute = [&](auto &v) {
            auto old = v;
            for (size_t j = 0; j < bvh.order.size(); ++j) v[j] = old[bvh.order[j]];
        };
        permute(sph);
        permute(sphf);
        permute(sphf2);
        permute(sph_cc);
        permute(sph_id);
        s->bvh_obound = bvh.obound;
        s->bvh_rbound = bvh.rbound;
        s->bvh_margin = bvh.margin;
        s->bvh_extent = bvh.extent;
        s->bvh_info.built = 1;
        s->bvh_info.nodes = (int32_t)bvh.nodes.size();
        s->bvh_info.leaves = bvh.leaves;
        s->bvh_info.depth = bvh.depth;
        s->bvh_info.lane_stack = bvh.lane_stack;
        s->bvh_info.margin = (float)bvh.margin;
        s->bvh_info.origin_bound = bvh.obound;
    }
    if (sph_cc.size() % 2) sph_cc.push_back(0.0);  // LDS staging copies 16-B units
    std::vector<RgLightDev> lights(d->n_lights);
    for (uint32_t i = 0; i < d->n_lights; ++i) {
        const rg_light &l = d->lights[i];
        lights[i].kind = (int32_t)l.kind;
        std::memcpy(lights[i].color, l.color, sizeof lights[i].color);
        lights[i].intensity = l.intensity;
        lights[i].pad = 0;
        std::memcpy(lights[i].v, l.v, sizeof lights[i].v);
        // Directional: normalize(-direction) (lights.rs:48) is a per-light constant.
        // Same IEEE ops in the same order as the device would run -> identical bits.
        double nx = -l.v[0], ny = -l.v[1], nz = -l.v[2];
        double inv = 1.0 / std::sqrt((nx * nx + ny * ny) + nz * nz);
        lights[i].dn[0] = nx * inv;
        lights[i].dn[1] = ny * inv;
        lights[i].dn[2] = nz * inv;
        lights[i].pad2 = 0.0;
    }
    s->n_sph = (int32_t)sph.size();
    s->n_pln = (int32_t)pln.size();
    s->n_dsk = (int32_t)dsk.size();
    s->n_box = (int32_t)box.size();
    s->n_bodies = (int32_t)d->n_bodies;
    s->n_lights = (int32_t)d->n_lights;
    s->n_textures = (int32_t)d->n_textures;

    rg_status st = RG_OK;
#define RG_UP(dst, vec) \
    if (st == RG_OK) st = upload(s, &s->dst, vec.data(), vec.size())
    RG_UP(sph, sph);
    RG_UP(sph_cc, sph_cc);
    RG_UP(sphf, sphf);
    RG_UP(sphf2, sphf2);
    RG_UP(sph_id, sph_id);
    RG_UP(pln, pln);
    RG_UP(pln_id, pln_id);
    RG_UP(dsk, dsk);
    RG_UP(dsk_id, dsk_id);
    RG_UP(box, box);
    RG_UP(box_id, box_id);
    RG_UP(bodies, bodies);
    RG_UP(mats, mats);
    RG_UP(lights, lights);
    RG_UP(nodes, bvh.nodes);
#undef RG_UP
    s->n_nodes = (int32_t)bvh.nodes.size();
    // the stack entry keeps the node index in its low RG_LANE_NODE_BITS bits
    s->lane_stack = (s->n_nodes <= (1 << RG_LANE_NODE_BITS) && bvh.lane_stack <= RG_LANE_STACK_MAX)
                        ? std::max(bvh.lane_stack, 1) : 0;
    // textures: RGBA8 -> one u32 per texel (one 4-byte gather per lookup)
    std::vector<RgTexDev> texs(d->n_textures);
    for (uint32_t i = 0; st == RG_OK && i < d->n_textures; ++i) {
        const rg_texture &t = d->textures[i];
        texs[i].w = (int32_t)t.width;
        texs[i].h = (int32_t)t.height;
        texs[i].texels = nullptr;
        size_t n = (size_t)t.width * t.height;
        if (n == 0 || !t.rgba) continue;
        uint32_t *dp = nullptr;
        st = upload(s, &dp, reinterpret_cast<const uint32_t *>(t.rgba), n);
        texs[i].texels = dp;
    }
    if (st == RG_OK) st = upload(s, &s->texs, texs.data(), texs.size());
    if (st == RG_OK && !(s->last = ctx_for(s, nullptr))) st = RG_ERR_OUT_OF_MEMORY;  // default-stream context
    if (st != RG_OK) { release(s); return st; }
    *out = s;
    return RG_OK;
}

void rg_scene_destroy(rg_scene *s) { release(s); }

rg_status rg_scene_set_max_depth(rg_scene *s, uint32_t max_depth) {
    if (!s) return RG_ERR_INVALID_ARGUMENT;
    s->max_depth = max_depth;
    return RG_OK;
}

rg_status rg_render_tiles_async(const rg_scene *s, uint32_t width, uint32_t height, const rg_tiling *tiling,
                                uint8_t *rgba_dev, float *rgb_dev, void *stream, rg_stats *stats) {
    if (!s || !rgba_dev || width == 0 || height == 0 || !tiling_valid(tiling)) return RG_ERR_INVALID_ARGUMENT;
    if (width < height) return RG_ERR_PORTRAIT;  // ray.rs:42
    if (frames_needed(s->max_depth) > kMaxFrames) return RG_ERR_INVALID_ARGUMENT;
    uint32_t out_rows = rg_tiling_rows(height, tiling);
    if ((unsigned long long)out_rows * width >= (1ull << 32) || (unsigned long long)height * width >= (1ull << 32))
        return RG_ERR_INVALID_ARGUMENT;  // the reference's u32 pixel index (rendering.rs:27)
    if (!ok(hipSetDevice(s->device))) return RG_ERR_DEVICE;
    hipStream_t st = static_cast<hipStream_t>(stream);
    rg_launch_ctx *cx = ctx_for(s, st);
    if (!cx) return RG_ERR_OUT_OF_MEMORY;
    s->last = cx;
    RgKernelArgs a = make_args(s);
    a.counters = cx->counters;
    a.width = width;
    a.height = height;
    a.tile_rows = tiling->tile_rows;
    a.tile_stride = tiling->tile_stride;
    a.tile_offset = tiling->tile_offset;
    a.out_rows = out_rows;
    a.aspect = (double)width / (double)height;
    a.rgba = reinterpret_cast<uint32_t *>(rgba_dev);
    a.rgb = rgb_dev;
    if (!ok(hipMemsetAsync(cx->counters, 0, RG_COUNTER_WORDS * sizeof(unsigned long long), st))) return RG_ERR_DEVICE;
    if (stats && !ok(hipEventRecord(cx->ev0, st))) return RG_ERR_DEVICE;  // kernel_ms includes the tile probe
    if (s->tile_order == 1 || (s->tile_order < 0 && rg_heavy_path(a))) {
        const size_t ntiles = (size_t)((width + 7u) / 8u) * ((out_rows + 7u) / 8u);
        if (ntiles > cx->tile_cap) {
            if (cx->tile_cost) (void)hipFree(cx->tile_cost);
            if (cx->tile_perm) (void)hipFree(cx->tile_perm);
            cx->tile_cost = cx->tile_perm = nullptr;
            cx->tile_cap = 0;
            if (!ok(hipMalloc(&cx->tile_cost, rg_tile_order_scratch_words((uint32_t)ntiles) * 4)) ||
                !ok(hipMalloc(&cx->tile_perm, ntiles * 4)))
                return RG_ERR_OUT_OF_MEMORY;
            cx->tile_cap = ntiles;
        }
        if (!ok(rg_launch_tile_order(&a, cx->tile_cost, cx->tile_perm, st))) return RG_ERR_DEVICE;
        a.tile_perm = cx->tile_perm;
    }
    if (out_rows == 0) return RG_OK;
    if (!ok(rg_launch_render(&a, frames_needed(s->max_depth), st))) return RG_ERR_DEVICE;
    if (!stats) return RG_OK;
    if (!ok(hipEventRecord(cx->ev1, st))) return RG_ERR_DEVICE;
    unsigned long long c[4];
    if (!ok(hipMemcpyAsync(c, cx->counters, sizeof c, hipMemcpyDeviceToHost, st))) return RG_ERR_DEVICE;
    if (!ok(hipStreamSynchronize(st))) return RG_ERR_DEVICE;
    float ms = 0.0f;
    (void)hipEventElapsedTime(&ms, cx->ev0, cx->ev1);
    stats->rays.primary = c[0];
    stats->rays.shadow = c[1];
    stats->rays.secondary = c[2];
    stats->kernel_ms = ms;
    stats->error_pixel = -1;
    if (c[3] != 0) {
        unsigned long long key = ~c[3];
        stats->error_pixel = (int32_t)(key >> 8);
        return (rg_status)(-(int32_t)(key & 0xff));
    }
    return RG_OK;
}

rg_status rg_render_tiles(const rg_scene *s, uint32_t width, uint32_t height, const rg_tiling *tiling,
                          uint8_t *rgba_out, float *rgb_out, rg_stats *stats) {
    if (!s || !rgba_out || width == 0 || height == 0 || !tiling_valid(tiling)) return RG_ERR_INVALID_ARGUMENT;
    if (width < height) return RG_ERR_PORTRAIT;
    if (!ok(hipSetDevice(s->device))) return RG_ERR_DEVICE;
    uint32_t rows = rg_tiling_rows(height, tiling);
    size_t npx = (size_t)rows * width;
    void *d_rgba = nullptr, *d_rgb = nullptr;
    if (!ok(hipMalloc(&d_rgba, npx * 4 + 4))) return RG_ERR_OUT_OF_MEMORY;
    if (rgb_out && !ok(hipMalloc(&d_rgb, npx * 12 + 4))) { (void)hipFree(d_rgba); return RG_ERR_OUT_OF_MEMORY; }
    rg_stats local;
    rg_stats *sp = stats ? stats : &local;
    rg_status st = rg_render_tiles_async(s, width, height, tiling, (uint8_t *)d_rgba, (float *)d_rgb, nullptr, sp);
    if (st == RG_OK || st < RG_ERR_INVALID_ARGUMENT) {
        if (!ok(hipMemcpy(rgba_out, d_rgba, npx * 4, hipMemcpyDeviceToHost))) st = RG_ERR_DEVICE;
        if (rgb_out && !ok(hipMemcpy(rgb_out, d_rgb, npx * 12, hipMemcpyDeviceToHost))) st = RG_ERR_DEVICE;
    }
    (void)hipFree(d_rgba);
    if (d_rgb) (void)hipFree(d_rgb);
    return st;
}

rg_status rg_render_image(const rg_scene *s, uint32_t width, uint32_t height, uint8_t *rgba_out, rg_stats *stats) {
    rg_tiling whole = {height ? height : 1, 1, 0};
    return rg_render_tiles(s, width, height, &whole, rgba_out, nullptr, stats);
}

rg_status rg_render_stream(const rg_scene *s, uint32_t width, uint32_t height, uint32_t tile_rows,
                           rg_tile_callback on_tile, void *user, rg_stats *stats) {
    if (!s || !on_tile || width == 0 || height == 0 || tile_rows == 0) return RG_ERR_INVALID_ARGUMENT;
    if (width < height) return RG_ERR_PORTRAIT;
    if (!ok(hipSetDevice(s->device))) return RG_ERR_DEVICE;
    // Bands are rendered one after another on one stream; while the host hands
    // band b to the callback, band b+1 is already rendering (double-buffered
    // pinned staging).  Counters accumulate on the host.
    uint32_t nb = (height + tile_rows - 1) / tile_rows;
    size_t band_px = (size_t)tile_rows * width;
    void *d_buf[2] = {nullptr, nullptr};
    void *h_buf[2] = {nullptr, nullptr};
    hipStream_t stream = nullptr;
    hipEvent_t done[2] = {nullptr, nullptr};
    rg_status st = RG_OK;
    rg_ray_counts total = {0, 0, 0};
    float total_ms = 0.0f;
    int32_t err_pixel = -1;
    rg_status err_status = RG_OK;
    for (int i = 0; i < 2 && st == RG_OK; ++i) {
        if (!ok(hipMalloc(&d_buf[i], band_px * 4 + 4)) || !ok(hipHostMalloc(&h_buf[i], band_px * 4 + 4)))
            st = RG_ERR_OUT_OF_MEMORY;
        else if (!ok(hipEventCreate(&done[i])))
            st = RG_ERR_DEVICE;
    }
    if (st == RG_OK && !ok(hipStreamCreate(&stream))) st = RG_ERR_DEVICE;
    for (uint32_t b = 0; st == RG_OK && b < nb; ++b) {
        int k = b & 1;
        rg_tiling t = {tile_rows, nb, b};
        rg_stats bs;
        st = rg_render_tiles_async(s, width, height, &t, (uint8_t *)d_buf[k], nullptr, stream, &bs);
        if (st < RG_ERR_INVALID_ARGUMENT && st != RG_ERR_DEVICE && st != RG_ERR_OUT_OF_MEMORY) {
            if (err_status == RG_OK) { err_status = st; err_pixel = bs.error_pixel; }
            st = RG_OK;
        }
        if (st != RG_OK) break;
        total.primary += bs.rays.primary;
        total.shadow += bs.rays.shadow;
        total.secondary += bs.rays.secondary;
        total_ms += bs.kernel_ms;
        uint32_t rows = (b + 1) * tile_rows <= height ? tile_rows : height - b * tile_rows;
        if (!ok(hipMemcpyAsync(h_buf[k], d_buf[k], (size_t)rows * width * 4, hipMemcpyDeviceToHost, stream)) ||
            !ok(hipStreamSynchronize(stream))) {
            st = RG_ERR_DEVICE;
            break;
        }
        if (on_tile(b * tile_rows, rows, width, (const uint8_t *)h_buf[k], user) != 0) {
            st = RG_ERR_CANCELLED;
            break;
        }
    }
    if (stream) (void)hipStreamDestroy(stream);
    for (int i = 0; i < 2; ++i) {
        if (d_buf[i]) (void)hipFree(d_buf[i]);
        if (h_buf[i]) (void)hipHostFree(h_buf[i]);
        if (done[i]) (void)hipEventDestroy(done[i]);
    }
    if (stats) {
        stats->rays = total;
        stats->kernel_ms = total_ms;
        stats->error_pixel = err_pixel;
    }
    if (st == RG_OK && err_status != RG_OK) return err_status;
    return st;
}

rg_status rg_debug_set_path(rg_scene *s, int32_t path) {
    if (!s || path < RG_PATH_AUTO || path > RG_PATH_HEAVY) return RG_ERR_INVALID_ARGUMENT;
    s->path = path;
    return RG_OK;
}

rg_status rg_debug_set_bvh(rg_scene *s, int32_t enable) {
    if (!s || (enable != 0 && enable != 1)) return RG_ERR_INVALID_ARGUMENT;
    s->bvh_enabled = enable != 0;
    return RG_OK;
}

rg_status rg_debug_bvh_info(const rg_scene *s, rg_bvh_info *info) {
    if (!s || !info) return RG_ERR_INVALID_ARGUMENT;
    *info = s->bvh_info;
    info->enabled = s->bvh_enabled && s->n_nodes > 0;
    return RG_OK;
}

rg_status rg_debug_set_lane_depth(rg_scene *s, int32_t min_depth) {
    if (!s) return RG_ERR_INVALID_ARGUMENT;
    s->lane_min_depth = min_depth < 0 ? RG_LANE_MIN_DEPTH : min_depth;
    return RG_OK;
}

rg_status rg_debug_set_tile_order(rg_scene *s, int32_t mode) {
    if (!s || mode < -1 || mode > 1) return RG_ERR_INVALID_ARGUMENT;
    s->tile_order = mode;
    return RG_OK;
}

rg_status rg_debug_counters(const rg_scene *s, uint64_t out[16]) {
    if (!s || !out) return RG_ERR_INVALID_ARGUMENT;
    if (!ok(hipSetDevice(s->device))) return RG_ERR_DEVICE;
    if (!ok(hipStreamSynchronize(s->last->stream)) ||
        !ok(hipMemcpy(out, s->last->counters, 16 * sizeof(uint64_t), hipMemcpyDeviceToHost)))
        return RG_ERR_DEVICE;
    return RG_OK;
}

rg_status rg_trace(const rg_scene *s, const double *rays, uint32_t n, double *dist, int32_t *body) {
    if (!s || (n && (!rays || !dist || !body))) return RG_ERR_INVALID_ARGUMENT;
    if (n == 0) return RG_OK;
    if (!ok(hipSetDevice(s->device))) return RG_ERR_DEVICE;
    void *d_rays = nullptr, *d_dist = nullptr, *d_body = nullptr;
    rg_status st = RG_OK;
    if (!ok(hipMalloc(&d_rays, (size_t)n * 48)) || !ok(hipMalloc(&d_dist, (size_t)n * 8)) ||
        !ok(hipMalloc(&d_body, (size_t)n * 4)))
        st = RG_ERR_OUT_OF_MEMORY;
    rg_launch_ctx *cx = ctx_for(s, nullptr);
    if (!cx) st = RG_ERR_OUT_OF_MEMORY;
    RgKernelArgs a = make_args(s);
    unsigned long long c[4] = {0, 0, 0, 0};
    if (st == RG_OK) { s->last = cx; a.counters = cx->counters; }
    if (st == RG_OK && (!ok(hipMemcpy(d_rays, rays, (size_t)n * 48, hipMemcpyHostToDevice)) ||
                        !ok(hipMemset(cx->counters, 0, sizeof c)) ||
                        !ok(rg_launch_trace(&a, (const double *)d_rays, n, (double *)d_dist, (int32_t *)d_body, nullptr)) ||
                        !ok(hipMemcpy(dist, d_dist, (size_t)n * 8, hipMemcpyDeviceToHost)) ||
                        !ok(hipMemcpy(body, d_body, (size_t)n * 4, hipMemcpyDeviceToHost)) ||
                        !ok(hipMemcpy(c, cx->counters, sizeof c, hipMemcpyDeviceToHost))))
        st = RG_ERR_DEVICE;
    if (d_rays) (void)hipFree(d_rays);
    if (d_dist) (void)hipFree(d_dist);
    if (d_body) (void)hipFree(d_body);
    if (st == RG_OK && c[3] != 0) st = (rg_status)(-(int32_t)((~c[3]) & 0xff));
    return st;
}

}  // extern "C"
