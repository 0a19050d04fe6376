// rg_capi.hip — host side of libraingun_hip.so: the C ABI declared in
// include/raingun.h.  Scene upload (SoA hot tables + cold shading tables),
// tiled launches, ray counters, device error words, the host-visible image
// path (banded renders overlapped with their device-to-host copies),
// streaming bands and the batch closest-hit query.  The single-process
// multi-GPU entry (rg_render_multi) is in rg_multi.hip.  No exception or
// abort crosses the ABI.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "../../include/raingun.h"
#include "../../include/raingun_debug.h"
#include "rg_bvh.h"
#include "rg_device.h"
#include "rg_lightbuf.h"
#include "rg_internal.h"

#pragma clang fp contract(off)

#ifndef RG_BVH_MIN_SPHERES
#define RG_BVH_MIN_SPHERES 16  // below this a scan of the sphere table is as cheap as a traversal
#endif
#ifndef RG_LANE_MIN_DEPTH
#define RG_LANE_MIN_DEPTH 1
#endif
#ifndef RG_TILE_ORDER
#define RG_TILE_ORDER -1
#endif

extern "C" hipError_t rg_launch_render(const RgKernelArgs *a, int maxd, hipStream_t stream);
extern "C" int rg_host_array_frames(void);
extern "C" hipError_t rg_render_grid_threads(const RgKernelArgs *a, int maxd, size_t *threads);
extern "C" int rg_max_array_frames(void);
extern "C" int rg_launch_global_frames(const RgKernelArgs *a, int maxd);
extern "C" hipError_t rg_launch_tile_order(const RgKernelArgs *a, uint32_t *scratch, uint32_t *perm, hipStream_t stream);
extern "C" size_t rg_tile_order_scratch_words(uint32_t ntiles);
extern "C" hipError_t rg_launch_trace(const RgKernelArgs *a, const double *rays, uint32_t n, double *dist,
                                      int32_t *body, hipStream_t stream);

namespace {

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
    f2.id = -1;  // set with sph_id
}

// f64::to_radians (2017 std: self * (PI / 180)), then libm tan (ray.rs:45).
double fov_adjustment(double fov) { return std::tan(fov * (3.14159265358979323846 / 180.0) / 2.0); }

// Parameters the body tests read (bodies.rs): sphere 4, plane 6, disk 7, AABB 6.
int body_params(uint32_t kind) { return kind == RG_BODY_SPHERE ? 4 : kind == RG_BODY_DISK ? 7 : 6; }

// A body or light parameter that is non-finite or >= 1e100 in magnitude: ray
// arithmetic may then overflow to NaN distances (rg_kernels.hip ray_exotic).
bool exotic_value(double v) { return !(std::fabs(v) < 1e100); }

void destroy_ctx(rg_launch_ctx *c) {
    if (c->counters) (void)hipFree(c->counters);
    if (c->sticky) (void)hipFree(c->sticky);
    if (c->tile_cost) (void)hipFree(c->tile_cost);
    if (c->tile_perm) (void)hipFree(c->tile_perm);
    if (c->deep) (void)hipFree(c->deep);
    if (c->prim) (void)hipFree(c->prim);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    delete c;
}

void release_image_res(rg_image_res &r) {
    for (hipStream_t &st : r.rs)
        if (st) { (void)hipStreamSynchronize(st); (void)hipStreamDestroy(st); st = nullptr; }
    if (r.cs) { (void)hipStreamSynchronize(r.cs); (void)hipStreamDestroy(r.cs); r.cs = nullptr; }
    for (hipEvent_t &e : r.ev_done) if (e) { (void)hipEventDestroy(e); e = nullptr; }
    for (hipEvent_t &e : r.ev_copy) if (e) { (void)hipEventDestroy(e); e = nullptr; }
    for (hipEvent_t *e : {&r.ev_t0, &r.ev_t1, &r.ev_join})
        if (*e) { (void)hipEventDestroy(*e); *e = nullptr; }
    if (r.d_rgba) (void)hipFree(r.d_rgba);
    if (r.d_rgb) (void)hipFree(r.d_rgb);
    if (r.h_stage) (void)hipHostFree(r.h_stage);
    if (r.h_frame) (void)hipHostFree(r.h_frame);
    if (r.h_flags) (void)hipHostFree(r.h_flags);
    if (r.h_cancel) (void)hipHostFree(r.h_cancel);
    if (r.h_snap) (void)hipHostFree(r.h_snap);
    r = rg_image_res{};
}

void release(rg_scene *s) {
    if (!s) return;
    (void)hipSetDevice(s->device);
    for (rg_frames *f : s->frames) rg_frames_detach_scene(f);
    s->frames.clear();
    rg_multi_release(s);
    release_image_res(s->img);
    for (void *p : s->allocations) (void)hipFree(p);
    s->allocations.clear();
    if (s->lds_blob) (void)hipFree(s->lds_blob);
    s->lds_blob = nullptr;
    for (rg_launch_ctx *c : s->ctxs) destroy_ctx(c);
    s->ctxs.clear();
    delete s;
}

// The launch context of `stream`, created on first use (nullptr: out of memory / device error).
rg_launch_ctx *ctx_for(const rg_scene *s, hipStream_t stream) {
    for (rg_launch_ctx *c : s->ctxs)
        if (c->stream == stream) return c;
    rg_launch_ctx *c = new (std::nothrow) rg_launch_ctx();
    if (!c) return nullptr;
    c->stream = stream;
    void *p = nullptr, *q = nullptr;
    if (!ok(hipMalloc(&p, 2 * RG_COUNTER_WORDS * sizeof(unsigned long long)))) { delete c; return nullptr; }
    c->counters = static_cast<unsigned long long *>(p);
    c->last_counters = c->counters;
    // stream-ordered: hipMemset on the null stream does not order against a
    // non-blocking stream's first launch
    if (!ok(hipMemsetAsync(p, 0, 2 * RG_COUNTER_WORDS * sizeof(unsigned long long), stream))) {
        destroy_ctx(c);
        return nullptr;
    }
    if (!ok(hipMalloc(&q, sizeof(unsigned long long))) || !ok(hipMemsetAsync(q, 0, sizeof(unsigned long long), stream))) {
        if (q) (void)hipFree(q);
        destroy_ctx(c);
        return nullptr;
    }
    c->sticky = static_cast<unsigned long long *>(q);
    if (!ok(hipEventCreate(&c->ev0)) || !ok(hipEventCreate(&c->ev1))) {
        destroy_ctx(c);
        return nullptr;
    }
    s->ctxs.push_back(c);
    return c;
}

bool tiling_valid(const rg_tiling *t) {
    return t && t->tile_rows > 0 && t->tile_stride > 0 && t->tile_offset < t->tile_stride;
}

int frames_needed(uint32_t max_depth) { return max_depth > 1 ? (int)max_depth - 1 : 1; }

const void *lds_blob_for(const rg_scene *s, const RgKernelArgs &a);  // below

// decode the complemented error key of counters[3] / a sticky word
rg_status decode_error(unsigned long long word, int32_t *pixel) {
    if (word == 0) return RG_OK;
    const unsigned long long key = ~word;
    if (pixel) *pixel = (int32_t)(key >> 8);
    return (rg_status)(-(int32_t)(key & 0xff));
}

}  // namespace

// ---------------------------------------------------------------- internal (rg_internal.h)

RgKernelArgs rg_make_args(const rg_scene *s) {
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
    // light buffers only with the BVH (the margins use its bounds; the kernel takes them on the BVH path)
    const bool lbuf = bvh && s->lbuf_enabled && (s->n_lbuf > 0 || s->lb_cam >= 0);
    a.lbuf = lbuf ? s->lbuf : nullptr;
    a.lb_start = lbuf ? s->lb_start : nullptr;
    a.lb_ent = lbuf ? s->lb_ent : nullptr;
    a.n_lbuf = lbuf ? s->n_lbuf : 0;
    a.lb_cam = lbuf ? s->lb_cam : -1;
    a.bodies = s->bodies;
    a.mats = s->mats;
    a.lights = s->lights;
    a.texs = s->texs;
    a.n_bodies = s->n_bodies;
    a.n_lights = s->n_lights;
    a.n_textures = s->n_textures;
    a.nan_scene = s->nan_scene ? 1 : 0;
    // per-lane BVH walk (heavy path only): stacks of lane_stack entries per thread at LDS offset 0
    const bool lane = bvh && rg_heavy_path(a) && s->lane_stack > 0 && s->lane_min_depth < 1 << 20;
    a.lane_stack = lane ? s->lane_stack : 0;
    a.lane_min_depth = lane ? s->lane_min_depth : 1 << 30;
    // lane_stack entries + one spare slot per lane (rg_kernels.hip bvh_lane, RG_LANE_BRANCHFREE)
    a.lds_lstack_bytes = lane ? ((uint32_t)(a.lane_stack + 1) * 4u) * 256u * RG_HEAVY_WPS : 0u;
    // LDS arena: [lane stacks | sphf | sphf2 | sph | cc (padded to 16 B) | nodes | pln | dsk | box (padded) |
    //             lights | texs (padded) | bodies | mats].  The hot part (staged whenever the sphere
    //             tables are) ends after the texture descriptors: lights and texture descriptors are a
    //             few hundred bytes that every shadow ray / textured hit reads with a per-lane index.
    auto al16 = [](uint32_t v) { return (v + 15u) & ~15u; };
    a.lds_sphf = a.lds_lstack_bytes;
    a.lds_sph = a.lds_sphf + (uint32_t)s->n_sph * (uint32_t)(sizeof(RgSphF) + sizeof(RgSphF2));
    a.lds_cc = a.lds_sph + (uint32_t)s->n_sph * (uint32_t)sizeof(RgSph);
    a.lds_nodes = al16(a.lds_cc + (uint32_t)s->n_sph * 8u);
    a.lds_pln = a.lds_nodes + (uint32_t)a.n_nodes * (uint32_t)sizeof(RgBvhNode);
    a.lds_dsk = a.lds_pln + (uint32_t)s->n_pln * (uint32_t)sizeof(RgPln);
    a.lds_box = a.lds_dsk + (uint32_t)s->n_dsk * (uint32_t)sizeof(RgDsk);
    a.lds_lights = al16(a.lds_box + (uint32_t)s->n_box * (uint32_t)sizeof(RgBox));
    a.lds_texs = a.lds_lights + (uint32_t)s->n_lights * (uint32_t)sizeof(RgLightDev);
    a.lds_lbuf = al16(a.lds_texs + (uint32_t)s->n_textures * (uint32_t)sizeof(RgTexDev));
    a.lds_bodies = a.lds_lbuf + (a.lbuf ? (uint32_t)s->n_lbdesc * (uint32_t)sizeof(RgLightBufDev) : 0u);
    a.lds_hot_bytes = a.lds_bodies;
    a.lds_mats = a.lds_bodies + (uint32_t)s->n_bodies * (uint32_t)sizeof(RgBodyDev);
    a.lds_total_bytes = a.lds_mats + (uint32_t)s->n_bodies * (uint32_t)sizeof(RgMatDev);
    a.def[0] = s->def[0];
    a.def[1] = s->def[1];
    a.def[2] = s->def[2];
    a.max_depth = s->max_depth;
    a.fov_adjustment = fov_adjustment(s->fov);
    a.tile_wlog = 3;  // 8x8 tiles
    return a;
}

rg_status rg_launch_tiles(const rg_scene *s, uint32_t width, uint32_t height, const rg_tiling *tiling,
                          uint8_t *rgba_dev, float *rgb_dev, hipStream_t st, unsigned long long *snap,
                          rg_launch_ctx **ctx_out, bool timed, uint32_t *tile_flags, uint32_t frame_seq,
                          const uint32_t *cancel, uint32_t tile_wlog, bool host_frame, bool pipelined,
                          uint32_t tile_first, uint32_t tile_count, bool image_rows, uint32_t tile_group) {
    if (tile_wlog < 3 || tile_wlog > 6) return RG_ERR_INVALID_ARGUMENT;
    if (image_rows && (!host_frame || rgb_dev)) return RG_ERR_INVALID_ARGUMENT;
    if (!s || !rgba_dev || width == 0 || height == 0 || !tiling_valid(tiling)) return RG_ERR_INVALID_ARGUMENT;
    if (tile_group < 1 || tiling->tile_offset + tile_group > tiling->tile_stride + (tile_group == 1 ? 1u : 0u))
        return RG_ERR_INVALID_ARGUMENT;
    if (width < height) return RG_ERR_PORTRAIT;  // ray.rs:42
    const uint32_t sel_rows = rg_tiling_rows_grouped(height, tiling, tile_group);  // every selected tile
    const uint32_t sel_tiles = sel_rows / tiling->tile_rows;
    if (tile_first > sel_tiles) return RG_ERR_INVALID_ARGUMENT;
    const uint32_t out_rows = std::min(sel_tiles - tile_first, tile_count) * tiling->tile_rows;
    if ((unsigned long long)out_rows * width >= (1ull << 32) || (unsigned long long)height * width >= (1ull << 32))
        return RG_ERR_INVALID_ARGUMENT;  // the reference's u32 pixel index (rendering.rs:27)
    if (!ok(hipSetDevice(s->device))) return RG_ERR_DEVICE;
    rg_launch_ctx *cx = ctx_for(s, st);
    if (!cx) return RG_ERR_OUT_OF_MEMORY;
    s->last = cx;
    if (ctx_out) *ctx_out = cx;
    RgKernelArgs a = rg_make_args(s);
    a.counters = cx->counters + (size_t)cx->cur * RG_COUNTER_WORDS;  // zero (see rg_launch_ctx::counters)
    a.counters_next = cx->counters + (size_t)(1 - cx->cur) * RG_COUNTER_WORDS;
    a.err_sticky = cx->sticky;
    a.width = width;
    a.height = height;
    a.tile_rows = tiling->tile_rows;
    a.tile_stride = tiling->tile_stride;
    a.tile_offset = tiling->tile_offset;
    a.tile_group = tile_group;
    a.tile_base = tile_first;
    a.out_rows = out_rows;
    a.aspect = (double)width / (double)height;
    a.width_d = (double)width;
    a.height_d = (double)height;
    a.rgba = reinterpret_cast<uint32_t *>(rgba_dev);
    a.rgb = rgb_dev;
    a.tile_flags = tile_flags;
    a.frame_seq = frame_seq;
    a.cancel = cancel;
    a.tile_wlog = tile_wlog;
    a.defer_px = host_frame ? 1u : 0u;
    a.image_rows = image_rows ? 1u : 0u;
    a.pipelined = pipelined ? 1u : 0u;
    const int frames = frames_needed(s->max_depth);
    // host-frame launches of heavy-path scenes run array-frame kernels with the
    // host-frame features (rg_kernels.hip HF) up to rg_host_array_frames() frames;
    // the others the MAXD == 0 kernels, whose frames live in a global buffer
    const bool host_arrays = frames <= rg_host_array_frames() && rg_heavy_path(a);
    if (host_frame) {  // the light path's LDS tile ring (rg_device.h RG_RING_*)
        const bool big = rg_tile_count(a) >= RG_RING_BIG_TILES;
        a.ring_flush = (uint32_t)std::max(0, big ? s->ring_flush_big : s->ring_flush_small);
        a.ring_group = (uint32_t)std::max(0, big ? s->ring_group_big : s->ring_group_small);
    }
    const int disp = (host_frame && !host_arrays) ? std::max(frames, rg_max_array_frames() + 1) : frames;
    if (rg_launch_global_frames(&a, disp) && out_rows > 0) {
        // frames in a global buffer sized for this launch's (persistent) grid
        size_t threads = 0;
        if (!ok(rg_render_grid_threads(&a, disp, &threads)) || threads == 0 || threads > 0xFFFFFFFFull)
            return RG_ERR_DEVICE;
        const size_t per_thread = (size_t)frames * RG_FRAME_BYTES;
        if (threads * per_thread > ((size_t)1 << 30)) {
            // very deep recursion (scene.rs:16 is a u32): a persistent grid that fits half the free
            // device memory (at most 16 GiB of frames) -- fewer waves, every depth still renders
            size_t free_b = 0, total_b = 0;
            if (!ok(hipMemGetInfo(&free_b, &total_b))) return RG_ERR_DEVICE;
            const size_t budget = std::min<size_t>(free_b / 2, (size_t)16 << 30);
            if (threads * per_thread > budget) {
                a.max_grid_threads = (uint32_t)std::min<size_t>(budget / per_thread, 0xFFFFFFFFu);
                if (!ok(rg_render_grid_threads(&a, disp, &threads)) || threads == 0) return RG_ERR_DEVICE;
                if (threads * per_thread > budget) return RG_ERR_OUT_OF_MEMORY;  // not even one block fits
            }
        }
        const size_t bytes = threads * per_thread;
        if (bytes > cx->deep_bytes) {
            if (cx->deep) (void)hipFree(cx->deep);
            cx->deep = nullptr;
            cx->deep_bytes = 0;
            if (!ok(hipMalloc(&cx->deep, bytes))) { (void)hipGetLastError(); cx->deep = nullptr; return RG_ERR_OUT_OF_MEMORY; }
            cx->deep_bytes = bytes;
        }
        a.deep_stack = cx->deep;
        a.deep_stride = (uint32_t)threads;
    }
    // primary-ray sensor coordinates per column / row (ray.rs:46-51), the
    // kernel's expressions evaluated here once per frame size (same IEEE
    // operations in the same order, no contraction: identical doubles)
    if (cx->prim_w != width || cx->prim_h != height || cx->prim_fov != a.fov_adjustment || !cx->prim) {
        const size_t n = (size_t)width + height;
        if (n > cx->prim_cap) {
            if (cx->prim) (void)hipFree(cx->prim);
            cx->prim = nullptr;
            cx->prim_cap = 0;
            void *q = nullptr;
            if (!ok(hipMalloc(&q, n * sizeof(double)))) { (void)hipGetLastError(); return RG_ERR_OUT_OF_MEMORY; }
            cx->prim = static_cast<double *>(q);
            cx->prim_cap = n;
        }
        std::vector<double> tab(n);
        for (uint32_t x = 0; x < width; ++x)
            tab[x] = ((((double)x + 0.5) / (double)width) * 2.0 - 1.0) * a.aspect * a.fov_adjustment;
        for (uint32_t y = 0; y < height; ++y)
            tab[(size_t)width + y] = (1.0 - (((double)y + 0.5) / (double)height) * 2.0) * a.fov_adjustment;
        // stream-ordered: earlier launches on this stream are done with the old table
        if (!ok(hipMemcpyAsync(cx->prim, tab.data(), n * sizeof(double), hipMemcpyHostToDevice, st)) ||
            !ok(hipStreamSynchronize(st)))
            return RG_ERR_DEVICE;
        cx->prim_w = width;
        cx->prim_h = height;
        cx->prim_fov = a.fov_adjustment;
    }
    a.prim_sx = cx->prim;
    a.prim_sy = cx->prim + width;
    if (!rg_heavy_path(a)) a.lds_blob = lds_blob_for(s, a);  // light path: one staging loop per block
    if (timed && !ok(hipEventRecord(cx->ev0, st))) return RG_ERR_DEVICE;  // kernel_ms includes the tile probe
    // expensive tiles first on the heavy path (probe-ordered light tiles measured slower:
    // DESIGN.md 4g); rg_debug_set_tile_order overrides
    if (s->tile_order == 1 || (s->tile_order < 0 && rg_heavy_path(a))) {
        const size_t ntiles = (size_t)rg_tile_count(a);
        const rg_launch_ctx::PermKey key{width, height, tiling->tile_rows, tiling->tile_stride, tiling->tile_offset,
                                         tile_first, out_rows, tile_wlog, s->max_depth, (uint32_t)s->n_lights,
                                         tile_group, a.fov_adjustment, s->mats};
        if (!(cx->perm_valid && cx->perm_key == key) && ntiles > cx->tile_cap) {
            if (cx->tile_cost) (void)hipFree(cx->tile_cost);
            if (cx->tile_perm) (void)hipFree(cx->tile_perm);
            cx->tile_cost = cx->tile_perm = nullptr;
            cx->tile_cap = 0;
            if (!ok(hipMalloc(&cx->tile_cost, rg_tile_order_scratch_words((uint32_t)ntiles) * 4)) ||
                !ok(hipMalloc(&cx->tile_perm, ntiles * 4)))
                return RG_ERR_OUT_OF_MEMORY;
            cx->tile_cap = ntiles;
        }
        if (ntiles > 0) {
            // the order depends only on the frame geometry and the scene: made once per
            // launch context and key, so a steady stream of frames runs ONE kernel each
            if (!(cx->perm_valid && cx->perm_key == key)) {
                cx->perm_valid = false;
                if (!ok(rg_launch_tile_order(&a, cx->tile_cost, cx->tile_perm, st))) return RG_ERR_DEVICE;
                cx->perm_valid = true;
                cx->perm_key = key;
            }
            a.tile_perm = cx->tile_perm;
        }
    }
    cx->last_counters = a.counters;
    // statistics words: written into page-locked host memory by the kernel's last wave, or copied
    unsigned long long *snap_dev = (snap && out_rows > 0)
                                       ? static_cast<unsigned long long *>(rg_host_device_ptr(snap, 4 * sizeof(*snap)))
                                       : nullptr;
    a.snap_out = snap_dev;
    if (out_rows > 0) {
        if (!ok(rg_launch_render(&a, disp, st))) return RG_ERR_DEVICE;
        cx->cur = 1 - cx->cur;  // the kernel zeroes the other set for the next launch
    }
    if (timed && !ok(hipEventRecord(cx->ev1, st))) return RG_ERR_DEVICE;
    if (snap && !snap_dev &&
        !ok(hipMemcpyAsync(snap, a.counters, 4 * sizeof(unsigned long long), hipMemcpyDeviceToHost, st)))
        return RG_ERR_DEVICE;
    return RG_OK;
}

rg_status rg_snap_status(const unsigned long long *snap, rg_stats *stats) {
    if (stats) {
        stats->rays.primary = snap[0];
        stats->rays.shadow = snap[1];
        stats->rays.secondary = snap[2];
        stats->error_pixel = -1;
    }
    return decode_error(snap[3], stats ? &stats->error_pixel : nullptr);
}

void *rg_host_device_ptr(void *p, size_t bytes) {
    if (!p || bytes == 0) return nullptr;
    auto dev = [](void *q) -> char * {
        hipPointerAttribute_t at;
        std::memset(&at, 0, sizeof at);
        if (hipPointerGetAttributes(&at, q) != hipSuccess) {
            (void)hipGetLastError();
            return nullptr;
        }
        return at.type == hipMemoryTypeHost ? static_cast<char *>(at.devicePointer) : nullptr;
    };
    char *d0 = dev(p), *d1 = dev(static_cast<char *>(p) + bytes - 1);
    // one mapping: the last byte's device address continues the first's
    return (d0 && d1 && d1 == d0 + (bytes - 1)) ? d0 : nullptr;
}

bool rg_host_is_pinned(const void *p, size_t bytes) {
    if (!p || bytes == 0) return false;
    auto one = [](const void *q) {
        hipPointerAttribute_t at;
        std::memset(&at, 0, sizeof at);
        if (hipPointerGetAttributes(&at, q) != hipSuccess) {
            (void)hipGetLastError();
            return false;
        }
        return at.type == hipMemoryTypeHost;
    };
    return one(p) && one(static_cast<const char *>(p) + bytes - 1);
}

namespace {

// Host tables of a scene: everything rg_scene_create uploads, kept so that
// rg_render_multi can place replicas on other devices.
rg_status upload_tables(rg_scene *s, const rg_host_tables &h) {
    rg_status st = RG_OK;
#define RG_UP(dst, vec) \
    if (st == RG_OK) st = upload(s, &s->dst, h.vec.data(), h.vec.size())
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
    RG_UP(nodes, nodes);
    RG_UP(lbuf, lbuf);
    RG_UP(lb_start, lb_start);
    RG_UP(lb_ent, lb_ent);
#undef RG_UP
    // textures: RGBA8 -> one u32 per texel (one 4-byte gather per lookup)
    std::vector<RgTexDev> texs(h.tex_w.size());
    for (size_t i = 0; st == RG_OK && i < texs.size(); ++i) {
        texs[i].w = (int32_t)h.tex_w[i];
        texs[i].h = (int32_t)h.tex_h[i];
        texs[i].texels = nullptr;
        if (h.texels[i].empty()) continue;
        uint32_t *dp = nullptr;
        st = upload(s, &dp, h.texels[i].data(), h.texels[i].size());
        texs[i].texels = dp;
    }
    if (st == RG_OK) st = upload(s, &s->texs, texs.data(), texs.size());
    s->tex_desc = texs;
    return st;
}

// The LDS arena of launch args `a` as one device image (light path: RgKernelArgs::lds_blob),
// built from the host tables once per arena layout; nullptr if it cannot be made.
const void *lds_blob_for(const rg_scene *s, const RgKernelArgs &a) {
    const uint32_t layout[14] = {a.lds_sphf, a.lds_sph, a.lds_cc, a.lds_nodes, a.lds_pln, a.lds_dsk, a.lds_box,
                                 a.lds_bodies, a.lds_mats, a.lds_lights, a.lds_texs, a.lds_total_bytes,
                                 (uint32_t)a.n_nodes, (uint32_t)a.n_sph};
    rg_scene *m = const_cast<rg_scene *>(s);
    if (m->lds_blob && std::memcmp(layout, m->lds_blob_layout, sizeof layout) == 0) return m->lds_blob;
    if (!s->host || a.lds_total_bytes == 0 || a.lds_total_bytes % 16u != 0u) return nullptr;
    const rg_host_tables &h = *s->host;
    std::vector<unsigned char> img(a.lds_total_bytes, 0);
    auto put = [&](uint32_t off, const void *src, size_t bytes) {
        if (bytes && off + bytes <= img.size()) std::memcpy(img.data() + off, src, bytes);
    };
    put(a.lds_sphf, h.sphf.data(), h.sphf.size() * sizeof(RgSphF));
    put(a.lds_sphf + (uint32_t)(h.sphf.size() * sizeof(RgSphF)), h.sphf2.data(), h.sphf2.size() * sizeof(RgSphF2));
    put(a.lds_sph, h.sph.data(), h.sph.size() * sizeof(RgSph));
    put(a.lds_cc, h.sph_cc.data(), h.sph_cc.size() * sizeof(double));
    if (a.n_nodes > 0) put(a.lds_nodes, h.nodes.data(), h.nodes.size() * sizeof(RgBvhNode));
    put(a.lds_pln, h.pln.data(), h.pln.size() * sizeof(RgPln));
    put(a.lds_dsk, h.dsk.data(), h.dsk.size() * sizeof(RgDsk));
    put(a.lds_box, h.box.data(), h.box.size() * sizeof(RgBox));
    put(a.lds_bodies, h.bodies.data(), h.bodies.size() * sizeof(RgBodyDev));
    put(a.lds_mats, h.mats.data(), h.mats.size() * sizeof(RgMatDev));
    put(a.lds_lights, h.lights.data(), h.lights.size() * sizeof(RgLightDev));
    put(a.lds_texs, s->tex_desc.data(), s->tex_desc.size() * sizeof(RgTexDev));
    if (a.lbuf) put(a.lds_lbuf, h.lbuf.data(), h.lbuf.size() * sizeof(RgLightBufDev));
    void *p = nullptr;
    if (!ok(hipMalloc(&p, img.size()))) { (void)hipGetLastError(); return nullptr; }
    if (!ok(hipMemcpy(p, img.data(), img.size(), hipMemcpyHostToDevice))) { (void)hipFree(p); return nullptr; }
    if (m->lds_blob) {
        // stream-ordered launches may still read the old image: keep it with the scene's allocations
        m->allocations.push_back(m->lds_blob);
    }
    m->lds_blob = p;
    std::memcpy(m->lds_blob_layout, layout, sizeof layout);
    return p;
}

void copy_scalars(rg_scene *dst, const rg_scene *src) {
    dst->fov = src->fov;
    std::memcpy(dst->def, src->def, sizeof dst->def);
    dst->max_depth = src->max_depth;
    dst->n_sph = src->n_sph;
    dst->n_pln = src->n_pln;
    dst->n_dsk = src->n_dsk;
    dst->n_box = src->n_box;
    dst->n_bodies = src->n_bodies;
    dst->n_lights = src->n_lights;
    dst->n_textures = src->n_textures;
    dst->n_nodes = src->n_nodes;
    dst->n_lbuf = src->n_lbuf;
    dst->lb_cam = src->lb_cam;
    dst->n_lbdesc = src->n_lbdesc;
    dst->lane_stack = src->lane_stack;
    dst->nan_scene = src->nan_scene;
    dst->bvh_obound = src->bvh_obound;
    dst->bvh_rbound = src->bvh_rbound;
    dst->bvh_margin = src->bvh_margin;
    dst->bvh_extent = src->bvh_extent;
    dst->bvh_info = src->bvh_info;
}

}  // namespace

rg_status rg_scene_replica(const rg_scene *src, int32_t device, rg_scene **out) {
    *out = nullptr;
    if (!src->host) return RG_ERR_INVALID_ARGUMENT;
    rg_scene *s = new (std::nothrow) rg_scene();
    if (!s) return RG_ERR_OUT_OF_MEMORY;
    s->device = device;
    copy_scalars(s, src);
    rg_sync_settings(s, src);
    s->host = src->host;
    if (!ok(hipSetDevice(device))) { release(s); return RG_ERR_DEVICE; }
    rg_status st = upload_tables(s, *src->host);
    if (st == RG_OK && !(s->last = ctx_for(s, nullptr))) st = RG_ERR_OUT_OF_MEMORY;
    if (st != RG_OK) { release(s); return st; }
    *out = s;
    return RG_OK;
}

void rg_scene_free(rg_scene *s) { release(s); }

void rg_sync_settings(rg_scene *dst, const rg_scene *src) {
    dst->max_depth = src->max_depth;
    dst->path = src->path;
    dst->bvh_enabled = src->bvh_enabled;
    dst->lbuf_enabled = src->lbuf_enabled;
    dst->lane_min_depth = src->lane_min_depth;
    dst->tile_order = src->tile_order;
    dst->ring_flush_small = src->ring_flush_small;
    dst->ring_group_small = src->ring_group_small;
    dst->ring_flush_big = src->ring_flush_big;
    dst->ring_group_big = src->ring_group_big;
}

uint32_t rg_tiling_rows_grouped(uint32_t height, const rg_tiling *t, uint32_t group) {
    if (!tiling_valid(t) || height == 0 || group < 1 || (group > 1 && t->tile_offset + group > t->tile_stride)) return 0;
    const uint32_t tiles = (height + t->tile_rows - 1) / t->tile_rows;
    // per stride of image tiles: tiles offset .. offset + group - 1 (group 1: the round robin)
    const uint32_t full = tiles / t->tile_stride, rem = tiles % t->tile_stride;
    const uint32_t last = rem > t->tile_offset ? std::min(group, rem - t->tile_offset) : 0u;
    return (full * group + last) * t->tile_rows;
}

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
    case RG_ERR_COLLECTIVE: return "RCCL unavailable or failed (rg_render_multi)";
    case RG_ERR_PENDING: return "a frame batch waits for its gather: rg_frames_flush on every rank first";
    default: return "unknown status";
    }
}

int32_t rg_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

uint32_t rg_tiling_rows(uint32_t height, const rg_tiling *t) { return rg_tiling_rows_grouped(height, t, 1); }

rg_status rg_scene_create(const rg_scene_desc *d, int32_t device, rg_scene **out) {
    if (!d || !out) return RG_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    if ((d->n_bodies && !d->bodies) || (d->n_lights && !d->lights) || (d->n_textures && !d->textures))
        return RG_ERR_INVALID_ARGUMENT;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return RG_ERR_DEVICE;
    // validate enums and textures on the host first
    bool nan_scene = false;
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
        for (int k = 0; k < body_params(b.kind); ++k) nan_scene |= exotic_value(b.p[k]);
    }
    for (uint32_t i = 0; i < d->n_lights; ++i) {
        if (d->lights[i].kind > RG_LIGHT_SPHERICAL) return RG_ERR_INVALID_ARGUMENT;
        for (int k = 0; k < 3; ++k) nan_scene |= exotic_value(d->lights[i].v[k]);
    }

    rg_scene *s = new (std::nothrow) rg_scene();
    if (!s) return RG_ERR_OUT_OF_MEMORY;
    std::shared_ptr<rg_host_tables> hp(new (std::nothrow) rg_host_tables());
    if (!hp) { delete s; return RG_ERR_OUT_OF_MEMORY; }
    rg_host_tables &h = *hp;
    s->device = device;
    s->fov = d->fov;
    std::memcpy(s->def, d->default_color, sizeof s->def);
    s->max_depth = d->max_recursion_depth;
    s->nan_scene = nan_scene;
    if (!ok(hipSetDevice(device))) { release(s); return RG_ERR_DEVICE; }

    std::vector<double> sph_raw;  // center xyz, radius (BVH build input)
    h.bodies.resize(d->n_bodies);
    h.mats.resize(d->n_bodies);
    for (uint32_t i = 0; i < d->n_bodies; ++i) {
        const rg_body &b = d->bodies[i];
        const double *p = b.p;
        h.bodies[i].kind = (int32_t)b.kind;
        h.bodies[i].pad = 0;
        std::memcpy(h.bodies[i].p, b.p, sizeof h.bodies[i].p);
        const rg_material &m = b.material;
        RgMatDev &md = h.mats[i];
        md.coloration = (int32_t)m.coloration;
        std::memcpy(md.color, m.color, sizeof md.color);
        md.tex = m.texture;
        md.xoff = m.x_offset;
        md.yoff = m.y_offset;
        md.albedo_pi = m.albedo / 3.14159265358979323846f;  // std::f32::consts::PI, IEEE f32 division
        md.surface = (int32_t)m.surface;
        md.reflectivity = m.reflectivity;
        md.index = m.index;
        md.transparency = m.transparency;
        switch (b.kind) {
        case RG_BODY_SPHERE:
            // r2 = radius * radius and cc = (c.c) evaluated exactly as the per-ray
            // reference expressions (bodies.rs:95,97) -> bit-identical.
            h.sph.push_back(RgSph{p[0], p[1], p[2], p[3] * p[3]});
            h.sphf.emplace_back();
            h.sphf2.emplace_back();
            make_filter_records(p, h.sphf.back(), h.sphf2.back());
            h.sphf2.back().id = (int32_t)i;  // the record a leaf test already holds carries the id
            h.sph_cc.push_back(dot3(p, p));  // padded to an even count after the loop
            h.sph_id.push_back((int32_t)i);
            sph_raw.insert(sph_raw.end(), p, p + 4);
            break;
        case RG_BODY_PLANE:
            h.pln.push_back(RgPln{p[0], p[1], p[2], p[3], p[4], p[5], dot3(p, p + 3), 0.0});
            h.pln_id.push_back((int32_t)i);
            break;
        case RG_BODY_DISK:
            h.dsk.push_back(RgDsk{p[0], p[1], p[2], p[3], p[4], p[5], p[6], dot3(p, p + 3)});
            h.dsk_id.push_back((int32_t)i);
            break;
        default:
            h.box.push_back(RgBox{{p[0], p[1], p[2]}, {p[3], p[4], p[5]}});
            h.box_id.push_back((int32_t)i);
            break;
        }
    }
    // Sphere BVH: reorder the sphere tables into leaf order (sph_id keeps the
    // YAML index, so the closest-hit tie-break is unaffected).  Not for scenes
    // whose arithmetic may produce NaN distances: the scene.rs:38 panic needs
    // every ray's hit count, which a pruned traversal does not see.
    RgBvhBuild bvh;
    if (!nan_scene && (int)h.sph.size() >= RG_BVH_MIN_SPHERES && rg_build_bvh(sph_raw.data(), (int)h.sph.size(), bvh)) {
        auto permute = [&](auto &v) {
            auto old = v;
            for (size_t j = 0; j < bvh.order.size(); ++j) v[j] = old[bvh.order[j]];
        };
        permute(h.sph);
        permute(h.sphf);
        permute(h.sphf2);
        permute(h.sph_cc);
        permute(h.sph_id);
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
        h.nodes = bvh.nodes;
    }
    if (h.sph_cc.size() % 2) h.sph_cc.push_back(0.0);  // LDS staging copies 16-B units
    h.lights.resize(d->n_lights);
    for (uint32_t i = 0; i < d->n_lights; ++i) {
        const rg_light &l = d->lights[i];
        RgLightDev &ld = h.lights[i];
        ld.kind = (int32_t)l.kind;
        std::memcpy(ld.color, l.color, sizeof ld.color);
        ld.intensity = l.intensity;
        ld.pad = 0;
        std::memcpy(ld.v, l.v, sizeof ld.v);
        // Directional: normalize(-direction) (lights.rs:48) is a per-light constant.
        // Same IEEE ops in the same order as the device would run -> identical bits.
        double nx = -l.v[0], ny = -l.v[1], nz = -l.v[2];
        double inv = 1.0 / std::sqrt((nx * nx + ny * ny) + nz * nz);
        ld.dn[0] = nx * inv;
        ld.dn[1] = ny * inv;
        ld.dn[2] = nz * inv;
        ld.pad2 = 0.0;
    }
    // Shadow-ray light buffers (rg_lightbuf.cpp) over the BVH-ordered sphere tables, for the first
    // RG_LB_MAX_LIGHTS lights; a light that cannot be served well keeps the BVH walk (kind NONE)
    if (!h.nodes.empty()) {
        std::vector<double> sp(4 * h.sph.size());
        for (size_t j = 0; j < h.sph.size(); ++j) {
            const double *p = &sph_raw[4 * (size_t)bvh.order[j]];  // centre, radius of BVH position j
            std::memcpy(&sp[4 * j], p, 4 * sizeof(double));
        }
        const uint32_t nl = std::min<uint32_t>(d->n_lights, RG_LB_MAX_LIGHTS);
        h.lbuf.assign(nl, RgLightBufDev{});
        int built = 0;
        for (uint32_t i = 0; i < nl; ++i) {
            RgLightBufBuild lb;
            if (!rg_build_lightbuf(sp.data(), (int)h.sph.size(), h.lights[i].kind, h.lights[i].dn, h.lights[i].v,
                                   bvh.extent, (double)bvh.obound, lb))
                continue;
            // a budget on all buffers together: past it, a light keeps the BVH walk
            if (h.lb_ent.size() + lb.ent.size() + h.lb_start.size() + lb.start.size() > RG_LB_TOTAL_WORDS) continue;
            const uint32_t ebase = (uint32_t)h.lb_ent.size(), cbase = (uint32_t)h.lb_start.size();
            for (uint32_t &v : lb.start) v += ebase;
            lb.dev.cell_off = cbase;
            lb.dev.always0 += ebase;
            lb.dev.always1 += ebase;
            h.lb_start.insert(h.lb_start.end(), lb.start.begin(), lb.start.end());
            h.lb_ent.insert(h.lb_ent.end(), lb.ent.begin(), lb.ent.end());
            h.lbuf[i] = lb.dev;
            ++built;
        }
        // the camera buffer: a light buffer around the camera (ray.rs:53: every primary ray starts at
        // the origin), behind the lights' slots; primary rays test their direction's cell
        const double zero[3] = {0.0, 0.0, 0.0};
        RgLightBufBuild cam;
        if (rg_build_lightbuf(sp.data(), (int)h.sph.size(), RG_LIGHT_SPHERICAL, zero, zero, bvh.extent,
                              (double)bvh.obound, cam) &&
            h.lb_ent.size() + cam.ent.size() + h.lb_start.size() + cam.start.size() <= RG_LB_TOTAL_WORDS) {
            const uint32_t ebase = (uint32_t)h.lb_ent.size(), cbase = (uint32_t)h.lb_start.size();
            for (uint32_t &v : cam.start) v += ebase;
            cam.dev.cell_off = cbase;
            cam.dev.always0 += ebase;
            cam.dev.always1 += ebase;
            h.lb_start.insert(h.lb_start.end(), cam.start.begin(), cam.start.end());
            h.lb_ent.insert(h.lb_ent.end(), cam.ent.begin(), cam.ent.end());
            s->lb_cam = (int32_t)h.lbuf.size();
            h.lbuf.push_back(cam.dev);
        }
        if (!built && s->lb_cam < 0) h.lbuf.clear();
        s->n_lbuf = built ? (int32_t)nl : 0;
        s->n_lbdesc = (int32_t)h.lbuf.size();
        s->bvh_info.lbuf_bytes = (int64_t)((h.lb_ent.size() + h.lb_start.size()) * sizeof(uint32_t) +
                                           h.lbuf.size() * sizeof(RgLightBufDev));
    }
    h.tex_w.resize(d->n_textures);
    h.tex_h.resize(d->n_textures);
    h.texels.resize(d->n_textures);
    for (uint32_t i = 0; i < d->n_textures; ++i) {
        const rg_texture &t = d->textures[i];
        h.tex_w[i] = t.width;
        h.tex_h[i] = t.height;
        const size_t n = (size_t)t.width * t.height;
        if (n == 0 || !t.rgba) continue;
        h.texels[i].resize(n);
        std::memcpy(h.texels[i].data(), t.rgba, n * 4);
    }
    s->n_sph = (int32_t)h.sph.size();
    s->n_pln = (int32_t)h.pln.size();
    s->n_dsk = (int32_t)h.dsk.size();
    s->n_box = (int32_t)h.box.size();
    s->n_bodies = (int32_t)d->n_bodies;
    s->n_lights = (int32_t)d->n_lights;
    s->n_textures = (int32_t)d->n_textures;
    s->n_nodes = (int32_t)h.nodes.size();
    // the stack entry keeps the node index in its low RG_LANE_NODE_BITS bits
    s->lane_stack = (s->n_nodes <= (1 << RG_LANE_NODE_BITS) && bvh.lane_stack <= RG_LANE_STACK_MAX)
                        ? std::max(bvh.lane_stack, 1) : 0;

    rg_status st = upload_tables(s, h);
    s->host = hp;
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

rg_status rg_scene_release_stream(rg_scene *s, void *stream) {
    if (!s) return RG_ERR_INVALID_ARGUMENT;
    hipStream_t hs = static_cast<hipStream_t>(stream);
    if (!hs) return RG_OK;  // the null-stream context lives as long as the scene
    if (!ok(hipSetDevice(s->device))) return RG_ERR_DEVICE;
    for (size_t i = 0; i < s->ctxs.size(); ++i) {
        if (s->ctxs[i]->stream != hs) continue;
        rg_launch_ctx *c = s->ctxs[i];
        (void)hipStreamSynchronize(hs);
        if (s->last == c) s->last = ctx_for(s, nullptr);
        s->ctxs.erase(s->ctxs.begin() + (std::ptrdiff_t)i);
        destroy_ctx(c);
        break;
    }
    return RG_OK;
}

rg_status rg_stream_status(const rg_scene *s, void *stream, int32_t *error_pixel) {
    if (!s) return RG_ERR_INVALID_ARGUMENT;
    if (error_pixel) *error_pixel = -1;
    if (!ok(hipSetDevice(s->device))) return RG_ERR_DEVICE;
    hipStream_t hs = static_cast<hipStream_t>(stream);
    for (rg_launch_ctx *c : s->ctxs) {
        if (c->stream != hs) continue;
        unsigned long long w = 0;
        if (!ok(hipStreamSynchronize(hs)) || !ok(hipMemcpy(&w, c->sticky, sizeof w, hipMemcpyDeviceToHost)) ||
            !ok(hipMemset(c->sticky, 0, sizeof w)))
            return RG_ERR_DEVICE;
        return decode_error(w, error_pixel);
    }
    return RG_OK;  // nothing was launched on this stream
}

rg_status rg_render_tiles_async(const rg_scene *s, uint32_t width, uint32_t height, const rg_tiling *tiling,
                                uint8_t *rgba_dev, float *rgb_dev, void *stream, rg_stats *stats) {
    hipStream_t st = static_cast<hipStream_t>(stream);
    rg_launch_ctx *cx = nullptr;
    rg_status r = rg_launch_tiles(s, width, height, tiling, rgba_dev, rgb_dev, st, nullptr, &cx, stats != nullptr,
                                  nullptr, 0, nullptr, 3, false, false);
    if (r != RG_OK || !stats) return r;
    unsigned long long c[4];
    if (!ok(hipMemcpyAsync(c, cx->last_counters, sizeof c, hipMemcpyDeviceToHost, st))) return RG_ERR_DEVICE;
    if (!ok(hipStreamSynchronize(st))) return RG_ERR_DEVICE;
    float ms = 0.0f;
    (void)hipEventElapsedTime(&ms, cx->ev0, cx->ev1);
    stats->kernel_ms = ms;
    return rg_snap_status(c, stats);
}

rg_status rg_render_tiles_pipelined(const rg_scene *s, uint32_t width, uint32_t height, const rg_tiling *tiling,
                                    uint8_t *rgba_dev, float *rgb_dev, void *stream) {
    // one of several frames in flight (rg_frames, bench.py): the heavy path sizes
    // its grid for throughput (rg_kernels.hip launch_one, RgKernelArgs::pipelined)
    return rg_launch_tiles(s, width, height, tiling, rgba_dev, rgb_dev, static_cast<hipStream_t>(stream), nullptr,
                           nullptr, false, nullptr, 0, nullptr, 3, false, true);
}

}  // extern "C"

// ---------------------------------------------------------------- host-visible frames
// The drop-in for rendering::render_image (rendering.rs:24-38) returns the
// frame in HOST memory.  A 4K RGBA8 frame is 33 MB, about as long on PCIe
// (~55 GB/s) as its render, so the frame is rendered in K row bands on two
// render streams and band b's device-to-host copy (on a copy stream) runs
// while bands b+1.. render.  A pinned caller buffer (hipHostMalloc'd, or
// registered with rg_host_register) receives the DMA directly; a pageable
// one is fed from a ring of pinned staging slots by host memcpy, overlapped
// with the following bands' DMA.  Device framebuffer, staging, streams and
// events belong to the scene and are reused across calls.
struct rg_copy_pool::Impl {
    std::vector<std::thread> th;
    std::mutex m;
    std::condition_variable cv;
    std::atomic<bool> stop{false}, active{false};
    std::atomic<uint64_t> gen{0};
    std::atomic<int> remaining{0};
    unsigned char *dst = nullptr;
    const unsigned char *src = nullptr;
    size_t bytes = 0;
    int parts = 1;
};

rg_copy_pool::rg_copy_pool(int helpers) : p_(new Impl) {
    p_->parts = helpers + 1;
    for (int i = 0; i < helpers; ++i) p_->th.emplace_back([this, i] { run(i + 1); });
}

rg_copy_pool::~rg_copy_pool() {
    {
        std::lock_guard<std::mutex> g(p_->m);
        p_->stop.store(true);
    }
    p_->cv.notify_all();
    for (std::thread &t : p_->th) t.join();
    delete p_;
}

void rg_copy_pool::begin() {
    {
        std::lock_guard<std::mutex> g(p_->m);
        p_->active.store(true);
    }
    p_->cv.notify_all();
}

void rg_copy_pool::end() { p_->active.store(false); }

namespace {
// Piece i of n of [0, bytes), 4 KiB aligned (the last piece takes the rest).
inline void piece(size_t bytes, int i, int n, size_t &off, size_t &len) {
    const size_t per = (bytes / (size_t)n + 4095) & ~(size_t)4095;
    off = std::min(bytes, per * (size_t)i);
    len = i == n - 1 ? bytes - off : std::min(bytes - off, per);
}
}  // namespace

namespace {
// A band's copy out of pinned staging into the caller's pageable frame (non-temporal AVX2 stores
// measured no consistent change: DESIGN.md 5)
void copy_band(unsigned char *dst, const unsigned char *src, size_t n) { std::memcpy(dst, src, n); }
}  // namespace

void rg_copy_pool::run(int id) {
    uint64_t seen = 0;
    for (;;) {
        uint64_t g = p_->gen.load(std::memory_order_acquire);
        if (g == seen) {
            if (p_->stop.load()) return;
            if (p_->active.load(std::memory_order_relaxed)) {
                __builtin_ia32_pause();
                continue;
            }
            std::unique_lock<std::mutex> lk(p_->m);
            p_->cv.wait(lk, [&] {
                return p_->stop.load() || p_->active.load() || p_->gen.load(std::memory_order_acquire) != seen;
            });
            continue;
        }
        seen = g;
        size_t off, len;
        piece(p_->bytes, id, p_->parts, off, len);
        if (len) copy_band(p_->dst + off, p_->src + off, len);
        p_->remaining.fetch_sub(1, std::memory_order_acq_rel);
    }
}

void rg_copy_pool::copy(void *dst, const void *src, size_t bytes) {
    if (p_->parts == 1 || bytes < (256u << 10)) {
        std::memcpy(dst, src, bytes);
        return;
    }
    p_->dst = static_cast<unsigned char *>(dst);
    p_->src = static_cast<const unsigned char *>(src);
    p_->bytes = bytes;
    p_->remaining.store(p_->parts - 1, std::memory_order_relaxed);
    {
        std::lock_guard<std::mutex> g(p_->m);  // a sleeping helper sees the new generation
        p_->gen.fetch_add(1, std::memory_order_release);
    }
    p_->cv.notify_all();
    size_t off, len;
    piece(bytes, 0, p_->parts, off, len);
    if (len) copy_band(p_->dst + off, p_->src + off, len);
    while (p_->remaining.load(std::memory_order_acquire) != 0) __builtin_ia32_pause();
}

namespace {

// Bands of a banded host-visible frame: the first band's copy starts while
// the later bands render (the frame's PCIe transfer alone: ~0.59 ms for 33 MB
// at the measured 56 GB/s, profiles/r02/host_visible/d2h_probe.jsonl).  ~2 Mpx
// per band, at most 3: a 4K frame in 3 bands 0.95 ms, in 16 bands 1.46 ms --
// small launches leave most of the GPU idle (hv_sweep_bands_before.jsonl).
int image_bands(const rg_scene *s, size_t px) {
    if (s->image_bands > 0) return s->image_bands;
    const size_t k = px / RG_IMAGE_BAND_PX;
    return (int)std::max<size_t>(1, std::min<size_t>(3, k));
}

rg_status ensure_image_res(const rg_scene *s) {
    rg_image_res &r = s->img;
    if (r.cs) return RG_OK;
    bool good = true;
#if RG_IMAGE_STREAM_CUMASK
    // The host frame's two render streams run concurrently (split frames: the device part on
    // rs[0], the one-launch part on rs[1]), so they must not share a hardware queue.  HIP hands a
    // plain new stream one of the process's shared queues, and where it lands depends on the
    // streams made before it: two of three test1 instances ran the split frame at 1.06 ms instead
    // of 0.76-0.80 (the parts serialised) after the bench reused its render streams
    // (profiles/r06/s32, s36).  A stream with a CU mask (every CU) gets a hardware queue of its
    // own: rs[1] is made so.  rs[0] stays a plain stream -- the heavy scenes' one-launch frame runs
    // there, and on a CU-masked queue it measured 2.32 instead of 2.03 ms in two of three runs (s37).
    {
        int cus = 0;
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, s->device);
        std::vector<uint32_t> mask((size_t)std::max(1, (cus + 31) / 32), 0xFFFFFFFFu);
        if (cus % 32) mask.back() = (1u << (cus % 32)) - 1u;
        good = good && ok(hipStreamCreateWithFlags(&r.rs[0], hipStreamNonBlocking)) &&
               ok(hipExtStreamCreateWithCUMask(&r.rs[1], (uint32_t)mask.size(), mask.data()));
    }
#else
    for (hipStream_t &st : r.rs) good = good && ok(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
#endif
    good = good && ok(hipStreamCreateWithFlags(&r.cs, hipStreamNonBlocking));
    for (hipEvent_t &e : r.ev_done) good = good && ok(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    for (hipEvent_t &e : r.ev_copy) good = good && ok(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    good = good && ok(hipEventCreate(&r.ev_t0)) && ok(hipEventCreate(&r.ev_t1)) &&
           ok(hipEventCreateWithFlags(&r.ev_join, hipEventDisableTiming));
    void *snap = nullptr;
    good = good && ok(hipHostMalloc(&snap, RG_IMAGE_MAX_BANDS * 4 * sizeof(unsigned long long), hipHostMallocDefault));
    r.h_snap = static_cast<unsigned long long *>(snap);
    if (!good) {
        release_image_res(r);
        return RG_ERR_DEVICE;
    }
    return RG_OK;
}

template <class P>
rg_status grow_device(P *&p, size_t &cap, size_t bytes) {
    if (bytes <= cap) return RG_OK;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    void *q = nullptr;
    if (!ok(hipMalloc(&q, bytes))) { (void)hipGetLastError(); return RG_ERR_OUT_OF_MEMORY; }
    p = static_cast<P *>(q);
    cap = bytes;
    return RG_OK;
}

// Pinned, coherent host buffer of at least `bytes` (grown, never shrunk).
template <class P>
rg_status grow_pinned(P *&p, size_t &cap, size_t bytes) {
    if (bytes <= cap) return RG_OK;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    void *q = nullptr;
    if (!ok(hipHostMalloc(&q, bytes, hipHostMallocCoherent))) { (void)hipGetLastError(); return RG_ERR_OUT_OF_MEMORY; }
    std::memset(q, 0, bytes);
    p = static_cast<P *>(q);
    cap = bytes;
    return RG_OK;
}

// Wait until tiles [t0, t1) of the launch carry `seq` (the kernel publishes a
// tile after a system-scope release of its pixels).  Polls the launch's done
// event now and then, so a failed launch returns instead of spinning.
rg_status wait_tiles(const uint32_t *flags, size_t t0, size_t t1, uint32_t seq, hipEvent_t done) {
    unsigned spins = 0;
    for (size_t i = t0; i < t1; ++i) {
        while (__atomic_load_n(&flags[i], __ATOMIC_ACQUIRE) != seq) {
            if ((++spins & 1023u) == 0u) {
                const hipError_t e = hipEventQuery(done);
                if (e == hipSuccess) {  // the kernel is done: the flag must be there now
                    if (__atomic_load_n(&flags[i], __ATOMIC_ACQUIRE) != seq) return RG_ERR_DEVICE;
                } else if (e != hipErrorNotReady) {
                    (void)hipGetLastError();
                    return RG_ERR_DEVICE;
                }
            }
            __builtin_ia32_pause();
        }
    }
    return RG_OK;
}

// Host-visible frame in ONE launch, no device framebuffer and no copy engine:
// the kernel's pixel stores go straight over PCIe into page-locked host memory
// (8x8-tile-shaped 4-B stores reach 52.7 GB/s of the 55.8 GB/s a DMA copy
// does: profiles/r02/host_visible/d2h_probe.jsonl), so the transfer overlaps the whole
// render.  A pinned caller buffer is written directly.  A pageable one
// (a Rust Vec, a numpy array) is fed from a pinned frame the kernel writes:
// the kernel publishes each finished 8x8 tile (RgKernelArgs::tile_flags) and
// the host copies every band of rows, on RG_COPY_HELPERS + 1 threads, as
// soon as its tiles are in, while the kernel renders the rest.
rg_status render_host_direct(const rg_scene *s, uint32_t W, uint32_t H, const rg_tiling *t, uint32_t rows,
                             uint8_t *rgba_out, rg_stats *stats) {
    rg_image_res &r = s->img;
    const size_t row4 = (size_t)W * 4, bytes = (size_t)rows * row4;
    hipStream_t rs = r.rs[0];
    void *dst = rg_host_device_ptr(rgba_out, std::max<size_t>(bytes, 1));
    const bool pageable = dst == nullptr;
    const bool light = !rg_heavy_path(rg_make_args(s));
    const uint32_t wl = (uint32_t)(s->host_tile_forced || !light ? s->host_tile_wlog : RG_HOST_TILE_WLOG_LIGHT),
                   TH = 64u >> wl;
    const size_t tiles_x = ((size_t)W + (1u << wl) - 1u) >> wl, tile_rows = (rows + TH - 1u) / TH,
                 ntiles = tiles_x * tile_rows;
    rg_status st = RG_OK;
    uint32_t seq = 0;
    if (pageable) {
        if ((st = grow_pinned(r.h_frame, r.h_frame_cap, bytes + 4)) != RG_OK) return st;
        if ((st = grow_pinned(r.h_flags, r.h_flags_cap, (ntiles + 1) * 4)) != RG_OK) return st;
        dst = rg_host_device_ptr(r.h_frame, std::max<size_t>(bytes, 1));
        if (!dst) return RG_ERR_DEVICE;
        if (++r.seq == 0) r.seq = 1;
        seq = r.seq;
    }
    uint32_t *flags_dev = nullptr;
    if (pageable && !(flags_dev = static_cast<uint32_t *>(rg_host_device_ptr(r.h_flags, ntiles * 4 + 4))))
        return RG_ERR_DEVICE;
    if (!ok(hipEventRecord(r.ev_t0, rs))) return RG_ERR_DEVICE;
    st = rg_launch_tiles(s, W, H, t, static_cast<uint8_t *>(dst), nullptr, rs, r.h_snap, nullptr, false, flags_dev,
                         seq, nullptr, wl, true);
    if (st != RG_OK) return st;
    if (!ok(hipEventRecord(r.ev_t1, rs))) return RG_ERR_DEVICE;
    if (pageable) {
        if (!r.pool) r.pool = std::make_shared<rg_copy_pool>(RG_COPY_HELPERS);
        struct Active {
            rg_copy_pool &p;
            explicit Active(rg_copy_pool &q) : p(q) { p.begin(); }
            ~Active() { p.end(); }
        } active(*r.pool);
        // bands of whole tile rows, ~RG_IMAGE_BAND_PX / 4 pixels each (the queue hands out tiles in raster order)
        const size_t band_tr = std::max<size_t>(1, (RG_IMAGE_BAND_PX / 4) / ((size_t)W * TH));
        for (size_t tr0 = 0; tr0 < tile_rows && st == RG_OK; tr0 += band_tr) {
            const size_t tr1 = std::min(tile_rows, tr0 + band_tr);
            if ((st = wait_tiles(r.h_flags, tr0 * tiles_x, tr1 * tiles_x, seq, r.ev_t1)) != RG_OK) break;
            const size_t y0 = tr0 * TH, y1 = std::min<size_t>(rows, tr1 * TH);
            r.pool->copy(rgba_out + y0 * row4, static_cast<uint8_t *>(r.h_frame) + y0 * row4, (y1 - y0) * row4);
        }
    }
    if (!ok(hipStreamSynchronize(rs))) return RG_ERR_DEVICE;
    if (st != RG_OK) return st;
    rg_stats total;
    std::memset(&total, 0, sizeof total);
    const rg_status err = rg_snap_status(r.h_snap, &total);
    float ms = 0.0f;
    (void)hipEventElapsedTime(&ms, r.ev_t0, r.ev_t1);
    total.kernel_ms = ms;
    if (stats) *stats = total;
    return err;
}

// Host-visible frame into a page-locked buffer, split in two concurrent parts
// that share the PCIe link: the top rows render into device memory (a plain
// device-resident launch) and go to the caller's buffer as one DMA copy, while
// the rest is ONE launch writing its pixels over PCIe itself
// (render_host_direct's kernel).  The one-launch kernel alone reaches ~38 GB/s
// of the ~55 GB/s a copy does; the copy of the first part runs beside it.
// The automatic choice for light-path scenes into page-locked buffers (test1
// 4K 0.90 -> 0.80 ms, test3 0.835 -> 0.80: profiles/r05/s31, s32); heavy
// scenes keep the one launch (north star 2.13 -> 2.23-2.70 ms split).
#ifndef RG_HOST_SPLIT_PCT
#define RG_HOST_SPLIT_PCT 35
#endif
#ifndef RG_HOST_SPLIT_B_FIRST
// part B's persistent host-frame launch first, part A's beside it: B's PCIe writes start at once
// (test1 4K pinned 0.854 -> 0.80 ms at 35 %; 30 % 0.83, 40 % 0.91: profiles/r05/s32)
#define RG_HOST_SPLIT_B_FIRST 1
#endif
rg_status render_host_split(const rg_scene *s, uint32_t W, uint32_t H, const rg_tiling *t, uint32_t rows,
                            uint8_t *rgba_out, rg_stats *stats) {
    (void)t;  // a whole-frame tiling (stride 1): output row = image row
    rg_image_res &r = s->img;
    const size_t row4 = (size_t)W * 4;
    void *dst = rg_host_device_ptr(rgba_out, (size_t)rows * row4);
    if (!dst) return RG_ERR_INVALID_ARGUMENT;  // pinned buffers only (the caller checked)
    // the frame re-cut into 8-row tiles (the caller's tiling is a whole-frame one: output row = image row)
    const rg_tiling t8 = {8u, 1u, 0u};
    const uint32_t TR = 8u, nt = (H + 7u) / 8u;
    const int pct = s->host_split_pct > 0 ? s->host_split_pct : RG_HOST_SPLIT_PCT;
    const uint32_t ja = std::min(nt - 1u, std::max(1u, (uint32_t)(((unsigned long long)nt * (unsigned)pct + 50u) / 100u)));
    const size_t a_bytes = (size_t)ja * TR * row4;  // rows [0, ja TR): below H (ja < nt)
    if (rows > H) std::memset(rgba_out + (size_t)H * row4, 0, (size_t)(rows - H) * row4);  // the tiling's padding
    rg_status st = grow_device(r.d_rgba, r.d_rgba_cap, a_bytes + 4);
    if (st != RG_OK) return st;
    const bool light = !rg_heavy_path(rg_make_args(s));
    const uint32_t wl = (uint32_t)(s->host_tile_forced || !light ? s->host_tile_wlog : RG_HOST_TILE_WLOG_LIGHT);
    if (!ok(hipEventRecord(r.ev_t0, r.rs[0])) || !ok(hipStreamWaitEvent(r.rs[1], r.ev_t0, 0))) return RG_ERR_DEVICE;
    // Once either part is enqueued, every exit first drains both render streams and the copy
    // stream: part B's kernel and part A's DMA store into the caller's buffer, which the caller
    // owns again when this call returns (rendering.rs:24-38 returns a finished ImageBuffer).
    auto drain = [&](rg_status e) -> rg_status {
        (void)hipStreamSynchronize(r.rs[1]);
        (void)hipStreamSynchronize(r.rs[0]);
        (void)hipStreamSynchronize(r.cs);
        (void)hipGetLastError();
        return e;
    };
    // part A (device memory) and part B (one launch writing host memory), in RG_HOST_SPLIT_B_FIRST order
    auto launch_a = [&]() -> rg_status {
        if (s->split_fail_a > 0) {  // rg_debug_fail_split_a: this launch reports failure without running
            --s->split_fail_a;
            return RG_ERR_DEVICE;
        }
        const rg_status e = rg_launch_tiles(s, W, H, &t8, static_cast<uint8_t *>(r.d_rgba), nullptr, r.rs[0], r.h_snap,
                                            nullptr, false, nullptr, 0, nullptr, 3, false, false, 0, ja);
        if (e != RG_OK) return e;
        return ok(hipEventRecord(r.ev_done[0], r.rs[0])) ? RG_OK : RG_ERR_DEVICE;
    };
    auto launch_b = [&]() -> rg_status {
        return rg_launch_tiles(s, W, H, &t8, static_cast<uint8_t *>(dst), nullptr, r.rs[1], r.h_snap + 4, nullptr,
                               false, nullptr, 0, nullptr, wl, true, false, ja, 0xFFFFFFFFu, true);  // image rows >= ja * 8
    };
    if (RG_HOST_SPLIT_B_FIRST) {
        if ((st = launch_b()) != RG_OK || (st = launch_a()) != RG_OK) return drain(st);
    } else {
        if ((st = launch_a()) != RG_OK || (st = launch_b()) != RG_OK) return drain(st);
    }
    if (!ok(hipStreamWaitEvent(r.cs, r.ev_done[0], 0)) ||
        !ok(hipMemcpyAsync(rgba_out, r.d_rgba, a_bytes, hipMemcpyDeviceToHost, r.cs)) ||
        !ok(hipEventRecord(r.ev_copy[0], r.cs)) || !ok(hipStreamWaitEvent(r.rs[1], r.ev_copy[0], 0)) ||
        !ok(hipEventRecord(r.ev_t1, r.rs[1])))
        return drain(RG_ERR_DEVICE);
    const bool synced1 = ok(hipStreamSynchronize(r.rs[1]));
    const bool synced0 = ok(hipStreamSynchronize(r.rs[0]));
    if (!synced1 || !synced0) return drain(RG_ERR_DEVICE);
    rg_stats total;
    std::memset(&total, 0, sizeof total);
    total.error_pixel = -1;
    rg_status err = RG_OK;
    for (int b = 0; b < 2; ++b) {  // part A holds the lower pixel indices: its error first
        rg_stats bs;
        const rg_status e = rg_snap_status(r.h_snap + 4 * b, &bs);
        total.rays.primary += bs.rays.primary;
        total.rays.shadow += bs.rays.shadow;
        total.rays.secondary += bs.rays.secondary;
        if (e != RG_OK && err == RG_OK) {
            err = e;
            total.error_pixel = bs.error_pixel;
        }
    }
    float ms = 0.0f;
    (void)hipEventElapsedTime(&ms, r.ev_t0, r.ev_t1);
    total.kernel_ms = ms;
    if (stats) *stats = total;
    return err;
}

}  // namespace

rg_status rg_render_host(const rg_scene *s, uint32_t W, uint32_t H, const rg_tiling *t, uint8_t *rgba_out,
                         float *rgb_out, rg_stats *stats) {
    if (!s || !rgba_out || W == 0 || H == 0 || !tiling_valid(t)) return RG_ERR_INVALID_ARGUMENT;
    if (W < H) return RG_ERR_PORTRAIT;
    const uint32_t rows = rg_tiling_rows(H, t);
    if ((unsigned long long)rows * W >= (1ull << 32) || (unsigned long long)H * W >= (1ull << 32))
        return RG_ERR_INVALID_ARGUMENT;
    if (!ok(hipSetDevice(s->device))) return RG_ERR_DEVICE;
    rg_status st = ensure_image_res(s);
    if (st != RG_OK) return st;
    rg_image_res &r = s->img;
    // Path choice (4K frames): into page-locked buffers one launch writing host
    // memory wins -- heavy scenes (synth1024: 2.99 vs 3.63 ms banded,
    // profiles/r02/host_visible/hv_sweep.jsonl) and, since the light path stores
    // its tiles through an LDS ring in contiguous 4-KB runs of 64x1 tiles, light
    // scenes too (test1 0.86 vs 0.93 ms, test3 0.82 vs 0.84:
    // profiles/r03/late/hv_ring_group.txt); into pageable memory the per-tile
    // publication costs more than the copies it overlaps (test1 2.5 vs 1.15
    // ms) -- banded there.
    if (!rgb_out) {
        const bool pinned = rg_host_device_ptr(rgba_out, std::max<size_t>((size_t)rows * W * 4, 1)) != nullptr;
        const bool split = s->image_bands == -2 || (s->image_bands == 0 && !rg_heavy_path(rg_make_args(s)));
        if (split && pinned && t->tile_stride == 1 && H >= 16)
            return render_host_split(s, W, H, t, rows, rgba_out, stats);
        bool direct = s->image_bands < 0;
        if (s->image_bands == 0) direct = pinned;
        if (direct) return render_host_direct(s, W, H, t, rows, rgba_out, stats);
    }

    // Bands.  A whole-frame tiling (stride 1) is re-cut into K bands of BR
    // rows (tiling {BR, K, b} renders exactly rows [b BR, (b+1) BR)); a sharded
    // tiling is rendered in one launch.
    const bool banded = t->tile_stride == 1;
    int K = 1;
    uint32_t BR = rows;
    if (banded) {
        K = image_bands(s, (size_t)H * W);
        BR = (H + (uint32_t)K - 1) / (uint32_t)K;
        BR = (BR + 7u) & ~7u;  // whole 8x8 tiles per band
        K = (int)((H + BR - 1) / BR);
    }
    const uint32_t dev_rows = banded ? (uint32_t)K * BR : rows;
    const bool want_rgb = rgb_out != nullptr;
    const size_t row4 = (size_t)W * 4, row12 = (size_t)W * 12;
    if ((st = grow_device(r.d_rgba, r.d_rgba_cap, (size_t)dev_rows * row4 + 4)) != RG_OK) return st;
    if (want_rgb && (st = grow_device(r.d_rgb, r.d_rgb_cap, (size_t)dev_rows * row12 + 4)) != RG_OK) return st;
    const bool direct = rg_host_is_pinned(rgba_out, (size_t)rows * row4) &&
                        (!want_rgb || rg_host_is_pinned(rgb_out, (size_t)rows * row12));
    const int R = RG_IMAGE_STAGE_SLOTS;
    const size_t slot_bytes = (size_t)BR * (row4 + (want_rgb ? row12 : 0));
    if (!direct && (size_t)R * slot_bytes > r.h_stage_cap) {
        if (r.h_stage) (void)hipHostFree(r.h_stage);
        r.h_stage = nullptr;
        r.h_stage_cap = 0;
        if (!ok(hipHostMalloc(&r.h_stage, (size_t)R * slot_bytes, hipHostMallocDefault))) {
            (void)hipGetLastError();
            r.h_stage = nullptr;
            return RG_ERR_OUT_OF_MEMORY;
        }
        r.h_stage_cap = (size_t)R * slot_bytes;
    }
    // host rows of band b: [b BR, min(H, (b+1) BR)) when banded, else all `rows`
    auto host_rows = [&](int b) -> uint32_t {
        if (!banded) return rows;
        const uint32_t r0 = (uint32_t)b * BR;
        return std::min(H, r0 + BR) - r0;
    };
    auto stage_rgba = [&](int b) { return static_cast<uint8_t *>(r.h_stage) + (size_t)(b % R) * slot_bytes; };
    auto stage_rgb = [&](int b) { return reinterpret_cast<float *>(stage_rgba(b) + (size_t)BR * row4); };

    if (!ok(hipEventRecord(r.ev_t0, r.rs[0])) || !ok(hipStreamWaitEvent(r.rs[1], r.ev_t0, 0))) return RG_ERR_DEVICE;
    for (int b = 0; b < K; ++b) {
        hipStream_t rs = r.rs[b & 1];
        rg_tiling bt = banded ? rg_tiling{BR, (uint32_t)K, (uint32_t)b} : *t;
        const size_t off = banded ? (size_t)b * BR : 0;
        st = rg_launch_tiles(s, W, H, &bt, static_cast<uint8_t *>(r.d_rgba) + off * row4,
                             want_rgb ? reinterpret_cast<float *>(static_cast<uint8_t *>(r.d_rgb) + off * row12) : nullptr,
                             rs, r.h_snap + 4 * b, nullptr);
        if (st != RG_OK) return st;
        if (!ok(hipEventRecord(r.ev_done[b], rs))) return RG_ERR_DEVICE;
    }
    if (!ok(hipEventRecord(r.ev_join, r.rs[1])) || !ok(hipStreamWaitEvent(r.rs[0], r.ev_join, 0)) ||
        !ok(hipEventRecord(r.ev_t1, r.rs[0])))
        return RG_ERR_DEVICE;
    auto enqueue_copy = [&](int b) -> bool {
        const size_t off = banded ? (size_t)b * BR : 0;
        const uint32_t n = host_rows(b);
        uint8_t *dst4 = direct ? rgba_out + off * row4 : stage_rgba(b);
        float *dst12 = want_rgb ? (direct ? rgb_out + off * (size_t)W * 3 : stage_rgb(b)) : nullptr;
        if (!ok(hipStreamWaitEvent(r.cs, r.ev_done[b], 0))) return false;
        if (n > 0 && !ok(hipMemcpyAsync(dst4, static_cast<uint8_t *>(r.d_rgba) + off * row4, (size_t)n * row4,
                                        hipMemcpyDeviceToHost, r.cs)))
            return false;
        if (n > 0 && dst12 && !ok(hipMemcpyAsync(dst12, static_cast<uint8_t *>(r.d_rgb) + off * row12,
                                                 (size_t)n * row12, hipMemcpyDeviceToHost, r.cs)))
            return false;
        return ok(hipEventRecord(r.ev_copy[b], r.cs));
    };
    if (direct) {
        for (int b = 0; b < K; ++b)
            if (!enqueue_copy(b)) return RG_ERR_DEVICE;
        if (!ok(hipStreamSynchronize(r.cs))) return RG_ERR_DEVICE;
    } else {
        // pageable destination: DMA into the pinned staging ring, then a
        // parallel host copy of each band while the next bands' DMA runs
        if (!r.pool) r.pool = std::make_shared<rg_copy_pool>(RG_COPY_HELPERS);
        struct Active {
            rg_copy_pool &p;
            explicit Active(rg_copy_pool &q) : p(q) { p.begin(); }
            ~Active() { p.end(); }
        } active(*r.pool);
        for (int b = 0; b < std::min(K, R); ++b)
            if (!enqueue_copy(b)) return RG_ERR_DEVICE;
        for (int b = 0; b < K; ++b) {
            if (!ok(hipEventSynchronize(r.ev_copy[b]))) return RG_ERR_DEVICE;
            const size_t off = banded ? (size_t)b * BR : 0;
            const uint32_t n = host_rows(b);
            r.pool->copy(rgba_out + off * row4, stage_rgba(b), (size_t)n * row4);
            if (want_rgb) r.pool->copy(rgb_out + off * (size_t)W * 3, stage_rgb(b), (size_t)n * row12);
            if (b + R < K && !enqueue_copy(b + R)) return RG_ERR_DEVICE;
        }
    }
    if (!ok(hipStreamSynchronize(r.rs[0])) || !ok(hipStreamSynchronize(r.rs[1]))) return RG_ERR_DEVICE;
    if (banded && rows > H) {  // padding rows of a whole-frame tiling whose tile_rows does not divide H
        std::memset(rgba_out + (size_t)H * row4, 0, (size_t)(rows - H) * row4);
        if (want_rgb) std::memset(rgb_out + (size_t)H * W * 3, 0, (size_t)(rows - H) * row12);
    }
    rg_stats total;
    std::memset(&total, 0, sizeof total);
    total.error_pixel = -1;
    rg_status err = RG_OK;
    for (int b = 0; b < K; ++b) {  // bands in row order: the first erroring band holds the lowest pixel
        rg_stats bs;
        const rg_status e = rg_snap_status(r.h_snap + 4 * b, &bs);
        total.rays.primary += bs.rays.primary;
        total.rays.shadow += bs.rays.shadow;
        total.rays.secondary += bs.rays.secondary;
        if (e != RG_OK && err == RG_OK) {
            err = e;
            total.error_pixel = bs.error_pixel;
        }
    }
    float ms = 0.0f;
    (void)hipEventElapsedTime(&ms, r.ev_t0, r.ev_t1);
    total.kernel_ms = ms;
    if (stats) *stats = total;
    return err;
}

extern "C" {

rg_status rg_render_tiles(const rg_scene *s, uint32_t width, uint32_t height, const rg_tiling *tiling,
                          uint8_t *rgba_out, float *rgb_out, rg_stats *stats) {
    return rg_render_host(s, width, height, tiling, rgba_out, rgb_out, stats);
}

rg_status rg_render_image(const rg_scene *s, uint32_t width, uint32_t height, uint8_t *rgba_out, rg_stats *stats) {
    rg_tiling whole = {height ? height : 1, 1, 0};
    return rg_render_host(s, width, height, &whole, rgba_out, nullptr, stats);
}

rg_status rg_host_register(void *ptr, size_t bytes) {
    if (!ptr || bytes == 0) return RG_ERR_INVALID_ARGUMENT;
    // portable: every device's DMA engine may write it (rg_render_multi's per-device copies)
    if (!ok(hipHostRegister(ptr, bytes, hipHostRegisterPortable))) {
        (void)hipGetLastError();
        return RG_ERR_DEVICE;
    }
    return RG_OK;
}

rg_status rg_host_unregister(void *ptr) {
    if (!ptr) return RG_ERR_INVALID_ARGUMENT;
    if (!ok(hipHostUnregister(ptr))) {
        (void)hipGetLastError();
        return RG_ERR_DEVICE;
    }
    return RG_OK;
}

// Tile-completion streaming (render_image_stream, rendering.rs:40-69): ONE
// launch of the whole frame writes its pixels over PCIe into a pinned,
// coherent host frame and publishes every finished 8x8 tile
// (RgKernelArgs::tile_flags); the host hands band after band of `tile_rows`
// rows to the callback, in row order, as soon as the band's tiles are in,
// while the kernel renders the rest.  A callback returning nonzero cancels:
// the kernel takes no further tiles (RgKernelArgs::cancel; the reference's
// `.all` short-circuits likewise) and the call returns RG_ERR_CANCELLED once
// the tiles in flight are done.
rg_status rg_render_stream(const rg_scene *s, uint32_t width, uint32_t height, uint32_t tile_rows,
                           rg_tile_callback on_tile, void *user, rg_stats *stats) {
    if (!s || !on_tile || width == 0 || height == 0 || tile_rows == 0) return RG_ERR_INVALID_ARGUMENT;
    if (width < height) return RG_ERR_PORTRAIT;
    if ((unsigned long long)height * width >= (1ull << 32)) return RG_ERR_INVALID_ARGUMENT;
    if (!ok(hipSetDevice(s->device))) return RG_ERR_DEVICE;
    rg_status st = ensure_image_res(s);
    if (st != RG_OK) return st;
    rg_image_res &r = s->img;
    const size_t row4 = (size_t)width * 4, bytes = (size_t)height * row4;
    const uint32_t wl = (uint32_t)s->host_tile_wlog, TH = 64u >> wl;
    const size_t tiles_x = ((size_t)width + (1u << wl) - 1u) >> wl, ntiles = tiles_x * ((height + TH - 1u) / TH);
    size_t cancel_cap = r.h_cancel ? 64 : 0;
    if ((st = grow_pinned(r.h_frame, r.h_frame_cap, bytes + 4)) != RG_OK ||
        (st = grow_pinned(r.h_flags, r.h_flags_cap, (ntiles + 1) * 4)) != RG_OK ||
        (st = grow_pinned(r.h_cancel, cancel_cap, 64)) != RG_OK)
        return st;
    void *frame_dev = rg_host_device_ptr(r.h_frame, bytes);
    uint32_t *flags_dev = static_cast<uint32_t *>(rg_host_device_ptr(r.h_flags, ntiles * 4 + 4));
    const uint32_t *cancel_dev = static_cast<const uint32_t *>(rg_host_device_ptr(r.h_cancel, 4));
    if (!frame_dev || !flags_dev || !cancel_dev) return RG_ERR_DEVICE;
    __atomic_store_n(r.h_cancel, 0u, __ATOMIC_RELEASE);
    if (++r.seq == 0) r.seq = 1;
    const uint32_t seq = r.seq;
    hipStream_t rs = r.rs[0];
    const rg_tiling whole = {height, 1, 0};
    if (!ok(hipEventRecord(r.ev_t0, rs))) return RG_ERR_DEVICE;
    st = rg_launch_tiles(s, width, height, &whole, static_cast<uint8_t *>(frame_dev), nullptr, rs, r.h_snap, nullptr,
                         false, flags_dev, seq, cancel_dev, wl, true);
    if (st != RG_OK) return st;
    if (!ok(hipEventRecord(r.ev_t1, rs))) return RG_ERR_DEVICE;
    const uint8_t *frame = static_cast<const uint8_t *>(r.h_frame);
    for (uint32_t y0 = 0; y0 < height; y0 += tile_rows) {
        const uint32_t n = std::min(tile_rows, height - y0);
        if ((st = wait_tiles(r.h_flags, (size_t)(y0 / TH) * tiles_x, ((size_t)(y0 + n) + TH - 1u) / TH * tiles_x, seq,
                             r.ev_t1)) != RG_OK)
            break;
        if (on_tile(y0, n, width, frame + (size_t)y0 * row4, user) != 0) {
            __atomic_store_n(r.h_cancel, 1u, __ATOMIC_RELEASE);
            st = RG_ERR_CANCELLED;
            break;
        }
    }
    if (!ok(hipStreamSynchronize(rs))) return RG_ERR_DEVICE;
    rg_stats total;
    std::memset(&total, 0, sizeof total);
    const rg_status err = rg_snap_status(r.h_snap, &total);
    float ms = 0.0f;
    (void)hipEventElapsedTime(&ms, r.ev_t0, r.ev_t1);
    total.kernel_ms = ms;
    if (stats) *stats = total;
    if (st == RG_OK && err != RG_OK) return err;
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

rg_status rg_debug_set_lightbuf(rg_scene *s, int32_t enable) {
    if (!s || (enable != 0 && enable != 1)) return RG_ERR_INVALID_ARGUMENT;
    s->lbuf_enabled = enable != 0;
    return RG_OK;
}

int32_t rg_debug_lightbuf_count(const rg_scene *s) {
    // buffers IN USE: none while the BVH or the buffers are switched off (rg_debug_set_lightbuf(0))
    if (!s || !s->host || !s->bvh_enabled || !s->lbuf_enabled || s->n_nodes == 0) return 0;
    int32_t n = 0;
    for (int32_t i = 0; i < s->n_lbuf; ++i) n += s->host->lbuf[(size_t)i].kind != RG_LB_NONE;
    return n;
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

rg_status rg_debug_set_image_bands(rg_scene *s, int32_t bands) {
    if (!s || bands < -2 || bands > RG_IMAGE_MAX_BANDS) return RG_ERR_INVALID_ARGUMENT;
    s->image_bands = bands;
    return RG_OK;
}

rg_status rg_debug_set_host_split(rg_scene *s, int32_t pct) {
    if (!s || pct < 0 || pct > 99) return RG_ERR_INVALID_ARGUMENT;
    s->host_split_pct = pct;
    return RG_OK;
}

rg_status rg_debug_set_host_ring(rg_scene *s, int32_t flush_small, int32_t group_small, int32_t flush_big,
                                  int32_t group_big, int32_t multi_light_one) {
    if (!s || flush_small < -1 || flush_small > 16 || group_small < -1 || flush_big < -1 || flush_big > 16 ||
        group_big < -1 || multi_light_one < -1 || multi_light_one > 1)
        return RG_ERR_INVALID_ARGUMENT;
    if (flush_small >= 0) s->ring_flush_small = flush_small;
    if (group_small >= 0) s->ring_group_small = group_small;
    if (flush_big >= 0) s->ring_flush_big = flush_big;
    if (group_big >= 0) s->ring_group_big = group_big;
    if (multi_light_one >= 0) s->multi_light_one = multi_light_one != 0;
    return RG_OK;
}

rg_status rg_debug_fail_split_a(rg_scene *s, int32_t count) {
    if (!s || count < 0) return RG_ERR_INVALID_ARGUMENT;
    s->split_fail_a = count;
    return RG_OK;
}

rg_status rg_debug_set_host_tile_shape(rg_scene *s, int32_t tile_wlog) {
    if (!s || !(tile_wlog == 0 || (tile_wlog >= 3 && tile_wlog <= 6))) return RG_ERR_INVALID_ARGUMENT;
    s->host_tile_wlog = tile_wlog == 0 ? RG_HOST_TILE_WLOG : tile_wlog;
    s->host_tile_forced = tile_wlog != 0;
    return RG_OK;
}

rg_status rg_debug_counters(const rg_scene *s, uint64_t out[16]) {
    if (!s || !out) return RG_ERR_INVALID_ARGUMENT;
    if (!ok(hipSetDevice(s->device))) return RG_ERR_DEVICE;
    if (!ok(hipStreamSynchronize(s->last->stream)) ||
        !ok(hipMemcpy(out, s->last->last_counters, 16 * sizeof(uint64_t), hipMemcpyDeviceToHost)))
        return RG_ERR_DEVICE;
    return RG_OK;
}

rg_status rg_debug_counter_words(const rg_scene *s, int32_t first, int32_t n, uint64_t *out) {
    if (!s || !out || first < 0 || n < 0 || first + n > RG_COUNTER_WORDS) return RG_ERR_INVALID_ARGUMENT;
    if (!ok(hipSetDevice(s->device))) return RG_ERR_DEVICE;
    if (!ok(hipStreamSynchronize(s->last->stream)) ||
        !ok(hipMemcpy(out, s->last->last_counters + first, (size_t)n * sizeof(uint64_t), hipMemcpyDeviceToHost)))
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
    RgKernelArgs a = rg_make_args(s);
    unsigned long long c[4] = {0, 0, 0, 0};
    // the trace kernel counts into the set the context's next render launch will
    // use, and re-zeroes it after the read-back (that launch expects it zeroed)
    unsigned long long *cs = cx ? cx->counters + (size_t)cx->cur * RG_COUNTER_WORDS : nullptr;
    if (st == RG_OK) { s->last = cx; a.counters = cs; }
    if (st == RG_OK && (!ok(hipMemcpy(d_rays, rays, (size_t)n * 48, hipMemcpyHostToDevice)) ||
                        !ok(hipMemset(cs, 0, sizeof c)) ||
                        !ok(rg_launch_trace(&a, (const double *)d_rays, n, (double *)d_dist, (int32_t *)d_body, nullptr)) ||
                        !ok(hipMemcpy(dist, d_dist, (size_t)n * 8, hipMemcpyDeviceToHost)) ||
                        !ok(hipMemcpy(body, d_body, (size_t)n * 4, hipMemcpyDeviceToHost)) ||
                        !ok(hipMemcpy(c, cs, sizeof c, hipMemcpyDeviceToHost)) ||
                        !ok(hipMemset(cs, 0, RG_COUNTER_WORDS * sizeof(unsigned long long)))))
        st = RG_ERR_DEVICE;
    if (d_rays) (void)hipFree(d_rays);
    if (d_dist) (void)hipFree(d_dist);
    if (d_body) (void)hipFree(d_body);
    if (st == RG_OK && c[3] != 0) st = decode_error(c[3], nullptr);
    return st;
}

}  // extern "C"
