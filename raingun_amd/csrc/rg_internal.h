// rg_internal.h — host-side state behind the opaque rg_scene handle, shared
// by rg_capi.hip (scene upload, launches, host-visible frames, streaming),
// rg_frames.hip (frames in flight over N processes) and rg_multi.hip (one
// process driving N devices).  Not part of the ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <memory>
#include <vector>

#include "../../include/raingun.h"
#include "../../include/raingun_debug.h"
#include "rg_device.h"
#include "rg_lightbuf_ray.h"

// Per-stream launch state (ray counters, tile-queue heads, error words, tile
// ordering scratch, deep frame buffer, timing events).  Launches on distinct
// streams may run concurrently (frames in flight), so they must not share it;
// launches on one stream are ordered by the stream and reuse it.
struct rg_launch_ctx {
    hipStream_t stream = nullptr;
    // Two sets of RG_COUNTER_WORDS words (rg_device.h), used by alternate
    // launches: a render kernel counts into set `cur` and zeroes the other set
    // (the previous launch's, already read back: same stream), so the next
    // launch finds its set zeroed without a memset of its own.
    unsigned long long *counters = nullptr;
    int cur = 0;
    unsigned long long *last_counters = nullptr;  // the set of the latest launch (rg_debug_counters)
    unsigned long long *sticky = nullptr;    // first error of any launch since rg_stream_status cleared it
    uint32_t *tile_cost = nullptr, *tile_perm = nullptr;  // probe/sort scratch (rg_launch_tile_order), order
    size_t tile_cap = 0;
    // the launch the cached tile_perm was made for: the order is a function of
    // the frame geometry and the scene (probe rays, materials, lights, depth)
    struct PermKey {
        uint32_t width, height, tile_rows, tile_stride, tile_offset, tile_base, out_rows, tile_wlog, max_depth, n_lights,
            tile_group;
        double fov;
        const void *mats;
        bool operator==(const PermKey &o) const {
            return width == o.width && height == o.height && tile_rows == o.tile_rows && tile_stride == o.tile_stride &&
                   tile_offset == o.tile_offset && tile_base == o.tile_base && out_rows == o.out_rows &&
                   tile_group == o.tile_group &&
                   tile_wlog == o.tile_wlog && max_depth == o.max_depth &&
                   n_lights == o.n_lights && fov == o.fov && mats == o.mats;
        }
    };
    bool perm_valid = false;
    PermKey perm_key{};
    void *deep = nullptr;  // frames for depths above the compiled arrays (rg_kernels.hip FrameStack<0>)
    size_t deep_bytes = 0;
    double *prim = nullptr;  // sensor x per column then sensor y per row (RgKernelArgs::prim_sx / prim_sy)
    size_t prim_cap = 0;     // doubles
    uint32_t prim_w = 0, prim_h = 0;
    double prim_fov = 0.0;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
};

#ifndef RG_IMAGE_STREAM_CUMASK
#define RG_IMAGE_STREAM_CUMASK 1  // host-frame render streams with a CU mask: a hardware queue each (rg_capi.hip)
#endif
#define RG_IMAGE_STAGE_SLOTS 4  // pinned staging slots of the host-visible image path
#define RG_IMAGE_MAX_BANDS 16   // events / counter snapshots per host-visible render or stream ring
#define RG_IMAGE_BAND_PX (2u << 20)    // ~pixels per band of a banded host-visible frame
#ifndef RG_HOST_TILE_WLOG_LIGHT
// one-launch host-visible frames of light-path scenes: 64x1 tiles, so that a wave's ring of
// consecutive tiles (rg_kernels.hip RG_HOST_RING) is one contiguous run of host memory
#define RG_HOST_TILE_WLOG_LIGHT 6
#endif
#ifndef RG_HOST_TILE_WLOG
// one-launch host-visible frames of heavy-path scenes: 16x4 tiles (RgKernelArgs::tile_wlog) --
// 64-B row segments per PCIe write, where 8x8 tiles send 32-B ones and 64x1 tiles lose the BVH
// walk's coherence: north star into pinned memory 2.53 -> 2.14 ms (8x8 -> 16x4; 32x2 2.22,
// 64x1 2.66: profiles/r05/s13, s14, s15)
#define RG_HOST_TILE_WLOG 4
#endif
#ifndef RG_COPY_HELPERS
#define RG_COPY_HELPERS 3       // helper threads of the pageable host copy (plus the calling thread)
#endif

// Parallel host memcpy for frames delivered into PAGEABLE caller memory: one
// thread moves a band out of pinned staging at ~10-17 GB/s, a third of what
// PCIe delivers (~56 GB/s), so the band is split over the calling thread and
// RG_COPY_HELPERS helpers.  Helpers spin while a render call is in progress
// (fork/join per band in ~1 us) and sleep between calls.
class rg_copy_pool {
  public:
    explicit rg_copy_pool(int helpers);
    ~rg_copy_pool();
    rg_copy_pool(const rg_copy_pool &) = delete;
    rg_copy_pool &operator=(const rg_copy_pool &) = delete;
    void begin();  // a render call starts: helpers spin
    void end();    // ... ends: helpers sleep
    void copy(void *dst, const void *src, size_t bytes);  // blocking, split over all threads

  private:
    void run(int id);
    struct Impl;
    Impl *p_;
};

// Resources of the host-visible paths (rg_render_image / rg_render_tiles /
// rg_render_stream), owned by the scene and reused across calls.
struct rg_image_res {
    std::shared_ptr<rg_copy_pool> pool;      // pageable destinations (created on first use)
    hipStream_t rs[2] = {nullptr, nullptr};  // render streams (bands alternate)
    hipStream_t cs = nullptr;                // device-to-host copies
    hipEvent_t ev_done[RG_IMAGE_MAX_BANDS] = {};
    hipEvent_t ev_copy[RG_IMAGE_MAX_BANDS] = {};
    hipEvent_t ev_t0 = nullptr, ev_t1 = nullptr, ev_join = nullptr;
    void *d_rgba = nullptr;
    size_t d_rgba_cap = 0;
    void *d_rgb = nullptr;
    size_t d_rgb_cap = 0;
    void *h_stage = nullptr;  // pinned
    size_t h_stage_cap = 0;
    void *h_frame = nullptr;  // pinned, coherent: whole frames the kernel writes over PCIe (pageable destinations)
    size_t h_frame_cap = 0;
    uint32_t *h_flags = nullptr;  // pinned, coherent: per-tile publication words (RgKernelArgs::tile_flags)
    size_t h_flags_cap = 0;       // bytes
    uint32_t seq = 0;             // frame sequence number the flags carry
    uint32_t *h_cancel = nullptr; // pinned, coherent: streaming cancellation word (RgKernelArgs::cancel)
    unsigned long long *h_snap = nullptr;  // pinned: 4 counter words per band
};

// Everything rg_scene_create uploads, as host tables (kept for replicas on
// other devices: rg_render_multi).
struct rg_host_tables {
    std::vector<RgSph> sph;
    std::vector<RgSphF> sphf;
    std::vector<RgSphF2> sphf2;
    std::vector<double> sph_cc;
    std::vector<int32_t> sph_id, pln_id, dsk_id, box_id;
    std::vector<RgPln> pln;
    std::vector<RgDsk> dsk;
    std::vector<RgBox> box;
    std::vector<RgBodyDev> bodies;
    std::vector<RgMatDev> mats;
    std::vector<RgLightDev> lights;
    std::vector<RgBvhNode> nodes;
    std::vector<RgLightBufDev> lbuf;           // per light (kind RG_LB_NONE: no buffer), first RG_LB_MAX_LIGHTS lights
    std::vector<uint32_t> lb_start, lb_ent;    // every light's cell starts / list entries, concatenated
    std::vector<uint32_t> tex_w, tex_h;
    std::vector<std::vector<uint32_t>> texels;
};

struct rg_multi_res;  // rg_multi.hip
struct rg_frames;     // rg_frames.hip (include/raingun_frames.h)

struct rg_scene {
    int device = 0;
    double fov = 90.0;
    float def[3] = {0, 0, 0};
    uint32_t max_depth = 10;
    int32_t n_sph = 0, n_pln = 0, n_dsk = 0, n_box = 0, n_bodies = 0, n_lights = 0, n_textures = 0;
    bool nan_scene = false;  // NaN distances possible (rg_kernels.hip ray_exotic)
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
    int32_t lane_min_depth = 1;  // rays of this depth and deeper walk the BVH per lane
    bool bvh_enabled = true;
    RgLightBufDev *lbuf = nullptr;  // shadow-ray light buffers (rg_lightbuf.cpp), n_lbuf lights
    uint32_t *lb_start = nullptr, *lb_ent = nullptr;
    int32_t n_lbuf = 0;             // light slots (the first n_lbuf lights; kind NONE: no buffer)
    int32_t lb_cam = -1;            // the camera buffer's index in lbuf (primary rays), -1: none
    int32_t n_lbdesc = 0;           // descriptors in lbuf (light slots + the camera buffer)
    bool lbuf_enabled = true;       // rg_debug_set_lightbuf
    float bvh_obound = 0.0f;
    double bvh_rbound = 0.0, bvh_margin = 0.0, bvh_extent = 0.0;
    rg_bvh_info bvh_info{};
    int tile_order = -1;  // expensive tiles first (rg_kernels.hip "tile ordering"): -1 auto (heavy path), 0, 1
    int image_bands = 0;  // host-visible frames: 0 auto, -1 one launch writing host memory, -2 split, 1..16 row bands
    int host_split_pct = 0;  // -2 (split): percent of the frame's rows rendered into device memory + DMA (0: default)
    mutable int split_fail_a = 0;
    // light-path host frames (rg_debug_set_host_ring): LDS-ring flush size and queue group of small
    // (< RG_RING_BIG_TILES tiles) and big launches; rg_render_multi's automatic mode runs light
    // scenes' shares as one launch per device (else bands + DMA)
    int ring_flush_small = RG_RING_FLUSH_SMALL, ring_group_small = RG_RING_GROUP_SMALL;
    int ring_flush_big = RG_RING_FLUSH_BIG, ring_group_big = RG_RING_GROUP_BIG;
    bool multi_light_one = RG_MULTI_LIGHT_ONE != 0;  // debug: the next N split renders report part A's launch as failed (rg_debug_fail_split_a)
    int host_tile_wlog = RG_HOST_TILE_WLOG;  // tile shape of the one-launch host-visible path
    bool host_tile_forced = false;           // set by rg_debug_set_host_tile_shape (else light scenes: 64x1)
    // rg_render_multi (rg_debug_set_multi): 0 each device copies its rows to the host, 1 RCCL gather;
    // stand-in: every "device" is this one, gathers through a stand-in (tests on one GPU);
    // bands per device share in the direct mode (0: automatic)
    int multi_mode = 0;
    bool multi_stand_in = false;
    int multi_bands = 0;
    int multi_only_rank = -1;  // stand-in direct mode: issue only this device's work (timeline rehearsal)
    std::shared_ptr<const rg_host_tables> host;
    std::vector<RgTexDev> tex_desc;  // the uploaded texture descriptors (device texel pointers)
    // the LDS arena as one device image (RgKernelArgs::lds_blob), for the layout it was built for
    void *lds_blob = nullptr;
    uint32_t lds_blob_layout[14] = {};
    mutable std::vector<rg_launch_ctx *> ctxs;  // one per stream used
    mutable rg_launch_ctx *last = nullptr;       // the context of the latest launch (rg_debug_counters)
    mutable rg_image_res img;
    mutable rg_multi_res *multi = nullptr;
    // frame pipelines built on this scene: a scene destroyed first detaches them
    // (rg_frames_destroy then no longer touches it), in either destruction order
    mutable std::vector<rg_frames *> frames;
};

// rg_frames.hip: the scene of `f` is going away (rg_scene_destroy)
void rg_frames_detach_scene(rg_frames *f);

// Kernel arguments of a scene (tables, LDS arena, frame constants).
RgKernelArgs rg_make_args(const rg_scene *s);

// Enqueue one tiled render on `stream` (the body of rg_render_tiles_async).
// snap (nullable, host memory, pinned for a truly asynchronous copy): the
// launch's 4 counter words (rays by class, error key) are copied there after
// the kernel.  ctx_out (nullable): the stream's launch context.  timed: record
// the context's ev0/ev1 around the launch (kernel_ms).
rg_status rg_launch_tiles(const rg_scene *s, uint32_t width, uint32_t height, const rg_tiling *tiling,
                          uint8_t *rgba_dev, float *rgb_dev, hipStream_t stream, unsigned long long *snap,
                          rg_launch_ctx **ctx_out, bool timed = false, uint32_t *tile_flags = nullptr,
                          uint32_t frame_seq = 0, const uint32_t *cancel = nullptr, uint32_t tile_wlog = 3,
                          bool host_frame = false,   // host_frame: rgba_dev is page-locked host memory
                          bool pipelined = false,    // frames in flight: size the grid for throughput
                          // a band of the tiling's selection: selected tiles [tile_first, tile_first + tile_count),
                          // rgba_dev / rgb_dev pointing at tile_first's first row
                          uint32_t tile_first = 0, uint32_t tile_count = 0xFFFFFFFFu,
                          // host_frame only: rgba_dev is the whole image, pixels go to their image rows
                          bool image_rows = false,
                          // groups of tile_group consecutive image tiles per stride (RgKernelArgs::tile_group)
                          uint32_t tile_group = 1);

// Rows a tiling selects when its tiles come in groups of `group` consecutive image tiles per
// stride (group 1: rg_tiling_rows); 0 for an invalid tiling or group (offset + group > stride).
uint32_t rg_tiling_rows_grouped(uint32_t height, const rg_tiling *t, uint32_t group);

// Ray counts and status of a counter snapshot (stats nullable).
rg_status rg_snap_status(const unsigned long long *snap, rg_stats *stats);

// Host-visible render of `tiling` into host buffers (rg_render_tiles / rg_render_image).
rg_status rg_render_host(const rg_scene *s, uint32_t width, uint32_t height, const rg_tiling *tiling,
                         uint8_t *rgba_out, float *rgb_out, rg_stats *stats);

// Is [p, p + bytes) page-locked host memory the DMA engine can write directly?
bool rg_host_is_pinned(const void *p, size_t bytes);
// The device address of page-locked host memory [p, p + bytes) (nullptr: not pinned).
void *rg_host_device_ptr(void *p, size_t bytes);

// A copy of `src` on `device` (same tables, same settings).
rg_status rg_scene_replica(const rg_scene *src, int32_t device, rg_scene **out);
void rg_scene_free(rg_scene *s);
void rg_sync_settings(rg_scene *dst, const rg_scene *src);  // depth, path, BVH, lane depth, tile order

// rg_multi.hip: free the scene's multi-GPU resources (replicas, communicators).
void rg_multi_release(const rg_scene *s);
