/*
 * raingun_debug.h — test/diagnostic entry points of libraingun_hip.so.
 * Not part of the reference's interface; used by tests/ to exercise every
 * kernel path on every scene.
 */
#ifndef RAINGUN_DEBUG_H
#define RAINGUN_DEBUG_H

#include "raingun.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Force the kernel path used for this scene: -1 = automatic (by body count),
 * 0 = light path (2 waves/SIMD, batched shadow rays, exact f64 tests),
 * 1 = heavy path (4 waves/SIMD, one ray per lane, f32 pre-filter + exact f64). */
rg_status rg_debug_set_path(rg_scene *scene, int32_t path);

/* Sphere BVH (built by rg_scene_create for scenes with at
 * least 16 spheres and used by the heavy path and rg_trace).  Disabling it
 * makes every ray scan all spheres; results are identical either way. */
typedef struct rg_bvh_info {
    int32_t built;         /* a BVH exists for this scene */
    int32_t enabled;       /* and is used by the render/trace launches */
    int32_t nodes;         /* 4-wide nodes (128 B each) */
    int32_t leaves;        /* leaves (<= 4 spheres each) */
    int32_t depth;         /* levels */
    float margin;          /* box inflation, scene units */
    float origin_bound;    /* rays with |o_k| above this scan all spheres */
    int32_t lane_stack;    /* per-lane walk: worst-case stack entries per lane */
    int64_t lbuf_bytes;    /* shadow-ray light buffers + camera buffer, device bytes (capped:
                            * RG_LB_TOTAL_WORDS words; lights past the cap keep the BVH walk) */
} rg_bvh_info;
rg_status rg_debug_set_bvh(rg_scene *scene, int32_t enable);
rg_status rg_debug_bvh_info(const rg_scene *scene, rg_bvh_info *info);

/* Shadow-ray light buffers (heavy path, BVH scenes; rg_lightbuf.cpp): per light,
 * a grid whose cells list every sphere a shadow ray starting there could hit,
 * so a shadow ray tests its cell's spheres instead of walking the BVH.  enable
 * 1 (default) / 0 (the BVH walk for every shadow ray); results are identical
 * either way.  rg_debug_lightbuf_count: lights whose buffer is in use (0 when
 * none was built, the BVH is off, or the buffers are switched off). */
rg_status rg_debug_set_lightbuf(rg_scene *scene, int32_t enable);
int32_t rg_debug_lightbuf_count(const rg_scene *scene);

/* BVH walk per ray kind: rays at recursion depth >= min_depth (secondary rays
 * and the shadow rays of their hits: incoherent) walk the tree per lane with a
 * nearest-first stack; shallower rays walk it wave-coherently.  0 = every
 * non-primary ray per lane, a large value = wave-coherent only, -1 = default
 * (1).  Heavy path only; results are identical either way. */
rg_status rg_debug_set_lane_depth(rg_scene *scene, int32_t min_depth);

/* Tile scheduling: 1 = a primary-ray probe orders each frame's 8x8 tiles by
 * estimated cost, most expensive first (stable within a cost class);
 * 0 = raster order; -1 (default) = ordered on the heavy (trace-dominated)
 * path only.  Results are identical either way. */
rg_status rg_debug_set_tile_order(rg_scene *scene, int32_t mode);

/* Host-visible frames (rg_render_image / rg_render_tiles without f32 RGB):
 * -1 = ONE launch whose pixel stores go over PCIe straight into page-locked
 * host memory (the caller's, or a pinned frame copied band by band into a
 * pageable caller buffer as the kernel publishes finished tiles);
 * 1..16 = render in this many row bands into device memory, each band's
 * device-to-host copy overlapping the next bands' renders; -2 = split (below);
 * 0 (default) = into page-locked buffers: split for light-path scenes, one
 * launch for heavy-path scenes; into pageable buffers: bands (~2 Mpx each, at
 * most 3).  Results are identical for every value. */
rg_status rg_debug_set_image_bands(rg_scene *scene, int32_t bands);

/* bands = -2 (page-locked whole-frame renders; otherwise as -1): the frame in two
 * concurrent parts sharing the PCIe link -- the top `pct` percent of the rows
 * rendered into device memory and copied by DMA, the rest in one launch writing
 * host memory.  pct 1..99, 0 = the library default.  Results are identical. */
rg_status rg_debug_set_host_split(rg_scene *scene, int32_t pct);

/* Fault injection for the split path's error exits: the next `count` split renders
 * report part A's launch as failed (RG_ERR_DEVICE) after part B -- the launch
 * storing into the caller's buffer -- is already enqueued.  The call must still
 * return only once nothing writes that buffer any more.  0 = off (default). */
rg_status rg_debug_fail_split_a(rg_scene *scene, int32_t count);

/* Light-path frames into page-locked host memory (the one-launch host-frame kernels; -1 keeps a
 * setting): finished tiles per LDS-ring flush (1..16, 0 = 16) and consecutive tiles the tile
 * queue hands a wave at a time (0 = the flush size), for launches below 50,000 tiles (`_small`:
 * rg_render_multi's device shares) and from it (`_big`: whole frames);
 * `multi_light_one` 1 (default) = rg_render_multi's automatic mode renders a light scene's device
 * shares as one launch each, 0 = bands + DMA copies.  Results are identical for every setting. */
rg_status rg_debug_set_host_ring(rg_scene *scene, int32_t flush_small, int32_t group_small, int32_t flush_big,
                                 int32_t group_big, int32_t multi_light_one);

/* Tile shape of the one-launch host-visible path: log2 of the tile width,
 * 3 (8x8) .. 6 (64x1), every tile 64 pixels; wider tiles give whole row
 * segments per PCIe write.  0 = automatic (the default: 16x4 for heavy-path
 * scenes, 64x1 for light-path scenes).  Device-resident renders always use 8x8. */
rg_status rg_debug_set_host_tile_shape(rg_scene *scene, int32_t tile_wlog);

/* rg_render_multi: mode 0 (default) = every device delivers its rows of the
 * frame to the host buffer itself, over its own PCIe link: `bands` = -1 one
 * launch per device whose kernel stores its rows straight into a page-locked
 * frame, 1..4 row bands per device, each band's rows copied while the later
 * bands render, 0 = automatic (one launch for heavy-path scenes into a
 * page-locked frame, else bands); mode 1 = ONE RCCL ncclGather of the parts to the scene's device,
 * re-interleave there, one copy to the host.  stand_in = 1 places every
 * "device" on the scene's device (a replica each) and routes mode 1's gather
 * through a stand-in with ncclGather's signature and group semantics, so
 * ngpus > 1 runs on one GPU (tests).  Results are identical for every setting.
 * only_rank >= 0 (stand-in, mode 0 only) issues only that device's work -- its
 * banded render and its rows' copies to the host -- so one GPU times the
 * timeline one device of an N-GPU node runs (the frame is then incomplete);
 * -1 = every device. */
rg_status rg_debug_set_multi(rg_scene *scene, int32_t mode, int32_t stand_in, int32_t bands, int32_t only_rank);

/* An rg_gather_fn (raingun_frames.h) that does nothing and returns 0: the
 * frame loop's own host cost per frame without a collective (probes). */
int rg_debug_gather_noop(const void *send, void *recv, size_t count, int datatype, int root, void *comm,
                         void *stream);

/* Copy the scene's 16 statistics words after the last render: [0..2] ray
 * counts, [4..8] BVH traversal statistics when the library was built with
 * -DRG_BVH_STATS (zero otherwise). */
rg_status rg_debug_counters(const rg_scene *scene, uint64_t out[16]);

/* Words [first, first + n) of the last render's counter set (RG_COUNTER_WORDS words):
 * diagnostic builds' extra statistics, e.g. -DRG_REGION_STATS region visits at 144.. */
rg_status rg_debug_counter_words(const rg_scene *scene, int32_t first, int32_t n, uint64_t *out);

#ifdef __cplusplus
}
#endif

#endif /* RAINGUN_DEBUG_H */
