/*
 * raingun.h — C ABI of the MI355X-native renderer for raingun's per-pixel
 * ray-trace path (libraingun_hip.so).
 *
 * The reference has no FFI layer: the seam this ABI replaces is the Rust
 * function
 *     rendering::render_image(scene: &Scene, width: u32, height: u32)
 *         -> ImageBuffer<Rgba<u8>, Vec<u8>>          raingun-lib/src/rendering.rs:24-38
 * reached through Scene::render_image (raingun-lib/src/scene.rs:41-43) from
 * the batch driver (src/render.rs:55).  Everything below that call
 * (render_pixel / get_color / cast_ray / shade_diffuse / fresnel and the body,
 * ray, light, material and colour primitives) runs inside one HIP megakernel
 * for gfx950.
 *
 * All plain C: pointers, sizes, POD structs.  No torch types, no C++.
 * Paths are relative to /root/reference.
 */
#ifndef RAINGUN_H
#define RAINGUN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RG_ABI_VERSION 1

/* ------------------------------------------------------------------------
 * Status codes.  The reference panics; the ABI returns one negative code per
 * panic site instead (no exception or abort ever crosses the boundary).
 * ---------------------------------------------------------------------- */
typedef enum rg_status {
    RG_OK = 0,
    RG_ERR_INVALID_ARGUMENT = -1,   /* null pointers, zero sizes, bad enum values */
    RG_ERR_PORTRAIT = -2,           /* assert!(width >= height)          ray.rs:42 */
    RG_ERR_AABB_NORMAL = -3,        /* "Could not determine normal"       bodies.rs:324 */
    RG_ERR_NAN_DISTANCE = -4,       /* partial_cmp(..).unwrap() on NaN    scene.rs:38 */
    RG_ERR_TRANSMISSION = -5,       /* create_transmission(..).unwrap()   rendering.rs:106 */
    RG_ERR_TEXTURE = -6,            /* texture index out of range / empty image (material.rs:34-47) */
    RG_ERR_DEVICE = -10,            /* HIP runtime error */
    RG_ERR_OUT_OF_MEMORY = -11,
    RG_ERR_CANCELLED = -12,         /* streaming receiver dropped         rendering.rs:53-54 */
    RG_ERR_COLLECTIVE = -13,        /* rg_render_multi: RCCL missing or a collective failed */
    RG_ERR_PENDING = -14            /* rg_frames_read_image: a frame batch still waits for its gather
                                       (call rg_frames_flush on every rank first) */
} rg_status;

/* ------------------------------------------------------------------------
 * Flat POD scene description — mirrors `Scene` (scene.rs:11-19) after serde
 * has run: bodies and lights in YAML order, textures already decoded to RGBA8
 * (material.rs:34-47 decodes eagerly at load time).
 * ---------------------------------------------------------------------- */
enum rg_body_kind {            /* bodies.rs:41-47 */
    RG_BODY_SPHERE = 0,        /* p = {center.x, center.y, center.z, radius}                 */
    RG_BODY_PLANE = 1,         /* p = {origin.x, origin.y, origin.z, normal.x, normal.y, normal.z} */
    RG_BODY_DISK = 2,          /* p = {origin.xyz, normal.xyz, radius}                        */
    RG_BODY_AABB = 3           /* p = {bounds[0].xyz, bounds[1].xyz}                          */
};

enum rg_coloration_kind {      /* material.rs:20-24 */
    RG_COLORATION_COLOR = 0,
    RG_COLORATION_TEXTURE = 1
};

enum rg_surface_kind {         /* material.rs:49-54 */
    RG_SURFACE_DIFFUSE = 0,
    RG_SURFACE_REFLECTING = 1,
    RG_SURFACE_REFRACTIVE = 2
};

enum rg_light_kind {           /* lights.rs:22-26 */
    RG_LIGHT_DIRECTIONAL = 0,  /* v = direction */
    RG_LIGHT_SPHERICAL = 1     /* v = position  */
};

typedef struct rg_material {   /* material.rs:7-12 */
    uint32_t coloration;       /* rg_coloration_kind */
    float color[3];            /* Coloration::Color, f32 RGB in [0,1] (color.rs:7-11) */
    int32_t texture;           /* Coloration::Texture: index into rg_scene_desc.textures */
    float x_offset, y_offset;  /* Texture::{x_offset,y_offset} (material.rs:30-31) */
    float albedo;
    uint32_t surface;          /* rg_surface_kind */
    float reflectivity;        /* Surface::Reflecting */
    float index;               /* Surface::Refractive */
    float transparency;        /* Surface::Refractive */
} rg_material;

typedef struct rg_body {
    uint32_t kind;             /* rg_body_kind */
    uint32_t _pad;
    double p[7];
    rg_material material;
} rg_body;

typedef struct rg_light {      /* lights.rs:8-20 */
    uint32_t kind;             /* rg_light_kind */
    float color[3];
    float intensity;
    uint32_t _pad;
    double v[3];
} rg_light;

typedef struct rg_texture {    /* decoded DynamicImage, RGBA8 row-major, width*height*4 bytes */
    uint32_t width, height;
    const uint8_t *rgba;
} rg_texture;

typedef struct rg_scene_desc { /* scene.rs:11-19; defaults scene.rs:21-31 */
    double fov;                /* degrees, default 90 */
    float default_color[3];    /* default black */
    uint32_t max_recursion_depth; /* default 10 */
    uint32_t n_bodies;
    const rg_body *bodies;
    uint32_t n_lights;
    const rg_light *lights;
    uint32_t n_textures;
    const rg_texture *textures;
} rg_scene_desc;

/* Ray counts by class.  A ray is one Scene::trace call (scene.rs:34-39):
 * primary rendering.rs:73, shadow rendering.rs:150, secondary rendering.rs:126. */
typedef struct rg_ray_counts {
    uint64_t primary;
    uint64_t shadow;
    uint64_t secondary;
} rg_ray_counts;

typedef struct rg_stats {
    rg_ray_counts rays;
    float kernel_ms;           /* HIP-event time of the render launch(es) on the render stream */
    int32_t error_pixel;       /* first pixel (linear index) that raised a device error, or -1 */
    uint32_t _pad;
} rg_stats;

/* Row selection for sharded renders: the frame is cut into tiles of
 * `tile_rows` rows; this call renders tiles t with t % tile_stride == tile_offset,
 * packed densely into the output in increasing t (the last tile may be partial
 * and is zero-padded in the output to a full tile).  {tile_rows=height,
 * tile_stride=1, tile_offset=0} is the whole frame.  */
typedef struct rg_tiling {
    uint32_t tile_rows;
    uint32_t tile_stride;
    uint32_t tile_offset;
} rg_tiling;

typedef struct rg_scene rg_scene;   /* opaque device-resident scene */

/* ---------------------------------------------------------------- API */

int32_t rg_abi_version(void);
const char *rg_status_string(int32_t status);

/* Number of HIP devices visible (0 if none / runtime missing). */
int32_t rg_device_count(void);

/* Copy the scene to `device` (SoA body tables, material/light tables, RGBA8
 * textures).  The caller keeps ownership of `desc` and its arrays.
 * Replaces Scene's deserialised in-memory form (scene.rs:11-19). */
rg_status rg_scene_create(const rg_scene_desc *desc, int32_t device, rg_scene **out);
void rg_scene_destroy(rg_scene *scene);

/* Override the recursion cap of an uploaded scene (main.rs:119-123 clamps it;
 * the depth-5 configs set it directly, scene.rs:16 is a pub field). */
rg_status rg_scene_set_max_depth(rg_scene *scene, uint32_t max_recursion_depth);

/* Blocking whole-frame render into a caller-owned host buffer of
 * width*height*4 bytes (row-major RGBA8, alpha 255).
 * Replaces rendering::render_image (rendering.rs:24-38). `stats` may be NULL.
 * Into a pinned `rgba_out` (rg_host_register, or memory from hipHostMalloc)
 * a heavy (trace-dominated) scene renders in ONE launch whose pixel stores go
 * over PCIe straight into the buffer; otherwise the frame renders in row
 * bands whose device-to-host copies overlap the later bands' renders (the DMA
 * lands directly in a pinned buffer; a pageable one is filled from pinned
 * staging by several host threads).  Any max_recursion_depth renders (scene.rs:16 is a u32): depths
 * above 65 keep their shading frames in device memory, 88 B per open frame
 * per thread of a persistent grid; when that exceeds half the free device
 * memory (capped at 16 GiB) the grid shrinks to fit -- slower, same frame --
 * and only when a single block's frames do not fit does the call return
 * RG_ERR_OUT_OF_MEMORY (depth ~ 10^6 and up).  On a device error
 * (RG_ERR_AABB_NORMAL / _NAN_DISTANCE / _TRANSMISSION: the reference's
 * panics) the frame is still delivered and stats->error_pixel names the first
 * (lowest-index) pixel that raised it. */
rg_status rg_render_image(const rg_scene *scene, uint32_t width, uint32_t height,
                          uint8_t *rgba_out, rg_stats *stats);

/* Page-lock a caller buffer (hipHostRegister) so rg_render_image / rg_render_tiles
 * / rg_render_multi DMA straight into it; unregister before freeing it.  Optional:
 * pageable buffers work too (staged).  A Rust caller registers its
 * ImageBuffer's Vec once and reuses it across frames. */
rg_status rg_host_register(void *ptr, size_t bytes);
rg_status rg_host_unregister(void *ptr);

/* Device-resident variant used by sharded / benchmark callers: renders the
 * tiles selected by `tiling` into `rgba_dev` (device pointer on the scene's
 * device, tiles_selected*tile_rows*width*4 bytes), on HIP stream `stream`
 * (a hipStream_t; NULL = null stream).  `rgb_dev` (nullable, device) receives
 * the pre-quantisation f32 RGB (3 floats per pixel, same packing) for float
 * parity checks.  Asynchronous unless `stats` is non-NULL, in which case the
 * call synchronises `stream` and fills ray counts, kernel time and errors.
 * Launches of one scene on DISTINCT streams may be in flight together (frames
 * in flight): each stream has its own launch state (ray counters, tile queue,
 * error word), created on the stream's first use.  Calls on one scene must
 * come from one host thread at a time.  The launch is sized for its own
 * latency (the whole GPU for this one frame). */
rg_status rg_render_tiles_async(const rg_scene *scene, uint32_t width, uint32_t height,
                                const rg_tiling *tiling, uint8_t *rgba_dev, float *rgb_dev,
                                void *stream, rg_stats *stats);

/* rg_render_tiles_async for a caller that keeps several frames in flight on
 * distinct streams (rg_frames, bench.py): asynchronous, and trace-heavy scenes
 * size their persistent grid for throughput -- a small launch takes a third
 * of the GPU or more with at least 32 tiles per wave, and the other frames in
 * flight fill the rest -- rather than for one launch's latency.  Same output. */
rg_status rg_render_tiles_pipelined(const rg_scene *scene, uint32_t width, uint32_t height,
                                    const rg_tiling *tiling, uint8_t *rgba_dev, float *rgb_dev,
                                    void *stream);

/* Forget the launch state of `stream` (before the caller destroys that stream);
 * the null stream's state lives as long as the scene. */
rg_status rg_scene_release_stream(rg_scene *scene, void *stream);

/* Status of the launches enqueued on `stream` since the previous call:
 * synchronises the stream, returns the first (lowest-pixel) device error any
 * of them raised (RG_OK if none) with its pixel in *error_pixel (nullable;
 * -1 if none), and clears it.  For asynchronous callers (stats == NULL),
 * whose launches otherwise report nothing. */
rg_status rg_stream_status(const rg_scene *scene, void *stream, int32_t *error_pixel);

/* Host-buffer variant of rg_render_tiles_async (blocking).  rgb_out nullable. */
rg_status rg_render_tiles(const rg_scene *scene, uint32_t width, uint32_t height,
                          const rg_tiling *tiling, uint8_t *rgba_out, float *rgb_out,
                          rg_stats *stats);

/* Number of output rows a tiling produces for `height` (tiles selected * tile_rows). */
uint32_t rg_tiling_rows(uint32_t height, const rg_tiling *tiling);

/* Tile-completion streaming (replaces render_image_stream, rendering.rs:40-69,
 * which sends one RenderedPixel per pixel over an mpsc channel): ONE launch
 * renders the frame into page-locked host memory and publishes every finished
 * tile; `on_tile` receives each band of `tile_rows` rows, in row order, as soon
 * as the band is complete, while the kernel renders on.  A non-zero return
 * from `on_tile` cancels: the kernel takes no further tiles (the reference's
 * `.all` stops when the channel closes) and the call returns RG_ERR_CANCELLED.
 * The band pointer is valid only during the callback. */
typedef int32_t (*rg_tile_callback)(uint32_t row_begin, uint32_t rows, uint32_t width,
                                    const uint8_t *rgba, void *user);
rg_status rg_render_stream(const rg_scene *scene, uint32_t width, uint32_t height,
                           uint32_t tile_rows, rg_tile_callback on_tile, void *user,
                           rg_stats *stats);

/* Closest-hit query over all bodies (Scene::trace, scene.rs:34-39) for n rays
 * given as {origin.xyz, direction.xyz} doubles (host buffers).  dist[i] is the
 * hit distance and body[i] the body index, or body[i] = -1 on a miss. */
rg_status rg_trace(const rg_scene *scene, const double *rays, uint32_t n,
                   double *dist, int32_t *body);

/* Single-process multi-GPU render (SURVEY.md §8(b),(e)): the same frame as
 * rg_render_image, split over `ngpus` devices -- the scene's device first,
 * then the next visible devices in order -- in `tile_rows`-row tiles dealt
 * round-robin (tile t -> device t % ngpus; 0 = 8 rows).  Each device renders
 * its tiles with its own replica of the scene (made on first use and kept)
 * in row bands, and after each band copies that band's tiles straight to
 * their image rows of `rgba_out` (width*height*4 bytes, host) with one
 * strided copy over its OWN PCIe link, overlapped with its later bands: N
 * links carry 1/N of the frame each (a pageable buffer is fed from a pinned
 * frame by host threads).  The RCCL path -- one ncclGather over xGMI to the
 * scene's device, re-interleave, one copy -- remains available through
 * rg_debug_set_multi (mode 1); its communicators come from ncclCommInitAll in
 * this process (RCCL loaded at run time: the librccl already in the process,
 * else $RG_RCCL_LIBRARY, else librccl.so.1; RG_ERR_COLLECTIVE if it cannot be
 * loaded).  No torch, no launcher: the drop-in for the reference's one
 * blocking call (rendering.rs:24-38, src/render.rs:55) on a whole node.
 * `stats` sums the devices' rays; on device errors error_pixel is the lowest
 * failing pixel of any device; kernel_ms is device 0's render span (its
 * launches, not the other devices' work or the copies to the host).  Every
 * copy into rgba_out has landed when the call returns, on errors too. */
rg_status rg_render_multi(const rg_scene *scene, uint32_t width, uint32_t height, int32_t ngpus,
                          uint32_t tile_rows, uint8_t *rgba_out, rg_stats *stats);

#ifdef __cplusplus
}
#endif

#endif /* RAINGUN_H */
