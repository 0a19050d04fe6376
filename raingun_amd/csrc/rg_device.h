// rg_device.h — device-side scene layout shared by the render kernels and the
// C-ABI host code in rg_capi.hip.  gfx950 only.
//
// HBM layout of an uploaded scene (one rg_scene per device):
//   * hot tables (read by every ray, wave-uniform index -> scalar loads through
//     the constant address space, SGPR operands straight into v_*_f64):
//       sph[n_sph]   {cx, cy, cz, r*r}                 32 B  (bodies.rs:92-97)
//       sph_cc[n_sph] (cx*cx + cy*cy) + cz*cz           8 B   primary-ray shortcut
//       pln[n_pln]   {ox,oy,oz, nx,ny,nz, o.n, -}       64 B  (bodies.rs:136-149)
//       dsk[n_dsk]   {ox,oy,oz, nx,ny,nz, r, o.n}       64 B  (bodies.rs:173-192)
//       box[n_box]   {lo.xyz, hi.xyz}                   48 B  (bodies.rs:242-282)
//     each with an int id table giving the body's index in YAML order (the
//     closest-hit tie-break of scene.rs:34-39 is "first minimum in list order").
//   * cold tables (per-lane gathers at shading time, L2 resident):
//       bodies[n] {kind, params[7]}, mats[n] (one material per body),
//       lights[n_lights], textures (RGBA8 texels, one u32 per texel).
#pragma once
#include <stdint.h>

#if !defined(__HIP__) && !defined(__HIPCC__)  // plain C++ (host-only builds and tests of rg_bvh.cpp)
#define __device__
#define __host__
#define __forceinline__ inline
#endif

// Hot tables are read through the constant address space (addrspace 4) in
// device code: with a wave-uniform index that always lowers to s_load_* (SGPR
// operands, scalar cache), never to per-lane vector loads.
#ifdef __HIP_DEVICE_COMPILE__
#define RG_CONST __attribute__((address_space(4)))
#else
#define RG_CONST
#endif
template <class T>
__device__ __forceinline__ const RG_CONST T *rg_cptr(const T *p) { return (const RG_CONST T *)p; }

struct alignas(16) RgSph { double cx, cy, cz, r2; };
// f32 pre-filter records (see rg_kernels.hip, "f32 pre-filter"): conservative
// bounds, never values the exact test uses.
struct alignas(16) RgSphF { float cx, cy, cz, r2hi; };       // c rounded to f32; r2 rounded up (+slack)
struct alignas(16) RgSphF2 { float cchi, thrp, cc32; int32_t id; };  // |c|^2 rounded up; primary-ray threshold; fl32(c.c); YAML body id (= sph_id)
struct alignas(16) RgPln { double ox, oy, oz, nx, ny, nz, on, pad; };
struct alignas(16) RgDsk { double ox, oy, oz, nx, ny, nz, r, on; };
struct alignas(16) RgBox { double lo[3], hi[3]; };

// 4-wide BVH over the sphere table (built on the host, rg_bvh.cpp).  Child
// boxes are f32, inflated and rounded outward so that the f32 slab test can
// only err towards "visit" (derivation: rg_kernels.hip, "BVH traversal").
// child[k] >= 0: internal node; child[k] < 0: leaf, v = ~child[k], spheres
// [v >> 3, (v >> 3) + (v & 7) + 1) of the (BVH-ordered) sphere tables.
struct alignas(16) RgBvhNode {
    float lox[4], loy[4], loz[4], hix[4], hiy[4], hiz[4];
    int32_t child[4];
    int32_t nchild;        // valid children (2..4)
    int32_t pad[3];
};

// Per-lane traversal (incoherent rays, rg_kernels.hip "bvh_lane") walks the
// same 4-wide nodes with a per-lane stack in LDS.  Stack entry: the f32 bits
// of the child's entry distance with the low RG_LANE_NODE_BITS cleared (a
// lower bound, so pruning at pop is conservative) | the child's node index.
#define RG_LANE_NODE_BITS 12
#define RG_LANE_STACK_MAX 16      // entries per lane the LDS arena may hold

struct RgBodyDev {         // per body, YAML order
    int32_t kind;
    int32_t pad;
    double p[7];
};

struct RgMatDev {          // material.rs:7-12 (+ Coloration 20-24, Surface 49-54), flattened
    int32_t coloration;
    float color[3];
    int32_t tex;
    float xoff, yoff;
    float albedo_pi;       // albedo / f32::consts::PI (rendering.rs:164), the host's f32 division
    int32_t surface;
    float reflectivity;
    float index;
    float transparency;
};

struct RgLightDev {        // lights.rs:8-26
    int32_t kind;
    float color[3];
    float intensity;
    int32_t pad;
    double v[3];              // direction (Directional) or position (Spherical)
    double dn[3];             // Directional: normalize(-direction) (lights.rs:48), a per-light constant
    double pad2;              // 80 B: 16-B multiple for LDS staging
};

struct RgLightBufDev;  // rg_lightbuf_ray.h

struct RgTexDev {
    const uint32_t *texels;  // RGBA8 packed little-endian: r | g<<8 | b<<16 | a<<24
    int32_t w, h;
};

// Everything a render launch needs, passed by value as the kernel argument.
struct RgKernelArgs {
    // hot tables
    const RgSph *sph;
    const double *sph_cc;
    const RgSphF *sphf;
    const RgSphF2 *sphf2;
    const int32_t *sph_id;
    const RgPln *pln;
    const int32_t *pln_id;
    const RgDsk *dsk;
    const int32_t *dsk_id;
    const RgBox *box;
    const int32_t *box_id;
    int32_t n_sph, n_pln, n_dsk, n_box;
    // BVH over the spheres (n_nodes == 0: none; brute-force sphere loops)
    const RgBvhNode *nodes;
    int32_t n_nodes;
    int32_t lane_stack;      // per-lane traversal stack entries (0: every lane walks wave-coherently)
    int32_t lane_min_depth;  // rays at this recursion depth or deeper walk per lane (if lane_stack > 0)
    float bvh_obound;        // near-ray origin bound |o_k| (rg_bvh_ray.h)
    double bvh_rbound;       // far rays: half-size of the region holding every inflated sphere box
    double bvh_margin;       // box inflation m
    double bvh_extent;       // S: max |coordinate| of any sphere bound
    // cold tables
    const RgBodyDev *bodies;
    const RgMatDev *mats;
    const RgLightDev *lights;
    const RgTexDev *texs;
    int32_t n_bodies, n_lights, n_textures;
    // LDS arena (byte offsets; used by the LDS-staged kernel variants)
    // [lane stacks | sphf | sphf2 | sph | cc | nodes | pln | dsk | box | bodies | mats | lights | texs] (byte offsets)
    uint32_t lds_lstack_bytes;  // per-lane traversal stacks at offset 0: lane_stack x block threads x 4 B
    uint32_t lds_sphf, lds_sph, lds_cc, lds_nodes, lds_pln, lds_dsk, lds_box, lds_bodies, lds_mats, lds_lights, lds_texs, lds_hot_bytes, lds_total_bytes;
    int32_t path;            // RG_PATH_* forced by rg_debug_set_path, or RG_PATH_AUTO
    // frame
    uint32_t width, height;
    uint32_t tile_rows, tile_stride, tile_offset, out_rows;
    // selected tiles in groups of tile_group consecutive image tiles (1: the plain round robin):
    // selected tile i is image tile (i / group) * stride + offset + i % group -- rank 0's larger
    // share of the N-rank frame loop (rg_frames_set_root_tiles)
    uint32_t tile_group;
    uint32_t tile_base;      // the launch renders selected tiles tile_base, tile_base + 1, ... (output row 0 = its first row)
    double fov_adjustment;   // tan(fov.to_radians() / 2), ray.rs:45 (host libm)
    double aspect;           // width / height, ray.rs:43
    float def[3];            // scene.default_color
    uint32_t max_depth;      // scene.max_recursion_depth
    // outputs
    uint32_t *rgba;          // packed RGBA8, out_rows * width
    float *rgb;              // nullable, out_rows * width * 3
    const uint32_t *tile_perm;     // nullable: dequeue order of the 8x8 tiles (expensive first)
    unsigned long long *counters;  // [0]=primary [1]=shadow [2]=secondary [3]=~error key [16+16q]=tile queue heads (RG_COUNTER_WORDS words)
    unsigned long long *counters_next;  // nullable: the other counter set of the launch context, zeroed by the render kernel
    // frames of the shading tree for depths above the compiled arrays (rg_kernels.hip FrameStack<0>)
    void *deep_stack;        // grid threads x (max_depth - 1) frames, frame i of thread g at [i * deep_stride + g]
    uint32_t deep_stride;    // threads of the grid the buffer was sized for
    int32_t nan_scene;       // a body or light parameter is non-finite or >= 1e100: NaN distances possible
    unsigned long long *err_sticky;  // nullable: the launch context's error word that survives launches
    // nullable: one word per 8x8 tile of the launch; when a wave has written a
    // tile (rgba in page-locked host memory) it stores frame_seq there after a
    // system-scope release, so the host can consume the tile's rows while the
    // kernel renders on (host-visible frames into pageable memory, streaming)
    uint32_t *tile_flags;
    uint32_t frame_seq;
    const uint32_t *cancel;  // nullable (host memory): nonzero = take no further tiles (streaming cancellation)
    // Tile shape: 64 pixels (a lane each), 2^tile_wlog wide and 64 >> tile_wlog
    // tall -- 3: 8x8 (default: ray coherence); 5: 32x2 and 6: 64x1 give whole
    // 128/256-B row segments per store, which PCIe writes into host memory need
    // (8x8 tiles finishing in scattered order: 29.6 GB/s, 32x2: 51-53, 64x1:
    // 55-56; profiles/r02/host_visible/d2h_probe.jsonl)
    uint32_t tile_wlog;
    uint32_t defer_px;  // 1: hold pixels in LDS, one store per finished tile (the frame is in host memory)
    // nullable: the primary rays' sensor coordinates (ray.rs:46-51) per image
    // column (prim_sx[x]) and row (prim_sy[y]), computed on the host with the
    // kernel's exact expressions -- two f64 divisions per pixel become two loads
    const double *prim_sx, *prim_sy;
    // 1: this launch is one of several frames in flight (rg_render_tiles_async):
    // the heavy path sizes its persistent grid for throughput, not latency (launch_one)
    uint32_t pipelined;
    // (double)width, (double)height (ray.rs:46-51 divisions): kernel arguments land in SGPRs,
    // where the kernel's own conversions would hold two loop-invariant VGPR pairs
    double width_d, height_d;
    // nullable, host memory the device can write: the last wave of the launch to finish copies
    // the 4 statistics words (rays by class, error key) there -- no copy after the kernel
    unsigned long long *snap_out;
    uint32_t max_grid_threads;  // nonzero: cap on the persistent grid (the deep frame buffer's memory bound)
    // 1 (host-frame launches only): rgba is the WHOLE image and every pixel goes to its image row
    // (y * width + x) instead of its dense output row -- a device of rg_render_multi writes its
    // interleaved row tiles straight into the caller's frame (padding rows are not stored)
    uint32_t image_rows;
    // > 1: this launch is part j = out_tile_add of a call split into out_tile_mul launches (the
    // call's selected tile i -> launch i % mul); its selected tile s is written as the call's
    // tile s * mul + add, so the parts together fill the call's dense output
    uint32_t out_tile_mul, out_tile_add;
    // nullable: the whole LDS arena [0, lds_total_bytes) as one device image (light path): a
    // block stages its scene copy with ONE unrolled loop instead of a loop per table
    const void *lds_blob;
    // nullable: shadow-ray light buffers of the first n_lbuf lights (rg_lightbuf_ray.h); a light's
    // shadow rays test only the spheres of their cell's list (heavy path, BVH scenes)
    const RgLightBufDev *lbuf;
    const uint32_t *lb_start;  // cell list starts (per light: cells + 1 words, at RgLightBufDev::cell_off)
    const uint32_t *lb_ent;    // sphere positions of every list
    int32_t n_lbuf;
    int32_t lb_cam;            // >= 0: lbuf[lb_cam] is the camera buffer (a light buffer at the origin, primary rays)
    uint32_t lds_lbuf;         // LDS arena: the light-buffer descriptors (hot tables, after the texture descriptors)
    // light path into page-locked host memory (defer_px, LDS tile ring): finished tiles per ring flush
    // (1 .. RG_HOST_RING) and consecutive tiles the queue hands a wave at a time (1 .. ring_flush);
    // 0 = RG_HOST_RING for both.  Small launches (rg_render_multi's shares) want small groups (balance),
    // whole frames long runs of host memory per flush (rg_capi.hip host_ring_for)
    uint32_t ring_flush, ring_group;
};

__host__ __device__ inline uint32_t rg_tile_w(const RgKernelArgs &a) { return 1u << a.tile_wlog; }
__host__ __device__ inline uint32_t rg_tile_h(const RgKernelArgs &a) { return 64u >> a.tile_wlog; }
__host__ __device__ inline uint32_t rg_tiles_x(const RgKernelArgs &a) { return (a.width + rg_tile_w(a) - 1u) >> a.tile_wlog; }
__host__ __device__ inline uint32_t rg_tiles_y(const RgKernelArgs &a) { return (a.out_rows + rg_tile_h(a) - 1u) / rg_tile_h(a); }
__host__ __device__ inline unsigned long long rg_tile_count(const RgKernelArgs &a) {
    return (unsigned long long)rg_tiles_x(a) * rg_tiles_y(a);
}

// sizeof(Frame) in rg_kernels.hip (the deep frame buffer is sized on the host)
#define RG_FRAME_BYTES 88

// Light-path frames into page-locked host memory (the one-launch host-frame kernels' LDS tile ring,
// rg_kernels.hip): finished tiles per ring flush and consecutive tiles per queue slot, for launches
// below RG_RING_BIG_TILES 64-pixel tiles (rg_render_multi's device shares: balance over the waves)
// and from it (whole frames, part B of split frames: long runs of host memory per flush).  test1 4K
// (profiles/r06/s5/hv_ring_sweep.out): 8-device rehearsal 0.2895 ms banded -> 0.207 ms one launch
// at 4 / 1 (16 / 16: 0.241, 4 / 4: 0.273); the 1-GPU pinned frame 0.805 -> 0.768 ms at 8 / 8.
#ifndef RG_RING_FLUSH_SMALL
#define RG_RING_FLUSH_SMALL 4
#endif
#ifndef RG_RING_GROUP_SMALL
#define RG_RING_GROUP_SMALL 1
#endif
#ifndef RG_RING_FLUSH_BIG
#define RG_RING_FLUSH_BIG 8
#endif
#ifndef RG_RING_GROUP_BIG
#define RG_RING_GROUP_BIG 8
#endif
#ifndef RG_RING_BIG_TILES
#define RG_RING_BIG_TILES 50000u
#endif
#ifndef RG_MULTI_LIGHT_ONE
#define RG_MULTI_LIGHT_ONE 1  // rg_render_multi, automatic mode: light scenes' shares as one launch per device
#endif
#ifndef RG_LB
#define RG_LB 3                   // lights per shadow batch on the light path (its LB template parameter)
#endif
#ifndef RG_LB_SMALL
#define RG_LB_SMALL 2             // light scenes with at most this many lights run a batch this wide (0: off)
#endif
#ifndef RG_LB_ONE
#define RG_LB_ONE 1               // light scenes with one light (or none) run a batch of one
#endif
#ifndef RG_HEAVY_WPS
#define RG_HEAVY_WPS 3            // heavy path: waves per SIMD (block = 256 * WPS threads; 168 VGPRs)
#endif
#ifndef RG_HEAVY_SCENE_BODIES
#define RG_HEAVY_SCENE_BODIES 32  // bodies per ray at which the trace loop, not shading, dominates
#endif

#define RG_PATH_AUTO -1
#define RG_PATH_LIGHT 0   // 2 waves/SIMD, batched shadow rays, exact f64 tests only
#define RG_PATH_HEAVY 1   // 4 waves/SIMD, one ray per lane, f32 pre-filter + exact f64 tests

// Kernel path of a launch (the launcher and the host's tile-order policy agree on it).
__host__ __device__ __forceinline__ bool rg_heavy_path(const RgKernelArgs &a) {
    bool heavy = a.n_sph + a.n_pln + a.n_dsk + a.n_box >= RG_HEAVY_SCENE_BODIES;
    if (a.path != RG_PATH_AUTO) heavy = a.path == RG_PATH_HEAVY;
    if (a.n_lights > RG_LB) heavy = true;  // the light path shades all lights in ONE batch
    return heavy;
}

#define RG_COUNTER_WORDS (16 + 16 * 16 + 16)  // stats + 16 queue heads, 128 B apart + the finished-wave count
#define RG_DONE_WORD (16 + 16 * 16)            // waves of the launch that finished (RgKernelArgs::snap_out)

// counters[3] holds ~((pixel << 8) | -status) of the lowest erroring pixel
// (atomicMax of the complement); 0 = no error, so one memset resets all four.
