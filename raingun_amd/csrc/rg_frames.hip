// rg_frames.hip — frames in flight over N ranks (include/raingun_frames.h).
//
// Per frame k, slot b = k % depth:
//   render stream b : wait done[b] -> render this rank's tiles into part[b] (off the root: pack it
//                     to RGB, 3 B per pixel) -> record rendered[b]
//   comm stream     : wait rendered[b] -> ncclGather(packed[b] -> gathered[b] on rank 0) -> record sent[b]
//   side stream     : (rank 0) wait sent[b] -> re-interleave gathered[b] into image[b] -> record done[b]
// (non-root ranks: done[b] = sent[b]).  All gathers go through ONE stream, so
// every rank issues and runs them in frame order; renders of consecutive frames
// overlap on their own streams.  Host work per frame is a handful of runtime
// calls (the Python pipeline spent ~70 us per frame on rank 0).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <new>
#include <vector>

#include "../../include/raingun.h"
#include "../../include/raingun_debug.h"
#include "../../include/raingun_frames.h"
#include "rg_internal.h"

namespace {

bool ok(hipError_t e) { return e == hipSuccess; }

// The gathered parts travel as packed RGB, 3 B per pixel: alpha is always
// 255 (color.rs rgba()), so a quarter of every gather's bytes over xGMI carried
// no information.  Non-root ranks pack their part after the render; the root
// re-interleaves its OWN rows straight from its RGBA part (its slot of the
// gather is not read) and the others' from the packed slots, re-adding alpha.
__global__ __launch_bounds__(256) void rg_pack_rgb_kernel(const uint32_t *rgba, uint8_t *rgb, size_t npx) {
    const size_t g = (size_t)blockIdx.x * 256u + threadIdx.x;  // pixels 4g .. 4g+3
    const size_t p0 = g * 4u;
    if (p0 >= npx) return;
    if (p0 + 4u <= npx) {
        const uint4 v = reinterpret_cast<const uint4 *>(rgba)[g];
        uint32_t *o = reinterpret_cast<uint32_t *>(rgb + p0 * 3u);  // 12 g bytes: dword aligned
        o[0] = (v.x & 0xFFFFFFu) | (v.y << 24);
        o[1] = ((v.y >> 8) & 0xFFFFu) | (v.z << 16);
        o[2] = ((v.z >> 16) & 0xFFu) | ((v.w & 0xFFFFFFu) << 8);
    } else {
        for (size_t p = p0; p < npx; ++p) {
            const uint32_t v = rgba[p];
            rgb[3 * p] = (uint8_t)v;
            rgb[3 * p + 1] = (uint8_t)(v >> 8);
            rgb[3 * p + 2] = (uint8_t)(v >> 16);
        }
    }
}

// Image row y lives in tile t = y / T.  The tiles are dealt in periods of
// P = root + world - 1: the first `root` tiles of each period to rank 0, then one
// to each other rank (root = 1: the round robin t -> rank t % world).  Tile t is
// that rank's (t / P * root + t % P)-th (rank 0) or (t / P)-th tile (the others):
// its row of the part is that index * T + y % T (distributed.py assemble).  Rank
// 0's rows come from root_part (RGBA), the others' from their packed slots
// (slot_bytes apart).  4 pixels per thread.
__global__ __launch_bounds__(256) void rg_reinterleave_kernel(const uint8_t *gathered, const uint32_t *root_part,
                                                              uint32_t *image, uint32_t width, uint32_t height,
                                                              uint32_t tile_rows, uint32_t world, uint32_t root,
                                                              size_t slot_bytes) {
    const uint32_t y = blockIdx.y;
    const uint32_t x0 = (blockIdx.x * 256u + threadIdx.x) * 4u;
    if (y >= height || x0 >= width) return;
    const uint32_t t = y / tile_rows, P = root + world - 1u;
    const uint32_t p = t / P, j = t - p * P;
    const uint32_t r = j < root ? 0u : j - root + 1u;
    const uint32_t src_row = (r == 0u ? p * root + j : p) * tile_rows + (y - t * tile_rows);
    uint32_t *dst = image + (size_t)y * width + x0;
    const size_t src_px = (size_t)src_row * width + x0;
    if (r == 0) {
        const uint32_t n = min(4u, width - x0);
        for (uint32_t k = 0; k < n; ++k) dst[k] = root_part[src_px + k];
        return;
    }
    const uint8_t *src = gathered + (size_t)r * slot_bytes + src_px * 3u;
    if ((width & 3u) == 0u) {  // whole, dword-aligned groups of 4 pixels
        const uint32_t *w = reinterpret_cast<const uint32_t *>(src);
        const uint32_t a = w[0], b = w[1], c = w[2];
        uint4 o;
        o.x = (a & 0xFFFFFFu) | 0xFF000000u;
        o.y = (a >> 24) | ((b & 0xFFFFu) << 8) | 0xFF000000u;
        o.z = (b >> 16) | ((c & 0xFFu) << 16) | 0xFF000000u;
        o.w = (c >> 8) | 0xFF000000u;
        *reinterpret_cast<uint4 *>(dst) = o;
    } else {
        const uint32_t n = min(4u, width - x0);
        for (uint32_t k = 0; k < n; ++k)
            dst[k] = (uint32_t)src[3 * k] | ((uint32_t)src[3 * k + 1] << 8) | ((uint32_t)src[3 * k + 2] << 16) |
                     0xFF000000u;
    }
}

}  // namespace

size_t rg_packed_slot_bytes(uint32_t slot_rows, uint32_t width) {
    return ((size_t)slot_rows * width * 3u + 15u) & ~(size_t)15u;
}

hipError_t rg_launch_pack_rgb(const void *rgba, void *rgb, size_t npx, hipStream_t stream) {
    const size_t groups = (npx + 3u) / 4u;
    hipLaunchKernelGGL(rg_pack_rgb_kernel, dim3((unsigned)((groups + 255u) / 256u)), dim3(256), 0, stream,
                       static_cast<const uint32_t *>(rgba), static_cast<uint8_t *>(rgb), npx);
    return hipGetLastError();
}

hipError_t rg_launch_reinterleave(const void *gathered, const void *root_part, void *image, uint32_t width,
                                  uint32_t height, uint32_t tile_rows, uint32_t world, size_t slot_bytes,
                                  hipStream_t stream, uint32_t root) {
    dim3 grid((((width + 3u) / 4u) + 255u) / 256u, height);
    hipLaunchKernelGGL(rg_reinterleave_kernel, grid, dim3(256), 0, stream, static_cast<const uint8_t *>(gathered),
                       static_cast<const uint32_t *>(root_part), static_cast<uint32_t *>(image), width, height,
                       tile_rows, world, root, slot_bytes);
    return hipGetLastError();
}

struct rg_frames {
    const rg_scene *scene = nullptr;
    int device = 0;
    uint32_t w = 0, h = 0, T = 0, slot_rows = 0;
    int rank = 0, world = 1, depth = 1;
    size_t part_bytes = 0;   // RGBA part of a frame
    size_t slot_bytes = 0;   // packed RGB part: what each rank sends (rg_packed_slot_bytes)
    rg_tiling tiling{};
    uint32_t root = 1;          // tiles of rank 0 per period (rg_frames_set_root_tiles)
    size_t root_part_rows = 0;  // rows of rank 0's part
    void *comm = nullptr;
    rg_gather_fn gather = nullptr;
    std::vector<hipStream_t> render;
    hipStream_t comm_stream = nullptr, side = nullptr;
    std::vector<void *> parts, packed, gathered, image;  // parts/image per slot; packed/gathered per batch
    std::vector<hipEvent_t> rendered, sent, done;
    unsigned long long k = 0;
    int last = -1;
    int batch = 1;              // frames per gather (consecutive slots of one batch)
    int pend_b0 = 0, pend_n = 0;  // rendered frames of the current batch not gathered yet
    rg_status err = RG_OK;     // first device error of any frame (sticky until destroy)
    int32_t err_pixel = -1;
};

namespace {

void frames_release(rg_frames *f) {
    if (!f) return;
    (void)hipSetDevice(f->device);
    for (hipStream_t s : f->render) (void)hipStreamSynchronize(s);
    if (f->comm_stream) (void)hipStreamSynchronize(f->comm_stream);
    if (f->side) (void)hipStreamSynchronize(f->side);
    for (void *p : f->parts) (void)hipFree(p);
    for (void *p : f->packed) (void)hipFree(p);
    for (void *p : f->gathered) (void)hipFree(p);
    for (void *p : f->image) (void)hipFree(p);
    for (hipEvent_t e : f->rendered) (void)hipEventDestroy(e);
    for (hipEvent_t e : f->sent) (void)hipEventDestroy(e);
    for (hipEvent_t e : f->done) (void)hipEventDestroy(e);
    rg_scene *sc = const_cast<rg_scene *>(f->scene);  // nullptr: the scene was destroyed first (it freed our launch state)
    if (sc) {
        auto &v = sc->frames;
        v.erase(std::remove(v.begin(), v.end(), f), v.end());
    }
    for (hipStream_t s : f->render) {
        if (sc) (void)rg_scene_release_stream(sc, s);  // its launch state goes with it
        (void)hipStreamDestroy(s);
    }
    if (f->comm_stream) (void)hipStreamDestroy(f->comm_stream);
    if (f->side) (void)hipStreamDestroy(f->side);
    delete f;
}

}  // namespace

void rg_frames_detach_scene(rg_frames *f) {
    if (!f) return;
    (void)hipSetDevice(f->device);
    for (hipStream_t s : f->render) (void)hipStreamSynchronize(s);
    f->scene = nullptr;
}

extern "C" {

rg_status rg_frames_create(const rg_scene *scene, uint32_t width, uint32_t height, uint32_t tile_rows, int32_t rank,
                           int32_t world, int32_t depth, void *comm, rg_gather_fn gather, rg_frames **out) {
    if (!out) return RG_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    if (!scene || !comm || !gather || width == 0 || height == 0 || tile_rows == 0 || world < 1 || rank < 0 ||
        rank >= world || depth < 1 || depth > 16)
        return RG_ERR_INVALID_ARGUMENT;
    if (width < height) return RG_ERR_PORTRAIT;  // ray.rs:42
    int dev = 0;
    if (!ok(hipGetDevice(&dev))) return RG_ERR_DEVICE;
    rg_frames *f = new (std::nothrow) rg_frames();
    if (!f) return RG_ERR_OUT_OF_MEMORY;
    f->scene = scene;
    f->device = dev;
    f->w = width;
    f->h = height;
    f->T = tile_rows;
    f->rank = rank;
    f->world = world;
    f->depth = depth;
    f->comm = comm;
    f->gather = gather;
    f->tiling = rg_tiling{tile_rows, (uint32_t)world, (uint32_t)rank};
    const uint32_t tiles = (height + tile_rows - 1) / tile_rows;
    f->slot_rows = (tiles + (uint32_t)world - 1) / (uint32_t)world * tile_rows;  // equal on every rank
    f->root_part_rows = f->slot_rows;
    f->part_bytes = (size_t)f->slot_rows * width * 4;
    f->slot_bytes = rg_packed_slot_bytes(f->slot_rows, width);
    bool good = true;
    auto stream = [&](hipStream_t &s) { good = good && ok(hipStreamCreateWithFlags(&s, hipStreamNonBlocking)); };
    auto event = [&](std::vector<hipEvent_t> &v) {
        hipEvent_t e = nullptr;
        good = good && ok(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        v.push_back(e);
    };
    auto alloc = [&](std::vector<void *> &v, size_t bytes) {
        void *p = nullptr;
        good = good && ok(hipMalloc(&p, bytes)) && ok(hipMemset(p, 0, bytes));  // padding rows stay zero
        v.push_back(p);
    };
    // two frames per gather halve rank 0's per-frame enqueue cost (RCCL's host work
    // is per call); a depth that is not even keeps one
    f->batch = (world > 1 && depth % 2 == 0) ? 2 : 1;
    const int B = 2;  // batch buffers hold the largest batch (rg_frames_set_batch); batch p = slots 2p, 2p+1
    f->render.assign(depth, nullptr);
    for (int b = 0; b < depth && good; ++b) {
        stream(f->render[b]);
        // the root sends (and ignores) the first batch * slot_bytes of its RGBA part
        alloc(f->parts, std::max(f->part_bytes, f->slot_bytes * B));
        event(f->rendered);
        event(f->sent);
        event(f->done);
        if (rank == 0) alloc(f->image, (size_t)height * width * 4);
        if (b % B != 0) continue;  // one send / receive buffer per batch of B slots
        if (rank == 0)
            alloc(f->gathered, f->slot_bytes * B * (size_t)world);
        else
            alloc(f->packed, f->slot_bytes * B);
    }
    stream(f->comm_stream);
    stream(f->side);
    if (!good) {
        frames_release(f);
        return RG_ERR_OUT_OF_MEMORY;
    }
    scene->frames.push_back(f);
    *out = f;
    return RG_OK;
}

void rg_frames_destroy(rg_frames *f) { frames_release(f); }

}  // extern "C"

namespace {

// ONE gather for the n consecutive frames of slots b0 .. b0 + n - 1 (one batch):
// rank r's chunk of the receive buffer holds its n packed parts back to back.
rg_status issue_gather(rg_frames *f, int b0, int n) {
    const int B = 2;
    const int p = b0 / B, h0 = b0 % B;  // the batch's buffers, the first frame's place in them
    const size_t count = (size_t)n * f->slot_bytes;
    void *send = f->rank == 0 ? f->parts[b0] : static_cast<uint8_t *>(f->packed[p]) + (size_t)h0 * f->slot_bytes;
    // a batch cut short by a flush leaves the batch's later frames their own part of the
    // buffers (send: slot h; receive: from h0 * world slots on), so the next frames'
    // gather never overwrites what the root's re-interleave of this one still reads
    void *recv = f->rank == 0 ? static_cast<uint8_t *>(f->gathered[p]) + (size_t)h0 * f->world * f->slot_bytes : nullptr;
    // ncclUint8 = 1 (rccl.h); recvbuff may be NULL off the root.  ncclSuccess = 0;
    // a non-blocking communicator may answer ncclInProgress = 7 with the operation enqueued
    const int gr = f->gather(send, recv, count, 1, 0, f->comm, f->comm_stream);
    if (gr != 0 && gr != 7) return RG_ERR_DEVICE;
    if (!ok(hipEventRecord(f->sent[b0], f->comm_stream))) return RG_ERR_DEVICE;
    if (f->rank == 0 && !ok(hipStreamWaitEvent(f->side, f->sent[b0], 0))) return RG_ERR_DEVICE;
    for (int h = 0; h < n; ++h) {
        const int b = b0 + h;
        if (f->rank == 0) {
            if (!ok(rg_launch_reinterleave(static_cast<uint8_t *>(recv) + (size_t)h * f->slot_bytes, f->parts[b],
                                           f->image[b], f->w, f->h, f->T, (uint32_t)f->world, count, f->side,
                                           f->root)) ||
                !ok(hipEventRecord(f->done[b], f->side)))
                return RG_ERR_DEVICE;
        } else if (!ok(hipEventRecord(f->done[b], f->comm_stream))) {
            return RG_ERR_DEVICE;
        }
    }
    f->last = b0 + n - 1;
    f->pend_n = 0;
    return RG_OK;
}

}  // namespace

extern "C" {

// raingun_debug.h: a gather that does nothing (host-overhead probes of the frame loop)
int rg_debug_gather_noop(const void *, void *, size_t, int, int, void *, void *) { return 0; }

rg_status rg_frames_set_root_tiles(rg_frames *f, int32_t root_tiles) {
    if (!f || root_tiles < 1 || root_tiles > 64 || f->k != 0) return RG_ERR_INVALID_ARGUMENT;
    if (f->world == 1) return root_tiles == 1 ? RG_OK : RG_ERR_INVALID_ARGUMENT;
    const uint32_t R = (uint32_t)root_tiles, P = R + (uint32_t)f->world - 1u;
    // rank 0: R consecutive tiles per period; rank r > 0: tile R + r - 1 of each period
    f->root = R;
    f->tiling = f->rank == 0 ? rg_tiling{f->T, P, 0u} : rg_tiling{f->T, P, R + (uint32_t)f->rank - 1u};
    const rg_tiling t1{f->T, P, R};  // rank 1 holds the most tiles of the other ranks
    const rg_tiling t0{f->T, P, 0u};
    const uint32_t slot_rows = rg_tiling_rows_grouped(f->h, &t1, 1);
    const size_t root_rows = rg_tiling_rows_grouped(f->h, &t0, R);
    const size_t part_rows = f->rank == 0 ? std::max<size_t>(root_rows, slot_rows) : slot_rows;
    if (part_rows * f->w * 4 > f->part_bytes) {  // rank 0's part grew: new part buffers
        for (void *&p : f->parts) {
            (void)hipFree(p);
            p = nullptr;
        }
        const size_t bytes = std::max(part_rows * f->w * 4, rg_packed_slot_bytes(slot_rows, f->w) * 2);
        for (void *&p : f->parts)
            if (!ok(hipMalloc(&p, bytes)) || !ok(hipMemset(p, 0, bytes))) return RG_ERR_OUT_OF_MEMORY;
        f->part_bytes = part_rows * f->w * 4;
    }
    f->slot_rows = slot_rows;  // smaller than before: the send / receive buffers stay large enough
    f->slot_bytes = rg_packed_slot_bytes(slot_rows, f->w);
    f->root_part_rows = root_rows;
    return RG_OK;
}

rg_status rg_frames_set_batch(rg_frames *f, int32_t batch) {
    if (!f || batch < 1 || batch > 2 || f->depth % batch != 0 || f->k != 0) return RG_ERR_INVALID_ARGUMENT;
    f->batch = batch;
    return RG_OK;
}

rg_status rg_frames_step(rg_frames *f) {
    if (!f || !f->scene) return RG_ERR_INVALID_ARGUMENT;
    const int b = (int)(f->k % (unsigned long long)f->depth);
    hipStream_t rs = f->render[b];
    if (f->k >= (unsigned long long)f->depth && !ok(hipStreamWaitEvent(rs, f->done[b], 0))) return RG_ERR_DEVICE;
    // (one of several frames in flight: the heavy path sizes its grid for throughput)
    rg_status st = rg_launch_tiles(f->scene, f->w, f->h, &f->tiling, static_cast<uint8_t *>(f->parts[b]), nullptr, rs,
                                   nullptr, nullptr, false, nullptr, 0, nullptr, 3, false, true, 0, 0xFFFFFFFFu, false,
                                   f->rank == 0 ? f->root : 1u);
    if (st != RG_OK) return st;
    // off the root the part travels packed (3 B per pixel) in its batch's send buffer;
    // the root's own part is read in place
    const int B = 2, p = b / B, h = b % B;
    if (f->rank != 0 && !ok(rg_launch_pack_rgb(f->parts[b], static_cast<uint8_t *>(f->packed[p]) + (size_t)h * f->slot_bytes,
                                               (size_t)f->slot_rows * f->w, rs)))
        return RG_ERR_DEVICE;
    if (!ok(hipEventRecord(f->rendered[b], rs)) || !ok(hipStreamWaitEvent(f->comm_stream, f->rendered[b], 0)))
        return RG_ERR_DEVICE;
    if (f->pend_n == 0) f->pend_b0 = b;
    f->pend_n++;
    f->k++;
    // a batch is gathered when its last slot is rendered (every rank issues the same gathers)
    if ((b + 1) % f->batch == 0) return issue_gather(f, f->pend_b0, f->pend_n);
    return RG_OK;
}

namespace {

// Wait for this rank's enqueued work and collect its device errors -- local only:
// never issues a collective (a gather that only one rank starts would hang).
rg_status frames_sync_local(rg_frames *f) {
    for (hipStream_t s : f->render) {
        if (!ok(hipStreamSynchronize(s))) return RG_ERR_DEVICE;
        // device errors of this rank's renders (the reference panics: rendering.rs, bodies.rs:324, scene.rs:38)
        int32_t px = -1;
        const rg_status e = rg_stream_status(f->scene, s, &px);
        if (e == RG_ERR_DEVICE) return e;
        if (e != RG_OK && (f->err == RG_OK || px < f->err_pixel)) {
            f->err = e;
            f->err_pixel = px;
        }
    }
    if (!ok(hipStreamSynchronize(f->comm_stream)) || !ok(hipStreamSynchronize(f->side))) return RG_ERR_DEVICE;
    return f->err;
}

}  // namespace

rg_status rg_frames_flush(rg_frames *f) {
    if (!f || !f->scene) return RG_ERR_INVALID_ARGUMENT;
    if (f->pend_n > 0) {  // a batch cut short: gather what was rendered (every rank flushes at the same frame)
        const rg_status st = issue_gather(f, f->pend_b0, f->pend_n);
        if (st != RG_OK) return st;
    }
    return frames_sync_local(f);
}

rg_status rg_frames_status(rg_frames *f, int32_t *error_pixel) {
    if (!f || !f->scene) return RG_ERR_INVALID_ARGUMENT;
    const rg_status st = frames_sync_local(f);  // local: a pending batch stays pending (no collective here)
    if (error_pixel) *error_pixel = f->err_pixel;
    return st;
}

const uint8_t *rg_frames_image(const rg_frames *f) {
    if (!f || f->rank != 0 || f->last < 0) return nullptr;
    return static_cast<const uint8_t *>(f->image[f->last]);
}

rg_status rg_frames_read_image(const rg_frames *f, uint8_t *host_out) {
    if (!f || !f->scene || !host_out || f->rank != 0) return RG_ERR_INVALID_ARGUMENT;
    // a batch still waiting for its gather needs rg_frames_flush on EVERY rank first: the
    // catch-up gather is a collective, which rank 0 must not start alone
    if (f->pend_n > 0) return RG_ERR_PENDING;
    if (f->last < 0) return RG_ERR_INVALID_ARGUMENT;  // no frame rendered yet
    const rg_status st = frames_sync_local(const_cast<rg_frames *>(f));
    if (st == RG_ERR_DEVICE) return st;
    if (!ok(hipMemcpy(host_out, f->image[f->last], (size_t)f->h * f->w * 4, hipMemcpyDeviceToHost)))
        return RG_ERR_DEVICE;
    return st;  // the frame is delivered; a device error any frame raised is reported
}

}  // extern "C"
