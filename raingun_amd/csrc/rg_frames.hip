// rg_frames.hip — frames in flight over N ranks (include/raingun_frames.h).
//
// Per frame k, slot b = k % depth:
//   render stream b : wait done[b] -> render this rank's tiles into part[b] -> record rendered[b]
//   comm stream     : wait rendered[b] -> ncclGather(part[b] -> gathered[b] on rank 0) -> record sent[b]
//   side stream     : (rank 0) wait sent[b] -> re-interleave gathered[b] into image[b] -> record done[b]
// (non-root ranks: done[b] = sent[b]).  All gathers go through ONE stream, so
// every rank issues and runs them in frame order; renders of consecutive frames
// overlap on their own streams.  Host work per frame is a handful of runtime
// calls (the Python pipeline spent ~70 us per frame on rank 0).
#include <hip/hip_runtime.h>

#include <new>
#include <vector>

#include "../../include/raingun.h"
#include "../../include/raingun_frames.h"

namespace {

bool ok(hipError_t e) { return e == hipSuccess; }

// Image row y lives in tile t = y / T, dealt to rank t % world as that rank's
// (t / world)-th tile: row (t / world) * T + y % T of its part (distributed.py assemble).
__global__ __launch_bounds__(256) void rg_reinterleave_kernel(const uint32_t *gathered, uint32_t *image, uint32_t width,
                                                              uint32_t height, uint32_t tile_rows, uint32_t world,
                                                              uint32_t slot_rows) {
    const uint32_t y = blockIdx.y;
    const uint32_t x = blockIdx.x * 256u + threadIdx.x;
    if (y >= height || x >= width) return;
    const uint32_t t = y / tile_rows;
    const uint32_t r = t % world;
    const uint32_t src_row = (t / world) * tile_rows + (y - t * tile_rows);
    image[(size_t)y * width + x] = gathered[((size_t)r * slot_rows + src_row) * width + x];
}

}  // namespace

hipError_t rg_launch_reinterleave(const void *gathered, void *image, uint32_t width, uint32_t height, uint32_t tile_rows,
                                  uint32_t world, uint32_t slot_rows, hipStream_t stream) {
    dim3 grid((width + 255u) / 256u, height);
    hipLaunchKernelGGL(rg_reinterleave_kernel, grid, dim3(256), 0, stream, static_cast<const uint32_t *>(gathered),
                       static_cast<uint32_t *>(image), width, height, tile_rows, world, slot_rows);
    return hipGetLastError();
}

struct rg_frames {
    const rg_scene *scene = nullptr;
    int device = 0;
    uint32_t w = 0, h = 0, T = 0, slot_rows = 0;
    int rank = 0, world = 1, depth = 1;
    size_t part_bytes = 0;
    rg_tiling tiling{};
    void *comm = nullptr;
    rg_gather_fn gather = nullptr;
    std::vector<hipStream_t> render;
    hipStream_t comm_stream = nullptr, side = nullptr;
    std::vector<void *> parts, gathered, image;
    std::vector<hipEvent_t> rendered, sent, done;
    unsigned long long k = 0;
    int last = -1;
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
    for (void *p : f->gathered) (void)hipFree(p);
    for (void *p : f->image) (void)hipFree(p);
    for (hipEvent_t e : f->rendered) (void)hipEventDestroy(e);
    for (hipEvent_t e : f->sent) (void)hipEventDestroy(e);
    for (hipEvent_t e : f->done) (void)hipEventDestroy(e);
    for (hipStream_t s : f->render) {
        (void)rg_scene_release_stream(const_cast<rg_scene *>(f->scene), s);  // its launch state goes with it
        (void)hipStreamDestroy(s);
    }
    if (f->comm_stream) (void)hipStreamDestroy(f->comm_stream);
    if (f->side) (void)hipStreamDestroy(f->side);
    delete f;
}

}  // namespace

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
    f->part_bytes = (size_t)f->slot_rows * width * 4;
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
    f->render.assign(depth, nullptr);
    for (int b = 0; b < depth && good; ++b) {
        stream(f->render[b]);
        alloc(f->parts, f->part_bytes);
        event(f->rendered);
        event(f->sent);
        event(f->done);
        if (rank == 0) {
            alloc(f->gathered, f->part_bytes * (size_t)world);
            alloc(f->image, (size_t)height * width * 4);
        }
    }
    stream(f->comm_stream);
    stream(f->side);
    if (!good) {
        frames_release(f);
        return RG_ERR_OUT_OF_MEMORY;
    }
    *out = f;
    return RG_OK;
}

void rg_frames_destroy(rg_frames *f) { frames_release(f); }

rg_status rg_frames_step(rg_frames *f) {
    if (!f) return RG_ERR_INVALID_ARGUMENT;
    const int b = (int)(f->k % (unsigned long long)f->depth);
    hipStream_t rs = f->render[b];
    if (f->k >= (unsigned long long)f->depth && !ok(hipStreamWaitEvent(rs, f->done[b], 0))) return RG_ERR_DEVICE;
    rg_status st = rg_render_tiles_async(f->scene, f->w, f->h, &f->tiling, static_cast<uint8_t *>(f->parts[b]),
                                         nullptr, rs, nullptr);
    if (st != RG_OK) return st;
    if (!ok(hipEventRecord(f->rendered[b], rs)) || !ok(hipStreamWaitEvent(f->comm_stream, f->rendered[b], 0)))
        return RG_ERR_DEVICE;
    // ncclUint8 = 1 (rccl.h); recvbuff may be NULL off the root.  ncclSuccess = 0;
    // a non-blocking communicator may answer ncclInProgress = 7 with the operation enqueued
    const int gr = f->gather(f->parts[b], f->rank == 0 ? f->gathered[b] : nullptr, f->part_bytes, 1, 0, f->comm,
                             f->comm_stream);
    if (gr != 0 && gr != 7) return RG_ERR_DEVICE;
    if (!ok(hipEventRecord(f->sent[b], f->comm_stream))) return RG_ERR_DEVICE;
    if (f->rank == 0) {
        if (!ok(hipStreamWaitEvent(f->side, f->sent[b], 0))) return RG_ERR_DEVICE;
        if (!ok(rg_launch_reinterleave(f->gathered[b], f->image[b], f->w, f->h, f->T, (uint32_t)f->world, f->slot_rows,
                                       f->side)) ||
            !ok(hipEventRecord(f->done[b], f->side)))
            return RG_ERR_DEVICE;
    } else if (!ok(hipEventRecord(f->done[b], f->comm_stream))) {
        return RG_ERR_DEVICE;
    }
    f->last = b;
    f->k++;
    return RG_OK;
}

rg_status rg_frames_flush(rg_frames *f) {
    if (!f) return RG_ERR_INVALID_ARGUMENT;
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

rg_status rg_frames_status(rg_frames *f, int32_t *error_pixel) {
    if (!f) return RG_ERR_INVALID_ARGUMENT;
    const rg_status st = rg_frames_flush(f);
    if (error_pixel) *error_pixel = f->err_pixel;
    return st;
}

const uint8_t *rg_frames_image(const rg_frames *f) {
    if (!f || f->rank != 0 || f->last < 0) return nullptr;
    return static_cast<const uint8_t *>(f->image[f->last]);
}

rg_status rg_frames_read_image(const rg_frames *f, uint8_t *host_out) {
    if (!f || !host_out || f->rank != 0 || f->last < 0) return RG_ERR_INVALID_ARGUMENT;
    const rg_status st = rg_frames_flush(const_cast<rg_frames *>(f));
    if (st == RG_ERR_DEVICE) return st;
    if (!ok(hipMemcpy(host_out, f->image[f->last], (size_t)f->h * f->w * 4, hipMemcpyDeviceToHost)))
        return RG_ERR_DEVICE;
    return st;  // the frame is delivered; a device error any frame raised is reported
}

}  // extern "C"
