/*
 * raingun_frames.h — frames in flight over N ranks (one process per GPU):
 * the native per-frame pipeline of the row-tile split.
 *
 * Frame k: this rank renders its row tiles (rg_render_tiles_async with tiling
 * {tile_rows, world, rank}) into part buffer k % depth on render stream
 * k % depth; ONE RCCL gather of the equal-size parts to rank 0 follows on a
 * communication stream (gathers stay in frame order on every rank), and rank 0
 * re-interleaves the gathered parts into image order on a side stream.  A part
 * buffer is reused only after its previous frame was sent (and, on rank 0,
 * assembled).  The reference has no multi-GPU path: this replaces the
 * one-process Rayon loop of rendering::render_image (rendering.rs:24-38) for a
 * sequence of frames over a node.
 *
 * The RCCL communicator and ncclGather are the caller's (e.g. PyTorch's
 * ProcessGroupNCCL communicator and the librccl it loaded), passed as opaque
 * pointers, so the library links no collective library of its own.
 */
#ifndef RAINGUN_FRAMES_H
#define RAINGUN_FRAMES_H

#include "raingun.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ncclGather (rccl.h): (sendbuff, recvbuff, sendcount, datatype, root, comm, stream) -> ncclResult_t */
typedef int (*rg_gather_fn)(const void *send, void *recv, size_t count, int datatype, int root, void *comm,
                            void *stream);

typedef struct rg_frames rg_frames;

/* Set up `depth` frames in flight of a width x height frame split into
 * tile_rows-row tiles over `world` ranks (this is rank `rank`).  `comm` is an
 * ncclComm_t over the same ranks, `gather` the matching ncclGather.
 * Lifetime: destroy the frames before their scene.  If the scene is destroyed
 * first, it waits for the frames' renders and detaches them: every later call
 * but rg_frames_destroy (which then frees only the frames' own resources)
 * returns RG_ERR_INVALID_ARGUMENT. */
rg_status rg_frames_create(const rg_scene *scene, uint32_t width, uint32_t height, uint32_t tile_rows, int32_t rank,
                           int32_t world, int32_t depth, void *comm, rg_gather_fn gather, rg_frames **out);
void rg_frames_destroy(rg_frames *frames);

/* Frames per gather: 2 (default when world > 1 and depth is even) gathers two
 * consecutive frames' parts in ONE ncclGather, halving rank 0's per-frame
 * enqueue cost; 1 gathers every frame on its own.  Call before the first
 * rg_frames_step; batch must divide depth.  Frames and their order are the
 * same either way (a batch cut short by rg_frames_flush is gathered then). */
rg_status rg_frames_set_batch(rg_frames *frames, int32_t batch);

/* Enqueue one frame (asynchronous: returns once its work is on the streams). */
rg_status rg_frames_step(rg_frames *frames);

/* Block until every enqueued frame is rendered, gathered and assembled.
 * Returns the first device error (RG_ERR_AABB_NORMAL, _NAN_DISTANCE,
 * _TRANSMISSION: the reference's panics) any of this rank's frames raised
 * so far, RG_OK if none; the frames are still delivered. */
rg_status rg_frames_flush(rg_frames *frames);

/* rg_frames_flush, plus the pixel of that first error (-1 if none). */
rg_status rg_frames_status(rg_frames *frames, int32_t *error_pixel);

/* Rank 0: device pointer of the latest frame's assembled image (height rows of
 * width RGBA8 pixels, row-major), valid after rg_frames_flush; NULL elsewhere. */
const uint8_t *rg_frames_image(const rg_frames *frames);

/* Rank 0: copy the latest assembled image to host memory (height*width*4
 * bytes); blocks until every enqueued frame is done.  Returns what
 * rg_frames_flush returns (the image is copied either way). */
rg_status rg_frames_read_image(const rg_frames *frames, uint8_t *host_out);

#ifdef __cplusplus
}
#endif

#endif /* RAINGUN_FRAMES_H */
