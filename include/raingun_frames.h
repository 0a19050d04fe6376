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
 * The communicator and the gather are passed as opaque pointers: normally
 * the library's own (rg_comm_init_rank / rg_comm_gather_fn below: RCCL loaded
 * at run time, so the library links no collective library), or any other
 * ncclComm_t with its ncclGather.
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

/* Rank 0's share: the frame's tile_rows-row tiles are dealt in periods of
 * root_tiles + world - 1 -- the first root_tiles of each period to rank 0, then
 * one to each other rank (1, the default: the round robin tile t -> rank t %
 * world).  Rank 0's rows never cross the interconnect, so a larger share
 * shrinks every other rank's part of each gather (and the root's receive
 * volume) at the cost of more rendering on rank 0.  Every rank must set the
 * same value, before the first rg_frames_step.  The assembled frame is the
 * same for every value. */
rg_status rg_frames_set_root_tiles(rg_frames *frames, int32_t root_tiles);

/* Enqueue one frame (asynchronous: returns once its work is on the streams). */
rg_status rg_frames_step(rg_frames *frames);

/* Block until every enqueued frame is rendered, gathered and assembled.
 * Returns the first device error (RG_ERR_AABB_NORMAL, _NAN_DISTANCE,
 * _TRANSMISSION: the reference's panics) any of this rank's frames raised
 * so far, RG_OK if none; the frames are still delivered. */
rg_status rg_frames_flush(rg_frames *frames);

/* Local status: waits for this rank's enqueued work and returns what
 * rg_frames_flush would, plus the pixel of that first error (-1 if none).
 * Never issues a collective: a batch still waiting for its gather stays
 * pending (only rg_frames_flush, called on every rank, gathers it). */
rg_status rg_frames_status(rg_frames *frames, int32_t *error_pixel);

/* Rank 0: device pointer of the latest frame's assembled image (height rows of
 * width RGBA8 pixels, row-major), valid after rg_frames_flush; NULL elsewhere. */
const uint8_t *rg_frames_image(const rg_frames *frames);

/* Rank 0: copy the latest assembled image to host memory (height*width*4
 * bytes).  Local: it issues no collective, so when a batch of frames is still
 * waiting for its gather (batch 2, an odd number of steps since the last
 * gather) it returns RG_ERR_PENDING -- call rg_frames_flush on EVERY rank
 * first (a null argument or a rank other than 0 is RG_ERR_INVALID_ARGUMENT).  Otherwise it blocks until this rank's enqueued work is done and
 * returns what rg_frames_flush returns (the image is copied either way). */
rg_status rg_frames_read_image(const rg_frames *frames, uint8_t *host_out);

/* ------------------------------------------------------------------------
 * The library's own RCCL communicator for N processes (one per GPU), so a
 * caller needs no collective library or torch internals of its own.  RCCL is
 * loaded at run time (the librccl already in the process, else
 * $RG_RCCL_LIBRARY, else librccl.so.1; RG_ERR_COLLECTIVE if none).
 *   rank 0:     rg_comm_unique_id(id)              ncclGetUniqueId
 *   caller:     hand the RG_COMM_ID_BYTES bytes of `id` to every rank
 *   every rank: rg_comm_init_rank(id, world, rank, device, &comm)   ncclCommInitRank
 *               (collective: all ranks call it; binds `device`)
 *   rg_frames_create(..., comm, rg_comm_gather_fn(), ...)
 *   rg_comm_destroy(comm) after rg_frames_destroy.
 * ---------------------------------------------------------------------- */
#define RG_COMM_ID_BYTES 128
int32_t rg_comm_id_bytes(void);
rg_status rg_comm_unique_id(uint8_t *id);
rg_status rg_comm_init_rank(const uint8_t *id, int32_t world, int32_t rank, int32_t device, void **comm);
/* ncclCommCount / ncclCommUserRank / ncclCommCuDevice of `comm` (each out pointer nullable). */
rg_status rg_comm_info(void *comm, int32_t *nranks, int32_t *rank, int32_t *device);
rg_status rg_comm_destroy(void *comm);
/* ncclGather of the RCCL the communicators come from (NULL if RCCL cannot be loaded). */
rg_gather_fn rg_comm_gather_fn(void);

#ifdef __cplusplus
}
#endif

#endif /* RAINGUN_FRAMES_H */
