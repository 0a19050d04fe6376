// rg_multi.hip — rg_render_multi: one process drives N devices (SURVEY.md
// §8(b), §5: "rg_render_multi ... ncclCommInitAll").
//
// The frame is cut into tile_rows-row tiles dealt round-robin (tile t ->
// device t % N, the balance argument of DESIGN.md §6); each device renders its
// tiles with its own replica of the scene.  The frame must end in HOST memory
// (rendering.rs:24-38 returns an ImageBuffer), and each device has its own
// PCIe link, so by default the devices deliver their own rows (DIRECT):
//   device i, render streams : its tiles in K bands (two streams, alternating)
//   device i, copy stream    : after band b, ONE strided copy (hipMemcpy2DAsync)
//                              of the band's tiles straight to their image rows
//                              in page-locked host memory (the caller's buffer,
//                              or a pinned frame fed to a pageable buffer band by
//                              band by host threads)
// -- N links carry 1/N of the frame each, overlapped with the later bands'
// renders.  The RCCL path (GATHER, rg_debug_set_multi mode 1) keeps the
// collective design of SURVEY.md §8(e):
//   all devices        : ONE ncclGather of the equal-size parts to device 0, packed to
//                        RGB (3 B per pixel: alpha is always 255) off device 0
//                        (ncclGroupStart/End: one thread issues N ranks' calls)
//   device 0, stream 0 : re-interleave gathered parts into the frame, then
//                        copy the frame to the caller's host buffer
// RCCL is loaded with dlopen, so libraingun_hip.so links no collective
// library and shares the one already in a process (PyTorch's) if there is one.
//
// Stand-in (rg_debug_set_multi stand_in = 1, for tests on one GPU): every
// "device" is the scene's device, each with its own replica, and the gather
// goes through a stand-in with ncclGather's signature and group semantics
// (device copies into the root's receive buffer, ordered after each rank's
// render) -- so every N > 1 code path runs on a single GPU.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <link.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "../../include/raingun.h"
#include "../../include/raingun_debug.h"
#include "../../include/raingun_frames.h"
#include "rg_internal.h"

// rg_frames.hip: parts travel as packed RGB (3 B per pixel); device 0 reads its own part in place
hipError_t rg_launch_reinterleave(const void *gathered, const void *root_part, void *image, uint32_t width,
                                  uint32_t height, uint32_t tile_rows, uint32_t world, size_t slot_bytes,
                                  hipStream_t stream, uint32_t root = 1);
hipError_t rg_launch_pack_rgb(const void *rgba, void *rgb, size_t npx, hipStream_t stream);
size_t rg_packed_slot_bytes(uint32_t slot_rows, uint32_t width);

namespace {

bool ok(hipError_t e) { return e == hipSuccess; }

// ---------------------------------------------------------------- RCCL, loaded at run time
typedef int (*pfn_comm_init_all)(void **comms, int ndev, const int *devlist);
typedef int (*pfn_comm_destroy)(void *comm);
typedef int (*pfn_gather)(const void *send, void *recv, size_t count, int dtype, int root, void *comm, hipStream_t s);
typedef int (*pfn_group)(void);
struct NcclUniqueId {  // ncclUniqueId (rccl.h): 128 opaque bytes, passed by value to ncclCommInitRank
    char internal[RG_COMM_ID_BYTES];
};
typedef int (*pfn_get_unique_id)(NcclUniqueId *id);
typedef int (*pfn_comm_init_rank)(void **comm, int nranks, NcclUniqueId id, int rank);
typedef int (*pfn_comm_query)(void *comm, int *out);  // ncclCommCount / ncclCommCuDevice / ncclCommUserRank

struct Rccl {
    bool tried = false;
    void *handle = nullptr;
    pfn_comm_init_all init_all = nullptr;
    pfn_comm_destroy destroy = nullptr;
    pfn_gather gather = nullptr;
    pfn_group group_start = nullptr, group_end = nullptr;
    pfn_get_unique_id get_unique_id = nullptr;
    pfn_comm_init_rank init_rank = nullptr;
    pfn_comm_query count = nullptr, cu_device = nullptr, user_rank = nullptr;
};
Rccl g_rccl;
std::mutex g_rccl_mu;

int find_loaded(struct dl_phdr_info *info, size_t, void *data) {
    if (info->dlpi_name && std::strstr(info->dlpi_name, "librccl")) {
        *static_cast<std::string *>(data) = info->dlpi_name;
        return 1;
    }
    return 0;
}

const Rccl *rccl() {
    std::lock_guard<std::mutex> g(g_rccl_mu);
    if (g_rccl.tried) return g_rccl.handle ? &g_rccl : nullptr;
    g_rccl.tried = true;
    std::string loaded;
    dl_iterate_phdr(find_loaded, &loaded);
    std::vector<std::string> cands;
    if (!loaded.empty()) cands.push_back(loaded);  // the instance already in the process (e.g. PyTorch's)
    if (const char *e = std::getenv("RG_RCCL_LIBRARY")) cands.push_back(e);
    cands.push_back("librccl.so.1");
    cands.push_back("/opt/rocm/lib/librccl.so.1");
    for (const std::string &c : cands) {
        void *h = dlopen(c.c_str(), RTLD_NOW | RTLD_LOCAL);
        if (!h) continue;
        g_rccl.init_all = reinterpret_cast<pfn_comm_init_all>(dlsym(h, "ncclCommInitAll"));
        g_rccl.destroy = reinterpret_cast<pfn_comm_destroy>(dlsym(h, "ncclCommDestroy"));
        g_rccl.gather = reinterpret_cast<pfn_gather>(dlsym(h, "ncclGather"));
        g_rccl.group_start = reinterpret_cast<pfn_group>(dlsym(h, "ncclGroupStart"));
        g_rccl.group_end = reinterpret_cast<pfn_group>(dlsym(h, "ncclGroupEnd"));
        g_rccl.get_unique_id = reinterpret_cast<pfn_get_unique_id>(dlsym(h, "ncclGetUniqueId"));
        g_rccl.init_rank = reinterpret_cast<pfn_comm_init_rank>(dlsym(h, "ncclCommInitRank"));
        g_rccl.count = reinterpret_cast<pfn_comm_query>(dlsym(h, "ncclCommCount"));
        g_rccl.cu_device = reinterpret_cast<pfn_comm_query>(dlsym(h, "ncclCommCuDevice"));
        g_rccl.user_rank = reinterpret_cast<pfn_comm_query>(dlsym(h, "ncclCommUserRank"));
        if (g_rccl.init_all && g_rccl.destroy && g_rccl.gather && g_rccl.group_start && g_rccl.group_end &&
            g_rccl.get_unique_id && g_rccl.init_rank && g_rccl.count && g_rccl.cu_device && g_rccl.user_rank) {
            g_rccl.handle = h;
            return &g_rccl;
        }
        dlclose(h);
    }
    return nullptr;
}

constexpr int kNcclUint8 = 1;       // ncclDataType_t (rccl.h)
constexpr int kNcclInProgress = 7;  // a non-blocking communicator's "enqueued"

// ---------------------------------------------------------------- stand-in gather
// ncclGather's signature and the semantics rg_render_multi relies on: within
// one group the root (rank 0) is called first with the receive buffer; rank
// r's `count` bytes land at recv + r * count once rank r's earlier work on its
// stream is done, and the root's stream is ordered after every copy.
struct StandInGroup {
    void *root_recv = nullptr;
    hipStream_t root_stream = nullptr;
    std::vector<hipEvent_t> ev;  // one per rank
};
struct StandInComm {
    int rank = 0;
    StandInGroup *g = nullptr;
};

int stand_in_gather(const void *send, void *recv, size_t count, int dtype, int root, void *comm, hipStream_t stream) {
    StandInComm *c = static_cast<StandInComm *>(comm);
    if (!c || dtype != kNcclUint8 || root != 0) return 1;
    StandInGroup *g = c->g;
    if (c->rank == 0) {
        if (!recv) return 1;
        g->root_recv = recv;
        g->root_stream = stream;
        return ok(hipMemcpyAsync(recv, send, count, hipMemcpyDeviceToDevice, stream)) ? 0 : 1;
    }
    if (!g->root_recv || c->rank >= (int)g->ev.size()) return 1;
    hipEvent_t e = g->ev[c->rank];
    if (!ok(hipEventRecord(e, stream)) || !ok(hipStreamWaitEvent(g->root_stream, e, 0))) return 1;
    return ok(hipMemcpyAsync(static_cast<char *>(g->root_recv) + (size_t)c->rank * count, send, count,
                             hipMemcpyDeviceToDevice, g->root_stream))
               ? 0
               : 1;
}

#ifndef RG_MULTI_BAND_PX
#define RG_MULTI_BAND_PX (1u << 20)  // a device's share is cut into bands of about this many pixels (at most 4)
#endif

}  // namespace

// Per-scene multi-GPU state for one (ngpus, width, height, tile_rows, mode).
struct rg_multi_res {
    int n = 0;
    uint32_t w = 0, h = 0, T = 0, slot_rows = 0;
    int mode = 0;            // 0: direct per-device copies to the host, 1: RCCL gather
    bool stand_in = false;
    size_t part_bytes = 0;   // RGBA part
    size_t slot_bytes = 0;   // packed RGB part each device sends (gather)
    std::vector<int> devs;
    std::vector<rg_scene *> reps;      // reps[0] = the scene itself (not owned)
    std::vector<void *> comms;
    std::vector<StandInComm> sic;      // stand-in communicators
    StandInGroup sig;
    std::vector<hipStream_t> streams;  // render stream A per device (gather: the only one)
    std::vector<hipStream_t> streams2; // direct: render stream B per device (bands alternate)
    std::vector<hipStream_t> copies;   // direct: device-to-host copy stream per device
    std::vector<std::vector<hipEvent_t>> ev_band, ev_copy;  // direct: per device, per band
    std::vector<void *> parts, packed;            // packed[0] unused: device 0's part is read in place
    void *gathered = nullptr, *image = nullptr;  // device 0 (gather)
    void *h_frame = nullptr;                     // direct into pageable memory: pinned, portable frame
    unsigned long long *snap = nullptr;          // pinned: 4 words per (device, band)
    hipEvent_t ev0 = nullptr, ev1 = nullptr;     // device 0: render start .. its last band / frame assembled
};

namespace {

void free_res(rg_multi_res *m) {
    if (!m) return;
    const Rccl *r = g_rccl.handle ? &g_rccl : nullptr;
    for (int i = 0; i < (int)m->devs.size(); ++i) {
        (void)hipSetDevice(m->devs[i]);
        for (auto *v : {&m->streams, &m->streams2, &m->copies})
            if (i < (int)v->size() && (*v)[i]) (void)hipStreamSynchronize((*v)[i]);
    }
    for (int i = 0; i < (int)m->devs.size(); ++i) {
        (void)hipSetDevice(m->devs[i]);
        if (!m->stand_in && i < (int)m->comms.size() && m->comms[i] && r) (void)r->destroy(m->comms[i]);
        if (i < (int)m->parts.size() && m->parts[i]) (void)hipFree(m->parts[i]);
        if (i < (int)m->packed.size() && m->packed[i]) (void)hipFree(m->packed[i]);
        // the render streams' launch state lives in the replicas; the scene's own
        // (reps[0]) outlives these streams, so forget it before they go
        for (auto *v : {&m->streams, &m->streams2}) {
            if (i >= (int)v->size() || !(*v)[i]) continue;
            if (i < (int)m->reps.size() && m->reps[i]) (void)rg_scene_release_stream(m->reps[i], (*v)[i]);
            (void)hipStreamDestroy((*v)[i]);
        }
        if (i < (int)m->copies.size() && m->copies[i]) (void)hipStreamDestroy(m->copies[i]);
        for (auto *v : {&m->ev_band, &m->ev_copy})
            if (i < (int)v->size())
                for (hipEvent_t e : (*v)[i]) if (e) (void)hipEventDestroy(e);
        if (i > 0 && i < (int)m->reps.size() && m->reps[i]) rg_scene_free(m->reps[i]);
    }
    if (!m->devs.empty()) {
        (void)hipSetDevice(m->devs[0]);
        if (m->gathered) (void)hipFree(m->gathered);
        if (m->image) (void)hipFree(m->image);
        if (m->ev0) (void)hipEventDestroy(m->ev0);
        if (m->ev1) (void)hipEventDestroy(m->ev1);
        for (hipEvent_t e : m->sig.ev) if (e) (void)hipEventDestroy(e);
    }
    if (m->snap) (void)hipHostFree(m->snap);
    if (m->h_frame) (void)hipHostFree(m->h_frame);
    delete m;
}

constexpr int kMaxBands = 4;

// Wait for everything a call enqueued on any device (render, copy streams).  An
// error exit from the band loop may leave earlier bands' copies into the
// caller's buffer in flight: they must land before the call returns.
void drain(rg_multi_res *m) {
    for (int i = 0; i < (int)m->devs.size(); ++i) {
        (void)hipSetDevice(m->devs[i]);
        for (auto *v : {&m->streams, &m->streams2, &m->copies})
            if (i < (int)v->size() && (*v)[i]) (void)hipStreamSynchronize((*v)[i]);
    }
    (void)hipGetLastError();
}

// Bands of a device's share (direct mode): K bands of J selected tiles each.
int multi_bands(const rg_scene *s, uint32_t W, uint32_t H, int n) {
    if (s->multi_bands > 0) return std::min(s->multi_bands, kMaxBands);
    const size_t share = ((size_t)W * H + (size_t)n - 1) / (size_t)n;
    return (int)std::max<size_t>(1, std::min<size_t>(kMaxBands, share / RG_MULTI_BAND_PX));
}

rg_status build_res(const rg_scene *s, int n, uint32_t W, uint32_t H, uint32_t T, rg_multi_res **out) {
    *out = nullptr;
    const bool stand_in = s->multi_stand_in;
    const int mode = s->multi_mode;
    const Rccl *r = nullptr;
    if (mode == 1 && !stand_in && !(r = rccl())) return RG_ERR_COLLECTIVE;
    int ndev = 0;
    if (!ok(hipGetDeviceCount(&ndev)) || (!stand_in && n > ndev) || n > 64) return RG_ERR_INVALID_ARGUMENT;
    rg_multi_res *m = new (std::nothrow) rg_multi_res();
    if (!m) return RG_ERR_OUT_OF_MEMORY;
    m->n = n;
    m->w = W;
    m->h = H;
    m->T = T;
    m->mode = mode;
    m->stand_in = stand_in;
    const uint32_t tiles = (H + T - 1) / T;
    m->slot_rows = (tiles + (uint32_t)n - 1) / (uint32_t)n * T;  // equal on every device
    m->part_bytes = (size_t)m->slot_rows * W * 4;
    m->slot_bytes = rg_packed_slot_bytes(m->slot_rows, W);
    for (int i = 0; i < n; ++i) m->devs.push_back(stand_in ? s->device : (s->device + i) % ndev);
    m->reps.assign(n, nullptr);
    m->comms.assign(n, nullptr);
    m->streams.assign(n, nullptr);
    m->parts.assign(n, nullptr);
    m->packed.assign(n, nullptr);
    if (mode == 0) {
        m->streams2.assign(n, nullptr);
        m->copies.assign(n, nullptr);
        m->ev_band.assign(n, std::vector<hipEvent_t>(kMaxBands, nullptr));
        m->ev_copy.assign(n, std::vector<hipEvent_t>(kMaxBands, nullptr));
    }
    m->reps[0] = const_cast<rg_scene *>(s);
    rg_status st = RG_OK;
    for (int i = 1; i < n && st == RG_OK; ++i) st = rg_scene_replica(s, m->devs[i], &m->reps[i]);
    auto mk_stream = [](hipStream_t &x) { return ok(hipStreamCreateWithFlags(&x, hipStreamNonBlocking)); };
    for (int i = 0; i < n && st == RG_OK; ++i) {
        if (!ok(hipSetDevice(m->devs[i])) || !mk_stream(m->streams[i]))
            st = RG_ERR_DEVICE;
        else if (!ok(hipMalloc(&m->parts[i], std::max(m->part_bytes, m->slot_bytes))) ||
                 !ok(hipMemset(m->parts[i], 0, std::max(m->part_bytes, m->slot_bytes))) ||
                 (mode == 1 && i > 0 && !ok(hipMalloc(&m->packed[i], m->slot_bytes))))
            st = RG_ERR_OUT_OF_MEMORY;  // padding rows of the last tiles stay zero
        if (st == RG_OK && mode == 0) {
            if (!mk_stream(m->streams2[i]) || !mk_stream(m->copies[i])) st = RG_ERR_DEVICE;
            for (int b = 0; b < kMaxBands && st == RG_OK; ++b)
                if (!ok(hipEventCreateWithFlags(&m->ev_band[i][b], hipEventDisableTiming)) ||
                    !ok(hipEventCreateWithFlags(&m->ev_copy[i][b], hipEventDisableTiming)))
                    st = RG_ERR_DEVICE;
        }
    }
    if (st == RG_OK) {
        void *snap = nullptr;
        (void)hipSetDevice(m->devs[0]);
        if ((mode == 1 && (!ok(hipMalloc(&m->gathered, m->slot_bytes * (size_t)n)) ||
                           !ok(hipMalloc(&m->image, (size_t)H * W * 4)))) ||
            !ok(hipHostMalloc(&snap, (size_t)n * kMaxBands * 4 * sizeof(unsigned long long), hipHostMallocPortable)))
            st = RG_ERR_OUT_OF_MEMORY;
        m->snap = static_cast<unsigned long long *>(snap);
        if (st == RG_OK && (!ok(hipEventCreate(&m->ev0)) || !ok(hipEventCreate(&m->ev1)))) st = RG_ERR_DEVICE;
    }
    if (st == RG_OK && mode == 1) {
        if (stand_in) {
            m->sic.resize(n);
            m->sig.ev.assign(n, nullptr);
            for (int i = 0; i < n && st == RG_OK; ++i) {
                m->sic[i] = StandInComm{i, &m->sig};
                m->comms[i] = &m->sic[i];
                if (!ok(hipEventCreateWithFlags(&m->sig.ev[i], hipEventDisableTiming))) st = RG_ERR_DEVICE;
            }
        } else if (r->init_all(m->comms.data(), n, m->devs.data()) != 0) {
            for (void *&c : m->comms) c = nullptr;  // not (fully) created
            st = RG_ERR_COLLECTIVE;
        }
    }
    if (st != RG_OK) {
        free_res(m);
        return st;
    }
    *out = m;
    return RG_OK;
}

// Stats of all (device, band) launches: rays summed, the lowest erroring pixel.
rg_status merge_snaps(const rg_multi_res *m, int per_dev, rg_stats *stats) {
    rg_stats total;
    std::memset(&total, 0, sizeof total);
    unsigned long long worst = 0;  // complemented keys: the max is the lowest erroring pixel
    for (int k = 0; k < m->n * per_dev; ++k) {
        total.rays.primary += m->snap[4 * k];
        total.rays.shadow += m->snap[4 * k + 1];
        total.rays.secondary += m->snap[4 * k + 2];
        worst = std::max(worst, m->snap[4 * k + 3]);
    }
    unsigned long long w4[4] = {0, 0, 0, worst};
    rg_stats es;
    const rg_status err = rg_snap_status(w4, &es);
    total.error_pixel = es.error_pixel;
    float ms = 0.0f;
    (void)hipSetDevice(m->devs[0]);
    (void)hipEventElapsedTime(&ms, m->ev0, m->ev1);
    total.kernel_ms = ms;
    if (stats) *stats = total;
    return err;
}

// RCCL path: render, ONE grouped gather to device 0, re-interleave, one copy to the host.
rg_status render_gather(const rg_scene *s, rg_multi_res *m, uint8_t *rgba_out, rg_stats *stats) {
    const uint32_t W = m->w, H = m->h, T = m->T;
    const int n = m->n;
    if (!ok(hipSetDevice(m->devs[0])) || !ok(hipEventRecord(m->ev0, m->streams[0]))) return RG_ERR_DEVICE;
    for (int i = 0; i < n; ++i) {
        const rg_tiling t = {T, (uint32_t)n, (uint32_t)i};
        rg_status st = rg_launch_tiles(m->reps[i], W, H, &t, static_cast<uint8_t *>(m->parts[i]), nullptr,
                                       m->streams[i], m->snap + 4 * i, nullptr);
        if (st != RG_OK) return st;
        if (i > 0 && !ok(rg_launch_pack_rgb(m->parts[i], m->packed[i], (size_t)m->slot_rows * W, m->streams[i])))
            return RG_ERR_DEVICE;
    }
    // one gather of the equal-size parts to device 0 (all ranks' calls in one group)
    const Rccl *r = m->stand_in ? nullptr : rccl();
    const pfn_gather gather = m->stand_in ? stand_in_gather : r->gather;
    if (r && r->group_start() != 0) return RG_ERR_COLLECTIVE;
    int gerr = 0;
    for (int i = 0; i < n; ++i) {
        (void)hipSetDevice(m->devs[i]);
        const int g = gather(i == 0 ? m->parts[i] : m->packed[i], i == 0 ? m->gathered : nullptr, m->slot_bytes,
                             kNcclUint8, 0, m->comms[i], m->streams[i]);
        if (g != 0 && g != kNcclInProgress && gerr == 0) gerr = g;
    }
    const int ge = r ? r->group_end() : 0;
    if (gerr != 0 || (ge != 0 && ge != kNcclInProgress)) return RG_ERR_COLLECTIVE;
    // device 0: re-interleave, copy to the host
    if (!ok(hipSetDevice(m->devs[0])) ||
        !ok(rg_launch_reinterleave(m->gathered, m->parts[0], m->image, W, H, T, (uint32_t)n, m->slot_bytes,
                                   m->streams[0])) ||
        !ok(hipEventRecord(m->ev1, m->streams[0])) ||
        !ok(hipMemcpyAsync(rgba_out, m->image, (size_t)H * W * 4, hipMemcpyDeviceToHost, m->streams[0])))
        return RG_ERR_DEVICE;
    for (int i = n - 1; i >= 0; --i)
        if (!ok(hipSetDevice(m->devs[i])) || !ok(hipStreamSynchronize(m->streams[i]))) return RG_ERR_DEVICE;
    return merge_snaps(m, 1, stats);
}

// Direct path into a page-locked caller frame, one launch per device: every
// device's kernel stores its finished tiles over its OWN PCIe link straight into
// their image rows (RgKernelArgs::image_rows; the host-frame kernels' LDS tile
// ring / per-tile stores, rg_kernels.hip), so the copy overlaps the render and
// no band waits for a DMA -- a device's time is its render latency or its rows'
// PCIe time, whichever is longer.
rg_status render_direct_one(const rg_scene *s, rg_multi_res *m, uint8_t *dst, rg_stats *stats) {
    const uint32_t W = m->w, H = m->h, T = m->T;
    const int n = m->n;
    const size_t frame_bytes = (size_t)H * W * 4;
    const bool light = !rg_heavy_path(rg_make_args(s));
    const uint32_t wl = (uint32_t)(s->host_tile_forced || !light ? s->host_tile_wlog : RG_HOST_TILE_WLOG_LIGHT);
    if (!ok(hipSetDevice(m->devs[0])) || !ok(hipEventRecord(m->ev0, m->streams[0]))) return RG_ERR_DEVICE;
    for (int i = 0; i < n; ++i) {
        unsigned long long *snap = m->snap + 4 * i;
        if (s->multi_only_rank >= 0 && i != s->multi_only_rank) {  // timeline rehearsal of one device
            std::memset(snap, 0, 4 * sizeof(unsigned long long));
            continue;
        }
        if (!ok(hipSetDevice(m->devs[i]))) return RG_ERR_DEVICE;
        void *d = rg_host_device_ptr(dst, frame_bytes);  // registered portable: mapped on every device
        if (!d) return RG_ERR_DEVICE;
        const rg_tiling t = {T, (uint32_t)n, (uint32_t)i};
        const rg_status st = rg_launch_tiles(m->reps[i], W, H, &t, static_cast<uint8_t *>(d), nullptr, m->streams[i],
                                             snap, nullptr, false, nullptr, 0, nullptr, wl, true, false, 0,
                                             0xFFFFFFFFu, true);
        if (st != RG_OK) return st;
    }
    (void)hipSetDevice(m->devs[0]);
    if (!ok(hipEventRecord(m->ev1, m->streams[0]))) return RG_ERR_DEVICE;
    for (int i = n - 1; i >= 0; --i)
        if (!ok(hipSetDevice(m->devs[i])) || !ok(hipStreamSynchronize(m->streams[i]))) return RG_ERR_DEVICE;
    return merge_snaps(m, 1, stats);
}

// Is the page-locked frame mapped into every device's address space (a buffer the
// library registered is portable; one pinned elsewhere may be mapped on its own device only)?
bool mapped_on_all(const rg_multi_res *m, uint8_t *dst, size_t bytes) {
    for (int i = 0; i < m->n; ++i)
        if (!ok(hipSetDevice(m->devs[i])) || rg_host_device_ptr(dst, bytes) == nullptr) {
            (void)hipGetLastError();
            return false;
        }
    return true;
}

// Direct path: every device renders its tiles in K bands and copies each band
// straight to its image rows in page-locked host memory over its own link.
rg_status render_direct(const rg_scene *s, rg_multi_res *m, uint8_t *rgba_out, rg_stats *stats) {
    const uint32_t W = m->w, H = m->h, T = m->T;
    const int n = m->n;
    const size_t row4 = (size_t)W * 4, frame_bytes = (size_t)H * row4;
    // destination: the caller's buffer if page-locked, else the pinned frame
    uint8_t *dst = rg_host_is_pinned(rgba_out, frame_bytes) ? rgba_out : nullptr;
    const bool pageable = dst == nullptr;
    // automatic (bands 0): into a page-locked frame every device renders its share in ONE launch
    // storing its rows over its own link -- trace-heavy scenes since round 4 (north star, one
    // device's timeline 0.97 -> 0.87 ms), light scenes since round 6, once the light kernel's LDS
    // tile ring flushed small launches every 4 tiles with single-tile queue slots (test1 0.29 ->
    // 0.20 ms, the copy now overlapping the render: profiles/r06/s6; with 16-tile groups it was
    // 0.49-0.52 ms).  Only when every device can store into the frame: otherwise the
    // banded DMA copies, which work for any page-locked buffer.
    if (!pageable && (s->multi_bands < 0 || (s->multi_bands == 0 && (s->multi_light_one || rg_heavy_path(rg_make_args(s))))) &&
        mapped_on_all(m, dst, frame_bytes))
        return render_direct_one(s, m, dst, stats);
    if (pageable) {
        if (!m->h_frame) {
            (void)hipSetDevice(m->devs[0]);
            if (!ok(hipHostMalloc(&m->h_frame, frame_bytes, hipHostMallocPortable))) {
                (void)hipGetLastError();
                m->h_frame = nullptr;
                return RG_ERR_OUT_OF_MEMORY;
            }
        }
        dst = static_cast<uint8_t *>(m->h_frame);
    }
    const uint32_t tiles = (H + T - 1) / T;
    const uint32_t per_dev = (tiles + (uint32_t)n - 1) / (uint32_t)n;  // selected tiles of device 0 (the most)
    const uint32_t J = (per_dev + (uint32_t)multi_bands(s, W, H, n) - 1) / (uint32_t)multi_bands(s, W, H, n);
    const int K = (int)((per_dev + J - 1) / J);  // bands of J tiles per device (device 0's are all non-empty)
    if (!ok(hipSetDevice(m->devs[0])) || !ok(hipEventRecord(m->ev0, m->streams[0]))) return RG_ERR_DEVICE;
    for (int b = 0; b < K; ++b) {
        for (int i = 0; i < n; ++i) {
            const rg_tiling t = {T, (uint32_t)n, (uint32_t)i};
            const uint32_t sel = (tiles > (uint32_t)i) ? (tiles - (uint32_t)i + (uint32_t)n - 1) / (uint32_t)n : 0u;
            uint32_t j0 = std::min(sel, (uint32_t)b * J), j1 = std::min(sel, j0 + J);
            if (s->multi_only_rank >= 0 && i != s->multi_only_rank) j1 = j0;  // timeline rehearsal of one device
            unsigned long long *snap = m->snap + 4 * ((size_t)i * K + b);
            if (!ok(hipSetDevice(m->devs[i]))) return RG_ERR_DEVICE;
            hipStream_t rs = (b & 1) ? m->streams2[i] : m->streams[i];
            if (b == 1 && i == 0 && !ok(hipStreamWaitEvent(rs, m->ev0, 0))) return RG_ERR_DEVICE;
            if (j1 == j0) {  // nothing of this device in this band
                std::memset(snap, 0, 4 * sizeof(unsigned long long));
                if (!ok(hipEventRecord(m->ev_copy[i][b], m->copies[i]))) return RG_ERR_DEVICE;
                continue;
            }
            uint8_t *part = static_cast<uint8_t *>(m->parts[i]) + (size_t)j0 * T * row4;
            rg_status st = rg_launch_tiles(m->reps[i], W, H, &t, part, nullptr, rs, snap, nullptr, false, nullptr,
                                           0, nullptr, 3, false, false, j0, j1 - j0);
            if (st != RG_OK) return st;
            if (!ok(hipEventRecord(m->ev_band[i][b], rs)) || !ok(hipStreamWaitEvent(m->copies[i], m->ev_band[i][b], 0)))
                return RG_ERR_DEVICE;
            // selected tile j of device i is image tile j*n + i: whole tiles in one strided
            // copy, the image's last (partial) tile, if it is this device's, on its own
            const uint32_t last_j = (tiles - 1u - (uint32_t)i) / (uint32_t)n;  // valid: sel > 0
            const bool has_partial = (tiles - 1u) % (uint32_t)n == (uint32_t)i && j1 - 1 == last_j && H % T != 0;
            const uint32_t full = (j1 - j0) - (has_partial ? 1u : 0u);
            uint8_t *d0 = dst + ((size_t)j0 * n + (size_t)i) * T * row4;
            if (full > 0 && !ok(hipMemcpy2DAsync(d0, (size_t)n * T * row4, part, (size_t)T * row4, (size_t)T * row4,
                                                 full, hipMemcpyDeviceToHost, m->copies[i])))
                return RG_ERR_DEVICE;
            if (has_partial) {
                const uint32_t y0 = (tiles - 1u) * T;
                if (!ok(hipMemcpyAsync(dst + (size_t)y0 * row4, part + (size_t)full * T * row4, (size_t)(H - y0) * row4,
                                       hipMemcpyDeviceToHost, m->copies[i])))
                    return RG_ERR_DEVICE;
            }
            if (!ok(hipEventRecord(m->ev_copy[i][b], m->copies[i]))) return RG_ERR_DEVICE;
        }
    }
    // kernel_ms: device 0's renders (its last band on the second stream joined)
    (void)hipSetDevice(m->devs[0]);
    const int last_b = (K - 1) & 1 ? K - 1 : K - 2;  // last band on streams2 (odd index), -1: none
    if (last_b > 0 && !ok(hipStreamWaitEvent(m->streams[0], m->ev_band[0][last_b], 0))) return RG_ERR_DEVICE;
    if (!ok(hipEventRecord(m->ev1, m->streams[0]))) return RG_ERR_DEVICE;
    if (pageable) {
        // band b's image rows [b J n T, (b + 1) J n T) are complete once every device copied its part
        rg_image_res &img = s->img;
        if (!img.pool) img.pool = std::make_shared<rg_copy_pool>(RG_COPY_HELPERS);
        struct Active {
            rg_copy_pool &p;
            explicit Active(rg_copy_pool &q) : p(q) { p.begin(); }
            ~Active() { p.end(); }
        } active(*img.pool);
        for (int b = 0; b < K; ++b) {
            for (int i = 0; i < n; ++i)
                if (!ok(hipSetDevice(m->devs[i])) || !ok(hipEventSynchronize(m->ev_copy[i][b]))) return RG_ERR_DEVICE;
            const size_t y0 = std::min<size_t>(H, (size_t)b * J * n * T), y1 = std::min<size_t>(H, (size_t)(b + 1) * J * n * T);
            if (y1 > y0) img.pool->copy(rgba_out + y0 * row4, dst + y0 * row4, (y1 - y0) * row4);
        }
    }
    for (int i = n - 1; i >= 0; --i) {
        if (!ok(hipSetDevice(m->devs[i]))) return RG_ERR_DEVICE;
        for (hipStream_t x : {m->streams[i], m->streams2[i], m->copies[i]})
            if (!ok(hipStreamSynchronize(x))) return RG_ERR_DEVICE;
    }
    return merge_snaps(m, K, stats);
}

}  // namespace

void rg_multi_release(const rg_scene *s) {
    if (!s || !s->multi) return;
    free_res(s->multi);
    s->multi = nullptr;
    (void)hipSetDevice(s->device);
}

extern "C" rg_status rg_render_multi(const rg_scene *s, uint32_t W, uint32_t H, int32_t ngpus, uint32_t tile_rows,
                                     uint8_t *rgba_out, rg_stats *stats) {
    if (!s || !rgba_out || W == 0 || H == 0 || ngpus < 1) return RG_ERR_INVALID_ARGUMENT;
    if (W < H) return RG_ERR_PORTRAIT;  // ray.rs:42
    if ((unsigned long long)H * W >= (1ull << 32)) return RG_ERR_INVALID_ARGUMENT;
    const uint32_t T = tile_rows ? tile_rows : 8u;
    rg_multi_res *m = s->multi;
    if (!m || m->n != ngpus || m->w != W || m->h != H || m->T != T || m->mode != s->multi_mode ||
        m->stand_in != s->multi_stand_in) {
        rg_multi_release(s);
        rg_status st = build_res(s, ngpus, W, H, T, &m);
        if (st != RG_OK) {
            (void)hipSetDevice(s->device);
            return st;
        }
        s->multi = m;
    }
    for (int i = 1; i < m->n; ++i) rg_sync_settings(m->reps[i], s);
    const rg_status st = m->mode == 1 ? render_gather(s, m, rgba_out, stats) : render_direct(s, m, rgba_out, stats);
    if (st != RG_OK) drain(m);  // no copy into rgba_out may outlive the call
    (void)hipSetDevice(s->device);
    return st;
}

extern "C" rg_status rg_debug_set_multi(rg_scene *s, int32_t mode, int32_t stand_in, int32_t bands,
                                        int32_t only_rank) {
    if (!s || mode < 0 || mode > 1 || bands < -1 || bands > kMaxBands || only_rank < -1) return RG_ERR_INVALID_ARGUMENT;
    if (only_rank >= 0 && (mode != 0 || !stand_in)) return RG_ERR_INVALID_ARGUMENT;
    s->multi_mode = mode;
    s->multi_stand_in = stand_in != 0;
    s->multi_bands = bands;
    s->multi_only_rank = only_rank;
    return RG_OK;
}

// ---------------------------------------------------------------- communicators of N processes
// (include/raingun_frames.h): the library's own RCCL communicator for the
// one-process-per-GPU frame loop -- rank 0 makes the unique id, the caller
// hands it to every rank (any channel: torch.distributed's store, MPI, a file),
// and every rank joins with ncclCommInitRank on its device.  No torch internals.
extern "C" {

int32_t rg_comm_id_bytes(void) { return RG_COMM_ID_BYTES; }

rg_status rg_comm_unique_id(uint8_t *id) {
    if (!id) return RG_ERR_INVALID_ARGUMENT;
    const Rccl *r = rccl();
    if (!r) return RG_ERR_COLLECTIVE;
    NcclUniqueId u;
    if (r->get_unique_id(&u) != 0) return RG_ERR_COLLECTIVE;
    std::memcpy(id, u.internal, sizeof u.internal);
    return RG_OK;
}

rg_status rg_comm_init_rank(const uint8_t *id, int32_t world, int32_t rank, int32_t device, void **comm) {
    if (!comm) return RG_ERR_INVALID_ARGUMENT;
    *comm = nullptr;
    if (!id || world < 1 || rank < 0 || rank >= world || device < 0) return RG_ERR_INVALID_ARGUMENT;
    const Rccl *r = rccl();
    if (!r) return RG_ERR_COLLECTIVE;
    int ndev = 0;
    if (!ok(hipGetDeviceCount(&ndev)) || device >= ndev) return RG_ERR_INVALID_ARGUMENT;
    if (!ok(hipSetDevice(device))) return RG_ERR_DEVICE;  // ncclCommInitRank binds the current device
    NcclUniqueId u;
    std::memcpy(u.internal, id, sizeof u.internal);
    void *c = nullptr;
    if (r->init_rank(&c, world, u, rank) != 0 || !c) return RG_ERR_COLLECTIVE;
    *comm = c;
    return RG_OK;
}

rg_status rg_comm_info(void *comm, int32_t *nranks, int32_t *rank, int32_t *device) {
    const Rccl *r = g_rccl.handle ? &g_rccl : nullptr;
    if (!comm || !r) return RG_ERR_INVALID_ARGUMENT;
    const std::pair<pfn_comm_query, int32_t *> q[3] = {{r->count, nranks}, {r->user_rank, rank}, {r->cu_device, device}};
    for (const auto &e : q) {
        int v = 0;
        if (!e.second) continue;
        if (e.first(comm, &v) != 0) return RG_ERR_COLLECTIVE;
        *e.second = v;
    }
    return RG_OK;
}

rg_status rg_comm_destroy(void *comm) {
    const Rccl *r = g_rccl.handle ? &g_rccl : nullptr;
    if (!comm || !r) return RG_ERR_INVALID_ARGUMENT;
    return r->destroy(comm) == 0 ? RG_OK : RG_ERR_COLLECTIVE;
}

rg_gather_fn rg_comm_gather_fn(void) {
    const Rccl *r = rccl();
    return r ? reinterpret_cast<rg_gather_fn>(r->gather) : nullptr;
}

}  // extern "C"
