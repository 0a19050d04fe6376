// rg_multi.hip — rg_render_multi: one process drives N devices (SURVEY.md
// §8(b), §5: "rg_render_multi ... ncclCommInitAll").
//
// The frame is cut into tile_rows-row tiles dealt round-robin (tile t ->
// device t % N, the balance argument of DESIGN.md §6).  Per call:
//   device i, stream i : render its tiles into part[i] (its replica of the scene)
//   all devices        : ONE ncclGather of the equal-size parts to device 0, packed to
//                        RGB (3 B per pixel: alpha is always 255) off device 0
//                        (ncclGroupStart/End: one thread issues N ranks' calls)
//   device 0, stream 0 : re-interleave gathered parts into the frame, then
//                        copy the frame to the caller's host buffer
// RCCL is loaded with dlopen, so libraingun_hip.so links no collective
// library and shares the one already in a process (PyTorch's) if there is one.
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
#include "rg_internal.h"

// rg_frames.hip: parts travel as packed RGB (3 B per pixel); device 0 reads its own part in place
hipError_t rg_launch_reinterleave(const void *gathered, const void *root_part, void *image, uint32_t width,
                                  uint32_t height, uint32_t tile_rows, uint32_t world, size_t slot_bytes,
                                  hipStream_t stream);
hipError_t rg_launch_pack_rgb(const void *rgba, void *rgb, size_t npx, hipStream_t stream);
size_t rg_packed_slot_bytes(uint32_t slot_rows, uint32_t width);

namespace {

bool ok(hipError_t e) { return e == hipSuccess; }

// ---------------------------------------------------------------- RCCL, loaded at run time
typedef int (*pfn_comm_init_all)(void **comms, int ndev, const int *devlist);
typedef int (*pfn_comm_destroy)(void *comm);
typedef int (*pfn_gather)(const void *send, void *recv, size_t count, int dtype, int root, void *comm, hipStream_t s);
typedef int (*pfn_group)(void);

struct Rccl {
    bool tried = false;
    void *handle = nullptr;
    pfn_comm_init_all init_all = nullptr;
    pfn_comm_destroy destroy = nullptr;
    pfn_gather gather = nullptr;
    pfn_group group_start = nullptr, group_end = nullptr;
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
        if (g_rccl.init_all && g_rccl.destroy && g_rccl.gather && g_rccl.group_start && g_rccl.group_end) {
            g_rccl.handle = h;
            return &g_rccl;
        }
        dlclose(h);
    }
    return nullptr;
}

constexpr int kNcclUint8 = 1;       // ncclDataType_t (rccl.h)
constexpr int kNcclInProgress = 7;  // a non-blocking communicator's "enqueued"

}  // namespace

// Per-scene multi-GPU state for one (ngpus, width, height, tile_rows).
struct rg_multi_res {
    int n = 0;
    uint32_t w = 0, h = 0, T = 0, slot_rows = 0;
    size_t part_bytes = 0;   // RGBA part
    size_t slot_bytes = 0;   // packed RGB part each device sends
    std::vector<int> devs;
    std::vector<rg_scene *> reps;      // reps[0] = the scene itself (not owned)
    std::vector<void *> comms;
    std::vector<hipStream_t> streams;
    std::vector<void *> parts, packed;            // packed[0] unused: device 0's part is read in place
    void *gathered = nullptr, *image = nullptr;  // device 0
    unsigned long long *snap = nullptr;          // pinned: 4 words per device
    hipEvent_t ev0 = nullptr, ev1 = nullptr;     // device 0: render start .. frame assembled
};

namespace {

void free_res(rg_multi_res *m) {
    if (!m) return;
    const Rccl *r = g_rccl.handle ? &g_rccl : nullptr;
    for (int i = 0; i < (int)m->devs.size(); ++i) {
        (void)hipSetDevice(m->devs[i]);
        if (i < (int)m->streams.size() && m->streams[i]) (void)hipStreamSynchronize(m->streams[i]);
    }
    for (int i = 0; i < (int)m->devs.size(); ++i) {
        (void)hipSetDevice(m->devs[i]);
        if (i < (int)m->comms.size() && m->comms[i] && r) (void)r->destroy(m->comms[i]);
        if (i < (int)m->parts.size() && m->parts[i]) (void)hipFree(m->parts[i]);
        if (i < (int)m->packed.size() && m->packed[i]) (void)hipFree(m->packed[i]);
        if (i < (int)m->streams.size() && m->streams[i]) (void)hipStreamDestroy(m->streams[i]);
        if (i > 0 && i < (int)m->reps.size() && m->reps[i]) rg_scene_free(m->reps[i]);
    }
    if (!m->devs.empty()) {
        (void)hipSetDevice(m->devs[0]);
        if (m->gathered) (void)hipFree(m->gathered);
        if (m->image) (void)hipFree(m->image);
        if (m->ev0) (void)hipEventDestroy(m->ev0);
        if (m->ev1) (void)hipEventDestroy(m->ev1);
    }
    if (m->snap) (void)hipHostFree(m->snap);
    delete m;
}

rg_status build_res(const rg_scene *s, int n, uint32_t W, uint32_t H, uint32_t T, rg_multi_res **out) {
    *out = nullptr;
    const Rccl *r = rccl();
    if (!r) return RG_ERR_COLLECTIVE;
    int ndev = 0;
    if (!ok(hipGetDeviceCount(&ndev)) || n > ndev) return RG_ERR_INVALID_ARGUMENT;
    rg_multi_res *m = new (std::nothrow) rg_multi_res();
    if (!m) return RG_ERR_OUT_OF_MEMORY;
    m->n = n;
    m->w = W;
    m->h = H;
    m->T = T;
    const uint32_t tiles = (H + T - 1) / T;
    m->slot_rows = (tiles + (uint32_t)n - 1) / (uint32_t)n * T;  // equal on every device
    m->part_bytes = (size_t)m->slot_rows * W * 4;
    m->slot_bytes = rg_packed_slot_bytes(m->slot_rows, W);
    for (int i = 0; i < n; ++i) m->devs.push_back((s->device + i) % ndev);
    m->reps.assign(n, nullptr);
    m->comms.assign(n, nullptr);
    m->streams.assign(n, nullptr);
    m->parts.assign(n, nullptr);
    m->packed.assign(n, nullptr);
    m->reps[0] = const_cast<rg_scene *>(s);
    rg_status st = RG_OK;
    for (int i = 1; i < n && st == RG_OK; ++i) st = rg_scene_replica(s, m->devs[i], &m->reps[i]);
    for (int i = 0; i < n && st == RG_OK; ++i) {
        if (!ok(hipSetDevice(m->devs[i])) || !ok(hipStreamCreateWithFlags(&m->streams[i], hipStreamNonBlocking)))
            st = RG_ERR_DEVICE;
        else if (!ok(hipMalloc(&m->parts[i], std::max(m->part_bytes, m->slot_bytes))) ||
                 !ok(hipMemset(m->parts[i], 0, std::max(m->part_bytes, m->slot_bytes))) ||
                 (i > 0 && !ok(hipMalloc(&m->packed[i], m->slot_bytes))))
            st = RG_ERR_OUT_OF_MEMORY;  // padding rows of the last tiles stay zero
    }
    if (st == RG_OK) {
        void *snap = nullptr;
        (void)hipSetDevice(m->devs[0]);
        if (!ok(hipMalloc(&m->gathered, m->slot_bytes * (size_t)n)) || !ok(hipMalloc(&m->image, (size_t)H * W * 4)) ||
            !ok(hipHostMalloc(&snap, (size_t)n * 4 * sizeof(unsigned long long), hipHostMallocPortable)))
            st = RG_ERR_OUT_OF_MEMORY;
        m->snap = static_cast<unsigned long long *>(snap);
        if (st == RG_OK && (!ok(hipEventCreate(&m->ev0)) || !ok(hipEventCreate(&m->ev1)))) st = RG_ERR_DEVICE;
    }
    if (st == RG_OK && r->init_all(m->comms.data(), n, m->devs.data()) != 0) st = RG_ERR_COLLECTIVE;
    if (st != RG_OK) {
        for (void *&c : m->comms) c = nullptr;  // not (fully) created
        free_res(m);
        return st;
    }
    *out = m;
    return RG_OK;
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
    if (!m || m->n != ngpus || m->w != W || m->h != H || m->T != T) {
        rg_multi_release(s);
        rg_status st = build_res(s, ngpus, W, H, T, &m);
        if (st != RG_OK) {
            (void)hipSetDevice(s->device);
            return st;
        }
        s->multi = m;
    }
    const Rccl *r = rccl();
    const int n = m->n;
    for (int i = 1; i < n; ++i) rg_sync_settings(m->reps[i], s);
    // renders
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
    if (r->group_start() != 0) return RG_ERR_COLLECTIVE;
    int gerr = 0;
    for (int i = 0; i < n; ++i) {
        (void)hipSetDevice(m->devs[i]);
        const int g = r->gather(i == 0 ? m->parts[i] : m->packed[i], i == 0 ? m->gathered : nullptr, m->slot_bytes,
                                kNcclUint8, 0, m->comms[i],
                                m->streams[i]);
        if (g != 0 && g != kNcclInProgress && gerr == 0) gerr = g;
    }
    const int ge = r->group_end();
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
    rg_stats total;
    std::memset(&total, 0, sizeof total);
    total.error_pixel = -1;
    unsigned long long worst = 0;  // complemented keys: the max is the lowest erroring pixel
    for (int i = 0; i < n; ++i) {
        total.rays.primary += m->snap[4 * i];
        total.rays.shadow += m->snap[4 * i + 1];
        total.rays.secondary += m->snap[4 * i + 2];
        worst = std::max(worst, m->snap[4 * i + 3]);
    }
    unsigned long long w4[4] = {0, 0, 0, worst};
    rg_stats es;
    const rg_status err = rg_snap_status(w4, &es);
    total.error_pixel = es.error_pixel;
    float ms = 0.0f;
    (void)hipEventElapsedTime(&ms, m->ev0, m->ev1);
    total.kernel_ms = ms;
    if (stats) *stats = total;
    return err;
}
