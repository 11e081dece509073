// Host runtime of libpt_hip.so: the C ABI of include/pt_api.h.
//
// pt_scene_upload converts the host-built scene (reference-form BVH4s,
// primitives, materials, lights) into the device layout of pt_device.h:
// one node array for the TLAS and every BLAS, one leaf-ordered primitive slot
// array, and the light-sampler running sums.  pt_render runs the persistent
// wavefront (pt_kernels.hip) over sample chunks and gathers the film.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "pt_kernels.hip"
#include "pt_alpha_cov.h"

// The host keeps up to PT_LAG wavefront iterations queued ahead of the one
// whose counts it reads (no per-bounce round trip; iterations past the end of
// a chunk find zero paths and return at once)
#define PT_LAG 4
#define PT_RING (PT_LAG + 1)
// The tail (k_tail): at most this many live paths, and at most 1/PT_TAIL_SHARE
// of the wavefront, once every camera sample of the chunk has started
#ifndef PT_TAIL_PATHS
#define PT_TAIL_PATHS 65536u
#endif
#ifndef PT_TAIL_SHARE
#define PT_TAIL_SHARE 16u
#endif
// Any-hit rays of bounce k on a second stream, beside bounce k+1's closest-hit
// rays (the two only read the path state; the shading of k+1 waits for them):
// each persistent pool kernel's draining tail leaves CUs the other fills.
// Off by default (C4 -6.8 %, profiles/r03_ab_streams_shade.txt); the render
// flags or env PT_OVERLAP_SHADOW=1 turn it on.

struct pt_ctx {
    int device = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    // any-hit rays of bounce k traced on side_stream beside bounce k+1's
    // closest-hit rays (PT_RENDER_OVERLAP_SHADOW; see trace's loop)
    hipStream_t side_stream = nullptr;
    bool overlap = false;
    std::string err;
    // scene
    std::vector<void*> scene_bufs;
    uint64_t scene_bytes = 0;
    DevScene scene{};
    bool has_scene = false;
    uint32_t n_materials = 0;
    uint32_t n_media = 0;
    uint32_t trace_blocks = 0;  // resident traversal blocks on this device (persistent grid), max of the two
    uint32_t pool_blocks[2][2][2] = {};  // [any hit][instanced][quantized]: each pool kernel's resident blocks
    uint32_t sl_blocks = 0;              // ... of the stackless any-hit kernel (k_shadow_sl)
    uint64_t n_clusters = 0;    // BVH clusters of the uploaded scene (traversal choice)
    bool has_qnodes = false;    // the scene's nodes have a quantized copy (48-B records)
    int node_format = PT_NODES_AUTO;  // pt_set_node_format
    // wavefront buffers: two compacted path states (ping-pong), per-bounce hits,
    // the finished-path list and the shadow-ray queue
    uint32_t cap = 0;
    PathSoA PA{}, PB{};
    float4* hit = nullptr;
    uint32_t* qcnt = nullptr;
    uint32_t* ovf = nullptr;  // pool traversal stack entries beyond PT_POOL_LDS
    uint32_t* ovf_any = nullptr;  // the any-hit pool kernel's half of ovf (they may run together)
    uint32_t* ties = nullptr;     // closest-hit rays listed for the exact re-trace (k_closest_ties)
    float* sq_time = nullptr;     // motion blur: each queued shadow ray's time (with PA/PB.time)
    uint32_t* scratch = nullptr;  // instance traversal state, SCR_WORDS x scratch_lanes
    uint64_t scratch_lanes = 0;
    ShadowRec* sq = nullptr;
    unsigned long long* counters = nullptr;
    uint32_t* host_cnt = nullptr;  // pinned, PT_RING counter snapshots (SNAP_WORDS each)
    uint32_t* host_cnt_dev = nullptr;  // the same memory as the kernels address it
    float* sample_L = nullptr;
    uint64_t sample_cap = 0;  // floats
    double* film = nullptr;
    uint64_t film_cap = 0;  // doubles
    // adaptive sampling: per-pixel estimators / sample counts / active-list
    // entry, the two active lists and their counters
    AdaptEst* a_est = nullptr;
    uint32_t* a_counts = nullptr;
    int32_t* a_map = nullptr;
    uint32_t* a_list = nullptr;
    uint32_t* a_cnt = nullptr;
    uint64_t a_est_cap = 0, a_counts_cap = 0, a_map_cap = 0, a_list_cap = 0, a_cnt_cap = 0;
    // material sort (PT_RENDER_SORT_MATERIAL): shading order + bin counters
    uint32_t* sort_order = nullptr;
    uint32_t* sort_counts = nullptr;
    uint64_t sort_order_cap = 0, sort_counts_cap = 0;
    uint16_t* sort_bins = nullptr;  // each path's bin between k_sort_count and k_sort_scatter
    uint64_t sort_bins_cap = 0;
    uint32_t* ray_order = nullptr;  // PT_RENDER_SORT_RAYS: closest-hit claim order
    uint32_t* ray_counts = nullptr;
    uint64_t ray_order_cap = 0, ray_counts_cap = 0;
    uint2* nee_jobs = nullptr;  // PT_SHADE_SPLIT: k_shade's NEE jobs for k_shade_nee
    uint64_t nee_jobs_cap = 0;
    hipEvent_t ev[8] = {};
    hipEvent_t rev[PT_RING][5] = {};  // per in-flight iteration: kernel boundaries [0..2], end [4] ([3] unused)
    uint32_t* stack_drops = nullptr;  // device words: traversal pushes beyond the stack, exact-tie list drops
                                      // (DevScene::stack_drops / tie_drops)
    // multi-device context (pt_create with n_devices > 1): the other devices'
    // contexts (owned) and, per device, an RCCL communicator for the film reduce
    std::vector<pt_ctx*> peers;
    bool multi = false;  // renders through render_multi (n_devices > 1, or forced for tests)
    ncclComm_t comm = nullptr;
    bool comm_nonblocking = false;  // built by pt_comm_init_rank (non-blocking); else ncclCommInitAll's
    int comm_ranks = 0, comm_rank = 0;
    // where the last fixed-SPP frame's final sample chunk lies in sample_L
    // (pt_frame_samples); cleared by every other use of the buffer
    struct FrameRec {
        bool valid = false;
        uint32_t width = 0, npix = 0, tiled = 0, tiles_x = 0;
        uint32_t s_lo = 0, s_hi = 0, shard_index = 0, shard_count = 1;
        uint32_t height = 0;  // the film's: npix counts the padded 8x8 tiles when tiled
    } frame;
};

// The uploaded scene lives in the device's __constant__ DevScene S (one per
// device, not per context): calls that bind a context's scene and launch are
// serialized per device, so two contexts on one GPU used from two host
// threads cannot run kernels against each other's scene record.
static std::mutex g_device_mu[64];
struct DeviceLock {
    std::unique_lock<std::mutex> lk;
    explicit DeviceLock(int device) : lk(g_device_mu[(unsigned)device & 63u]) {}
};

static pt_status fail(pt_ctx* c, pt_status code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    if (c) c->err = buf;
    return code;
}
#define HIPCHK(c, x)                                                                                  \
    do {                                                                                              \
        hipError_t e_ = (x);                                                                          \
        if (e_ != hipSuccess) return fail(c, PT_ERR_HIP, "%s: %s (%s:%d)", #x, hipGetErrorString(e_), \
                                          __FILE__, __LINE__);                                        \
    } while (0)

static thread_local std::string g_err;

extern "C" int pt_version(void) { return PT_API_VERSION; }

extern "C" const char* pt_last_error(const pt_ctx* c) { return c ? c->err.c_str() : g_err.c_str(); }

extern "C" void pt_destroy(pt_ctx* c);

// One device's context (the whole context for n_devices = 1).
static pt_status create_dev(pt_ctx** out, int device) {
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
        g_err = "no HIP device";
        return PT_ERR_NODEV;
    }
    if (device < 0 || device >= n) {
        g_err = "device index out of range";
        return PT_ERR_ARG;
    }
    pt_ctx* c = new pt_ctx();
    c->device = device;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess) {
        g_err = "hip init failed";
        delete c;
        return PT_ERR_HIP;
    }
    c->stream = c->own_stream;
    if (hipStreamCreateWithFlags(&c->side_stream, hipStreamNonBlocking) != hipSuccess) {
        g_err = "hip init failed";
        hipStreamDestroy(c->own_stream);
        delete c;
        return PT_ERR_HIP;
    }
    {
        const char* ov = getenv("PT_OVERLAP_SHADOW");
        c->overlap = ov && atoi(ov) != 0;
    }
    for (hipEvent_t* e = &c->ev[0]; e != &c->ev[0] + 8; ++e)
        if (hipEventCreate(e) != hipSuccess) {
            g_err = "event create failed";
            delete c;
            return PT_ERR_HIP;
        }
    for (auto& r : c->rev)
        for (auto& e : r) {
        if (hipEventCreate(&e) != hipSuccess) {
            g_err = "event create failed";
            delete c;
            return PT_ERR_HIP;
        }
    }
    {
        // the persistent (pool) traversal grid of each pool kernel: its blocks
        // that are resident together (a variant's own figure: the instanced
        // kernels' registers must not shrink the grid of the others); the
        // overflow stack array covers the largest
        int cus = 0;
        const void* pool_kernels[2][2][2] = {
            {{reinterpret_cast<const void*>(&k_closest_pool<false, false, false>),
              reinterpret_cast<const void*>(&k_closest_pool<false, false, true>)},
             {reinterpret_cast<const void*>(&k_closest_pool<false, true, false>),
              reinterpret_cast<const void*>(&k_closest_pool<false, true, true>)}},
            {{reinterpret_cast<const void*>(&k_shadow_pool<false, false, false>),
              reinterpret_cast<const void*>(&k_shadow_pool<false, false, true>)},
             {reinterpret_cast<const void*>(&k_shadow_pool<false, true, false>),
              reinterpret_cast<const void*>(&k_shadow_pool<false, true, true>)}}};
        bool ok = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess;
        c->trace_blocks = 1;
        for (int a = 0; a < 2; a++)
            for (int i = 0; i < 2; i++)
                for (int q = 0; ok && q < 2; q++) {
                    int b = 0;
                    ok = hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, pool_kernels[a][i][q], PT_TRACE_BLOCK, 0) ==
                         hipSuccess;
                    c->pool_blocks[a][i][q] = (uint32_t)std::max(1, cus * std::max(1, b));
                    c->trace_blocks = std::max(c->trace_blocks, c->pool_blocks[a][i][q]);
                }
        if (ok) {
            int b = 0;
            ok = hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, reinterpret_cast<const void*>(&k_shadow_sl<false>),
                                                              PT_TRACE_BLOCK, 0) == hipSuccess;
            c->sl_blocks = (uint32_t)std::max(1, cus * std::max(1, b));
        }
        if (!ok) {
            g_err = "occupancy query failed";
            delete c;
            return PT_ERR_HIP;
        }
    }
    if (hipHostMalloc((void**)&c->host_cnt, PT_RING * SNAP_WORDS * 4, hipHostMallocCoherent | hipHostMallocMapped) !=
            hipSuccess ||
        hipHostGetDevicePointer((void**)&c->host_cnt_dev, c->host_cnt, 0) != hipSuccess) {
        g_err = "pinned alloc failed";
        pt_destroy(c);
        return PT_ERR_HIP;
    }
    if (hipMalloc((void**)&c->stack_drops, 128) != hipSuccess || hipMemset(c->stack_drops, 0, 128) != hipSuccess) {
        g_err = "device alloc failed";
        pt_destroy(c);
        return PT_ERR_OOM;
    }
    c->scene.stack_drops = c->stack_drops;
    c->scene.tie_drops = c->stack_drops + 1;
    *out = c;
    return PT_OK;
}

extern "C" pt_status pt_create(pt_ctx** out, int n_devices, const int* device_ids) {
    if (!out) return PT_ERR_ARG;
    *out = nullptr;
    if (n_devices < 1 || n_devices > 64) {
        g_err = "n_devices out of range";
        return PT_ERR_ARG;
    }
    std::vector<int> ids(n_devices);
    for (int i = 0; i < n_devices; i++) {
        ids[i] = device_ids ? device_ids[i] : i;
        for (int j = 0; j < i; j++)
            if (ids[j] == ids[i]) {
                g_err = "a device is listed twice";
                return PT_ERR_ARG;
            }
    }
    pt_ctx* c = nullptr;
    pt_status st = create_dev(&c, ids[0]);
    if (st) return st;
    for (int i = 1; i < n_devices; i++) {
        pt_ctx* p = nullptr;
        if ((st = create_dev(&p, ids[i])) != PT_OK) {
            pt_destroy(c);
            return st;
        }
        c->peers.push_back(p);
    }
    // PT_MULTI_DEVICE_PATH=1 (tests on a one-GPU box): a one-device context
    // still gets its communicator and renders through render_multi
    c->multi = n_devices > 1 || (getenv("PT_MULTI_DEVICE_PATH") && atoi(getenv("PT_MULTI_DEVICE_PATH")) != 0);
    if (c->multi) {  // one communicator per device, ranks in device_ids order
        std::vector<ncclComm_t> comms(n_devices);
        const ncclResult_t r = ncclCommInitAll(comms.data(), n_devices, ids.data());
        if (r != ncclSuccess) {
            g_err = std::string("ncclCommInitAll: ") + ncclGetErrorString(r);
            pt_destroy(c);
            return PT_ERR_COMM;
        }
        for (int i = 0; i < n_devices; i++) {
            pt_ctx* d = i ? c->peers[i - 1] : c;
            d->comm = comms[i];
            d->comm_ranks = n_devices;
            d->comm_rank = i;
        }
    }
    *out = c;
    return PT_OK;
}

extern "C" int pt_device_count(const pt_ctx* c) { return c ? 1 + (int)c->peers.size() : 0; }

extern "C" pt_status pt_comm_unique_id(uint8_t* id_out) {
    static_assert(sizeof(ncclUniqueId) == PT_COMM_ID_BYTES, "RCCL unique id size");
    if (!id_out) return PT_ERR_ARG;
    ncclUniqueId id;
    const ncclResult_t r = ncclGetUniqueId(&id);
    if (r != ncclSuccess) {
        g_err = std::string("ncclGetUniqueId: ") + ncclGetErrorString(r);
        return PT_ERR_COMM;
    }
    memcpy(id_out, &id, sizeof(id));
    return PT_OK;
}

static double comm_timeout_s() {
    double timeout_s = 120.0;
    if (const char* e = getenv("PT_COMM_TIMEOUT_S")) timeout_s = std::max(1.0, atof(e));
    return timeout_s;
}

// A per-rank communicator is built non-blocking (pt_comm_init_rank), and that
// mode stays with it: any later call on it (init, the reduce that sets up the
// connections, finalize) may return ncclInProgress while the work completes
// in the background.  Polls ncclCommGetAsyncError until the state leaves
// ncclInProgress or the deadline passes (then ncclInternalError: the caller
// aborts the communicator).  Test hook: PT_COMM_FAKE_INPROGRESS=n makes a
// reduce's enqueue report ncclInProgress and the first n polls after it too,
// as a real non-blocking communicator may (tests/test_gpu_distributed.py).
static int fake_inprogress() {
    const char* e = getenv("PT_COMM_FAKE_INPROGRESS");
    return e ? std::max(0, atoi(e)) : 0;
}
static ncclResult_t comm_wait(ncclComm_t comm, ncclResult_t r, double timeout_s, int fake_polls = 0) {
    const auto t0 = std::chrono::steady_clock::now();
    while (r == ncclInProgress && comm) {
        if (fake_polls > 0) {
            fake_polls--;
            r = ncclInProgress;
        } else if (ncclCommGetAsyncError(comm, &r) != ncclSuccess) {
            r = ncclInternalError;
        }
        if (r != ncclInProgress) break;
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s)
            return ncclInternalError;
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
    return r;
}

// Non-blocking ncclCommInitRankConfig polled up to a deadline (env
// PT_COMM_TIMEOUT_S, default 120 s): a rank whose peers never join (one failed
// before the collective init) aborts its half-built communicator and returns
// PT_ERR_COMM instead of blocking forever, so the caller's agreement step
// (pathtracing_amd/distributed.py init_film_comm) is always reached.
extern "C" pt_status pt_comm_init_rank(pt_ctx* c, int n_ranks, int rank, const uint8_t* id) {
    if (!c || !id || n_ranks < 1 || rank < 0 || rank >= n_ranks) return PT_ERR_ARG;
    if (c->multi) return fail(c, PT_ERR_STATE, "a multi-device context has its communicators");
    if (c->comm) return fail(c, PT_ERR_STATE, "communicator already initialised (pt_comm_destroy first)");
    HIPCHK(c, hipSetDevice(c->device));
    ncclUniqueId uid;
    memcpy(&uid, id, sizeof(uid));
    const double timeout_s = comm_timeout_s();
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    ncclComm_t comm = nullptr;
    ncclResult_t r = ncclCommInitRankConfig(&comm, n_ranks, uid, rank, &cfg);
    const bool pending = r == ncclInProgress && comm;
    r = comm_wait(comm, r, timeout_s);
    if (r != ncclSuccess) {
        if (comm) ncclCommAbort(comm);
        if (pending && r == ncclInternalError)
            return fail(c, PT_ERR_COMM, "ncclCommInitRank(%d of %d): peers did not join within %.0f s", rank,
                        n_ranks, timeout_s);
        return fail(c, PT_ERR_COMM, "ncclCommInitRank(%d of %d): %s", rank, n_ranks, ncclGetErrorString(r));
    }
    c->comm = comm;
    c->comm_nonblocking = true;
    c->comm_ranks = n_ranks;
    c->comm_rank = rank;
    return PT_OK;
}

// Drops the per-process communicator (ncclCommAbort: safe when its peers are
// gone or never finished joining), so a later pt_comm_init_rank can rejoin.
extern "C" pt_status pt_comm_destroy(pt_ctx* c) {
    if (!c) return PT_ERR_ARG;
    if (c->multi) return fail(c, PT_ERR_STATE, "a multi-device context owns its communicators");
    if (c->comm) {
        hipSetDevice(c->device);
        ncclCommAbort(c->comm);
    }
    c->comm = nullptr;
    c->comm_nonblocking = false;
    c->comm_ranks = 0;
    c->comm_rank = 0;
    return PT_OK;
}

// Orderly teardown of a per-rank (non-blocking) communicator: finalize (which
// may report ncclInProgress while it flushes), wait, then destroy; a finalize
// that fails or does not finish in time aborts instead.
static void comm_release(ncclComm_t comm, bool nonblocking) {
    if (!comm) return;
    if (!nonblocking) {
        ncclCommDestroy(comm);
        return;
    }
    ncclResult_t r = ncclCommFinalize(comm);
    r = comm_wait(comm, r, comm_timeout_s());
    if (r == ncclSuccess)
        ncclCommDestroy(comm);
    else
        ncclCommAbort(comm);
}

// In-place SUM reduce of n doubles onto `root` over the context's communicator,
// on its stream (replaces Film::Merge's atomic<double> adds, Film.hpp:125-132).
// On a non-blocking communicator the enqueue itself may report ncclInProgress
// (the first reduce sets up the connections): it is waited for, not treated as
// a failure, so this rank does not raise while its peers' reduce is queued.
static pt_status film_reduce_async(pt_ctx* c, double* film, uint64_t n, int root) {
    ncclResult_t r = ncclReduce(film, film, n, ncclDouble, ncclSum, root, c->comm, c->stream);
    const int fake = c->multi ? 0 : fake_inprogress();
    if (fake && r == ncclSuccess) r = ncclInProgress;
    if (r == ncclInProgress && !c->multi) r = comm_wait(c->comm, r, comm_timeout_s(), fake);
    if (r != ncclSuccess) return fail(c, PT_ERR_COMM, "ncclReduce: %s", ncclGetErrorString(r));
    return PT_OK;
}

extern "C" pt_status pt_film_reduce(pt_ctx* c, double* film, uint64_t n, int root) {
    if (!c || !film) return PT_ERR_ARG;
    if (!c->comm) return fail(c, PT_ERR_STATE, "no communicator (pt_comm_init_rank)");
    if (c->multi) return fail(c, PT_ERR_STATE, "multi-device contexts reduce inside pt_render");
    if (root < 0 || root >= c->comm_ranks) return fail(c, PT_ERR_ARG, "root out of range");
    HIPCHK(c, hipSetDevice(c->device));
    if (pt_status st = film_reduce_async(c, film, n, root)) return st;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return PT_OK;
}

static void free_scene(pt_ctx* c) {
    for (void* p : c->scene_bufs) hipFree(p);
    c->scene_bufs.clear();
    c->scene_bytes = 0;
    c->has_scene = false;
}
static void free_work(pt_ctx* c) {
    // (d shares o's allocation, L beta's: pt_kernels.h PathSoA)
    void* bufs[] = {c->PA.o.p, c->PA.beta.p, c->PA.sid, c->PA.time, c->PB.o.p, c->PB.beta.p, c->PB.sid,
                    c->PB.time, c->hit, c->qcnt, c->sq, c->counters, c->ovf, c->ties, c->sq_time};
    for (void* p : bufs)
        if (p) hipFree(p);
    c->PA = PathSoA{};
    c->PB = PathSoA{};
    c->hit = nullptr;
    c->qcnt = nullptr;
    c->sq = nullptr;
    c->counters = nullptr;
    c->ovf = nullptr;
    c->ovf_any = nullptr;
    c->ties = nullptr;
    c->sq_time = nullptr;
    c->cap = 0;
}

extern "C" void pt_destroy(pt_ctx* c) {
    if (!c) return;
    if (c->multi) {
        // the multi-device context's communicators (ncclCommInitAll: blocking,
        // one per device, every one owned by this thread) are finalized
        // together in one group -- one at a time, each finalize would wait for
        // peers that are not being finalized -- then destroyed
        std::vector<ncclComm_t> comms;
        for (size_t i = 0; i <= c->peers.size(); i++) {
            pt_ctx* d = i ? c->peers[i - 1] : c;
            if (d->comm) comms.push_back(d->comm);
            d->comm = nullptr;
        }
        if (!comms.empty()) {
            ncclGroupStart();
            for (ncclComm_t m : comms) ncclCommFinalize(m);
            ncclGroupEnd();
            for (ncclComm_t m : comms) ncclCommDestroy(m);
        }
    }
    for (pt_ctx* p : c->peers) pt_destroy(p);
    c->peers.clear();
    hipSetDevice(c->device);
    if (c->comm) comm_release(c->comm, c->comm_nonblocking);  // a per-rank communicator (pt_comm_init_rank)
    c->comm = nullptr;
    if (c->stream) hipStreamSynchronize(c->stream);
    if (c->side_stream) hipStreamSynchronize(c->side_stream);  // any-hit kernels of an overlapped frame
    free_scene(c);
    free_work(c);
    if (c->scratch) hipFree(c->scratch);
    if (c->sample_L) hipFree(c->sample_L);
    if (c->film) hipFree(c->film);
    for (void* p : {(void*)c->a_est, (void*)c->a_counts, (void*)c->a_map, (void*)c->a_list, (void*)c->a_cnt,
                    (void*)c->sort_order, (void*)c->sort_counts, (void*)c->ray_order, (void*)c->ray_counts,
                    (void*)c->sort_bins, (void*)c->nee_jobs})
        if (p) hipFree(p);
    if (c->host_cnt) hipHostFree(c->host_cnt);
    if (c->stack_drops) hipFree(c->stack_drops);
    for (auto& e : c->ev)
        if (e) hipEventDestroy(e);
    for (auto& r : c->rev)
        for (auto& e : r)
            if (e) hipEventDestroy(e);
    if (c->own_stream) hipStreamDestroy(c->own_stream);
    if (c->side_stream) hipStreamDestroy(c->side_stream);
    delete c;
}

extern "C" pt_status pt_set_stream(pt_ctx* c, void* s) {
    if (!c) return PT_ERR_ARG;
    c->stream = s ? (hipStream_t)s : c->own_stream;
    return PT_OK;
}

extern "C" pt_status pt_set_node_format(pt_ctx* c, int fmt) {
    if (!c || fmt < PT_NODES_AUTO || fmt > PT_NODES_QUANTIZED) return PT_ERR_ARG;
    c->node_format = fmt;
    for (pt_ctx* p : c->peers) p->node_format = fmt;
    return PT_OK;
}

extern "C" uint64_t pt_scene_device_bytes(const pt_ctx* c) { return c ? c->scene_bytes : 0; }

// ---- quantized nodes (DevQNode).  One axis of a cluster's four child boxes:
// origin = the smallest lower bound, step = the smallest power of two with
// which every bound fits 8 bits, each lower bound rounded down and each upper
// bound up, checked with the device's own decode fma(q, step, origin) so the
// decoded box always contains the reference's float box.  False when the
// bounds are not finite or no step fits (the scene then keeps full nodes).
// N children (4 per node); wlo / whi: 4 bytes per word
static bool quantize_axis_n(int N, const float* lo, const float* hi, uint32_t valid, float& org, uint32_t& e8,
                            uint32_t* wlo, uint32_t* whi) {
    for (int w = 0; w < N / 4; w++) {
        wlo[w] = 0;
        whi[w] = 0;
    }
    if (!valid) {
        org = 0.0f;
        e8 = 127;
        for (int w = 0; w < N / 4; w++) wlo[w] = 0xFFFFFFFFu;  // empty: lo 255 > hi 0 (refs REF_EMPTY anyway)
        return true;
    }
    float mn = INFINITY, mx = -INFINITY;
    for (int k = 0; k < N; k++)
        if (valid >> k & 1) {
            if (!std::isfinite(lo[k]) || !std::isfinite(hi[k])) return false;
            mn = std::min(mn, lo[k]);
            mx = std::max(mx, hi[k]);
        }
    org = mn;
    const double ext = (double)mx - (double)mn;
    int k0 = ext > 0 ? (int)std::ceil(std::log2(ext / 255.0)) : -126;
    for (int k = std::max(-126, k0 - 1); k <= 127; k++) {
        const float step = std::ldexp(1.0f, k);
        uint32_t ql[8] = {255, 255, 255, 255, 255, 255, 255, 255}, qh[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        bool ok = true;
        for (int c = 0; c < N && ok; c++) {
            if (!(valid >> c & 1)) continue;
            double a = std::floor(((double)lo[c] - (double)org) / step);
            a = std::min(255.0, std::max(0.0, a));
            while (a > 0 && std::fma((float)a, step, org) > lo[c]) a -= 1;
            if (std::fma((float)a, step, org) > lo[c]) ok = false;
            double b = std::ceil(((double)hi[c] - (double)org) / step);
            b = std::max(0.0, b);
            while (b <= 255 && std::fma((float)b, step, org) < hi[c]) b += 1;
            if (b > 255) ok = false;
            ql[c] = (uint32_t)a;
            qh[c] = (uint32_t)b;
        }
        if (!ok) continue;
        e8 = (uint32_t)(k + 127);
        for (int c = 0; c < N; c++) {
            wlo[c / 4] |= ql[c] << (8 * (c % 4));
            whi[c / 4] |= qh[c] << (8 * (c % 4));
        }
        return true;
    }
    return false;
}
static bool quantize_axis(const float* lo, const float* hi, uint32_t valid, float& org, uint32_t& e8, uint32_t& wlo,
                          uint32_t& whi) {
    return quantize_axis_n(4, lo, hi, valid, org, e8, &wlo, &whi);
}

static bool quantize_node(const DevCluster& n, DevQNode& q) {
    uint32_t valid = 0;
    for (int k = 0; k < 4; k++)
        if (n.child[k] != REF_EMPTY) valid |= 1u << k;
    const float* b = &n.xmin.x;  // xmin xmax ymin ymax zmin zmax, 4 floats each
    float org[3];
    uint32_t e[3], w[6];
    for (int a = 0; a < 3; a++)
        if (!quantize_axis(b + 8 * a, b + 8 * a + 4, valid, org[a], e[a], w[2 * a], w[2 * a + 1])) return false;
    q.a = make_float4(org[0], org[1], org[2], __builtin_bit_cast(float, e[0] | e[1] << 8 | e[2] << 16));
    for (int k = 0; k < 4; k++) q.b[k] = w[k];
    q.c[0] = w[4];
    q.c[1] = w[5];
    q.c[2] = n.order[0];
    q.c[3] = n.order[1];
    for (int k = 0; k < 4; k++) q.child[k] = n.child[k];
    return true;
}

template <class T>
static pt_status upload(pt_ctx* c, const T* src, size_t n, const T** dst, size_t pad = 0) {
    *dst = nullptr;
    size_t bytes = std::max<size_t>(n * sizeof(T) + pad, 16);
    void* p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) return fail(c, PT_ERR_OOM, "hipMalloc(%zu) failed", bytes);
    c->scene_bufs.push_back(p);
    c->scene_bytes += bytes;
    if (n && src) HIPCHK(c, hipMemcpy(p, src, n * sizeof(T), hipMemcpyHostToDevice));
    else HIPCHK(c, hipMemset(p, 0, bytes));
    *dst = (const T*)p;
    return PT_OK;
}

static bool is_perm(unsigned p) {
    unsigned seen = 0;
    for (int s = 0; s < 4; s++) seen |= 1u << ((p >> (2 * s)) & 3);
    return seen == 0xF;
}

// Is the material's alpha a constant, and what does the tester return then?
static bool tex_alpha_const(const pt_scene_desc* s, int id, float& a, int depth = 0) {
    if (id < 0 || (uint32_t)id >= s->n_textures || depth > 16) return false;
    const pt_texture& t = s->textures[id];
    if (t.kind == PT_TEX_SOLID) { a = 1.0f; return true; }
    if (t.kind == PT_TEX_CHECKER) {
        float a1, a2;
        if (tex_alpha_const(s, t.a, a1, depth + 1) && tex_alpha_const(s, t.b, a2, depth + 1) && a1 == a2) {
            a = a1;
            return true;
        }
        return false;
    }
    if (t.image < 0 || (uint32_t)t.image >= s->n_images) return false;
    if (s->images[t.image].channels != 4) { a = 1.0f; return true; }
    return false;
}
static void material_alpha_flags(const pt_scene_desc* s, int mid, uint32_t& flags) {
    if (mid < 0) return;
    const pt_material& m = s->materials[mid];
    if (m.kind != PT_MAT_DIFFUSE && m.kind != PT_MAT_DIELECTRIC) return;
    if (m.alpha_mode == PT_ALPHA_OPAQUE) return;
    flags |= GF_PRED_GLM;  // HasAlpha(): IntersectPred runs Intersect + Alpha
    float a = 0;
    bool known;
    if (m.alpha >= 0) {
        const pt_texture& t = s->textures[m.alpha];
        known = t.kind == PT_TEX_SOLID;
        a = t.value[0];
    } else {
        known = tex_alpha_const(s, m.tex, a);
    }
    bool always_true = known && (m.alpha_mode == PT_ALPHA_MASK ? (a > m.alpha_cutoff) : (a >= 1.0f));
    if (!always_true) flags |= GF_ALPHA;
}

// DevAlpha record of an alpha-tested triangle (pt_device.h): mat_alpha's
// source resolved here (Material.hpp:181-198, Texture.cpp:47-62); false where
// only the general path handles it (checker sources, float images, images
// wider or taller than 65535)
static bool alpha_record(const pt_scene_desc* s, const pt_prim& p, DevAlpha& r) {
    if (!s->uvs || p.material < 0) return false;
    const pt_material& m = s->materials[p.material];
    const uint32_t* v = s->tri_vidx + 3 * (size_t)p.index;
    const float* u0 = s->uvs + 2 * (size_t)v[0];
    const float* u1 = s->uvs + 2 * (size_t)v[1];
    const float* u2 = s->uvs + 2 * (size_t)v[2];
    r = DevAlpha{{u1[0], u2[0], u0[0]}, {u1[1], u2[1], u0[1]}, 0, 0, 0, 0, m.alpha_cutoff, 1.0f};
    uint32_t src;
    const pt_image* im = nullptr;
    const pt_texture& t = s->textures[m.alpha >= 0 ? m.alpha : m.tex];
    if (t.kind == PT_TEX_SOLID) {
        src = ALPHA_SRC_CONST;  // Evaluate(uv).x of a solid alpha texture; Texture::alpha of a solid is 1
        r.off_lo = __builtin_bit_cast(uint32_t, m.alpha >= 0 ? t.value[0] : 1.0f);
    } else if (t.kind == PT_TEX_IMAGE) {
        im = &s->images[t.image];
        if (m.alpha < 0 && im->channels != 4) {  // ImageTexture::alpha without an alpha channel: 1
            src = ALPHA_SRC_CONST;
            r.off_lo = __builtin_bit_cast(uint32_t, 1.0f);
            im = nullptr;
        } else {
            if (im->format != PT_IMAGE_U8 || im->width <= 0 || im->height <= 0 || im->width > 0xFFFF ||
                im->height > 0xFFFF || im->channels <= 0 || im->channels > 0xFF)
                return false;
            src = m.alpha >= 0 ? ALPHA_SRC_CH1 : ALPHA_SRC_CH4;
            r.scale = t.scale[0];
        }
    } else {
        return false;
    }
    if (im) {
        r.off_lo = (uint32_t)im->offset;
        r.off_hi = (uint32_t)(im->offset >> 32);
        r.wh = (uint32_t)im->width | (uint32_t)im->height << 16;
    }
    r.mode = (m.alpha_mode & 3u) | src << 2 | (im ? (uint32_t)im->channels : 0u) << 8;
    return true;
}

static PtAlphaRecord alpha_cov_record(const DevAlpha& r) {
    PtAlphaRecord a;
    std::memset(&a, 0, sizeof a);  // the coverage memo keys on the bytes
    for (int k = 0; k < 3; k++) a.su[k] = r.su[k], a.sv[k] = r.sv[k];
    a.src = (r.mode >> 2) & 3u;
    a.mode = r.mode & 3u;
    a.cut = r.cut;
    a.scale = r.scale;
    if (a.src == ALPHA_SRC_CONST) {
        a.constant = __builtin_bit_cast(float, r.off_lo);
    } else {
        a.off = (uint64_t)r.off_lo | (uint64_t)r.off_hi << 32;
        a.W = r.wh & 0xFFFFu, a.H = r.wh >> 16, a.C = (r.mode >> 8) & 0xFFu;
    }
    return a;
}

// The alpha records of the alpha-tested triangles among the slots `geom`
// (flags in a.w already set), each slot's record index and coverage mask set
// (pt_device.h) and the mask words (amask).  Test hook output (may be null):
// per slot PT_ALPHA_HOOK_WORDS words: the set handle, then its accept and
// reject masks (each max(1, n n / 32) words, padded to 512).
#define PT_ALPHA_HOOK_WORDS 1025
static void alpha_records(const pt_scene_desc* s, std::vector<DevGeom>& geom, std::vector<DevAlpha>* alpha,
                          std::vector<uint32_t>* amask, uint32_t* hook) {
#ifndef PT_ALPHA_MAXN  // the finest coverage subdivision (pt_alpha_cov.h)
#define PT_ALPHA_MAXN 128
#endif
    PtAlphaCoverage cov(s->texels, s->texels ? s->n_texel_bytes : 0, PT_ALPHA_MAXN, PT_ALPHA_IL != 0);
    uint32_t n = 0;
    for (uint32_t i = 0; i < s->n_prims; i++) {
        uint32_t* h = hook ? hook + (size_t)PT_ALPHA_HOOK_WORDS * i : nullptr;
        if (h) std::fill(h, h + PT_ALPHA_HOOK_WORDS, 0u), h[0] = PT_ALPHA_SET_NONE;
        const uint32_t fl = __builtin_bit_cast(uint32_t, geom[i].a.w);
        if ((fl & GF_KIND) != PT_PRIM_TRIANGLE || !(fl & GF_ALPHA)) continue;
        DevAlpha r;
        const bool fast = n < ALPHA_IDX_NONE && alpha_record(s, s->prims[i], r);
        const uint32_t idx = fast ? n++ : ALPHA_IDX_NONE;
        const uint32_t set = PT_ALPHA_COV && fast ? cov.set(alpha_cov_record(r)) : PT_ALPHA_SET_NONE;
        geom[i].a.w = __builtin_bit_cast(float, (fl & 0x1Fu) | (idx >> 16) << 5 | (set & 0xFFFFu) << 16);
        geom[i].b.w = __builtin_bit_cast(float, (idx & 0xFFFFu) | (set & 0xFFFF0000u));
        if (h && set != PT_ALPHA_SET_NONE) {
            const int cn = 4 << (set >> 29), wpm = std::max(1, cn * cn / 32);
            const uint32_t* w = cov.words().data() + (set & 0x1FFFFFFFu);
            h[0] = set;
            for (int k = 0; k < std::min(wpm, 512); k++) {  // (the hook's rows hold n <= 128)
                h[1 + k] = PT_ALPHA_IL ? w[2 * k] : w[k];
                h[513 + k] = PT_ALPHA_IL ? w[2 * k + 1] : w[wpm + k];
            }
        }
        if (fast && alpha) alpha->push_back(r);
    }
    if (amask) *amask = cov.words();
}

struct Conv {
    const pt_scene_desc* s;
    std::vector<DevCluster>& nodes;
    std::vector<DevGeom>& geom;
    std::vector<uint32_t>& cbase;
    uint8_t lut[8][135];
    std::string err;

    uint32_t convert(const pt_ref_bvh4_node& desc, uint32_t b) {
        const pt_bvh_desc& B = s->bvhs[b];
        if (desc.active == 0) {
            if (desc.count == 0) return REF_EMPTY;
            uint64_t slot0 = (uint64_t)B.prim_base + desc.cluster_idx;
            uint64_t last = slot0 + desc.count - 1;
            if (last >= s->n_prims || desc.cluster_idx + desc.count > B.n_prims) {
                err = "leaf primitive range out of bounds";
                return REF_EMPTY;
            }
            uint32_t w = __builtin_bit_cast(uint32_t, geom[last].a.w) | GF_LAST;
            geom[last].a.w = __builtin_bit_cast(float, w);
            return REF_LEAF | (uint32_t)slot0;
        }
        if (desc.cluster_idx >= B.n_clusters) {
            err = "cluster index out of bounds";
            return REF_EMPTY;
        }
        const uint32_t gi = cbase[b] + desc.cluster_idx;
        const pt_ref_bvh4_cluster& rc = B.clusters[desc.cluster_idx];
        DevCluster& dc = nodes[gi];
        memcpy(&dc.xmin, rc.xmin, 16);
        memcpy(&dc.xmax, rc.xmax, 16);
        memcpy(&dc.ymin, rc.ymin, 16);
        memcpy(&dc.ymax, rc.ymax, 16);
        memcpy(&dc.zmin, rc.zmin, 16);
        memcpy(&dc.zmax, rc.zmax, 16);
        uint32_t perm = desc.perm < 135 ? desc.perm : 0;
        dc.order[0] = dc.order[1] = 0;
        for (int o = 0; o < 8; o++) dc.order[o >> 2] |= (uint32_t)lut[o][perm] << (8 * (o & 3));
        dc.pad[0] = perm;  // the topology code itself (the quantized records look the order up)
        dc.pad[1] = 0;
        for (int k = 0; k < 4; k++) dc.child[k] = REF_EMPTY;
        for (int k = 0; k < 4; k++) {
            pt_ref_bvh4_node ch = rc.children[k];
            uint32_t r = convert(ch, b);
            nodes[gi].child[k] = r;  // re-index: the vector is pre-sized, no reallocation
        }
        return gi;
    }
};

extern "C" pt_status pt_bvh4_order_table(uint8_t* out);

// ---- quantized 48-B records (pt_device.h): every BVH's root gets a record first;
// then, depth first from each root, a node's children get one contiguous
// block (an inner child one record, a leaf child a copy of its slots in leaf
// order, c.w = the slot) and the node record names them by base + offsets.
// A child that is another BVH's root (a lone BLAS hop resolved at upload) is
// a copy of that root's record.  BLAS-hop slots push the BLAS root's record.
// False (the scene keeps 64-B nodes) when a block offset or the record count
// does not fit.
// esc (the stackless any-hit traversal's escape links, pt_pool.h
// trace_any_stackless): per record, its node's parent record and child slot,
// (parent << 2 | k); ESC_EXIT for every BVH's root record; a copy of a BLAS
// root in a TLAS child block also carries ESC_BLAS (entering it enters the
// BLAS, whose shared children escape to the original root record).
static bool build_q48(const std::vector<DevCluster>& nodes, const std::vector<DevGeom>& geom,
                      const std::vector<uint32_t>& roots, uint32_t n_prims, std::vector<DevGeom>& rec,
                      std::vector<uint32_t>& qroots, std::vector<uint32_t>& esc) {
    rec.clear();
    rec.reserve(nodes.size() + n_prims + 16);
    esc.clear();
    std::vector<uint32_t> node_rec(nodes.size(), REF_EMPTY);
    std::vector<std::pair<uint32_t, uint32_t>> copies;  // (record, cluster whose record it repeats)
    std::vector<std::pair<uint32_t, uint32_t>> work;    // (cluster, its record)
    auto alloc = [&](uint32_t n) {
        const uint32_t b = (uint32_t)rec.size();
        rec.resize(rec.size() + n);
        esc.resize(rec.size(), 0u);
        return b;
    };
    auto leaf_len = [&](uint32_t slot) {
        uint32_t n = 0;
        for (uint32_t s = slot; s < n_prims; s++) {
            n++;
            if (__builtin_bit_cast(uint32_t, geom[s].a.w) & GF_LAST) break;
        }
        return n;
    };
    auto is_hop = [&](uint32_t slot, uint32_t len) {
        for (uint32_t s = slot; s < slot + len; s++)
            if ((__builtin_bit_cast(uint32_t, geom[s].a.w) & GF_KIND) == PT_PRIM_BLAS) return true;
        return false;
    };
    // cluster-space root refs -> record-space (BLAS-hop slots carry them)
    std::vector<std::pair<uint32_t, uint32_t>> root_map;
    std::vector<uint32_t> hops;  // records of BLAS-hop slots
    auto copy_leaf = [&](uint32_t slot, uint32_t len, uint32_t at) {
        for (uint32_t k = 0; k < len; k++) {
            DevGeom g = geom[slot + k];
            g.c.w = __builtin_bit_cast(float, slot + k);
            rec[at + k] = g;  // BLAS-hop roots patched below, once every root has its record
            if ((__builtin_bit_cast(uint32_t, g.a.w) & GF_KIND) == PT_PRIM_BLAS) hops.push_back(at + k);
        }
    };
    qroots.assign(roots.size(), REF_EMPTY);
    for (size_t b = 0; b < roots.size(); b++) {
        const uint32_t r = roots[b];
        if (r == REF_EMPTY || r >= REF_SPECIAL) continue;
        if (r & REF_LEAF) {
            const uint32_t slot = r & ~REF_LEAF, len = leaf_len(slot), at = alloc(len);
            copy_leaf(slot, len, at);
            qroots[b] = REF_LEAF | (is_hop(slot, len) ? REF_BLOCK : 0u) | at;
        } else {
            if (r >= nodes.size()) return false;
            if (node_rec[r] == REF_EMPTY) {
                node_rec[r] = alloc(1);
                esc[node_rec[r]] = ESC_EXIT;
                work.push_back({r, node_rec[r]});
            }
            qroots[b] = node_rec[r];
        }
        root_map.push_back({r, qroots[b]});
    }
    // depth-first: each node's subtree contiguous
    while (!work.empty()) {
        const auto [gi, r] = work.back();
        work.pop_back();
        const DevCluster& n = nodes[gi];
        uint32_t size[4] = {0, 0, 0, 0};
        for (int k = 0; k < 4; k++) {
            const uint32_t ch = n.child[k];
            if (ch == REF_EMPTY) continue;
            if (ch >= REF_SPECIAL) return false;
            size[k] = (ch & REF_LEAF) ? leaf_len(ch & ~REF_LEAF) : 1u;
        }
        const uint32_t total = size[0] + size[1] + size[2] + size[3];
        const uint32_t base = alloc(total);
        uint32_t desc = 0, off = 0;
        for (int k = 0; k < 4; k++) {
            const uint32_t ch = n.child[k];
            uint32_t d = Q48_EMPTY;
            if (ch != REF_EMPTY) {
                if (off > Q48_MAX_OFFSET) return false;
                d = off;
                if (ch & REF_LEAF) {
                    const uint32_t slot = ch & ~REF_LEAF;
                    copy_leaf(slot, size[k], base + off);
                    d |= Q48_LEAF | (is_hop(slot, size[k]) ? Q48_HOP : 0u);
                } else if (node_rec[ch] != REF_EMPTY) {  // another BVH's root: a copy of its record
                    copies.push_back({base + off, ch});
                    esc[base + off] = (r << 2) | (uint32_t)k | ESC_BLAS;
                } else {
                    node_rec[ch] = base + off;
                    esc[base + off] = (r << 2) | (uint32_t)k;
                    work.push_back({ch, base + off});
                }
                off += size[k];
            }
            desc |= d << (8 * k);
        }
        // the node record: the cluster's quantized boxes, perm, base, desc
        DevQNode q;
        if (!quantize_node(n, q)) return false;
        DevGeom& o = rec[r];
        o.a = q.a;
        o.a.w = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, q.a.w) | (n.pad[0] & 0xFFu) << 24);
        o.b = make_float4(__builtin_bit_cast(float, q.b[0]), __builtin_bit_cast(float, q.b[1]),
                          __builtin_bit_cast(float, q.b[2]), __builtin_bit_cast(float, q.b[3]));
        o.c = make_float4(__builtin_bit_cast(float, q.c[0]), __builtin_bit_cast(float, q.c[1]),
                          __builtin_bit_cast(float, base), __builtin_bit_cast(float, desc));
        if (rec.size() >= REF_BLOCK) return false;
    }
    for (const auto& [at, ci] : copies) rec[at] = rec[node_rec[ci]];
    // BLAS-hop slots push the BLAS root's record (instance hops keep REF_INST_ENTER | slot)
    for (uint32_t h : hops) {
        DevGeom& g = rec[h];
        const uint32_t tgt = __builtin_bit_cast(uint32_t, g.b.x);
        if (tgt >= REF_SPECIAL) continue;
        uint32_t q = REF_EMPTY;
        for (const auto& [cr, qr] : root_map)
            if (cr == tgt) q = qr;
        if (q == REF_EMPTY) return false;
        g.b.x = __builtin_bit_cast(float, q);
    }
    // one pad record: leaf steps may read the record after the last one
    rec.push_back(DevGeom{});
    esc.push_back(0u);
    return !rec.empty() && rec.size() < REF_BLOCK;
}

static pt_status upload_dev(pt_ctx* c, const pt_scene_desc* s);
extern "C" pt_status pt_scene_upload(pt_ctx* c, const pt_scene_desc* s) {
    if (!c) return PT_ERR_ARG;
    // every device holds a full replica (C4 ~1 GB of 288 GB)
    if (pt_status st = upload_dev(c, s)) return st;
    for (pt_ctx* p : c->peers)
        if (pt_status st = upload_dev(p, s)) return fail(c, st, "device %d: %s", p->device, p->err.c_str());
    return PT_OK;
}
// Validate a scene description (pt_scene_upload's checks, also the host
// hooks' that read it)
static pt_status validate_scene(pt_ctx* c, const pt_scene_desc* s) {
    if (s->n_bvhs == 0 || !s->bvhs || s->n_prims == 0 || !s->prims)
        return fail(c, PT_ERR_ARG, "scene needs a TLAS and primitives");
    // ---- validate
    for (uint32_t i = 0; i < s->n_prims; i++) {
        const pt_prim& p = s->prims[i];
        bool ok = true;
        switch (p.kind) {
            case PT_PRIM_TRIANGLE: ok = p.index < s->n_triangles; break;
            case PT_PRIM_QUAD: ok = p.index < s->n_quads; break;
            case PT_PRIM_SPHERE: ok = p.index < s->n_spheres; break;
            case PT_PRIM_BLAS: ok = p.index > 0 && p.index < s->n_bvhs; break;
            case PT_PRIM_INSTANCE: ok = p.index < s->n_instances && s->instances; break;
            default: ok = false;
        }
        if (!ok) return fail(c, PT_ERR_ARG, "primitive %u: bad kind/index", i);
        if (p.material >= (int32_t)s->n_materials) return fail(c, PT_ERR_ARG, "primitive %u: bad material", i);
        if (p.medium < -1 || p.medium >= (int32_t)s->n_media) return fail(c, PT_ERR_ARG, "primitive %u: bad medium", i);
        if (p.light >= (int32_t)s->n_lights) return fail(c, PT_ERR_ARG, "primitive %u: bad light", i);
    }
    for (uint32_t t = 0; t < s->n_triangles; t++)
        for (int k = 0; k < 3; k++)
            if (s->tri_vidx[3 * t + k] >= s->n_vertices) return fail(c, PT_ERR_ARG, "triangle %u: bad vertex", t);
    for (uint32_t l = 0; l < s->n_lights; l++) {
        const pt_light& L = s->lights[l];
        if (L.kind == PT_LIGHT_TEX_INF &&
            (L.prim < 0 || (uint64_t)L.prim + (uint64_t)PT_TEXINF_X * PT_TEXINF_Y > s->n_light_dist || !s->light_dist ||
             L.tex < 0 || (uint32_t)L.tex >= s->n_textures))
            return fail(c, PT_ERR_ARG, "light %u: bad texture infinite light", l);
        if (L.kind == PT_LIGHT_AREA && (L.prim < 0 || (uint32_t)L.prim >= s->n_prims || L.tex < 0 ||
                                        (uint32_t)L.tex >= s->n_textures || L.instance < -1 ||
                                        (L.instance >= 0 && (uint32_t)L.instance >= s->n_instances)))
            return fail(c, PT_ERR_ARG, "light %u: bad area light", l);
    }
    // (the texel lookups index an image's elements in 32 bits, and the alpha
    // test reads an image's texels without a bound check: each image must lie
    // inside the texel buffer)
    for (uint32_t k = 0; k < s->n_images; k++) {
        const pt_image& im = s->images[k];
        const uint64_t elems = (uint64_t)std::max(im.width, 0) * (uint64_t)std::max(im.height, 0) *
                               (uint64_t)std::max(im.channels, 0);
        if (im.width <= 0 || im.height <= 0 || im.channels <= 0 || elems >= (1ull << 32))
            return fail(c, PT_ERR_ARG, "image %u: bad size (%d x %d x %d channels; below 2^32 elements)", k,
                        im.width, im.height, im.channels);
        const uint64_t bytes = elems * (im.format == PT_IMAGE_F32 ? 4ull : 1ull);
        if (im.offset > s->n_texel_bytes || bytes > s->n_texel_bytes - im.offset)
            return fail(c, PT_ERR_ARG, "image %u: texels past the texel buffer", k);
    }
    for (uint32_t k = 0; k < s->n_textures; k++) {
        const pt_texture& T = s->textures[k];
        if (T.kind == PT_TEX_IMAGE && (T.image < 0 || (uint32_t)T.image >= s->n_images))
            return fail(c, PT_ERR_ARG, "texture %u: bad image", k);
        if (T.kind == PT_TEX_CHECKER && (T.a < 0 || T.b < 0 || (uint32_t)T.a >= s->n_textures ||
                                         (uint32_t)T.b >= s->n_textures))
            return fail(c, PT_ERR_ARG, "texture %u: bad checker child", k);
    }
    for (uint32_t m = 0; m < s->n_materials; m++) {
        const pt_material& M = s->materials[m];
        int ids[5] = {M.tex, M.norm, M.rough, M.metal, M.alpha};
        for (int id : ids)
            if (id >= (int32_t)s->n_textures) return fail(c, PT_ERR_ARG, "material %u: bad texture", m);
        if ((M.kind == PT_MAT_DIFFUSE || M.kind == PT_MAT_DIELECTRIC || M.kind == PT_MAT_THIN) && M.tex < 0)
            return fail(c, PT_ERR_ARG, "material %u: missing texture", m);
        if ((M.kind == PT_MAT_DIFFUSE) && (M.rough < 0 || M.metal < 0))
            return fail(c, PT_ERR_ARG, "material %u: missing roughness/metallic texture", m);
        if ((M.kind == PT_MAT_DIELECTRIC) && M.rough < 0) return fail(c, PT_ERR_ARG, "material %u: missing roughness", m);
    }
    for (uint32_t i = 0; i < s->n_sampler_lights; i++)
        if (s->sampler_lights[i] >= s->n_lights) return fail(c, PT_ERR_ARG, "sampler light %u out of range", i);
    if (s->n_media && !s->media) return fail(c, PT_ERR_ARG, "media array missing");
    if (s->n_media > PT_MAX_MEDIA) return fail(c, PT_ERR_ARG, "more than %d media", PT_MAX_MEDIA);
    if (s->n_prims > REF_SLOT_MASK) return fail(c, PT_ERR_ARG, "too many primitives");
    {  // instances: chains of levels (pt_instance.inner) ending at a BLAS
       // without instances / nested BLAS; the records the TLAS names take
       // ascending virtual ranges past the real slots, level records none
        if (s->n_instances && !s->instances) return fail(c, PT_ERR_ARG, "instances array missing");
        std::vector<uint8_t> is_level(s->n_instances, 0);
        for (uint32_t k = 0; k < s->n_instances; k++) {
            const int32_t in = s->instances[k].inner;
            if (in < -1 || (in >= 0 && ((uint32_t)in <= k || (uint32_t)in >= s->n_instances)))
                return fail(c, PT_ERR_ARG, "instance %u: bad inner level %d", k, in);
            if (in >= 0) is_level[in] = 1;
        }
        for (uint32_t i = 0; i < s->n_prims; i++)
            if (s->prims[i].kind == PT_PRIM_INSTANCE &&
                (s->prims[i].index >= s->n_instances || is_level[s->prims[i].index]))
                return fail(c, PT_ERR_ARG, "prim %u: bad instance %u", i, s->prims[i].index);
        uint64_t next = s->n_prims;
        for (uint32_t k = 0; k < s->n_instances; k++) {
            const pt_instance& I = s->instances[k];
            if (I.bvh == 0 || I.bvh >= s->n_bvhs) return fail(c, PT_ERR_ARG, "instance %u: bad bvh", k);
            const pt_bvh_desc& B = s->bvhs[I.bvh];
            if ((uint64_t)B.prim_base + B.n_prims > s->n_prims) return fail(c, PT_ERR_ARG, "instance %u: bad bvh", k);
            for (uint32_t j = B.prim_base; j < B.prim_base + B.n_prims; j++)
                if (s->prims[j].kind == PT_PRIM_BLAS || s->prims[j].kind == PT_PRIM_INSTANCE)
                    return fail(c, PT_ERR_ARG, "instance %u: nested instance", k);
            int depth = 1;
            for (int32_t in = I.inner; in >= 0; in = s->instances[in].inner, depth++)
                if (s->instances[in].bvh != I.bvh)
                    return fail(c, PT_ERR_ARG, "instance %u: level %d names another bvh", k, in);
            if (depth > PT_MAX_INSTANCE_DEPTH)
                return fail(c, PT_ERR_ARG, "instance %u: %d levels (at most %d)", k, depth, PT_MAX_INSTANCE_DEPTH);
            if (is_level[k]) continue;
            if (I.virt_base < next || (uint64_t)I.virt_base + B.n_prims > REF_SLOT_MASK)
                return fail(c, PT_ERR_ARG, "instance %u: bad virtual slot range", k);
            next = (uint64_t)I.virt_base + B.n_prims;
        }
    }
    if (s->scene_medium < -1 || s->scene_medium >= (int32_t)s->n_media) return fail(c, PT_ERR_ARG, "bad scene medium");
    for (uint32_t i = 0; i < s->n_infinite_lights; i++)
        if (s->infinite_lights[i] >= s->n_lights) return fail(c, PT_ERR_ARG, "infinite light %u out of range", i);
    return PT_OK;
}

// The primitive slots' geometry and flags (DevGeom, pt_device.h) and info
static void slot_geometry(const pt_scene_desc* s, std::vector<DevGeom>& geom, std::vector<DevPrimInfo>& info) {
    for (uint32_t i = 0; i < s->n_prims; i++) {
        const pt_prim& p = s->prims[i];
        uint32_t flags = p.kind;
        DevGeom g{};
        if (p.kind == PT_PRIM_TRIANGLE) {
            const uint32_t* v = s->tri_vidx + 3 * (size_t)p.index;
            const float* P0 = s->positions + 3 * (size_t)v[0];
            const float* P1 = s->positions + 3 * (size_t)v[1];
            const float* P2 = s->positions + 3 * (size_t)v[2];
            g.a = make_float4(P0[0], P0[1], P0[2], 0);
            g.b = make_float4(P1[0] - P0[0], P1[1] - P0[1], P1[2] - P0[2], 0);  // edge1 = vert1 - vert0
            g.c = make_float4(P2[0] - P0[0], P2[1] - P0[1], P2[2] - P0[2], 0);  // edge2 = vert2 - vert0
        } else if (p.kind == PT_PRIM_QUAD) {
            const pt_quad& q = s->quads[p.index];
            g.a = make_float4(q.Q[0], q.Q[1], q.Q[2], 0);
            g.b = make_float4(q.u[0], q.u[1], q.u[2], 0);
            g.c = make_float4(q.v[0], q.v[1], q.v[2], 0);
        } else if (p.kind == PT_PRIM_SPHERE) {
            const pt_sphere& sp = s->spheres[p.index];
            g.a = make_float4(sp.center[0], sp.center[1], sp.center[2], 0);
            g.b = make_float4(sp.radius, 0, 0, 0);
        }
        if (p.kind == PT_PRIM_INSTANCE) flags = PT_PRIM_BLAS;  // device: a hop that pushes REF_INST_ENTER | slot
        if (p.kind != PT_PRIM_BLAS && p.kind != PT_PRIM_INSTANCE) material_alpha_flags(s, p.material, flags);
        g.a.w = __builtin_bit_cast(float, flags);
        geom[i] = g;
        info[i] = DevPrimInfo{p.material, p.light, p.medium, p.index};
    }
}

static pt_status upload_dev(pt_ctx* c, const pt_scene_desc* s) {
    if (!c || !s) return PT_ERR_ARG;
    DeviceLock dl(c->device);
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    free_scene(c);
    if (pt_status st = validate_scene(c, s)) return st;

    // ---- geometry slots
    // one zero pad slot past the end: pool leaf steps read slot + 1 unconditionally
    std::vector<DevGeom> geom(s->n_prims + 1);
    std::vector<DevPrimInfo> info(s->n_prims);
    slot_geometry(s, geom, info);
    // ---- alpha records of the alpha-tested triangles and their coverage
    // masks (pt_device.h alpha_index / alpha_cell, pt_alpha_cov.h)
    std::vector<DevAlpha> alpha;
    std::vector<uint32_t> amask;
    alpha_records(s, geom, &alpha, &amask, nullptr);
    if (amask.empty()) amask.push_back(0);
    // ---- nodes: TLAS then every BLAS, converted from the root descriptors
    std::vector<uint32_t> cbase(s->n_bvhs);
    uint64_t total = 0;
    for (uint32_t b = 0; b < s->n_bvhs; b++) {
        cbase[b] = (uint32_t)total;
        total += s->bvhs[b].n_clusters;
        if (s->bvhs[b].n_clusters && !s->bvhs[b].clusters) return fail(c, PT_ERR_ARG, "bvh %u: no clusters", b);
        if ((uint64_t)s->bvhs[b].prim_base + s->bvhs[b].n_prims > s->n_prims)
            return fail(c, PT_ERR_ARG, "bvh %u: primitive range out of bounds", b);
    }
    if (total >= REF_LEAF) return fail(c, PT_ERR_ARG, "too many clusters");
    std::vector<DevCluster> nodes(std::max<uint64_t>(total, 1));
    Conv cv{s, nodes, geom, cbase, {}, {}};
    pt_bvh4_order_table(&cv.lut[0][0]);
    std::vector<uint32_t> roots(s->n_bvhs);
    for (uint32_t b = 0; b < s->n_bvhs; b++) {
        roots[b] = cv.convert(s->bvhs[b].root, b);
        if (!cv.err.empty()) return fail(c, PT_ERR_ARG, "bvh %u: %s", b, cv.err.c_str());
    }
    for (uint32_t i = 0; i < s->n_prims; i++) {
        if (s->prims[i].kind == PT_PRIM_BLAS) {
            geom[i].b.x = __builtin_bit_cast(float, roots[s->prims[i].index]);
            info[i].index = roots[s->prims[i].index];
        } else if (s->prims[i].kind == PT_PRIM_INSTANCE) {
            geom[i].b.x = __builtin_bit_cast(float, REF_INST_ENTER | i);
            geom[i].b.y = __builtin_bit_cast(float, s->prims[i].index);
        }
    }
    // A leaf holding nothing but one BLAS hop (Scene -> Model, Scene.cpp:4-6)
    // only pushes that BLAS's root: the cluster refers to the root directly,
    // in the leaf's place, so the traversal visits the same nodes in the same
    // order one step sooner.
    for (DevCluster& n : nodes)
        for (int k = 0; k < 4; k++) {
            const uint32_t r = n.child[k];
            if (r == REF_EMPTY || !(r & REF_LEAF) || r >= REF_SPECIAL) continue;
            const uint32_t slot = r & ~REF_LEAF;
            if (slot >= s->n_prims || s->prims[slot].kind != PT_PRIM_BLAS) continue;
            if (!(__builtin_bit_cast(uint32_t, geom[slot].a.w) & GF_LAST)) continue;
            n.child[k] = __builtin_bit_cast(uint32_t, geom[slot].b.x);
        }
    std::vector<DevInstance> inst(s->n_instances);
    for (uint32_t k = 0; k < s->n_instances; k++) {
        const pt_instance& I = s->instances[k];
        DevInstance& D = inst[k];
        std::memcpy(D.T, I.transform, sizeof(D.T));
        std::memcpy(D.inv, I.inv, sizeof(D.inv));
        D.root = roots[I.bvh];
        D.qroot = REF_EMPTY;  // the quantized records: set with them
        D.prim_base = s->bvhs[I.bvh].prim_base;
        D.n_prims = s->bvhs[I.bvh].n_prims;
        D.virt_base = I.virt_base;
        D.inner = I.inner;
        D.anim = I.animated ? 1u : 0u;
        for (int j = 0; j < 3; j++) D.mdir[j] = I.motion[j];
        D.t0 = I.time_bounds[0];
        D.t1 = I.time_bounds[1];
    }
    // level records own no virtual slots: the hit's instance lookup
    // (hit_surface) finds the chain's outermost record
    for (uint32_t k = 0; k < s->n_instances; k++)
        if (s->instances[k].inner >= 0) inst[s->instances[k].inner].n_prims = 0;
    // ---- triangles: vertex indices + flags as uint4
    std::vector<uint4> tri(s->n_triangles);
    for (uint32_t t = 0; t < s->n_triangles; t++)
        tri[t] = make_uint4(s->tri_vidx[3 * t], s->tri_vidx[3 * t + 1], s->tri_vidx[3 * t + 2],
                            s->tri_flags ? s->tri_flags[t] : 0u);
    // ---- light sampler running sums (PowerLightSampler::Sample order)
    std::vector<float> cdf(s->n_sampler_lights);
    float acc = 0;
    for (uint32_t i = 0; i < s->n_sampler_lights; i++) {
        acc += s->lights[s->sampler_lights[i]].power;
        cdf[i] = acc;
    }
    DevScene& DS = c->scene;
    DS = DevScene{};
    pt_status st;
#define UP(dst, src, n) \
    if ((st = upload(c, src, n, &dst)) != PT_OK) return st;
    UP(DS.nodes, nodes.data(), nodes.size());
    {
        // nodes and leaf slots in one array of 48-B records (pt_device.h)
        std::vector<DevGeom> rec;
        std::vector<uint32_t> qroots, esc;
        bool ok = nodes.size() < REF_BLOCK && s->n_prims < REF_BLOCK &&
                  build_q48(nodes, geom, roots, s->n_prims, rec, qroots, esc);
        // 32-bit buffer offsets (pt_pool.h q48_buf_load) below the out-of-range marker
        if (ok && rec.size() * sizeof(DevGeom) >= (uint64_t)Q48_OOB_OFFSET) ok = false;
        DS.qrec_bytes = ok ? (uint32_t)(rec.size() * sizeof(DevGeom)) : 0u;
        c->has_qnodes = ok;
        if (ok) {
            UP(DS.qrec, rec.data(), rec.size());
            UP(DS.qesc, esc.data(), esc.size());
            DS.qroot = qroots[0];
            for (uint32_t k = 0; k < s->n_instances; k++) inst[k].qroot = qroots[s->instances[k].bvh];
            std::vector<uint32_t> lut(8 * Q48_LUT_STRIDE / 4, 0u);
            for (int o = 0; o < 8; o++)
                for (int p = 0; p < 135; p++)
                    reinterpret_cast<uint8_t*>(lut.data())[o * Q48_LUT_STRIDE + p] = cv.lut[o][p];
            UP(DS.qlut, lut.data(), lut.size());
        }
    }
    UP(DS.geom, geom.data(), geom.size());
    UP(DS.info, info.data(), info.size());
    UP(DS.tri, tri.data(), tri.size());
    UP(DS.positions, s->positions, 3 * (size_t)s->n_vertices);
    UP(DS.normals, s->normals, 3 * (size_t)s->n_vertices);
    UP(DS.uvs, s->uvs, 2 * (size_t)s->n_vertices);
    UP(DS.tangents, s->tangents, s->tangents ? 3 * (size_t)s->n_vertices : 0);
    UP(DS.tshade, (const DevTriShade*)nullptr, s->n_prims);  // per slot (k_tri_shade)
    UP(DS.alpha, alpha.data(), alpha.size());
    UP(DS.amask, amask.data(), amask.size());
    if (s->n_triangles) {
        hipLaunchKernelGGL(k_tri_shade, dim3((s->n_prims + 255) / 256), dim3(256), 0, c->stream, DS.geom, DS.info,
                           DS.tri, DS.normals, DS.uvs, s->tangents ? DS.tangents : nullptr, s->n_prims,
                           const_cast<DevTriShade*>(DS.tshade));
        HIPCHK(c, hipGetLastError());
        HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    UP(DS.quads, s->quads, s->n_quads);
    UP(DS.spheres, s->spheres, s->n_spheres);
    UP(DS.materials, s->materials, s->n_materials);
    UP(DS.textures, s->textures, s->n_textures);
    UP(DS.images, s->images, s->n_images);
    for (uint32_t k = 0; k < s->n_textures; k++) {
        const pt_texture& t = s->textures[k];
        if (t.kind != PT_TEX_SOLID && t.kind != PT_TEX_CHECKER) {
            const pt_image& im = s->images[t.image];  // (validated above)
            if (im.channels < 0 || im.channels > 0xFFFF || im.format < 0 || im.format > 0xFF)
                return fail(c, PT_ERR_ARG, "image %d: bad channels / format", t.image);
        }
    }
    // texels: 16 bytes of padding for the word loads of texel_pair_u8
    if ((st = upload(c, s->texels, s->n_texel_bytes, &DS.texels, 16)) != PT_OK) return st;
    UP(DS.lights, s->lights, s->n_lights);
    {  // each triangle area light's vertices and uvs (DevLightTri), beside its light record
        std::vector<DevLightTri> lt(std::max<uint32_t>(s->n_lights, 1));
        for (uint32_t k = 0; k < s->n_lights; k++) {
            const pt_light& L = s->lights[k];
            lt[k] = DevLightTri{};
            if (L.kind != PT_LIGHT_AREA || !s->uvs) continue;
            const pt_prim& p = s->prims[L.prim];
            if (p.kind != PT_PRIM_TRIANGLE) continue;
            const uint32_t* v = s->tri_vidx + 3 * (size_t)p.index;
            const float* P0 = s->positions + 3 * (size_t)v[0];
            const float* P1 = s->positions + 3 * (size_t)v[1];
            const float* P2 = s->positions + 3 * (size_t)v[2];
            const float* U0 = s->uvs + 2 * (size_t)v[0];
            const float* U1 = s->uvs + 2 * (size_t)v[1];
            const float* U2 = s->uvs + 2 * (size_t)v[2];
            lt[k].a = make_float4(P0[0], P0[1], P0[2], U0[0]);
            lt[k].b = make_float4(P1[0], P1[1], P1[2], U1[0]);
            lt[k].c = make_float4(P2[0], P2[1], P2[2], U2[0]);
            lt[k].d = make_float4(U0[1], U1[1], U2[1], __builtin_bit_cast(float, 1u));
        }
        UP(DS.ltri, lt.data(), lt.size());
    }
    UP(DS.sampler_lights, s->sampler_lights, s->n_sampler_lights);
    UP(DS.sampler_cdf, cdf.data(), cdf.size());
    {  // guide table (pt_device.h PT_LS_GUIDE): bucket b starts at the first
       // running sum >= fl(b / K * total), computed in float like ls_sample
        std::vector<uint32_t> guide(PT_LS_GUIDE + 1);
        uint32_t i = 0;
        for (uint32_t b = 0; b <= PT_LS_GUIDE; b++) {
            const float lo = b == PT_LS_GUIDE ? std::numeric_limits<float>::infinity()
                                              : ((float)b / (float)PT_LS_GUIDE) * acc;
            while (i < cdf.size() && !(cdf[i] >= lo)) i++;
            guide[b] = b == PT_LS_GUIDE ? (uint32_t)cdf.size() : i;
        }
        UP(DS.sampler_guide, guide.data(), guide.size());
    }
    UP(DS.infinite_lights, s->infinite_lights, s->n_infinite_lights);
    UP(DS.light_dist, s->light_dist, s->n_light_dist);
    UP(DS.media, s->media, s->n_media);
    UP(DS.instances, inst.data(), inst.size());
#undef UP
    DS.root = roots[0];
    DS.n_prims = s->n_prims;
    {  // scene box from the TLAS root cluster's child boxes (spatial hit sort)
        float lo[3] = {0, 0, 0}, hi[3] = {1, 1, 1};
        const pt_bvh_desc& T = s->bvhs[0];
        if (T.root.count == 0 && T.n_clusters > 0 && T.root.cluster_idx < T.n_clusters) {
            const pt_ref_bvh4_cluster& cl = T.clusters[T.root.cluster_idx];
            const float* mn[3] = {cl.xmin, cl.ymin, cl.zmin};
            const float* mx[3] = {cl.xmax, cl.ymax, cl.zmax};
            bool any = false;
            for (int k = 0; k < 4; k++) {
                bool ok = true;
                for (int a = 0; a < 3; a++) ok = ok && std::isfinite(mn[a][k]) && std::isfinite(mx[a][k]) && mn[a][k] <= mx[a][k];
                if (!ok) continue;
                for (int a = 0; a < 3; a++) {
                    lo[a] = any ? std::min(lo[a], mn[a][k]) : mn[a][k];
                    hi[a] = any ? std::max(hi[a], mx[a][k]) : mx[a][k];
                }
                any = true;
            }
        }
        for (int a = 0; a < 3; a++) {
            DS.bb_lo[a] = lo[a];
            DS.bb_scale[a] = hi[a] > lo[a] ? (float)(1 << PT_SORT_CELL_BITS) / (hi[a] - lo[a]) : 0.0f;
        }
    }
    DS.prim_cell = nullptr;
    if (s->n_prims) {  // each primitive's centroid cell, hit_cell's Morton code
        std::vector<uint16_t> cell(s->n_prims, 0);
        auto code = [&](const float* p) {
            uint32_t m = 0;
            for (int a = 0; a < 3; a++) {
                const float q = (p[a] - DS.bb_lo[a]) * DS.bb_scale[a];
                const uint32_t c = (uint32_t)std::min(std::max(q, 0.0f), (float)((1 << PT_SORT_CELL_BITS) - 1));
                for (int b = 0; b < PT_SORT_CELL_BITS; b++) m |= ((c >> b) & 1u) << (3 * b + a);
            }
            return (uint16_t)m;
        };
        for (uint32_t i = 0; i < s->n_prims; i++) {
            const pt_prim& pr = s->prims[i];
            float c[3];
            if (pr.kind == PT_PRIM_TRIANGLE) {
                const uint32_t* v = s->tri_vidx + 3 * (size_t)pr.index;
                for (int a = 0; a < 3; a++)
                    c[a] = (s->positions[3 * (size_t)v[0] + a] + s->positions[3 * (size_t)v[1] + a] +
                            s->positions[3 * (size_t)v[2] + a]) * (1.0f / 3.0f);
            } else if (pr.kind == PT_PRIM_QUAD) {
                const pt_quad& q = s->quads[pr.index];
                for (int a = 0; a < 3; a++) c[a] = q.Q[a] + 0.5f * (q.u[a] + q.v[a]);
            } else if (pr.kind == PT_PRIM_SPHERE) {
                for (int a = 0; a < 3; a++) c[a] = s->spheres[pr.index].center[a];
            } else {
                continue;  // a hop or an instance: never a hit's slot
            }
            cell[i] = code(c);
        }
        if ((st = upload(c, cell.data(), cell.size(), &DS.prim_cell)) != PT_OK) return st;
    }
    DS.n_nodes = (uint32_t)nodes.size();
    DS.n_texel_bytes = s->n_texel_bytes;
    DS.n_lights = s->n_lights;
    DS.light_sampler = s->light_sampler;
    DS.n_sampler_lights = s->n_sampler_lights;
    DS.sampler_total = acc;
    DS.n_infinite_lights = s->n_infinite_lights;
    DS.n_media = s->n_media;
    DS.scene_medium = s->scene_medium;
    DS.n_instances = s->n_instances;
    DS.motion = 0;  // an AnimatedPrimitive: rays carry their time (DevScene::motion)
    for (uint32_t k = 0; k < s->n_instances; k++)
        if (s->instances[k].animated) DS.motion = 1;
    DS.scratch = nullptr;
    DS.scratch_lanes = 0;
    DS.stack_drops = c->stack_drops;
    DS.tie_drops = c->stack_drops + 1;
    DS.n_materials = s->n_materials;
    DS.n_textures = s->n_textures;
    DS.n_images = s->n_images;
    c->has_scene = true;
    c->n_media = s->n_media;
    c->n_materials = s->n_materials;
    c->n_clusters = nodes.size();
    return PT_OK;
}

static bool is_device_ptr(const void* p) {
    if (!p) return false;
    hipPointerAttribute_t a;
    hipError_t e = hipPointerGetAttributes(&a, p);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeDevice;
}

template <class T>
static pt_status ensure(pt_ctx* c, T** p, uint64_t& cap, uint64_t n) {
    if (cap >= n && *p) return PT_OK;
    if (*p) hipFree(*p);
    *p = nullptr;
    cap = 0;
    if (hipMalloc((void**)p, std::max<uint64_t>(n, 4) * sizeof(T)) != hipSuccess)
        return fail(c, PT_ERR_OOM, "hipMalloc(%llu) failed", (unsigned long long)(n * sizeof(T)));
    cap = n;
    return PT_OK;
}

static pt_status ensure_work(pt_ctx* c, uint32_t cap) {
    if (c->cap >= cap) return PT_OK;
    free_work(c);
    size_t n = cap;
#define AL(p, bytes)                                                                         \
    if (hipMalloc((void**)&(p), (bytes)) != hipSuccess) {                                    \
        free_work(c);                                                                        \
        return fail(c, PT_ERR_OOM, "wavefront allocation of %zu paths failed", (size_t)n); \
    }
    for (PathSoA* P : {&c->PA, &c->PB}) {
        P->cap = (uint32_t)n;
        // {o, d} and {beta, L}: two 32-B records per path (pt_kernels.h PathSoA)
        AL(P->o.p, n * 32);
        P->d.p = P->o.p + 1;
        AL(P->beta.p, n * 32);
        P->L.p = P->beta.p + 1;
        AL(P->sid, n * 4);
    }
    AL(c->hit, n * 16);
    AL(c->ties, n * 4);  // a ray is listed at most once per launch
    // three counter sets, then pt_trace's pool and its tie count
    AL(c->qcnt, (3 * SET_WORDS + PT_POOL_WORDS + Q_STRIDE) * 4);
    AL(c->sq, n * sizeof(ShadowRecV));  // the larger record (VolPath's)
    AL(c->counters, (CNT_SHARDS + 1) * CNT_COUNT * 8);
    // stack entries past the LDS part: the pool kernels' resident grid x
    // (PT_POOL_STACK - their smaller LDS part); the one-ray-per-lane kernels
    // keep their whole stack in LDS unless PT_SIMPLE_LN splits it, and then
    // the array covers their grid (the capacity) too
    {
        constexpr bool simple_ovf = PT_SIMPLE_LN < PT_STACK;
        constexpr int ovf_entries = PT_POOL_STACK - std::min(PT_POOL_LDS, PT_SIMPLE_LN);
        size_t lanes = (size_t)c->trace_blocks * PT_TRACE_BLOCK;
        if (simple_ovf) lanes = std::max<size_t>(lanes, (n + PT_TRACE_BLOCK - 1) / PT_TRACE_BLOCK * PT_TRACE_BLOCK);
        const size_t half = lanes * ovf_entries;
        AL(c->ovf, 2 * half * 4);
        c->ovf_any = c->ovf + half;
    }
#undef AL
    if (hipMemset(c->qcnt, 0, (3 * SET_WORDS + PT_POOL_WORDS + Q_STRIDE) * 4) != hipSuccess) {
        free_work(c);
        return fail(c, PT_ERR_HIP, "hipMemset of the queue counters failed");
    }
    c->cap = cap;
    return PT_OK;
}

// Ray-time buffers of a scene with an AnimatedPrimitive (DevScene::motion):
// each path's time (PA / PB.time, ping-pong with the path state) and each
// queued shadow ray's (sq_time), sized with the wavefront; none otherwise.
static pt_status ensure_motion(pt_ctx* c) {
    if (c->scene.motion && c->cap && !(c->PA.time && c->PB.time && c->sq_time)) {
        for (float** p : {&c->PA.time, &c->PB.time, &c->sq_time})
            if (!*p && hipMalloc((void**)p, (size_t)c->cap * sizeof(float)) != hipSuccess) {
                (void)hipGetLastError();
                return fail(c, PT_ERR_OOM, "ray-time buffers of %u paths", c->cap);
            }
    }
    c->scene.sq_time = c->scene.motion ? c->sq_time : nullptr;
    return PT_OK;
}

// Frees every buffer sized by the wavefront's path count (alloc_paths' OOM retry).
static void free_paths(pt_ctx* c) {
    free_work(c);
    struct Buf {
        void** p;
        uint64_t* cap;
    } bufs[] = {{(void**)&c->sort_order, &c->sort_order_cap}, {(void**)&c->sort_bins, &c->sort_bins_cap},
                {(void**)&c->ray_order, &c->ray_order_cap}, {(void**)&c->nee_jobs, &c->nee_jobs_cap}};
    for (const Buf& b : bufs) {
        if (*b.p) hipFree(*b.p);
        *b.p = nullptr;
        *b.cap = 0;
    }
}

static double mitchell_int(float rx, float ry) { return rx * ry / 4.0; }
static double gauss_h(double x, double sigma) {
    return 0.56418958354775628695 / (sigma * 1.41421356237309504880) * std::exp(-(x * x) / (2 * sigma * sigma));
}

// Core loop shared by pt_render / pt_render_samples.  Renders local sample
// chunks; after each chunk either gathers into `film` (device) or hands the
// chunk's per-sample radiance to `on_chunk`.
// Makes this context's scene the one the kernels read (constant-memory `S`),
// ordered on the context's stream.  Called by every entry point that launches.
// Large scenes keep 128 M paths in flight and a whole 1024-spp 1080p frame in
// one sample chunk (≈ 52 GB of HBM): each traversal launch's tail is
// amortised over more rays and the spatial hit sort finds more rays per cell
// (C4: 16 M / 6 GiB 931 -> 64 M / 32 GiB 1015 -> 128 M / 32 GiB 1027 Mrays/s,
// profiles/r02_ab_c4.txt)
#ifndef PT_SAMPLE_GIB
#define PT_SAMPLE_GIB 32
#endif
// r04 (alpha records, tail kernel): 128 M 1655 -> 256 M 1671 -> 384 M 1673
// -> 512 M 1678 Mrays/s (≈ 150 GB of HBM with the sample chunk; 64 M 1619;
// profiles/r04_ab_traversal.txt); r06: 768 M 2145.4 vs 512 M 2136.3
// (≈ 210 GB; profiles/r06_ab_misc.txt).  A device short of memory halves it
#ifndef PT_PATHS_POOL
#define PT_PATHS_POOL (3u << 28)
#endif
#ifndef PT_PATHS_SIMPLE
#define PT_PATHS_SIMPLE (1u << 21)
#endif
#define PT_POOL_MIN_CLUSTERS (1u << 20)  // measured: C4 (2.6M clusters) gains 31%; 0.5M-cluster heightfield and C2/C3 lose

// Per-lane scratch rows for instance traversal (scenes with instances only):
// enough for the largest grid a traversal kernel launches with (the pool grid,
// the one-ray-per-lane grid of the wavefront, or a test hook's `lanes`).
static pt_status ensure_scratch(pt_ctx* c, uint64_t lanes) {
    if (c->scene.n_instances == 0) return PT_OK;
    lanes = std::max<uint64_t>({lanes, (uint64_t)c->trace_blocks * PT_TRACE_BLOCK,
                                (uint64_t)(c->cap + PT_TRACE_BLOCK - 1) / PT_TRACE_BLOCK * PT_TRACE_BLOCK});
    if (lanes <= c->scratch_lanes) return PT_OK;
    if (c->scratch) {
        HIPCHK(c, hipStreamSynchronize(c->stream));
        hipFree(c->scratch);
        c->scratch = nullptr;
        c->scratch_lanes = 0;
    }
    if (hipMalloc((void**)&c->scratch, lanes * SCR_WORDS * 4) != hipSuccess)
        return fail(c, PT_ERR_OOM, "instance scratch of %llu lanes", (unsigned long long)lanes);
    c->scratch_lanes = lanes;
    return PT_OK;
}

static pt_status ensure_motion(pt_ctx* c);
static pt_status bind_scene(pt_ctx* c, uint64_t lanes = 0) {
    if (pt_status st = ensure_scratch(c, lanes)) return st;
    if (pt_status st = ensure_motion(c)) return st;
    c->scene.scratch = c->scratch;
    c->scene.scratch_lanes = (uint32_t)c->scratch_lanes;
    HIPCHK(c, hipMemcpyToSymbolAsync(HIP_SYMBOL(S), &c->scene, sizeof(DevScene), 0, hipMemcpyHostToDevice, c->stream));
    return PT_OK;
}

// traversal kernel of one wavefront iteration
using ClosestFn = void (*)(PathSoA, const uint32_t*, float4*, uint32_t*, uint32_t*, uint32_t*, uint32_t*,
                           unsigned long long*, uint32_t*);
using ShadowFn = void (*)(PathSoA, float*, ShadowRec*, const uint32_t*, uint32_t*, uint32_t*,
                          unsigned long long*);
template <bool C, bool I>
static ClosestFn closest_fn(bool pool, bool qn) {
    return pool ? (qn ? k_closest_pool<C, I, true> : k_closest_pool<C, I, false>) : k_closest<C, I>;
}
template <bool C, bool I>
static ShadowFn shadow_fn(bool pool, bool qn) {
    return pool ? (qn ? k_shadow_pool<C, I, true> : k_shadow_pool<C, I, false>) : k_shadow<C, I>;
}
static ClosestFn pick_closest(bool pool, bool qn, bool inst, bool count) {
    return inst ? (count ? closest_fn<true, true>(pool, qn) : closest_fn<false, true>(pool, qn))
                : (count ? closest_fn<true, false>(pool, qn) : closest_fn<false, false>(pool, qn));
}
static ShadowFn pick_shadow(bool pool, bool qn, bool inst, bool count) {
    return inst ? (count ? shadow_fn<true, true>(pool, qn) : shadow_fn<false, true>(pool, qn))
                : (count ? shadow_fn<true, false>(pool, qn) : shadow_fn<false, false>(pool, qn));
}

// `drive(R, spp_local, s_chunk, trace)` decides which sample chunks are traced:
// trace(R) runs the wavefront over R's work pixels x samples [s_lo, s_hi) and
// leaves their radiance in c->sample_L (sample-major, R.npix_work per index).
template <class Drive>
static pt_status run(pt_ctx* c, const pt_camera_desc* cam, const pt_render_desc* rd, pt_stats* stats, Drive drive) {
    if (pt_status bs = bind_scene(c)) return bs;
    c->frame.valid = false;  // sample_L is about to be rewritten
    const uint32_t W = (uint32_t)cam->width, H = (uint32_t)cam->height;
    RenderParams R{};
    R.cam = *cam;
    R.seed = rd->seed;
    R.max_depth = rd->max_depth;
    R.strata_x = rd->strata[0];
    R.strata_y = rd->strata[1];
    R.shard_count = rd->shard_count ? rd->shard_count : 1;
    R.shard_index = rd->shard_index;
    if (R.shard_index >= R.shard_count) return fail(c, PT_ERR_ARG, "shard_index >= shard_count");
    if (rd->flags & PT_RENDER_ADAPTIVE) {  // adaptive: shards own whole pixels (32x32 tiles), not samples
        R.shard_index = 0;
        R.shard_count = 1;
    }
    if (rd->max_depth > PF_DEPTH_MASK - 1) return fail(c, PT_ERR_ARG, "max_depth too large");
    const bool ranged = !(rd->pixel_begin == 0 && rd->pixel_end == 0);
    if (ranged) {
        if (rd->pixel_end <= rd->pixel_begin || rd->pixel_end > W * H) return fail(c, PT_ERR_ARG, "bad pixel range");
        R.pixel_begin = rd->pixel_begin;
        R.npix_work = rd->pixel_end - rd->pixel_begin;
        R.tiled = 0;
    } else {
        R.npix_work = W * H;
        R.tiled = (W % 8 == 0 && H % 8 == 0) ? 1u : 0u;
        R.tiles_x = W / 8;
    }
    R.filter = rd->filter;
    R.frad[0] = rd->filter_radius[0];
    R.frad[1] = rd->filter_radius[1];
    R.fparam[0] = rd->filter_params[0];
    R.fparam[1] = rd->filter_params[1];
    R.rad_x = (int)std::ceil(rd->filter_radius[0] - 0.5f);
    R.rad_y = (int)std::ceil(rd->filter_radius[1] - 0.5f);
    double integral;
    if (rd->filter == PT_FILTER_BOX) integral = 4 * rd->filter_radius[0] * rd->filter_radius[1];
    else if (rd->filter == PT_FILTER_GAUSSIAN) {
        double sg = rd->filter_params[0];
        R.gauss_x = gauss_h(rd->filter_radius[0], sg);
        R.gauss_y = gauss_h(rd->filter_radius[1], sg);
        double s2 = sg * 1.41421356237309504880;
        double ix = 0.5 * (std::erf(rd->filter_radius[0] / s2) - std::erf(-rd->filter_radius[0] / s2));
        double iy = 0.5 * (std::erf(rd->filter_radius[1] / s2) - std::erf(-rd->filter_radius[1] / s2));
        integral = (ix - 2 * rd->filter_radius[0] * R.gauss_x) * (iy - 2 * rd->filter_radius[1] * R.gauss_y);
    } else if (rd->filter == PT_FILTER_LANCZOS) integral = rd->filter_params[1];  // the host object's Integral()
    else integral = mitchell_int(rd->filter_radius[0], rd->filter_radius[1]);
    R.inv_integral = 1.0 / integral;

    const uint32_t spp_local = rd->spp > R.shard_index ? (rd->spp - R.shard_index + R.shard_count - 1) / R.shard_count : 0;
    // sample chunk: keep the per-sample radiance buffer <= PT_SAMPLE_GIB
    const uint64_t max_floats = (uint64_t)PT_SAMPLE_GIB << 28;
    uint64_t per_s = 3ull * R.npix_work;
    uint32_t s_chunk = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(spp_local, max_floats / per_s));
    // a chunk's sample ids stay below the shadow records' flag bits: a
    // finished path's pending shadow record carries SHADOW_DONE_BIT | sid, and
    // VolPath's also SHADOW_MLE_BIT (pt_kernels.hip)
    const uint64_t sid_limit = rd->integrator == PT_INTEGRATOR_VOLPATH ? SHADOW_MLE_BIT : SHADOW_DONE_BIT;
    if ((uint64_t)R.npix_work >= sid_limit) return fail(c, PT_ERR_ARG, "film too large for the sample ids");
    s_chunk = (uint32_t)std::min<uint64_t>(s_chunk, (sid_limit - 1ull) / R.npix_work);
    // test hook: a smaller chunk (a frame in several chunks at test sizes)
    if (const char* e = getenv("PT_SAMPLE_CHUNK")) s_chunk = std::max(1u, std::min<uint32_t>(s_chunk, (uint32_t)atoi(e)));
    pt_status st;
    // a device with less free HBM (or a second context on it) gets smaller
    // chunks instead of PT_ERR_OOM
    while ((st = ensure(c, &c->sample_L, c->sample_cap, per_s * s_chunk)) == PT_ERR_OOM && s_chunk > 1) {
        (void)hipGetLastError();
        s_chunk = (s_chunk + 1) / 2;
    }
    if (st) return st;
    // wavefront size: large scenes (pool traversal) take 128 M paths in flight,
    // so each traversal launch's tail (the last, longest rays) is amortised
    // over more rays (C4 at 256 spp: 2 M -> 8 M paths +22 %, 8 M -> 16 M +5 %;
    // with the spatial hit sort at 1024 spp 16 M -> 128 M +10 %)
    const bool big_scene = c->n_clusters >= PT_POOL_MIN_CLUSTERS;
    uint32_t paths = rd->paths_in_flight ? rd->paths_in_flight : (big_scene ? PT_PATHS_POOL : PT_PATHS_SIMPLE);
    paths = (uint32_t)std::min<uint64_t>(paths, std::max<uint64_t>(1, (uint64_t)R.npix_work * s_chunk));
    paths = (paths + 255) & ~255u;
    const bool count = (rd->flags & PT_RENDER_COUNT_NODES) != 0;
    // traversal variant: pool (persistent, refilling) for deep trees where ray
    // lengths diverge, one ray per lane for small ones; flags override
    const bool use_pool = (rd->flags & PT_RENDER_TRAVERSAL_POOL)     ? true
                          : (rd->flags & PT_RENDER_TRAVERSAL_SIMPLE) ? false
                                                                     : c->n_clusters >= PT_POOL_MIN_CLUSTERS;
    const bool inst = c->scene.n_instances > 0;  // kernels with the instance step compiled in
    // node format of the pool kernels: quantized by default where it exists
    const bool qn = use_pool && c->has_qnodes && !(rd->flags & PT_RENDER_NODES_FULL) &&
                    ((rd->flags & PT_RENDER_NODES_QUANTIZED) || c->node_format != PT_NODES_FULL);
    const bool timing = (rd->flags & PT_RENDER_TIMING) != 0;
    // NEE rays through the stackless any-hit traversal (pt_pool.h
    // trace_any_stackless): quantized records without instances
    const bool sl = qn && !inst && (rd->flags & PT_RENDER_ANY_STACKLESS);
    // hit sort before shading: spatial by default for large scenes (C4 at 256
    // spp: 897 -> 949 Mrays/s, profiles/r02_ab_sort.txt), off for small ones
    // (the three passes cost ~0.1 ms a bounce, more than a small scene gains)
    const bool sort_rays = (rd->flags & PT_RENDER_SORT_RAYS) != 0;
    const bool sort_mat = (rd->flags & PT_RENDER_SORT_MATERIAL) != 0;
    const bool sort_sp = !sort_mat && !(rd->flags & PT_RENDER_NO_SORT) &&
                         ((rd->flags & PT_RENDER_SORT_SPATIAL) || big_scene);
    const bool keep_bins = sort_mat || sort_sp || sort_rays;
    // every buffer sized by the path count — the wavefront, the claim / hit
    // orders and bins, the instance scratch — is allocated in one step, and a
    // device short of HBM (or a second context on it) retries the whole step
    // with half the paths instead of failing the frame with PT_ERR_OOM
    auto alloc_paths = [&](uint32_t p) -> pt_status {
        pt_status s;
        if ((s = ensure_work(c, p)) != PT_OK) return s;
        if (sort_rays) {
            if ((s = ensure(c, &c->ray_order, c->ray_order_cap, p)) != PT_OK) return s;
            if ((s = ensure(c, &c->ray_counts, c->ray_counts_cap, PT_SORT_BINS_SPATIAL)) != PT_OK) return s;
        }
        if (sort_mat || sort_sp) {
            if ((s = ensure(c, &c->sort_order, c->sort_order_cap, p)) != PT_OK) return s;
            if ((s = ensure(c, &c->sort_counts, c->sort_counts_cap, PT_SORT_BINS_SPATIAL)) != PT_OK) return s;
        }
        if (keep_bins && (s = ensure(c, &c->sort_bins, c->sort_bins_cap, p)) != PT_OK) return s;
        if (PT_SHADE_SPLIT && rd->integrator == PT_INTEGRATOR_PATH &&
            (s = ensure(c, &c->nee_jobs, c->nee_jobs_cap, p)) != PT_OK)
            return s;
        return bind_scene(c);  // instance scratch and ray-time buffers sized for this wavefront
    };
    while ((st = alloc_paths(paths)) == PT_ERR_OOM && paths > (1u << 20)) {
        (void)hipGetLastError();
        free_paths(c);  // the larger buffers that did fit make room for the retry
        paths = ((paths >> 1) + 255) & ~255u;
    }
    if (st) return st;
    c->scene.ray_order = sort_rays ? c->ray_order : nullptr;
    struct ResetOrder {  // other entry points bind the scene without a claim order
        pt_ctx* c;
        ~ResetOrder() { c->scene.ray_order = nullptr; }
    } reset_order{c};
    if ((st = bind_scene(c)) != PT_OK) return st;
    uint16_t* bins = keep_bins ? c->sort_bins : nullptr;  // (shared by the claim-order and hit sorts: each pass pair runs in turn on sm)
    hipStream_t sm = c->stream;
    HIPCHK(c, hipMemsetAsync(c->counters, 0, (CNT_SHARDS + 1) * CNT_COUNT * 8, sm));
    HIPCHK(c, hipMemsetAsync(c->stack_drops, 0, 8, sm));  // stack and tie drops
    // the sample-id counter sits on its own line after the work-counter shards
    unsigned long long* next_sample = c->counters + CNT_SHARDS * CNT_COUNT + CNT_NEXT_SAMPLE;
    float t_cl = 0, t_sh = 0, t_an = 0;

    auto trace = [&](RenderParams& R) -> pt_status {
        pt_status st;
        R.chunk_total = (unsigned long long)R.npix_work * (R.s_hi - R.s_lo);
        if (R.max_depth == 0) {  // the Li loop never runs: every sample is black
            HIPCHK(c, hipMemsetAsync(c->sample_L, 0, 12ull * R.chunk_total, sm));
            if (stats) stats->paths += R.chunk_total;
            return PT_OK;
        }
        HIPCHK(c, hipMemsetAsync(next_sample, 0, 8, sm));
        // Counter sets rotate (pt_kernels.h SET_WORDS): iteration i reads its
        // path count from set[i % 3] (written by iteration i - 1, or the
        // initial fill), appends into set[(i + 1) % 3] and zeroes
        // set[(i + 2) % 3].  Every kernel reads its count from device memory,
        // so the host never waits for a bounce: it keeps PT_LAG iterations
        // queued ahead of the one whose counts it reads (the pinned snapshot
        // the iteration's first kernel writes, behind an event).
        uint32_t* set[3] = {c->qcnt, c->qcnt + SET_WORDS, c->qcnt + 2 * SET_WORDS};
        HIPCHK(c, hipMemsetAsync(c->qcnt, 0, 3 * SET_WORDS * 4, sm));
        // initial fill: one camera sample per wavefront entry
        PathSoA cur = c->PA, nxt = c->PB;
        // never more paths in flight than the chunk has samples (late adaptive
        // rounds hold a few active pixels): fill and grids sized to that
        const uint32_t pfill = (uint32_t)std::min<uint64_t>(paths, (R.chunk_total + 255) & ~255ull);
        hipLaunchKernelGGL(k_fill, dim3((pfill + 255) / 256), dim3(256), 0, sm, R, pfill, cur, set[0], next_sample);
        HIPCHK(c, hipGetLastError());
        uint32_t issued = 0, read = 0;
        bool drained = false;
        const bool ovl = ((c->overlap && !(rd->flags & PT_RENDER_SERIAL_SHADOW)) || (rd->flags & PT_RENDER_OVERLAP_SHADOW)) &&
                         use_pool && !inst && rd->integrator == PT_INTEGRATOR_PATH;  // (instance scratch is per grid lane, shared)
        hipStream_t sa = ovl ? c->side_stream : sm;  // the any-hit kernel's stream
        // Tail grids: once every camera sample of the chunk has been started
        // (read from the snapshots: the fill, then each iteration's new paths),
        // path counts can only fall, so the count entering the last iteration
        // read bounds every later one and the grids shrink to it (the kernels
        // still read their exact counts from device memory).
        uint64_t started = 0;
        uint32_t bound = pfill;
        // reads iteration `read`'s snapshot (after its event): stats, timing, end test
        auto consume = [&]() -> pt_status {
            const uint32_t slot = read % PT_RING;
            HIPCHK(c, hipEventSynchronize(c->rev[slot][4]));
            const volatile uint32_t* hc = c->host_cnt + slot * SNAP_WORDS;
            const uint32_t n_in = hc[SNAP_PATHS];
            started += read == 0 ? n_in : hc[SNAP_NEW];
            if (started >= R.chunk_total) bound = std::min(bound, n_in);
            if (stats) {
                stats->rays_any += hc[SNAP_SHADOW_PREV];
                if (n_in) {
                    stats->rays_closest += n_in;
                    stats->shade_hits += n_in;
                    stats->launches_closest++;
                    if (rd->integrator != PT_INTEGRATOR_SIMPLE) stats->launches_any++;
                }
            }
            if (timing && n_in) {
                float a, b, d;
                HIPCHK(c, hipEventElapsedTime(&a, c->rev[slot][0], c->rev[slot][1]));
                HIPCHK(c, hipEventElapsedTime(&b, c->rev[slot][1], c->rev[slot][2]));
                HIPCHK(c, hipEventElapsedTime(&d, c->rev[slot][2], c->rev[slot][4]));
                t_cl += a;
                t_sh += b;
                t_an += d;
            }
            if (n_in == 0) drained = true;  // and every later iteration finds none
            ++read;
            return PT_OK;
        };
        // the tail (k_tail): once every sample has started and the live paths
        // have fallen to a small share of the wavefront, one launch finishes them
        const bool tail_ok = PT_TAIL_PATHS > 0 && !inst && !(rd->flags & PT_RENDER_NO_TAIL) &&
                             (rd->integrator == PT_INTEGRATOR_PATH || rd->integrator == PT_INTEGRATOR_SIMPLE);
        const uint32_t tail_max = std::min<uint32_t>(PT_TAIL_PATHS, paths / PT_TAIL_SHARE);
        bool tail = false;
        while (!drained) {
            if (issued - read >= PT_LAG) {
                if ((st = consume()) != PT_OK) return st;
                continue;
            }
            if (tail_ok && read > 0 && started >= R.chunk_total && bound <= tail_max) {
                tail = true;
                break;
            }
            const uint32_t i = issued;
            const uint32_t nb = std::max(bound, 1u);
            const dim3 gt(use_pool ? std::min(c->pool_blocks[0][inst][qn], (nb + PT_TRACE_BLOCK - 1) / PT_TRACE_BLOCK)
                                   : (nb + PT_TRACE_BLOCK - 1) / PT_TRACE_BLOCK);
            const dim3 ga(use_pool ? std::min(sl ? c->sl_blocks : c->pool_blocks[1][inst][qn],
                                              (nb + PT_TRACE_BLOCK - 1) / PT_TRACE_BLOCK)
                                   : (nb + PT_TRACE_BLOCK - 1) / PT_TRACE_BLOCK);
            const dim3 gs((nb + 255) / 256), gsh((nb + PT_SHADE_BLOCK - 1) / PT_SHADE_BLOCK);
            const dim3 gsort((nb + 256 * PT_SORT_PER - 1) / (256 * PT_SORT_PER));  // k_sort_count / k_sort_scatter
            uint32_t* in = set[i % 3];
            uint32_t* out = set[(i + 1) % 3];
            uint32_t* spare = set[(i + 2) % 3];
            hipEvent_t* ev = c->rev[i % PT_RING];
            if (timing) HIPCHK(c, hipEventRecord(ev[0], sm));
            // (overlap: the previous bounce's any-hit kernel may still run on sa)
            if (sort_rays) {  // claim order of this bounce's closest-hit rays: origin cell + octant
                constexpr int NB = PT_SORT_BINS_SPATIAL;
                HIPCHK(c, hipMemsetAsync(c->ray_counts, 0, NB * 4, sm));
                hipLaunchKernelGGL((k_sort_count<PT_SORT_RAYS, NB>), gsort, dim3(256), 0, sm, cur, (const uint32_t*)in,
                                   (const float4*)c->hit, c->ray_counts, bins);
                hipLaunchKernelGGL((k_sort_scan<NB>), dim3(1), dim3(256), 0, sm, c->ray_counts);
                hipLaunchKernelGGL((k_sort_scatter<PT_SORT_RAYS, NB>), gsort, dim3(256), 0, sm, cur, (const uint32_t*)in,
                                   (const float4*)c->hit, c->ray_counts, c->ray_order, bins);
            }
            {
                auto kc = pick_closest(use_pool, qn, inst, count);
                hipLaunchKernelGGL(kc, gt, dim3(PT_TRACE_BLOCK), 0, sm, cur, (const uint32_t*)in, c->hit,
                                   out + Q_WORDS, c->ovf, spare, c->host_cnt_dev + (i % PT_RING) * SNAP_WORDS,
                                   c->counters, c->ties);
                if (use_pool)  // the rays that met an exact-t tie, re-traced in the reference's order
                    hipLaunchKernelGGL(inst ? k_closest_ties<true> : k_closest_ties<false>,
                                       dim3(std::min(PT_TIE_BLOCKS, gt.x)), dim3(PT_TRACE_BLOCK), 0, sm, cur,
                                       (const uint32_t*)in, c->hit, (const uint32_t*)(out + Q_WORDS),
                                       (const uint32_t*)c->ties);
            }
            if (timing) HIPCHK(c, hipEventRecord(ev[1], sm));
            // the hit sort and the shading rewrite the shadow queue, the sample
            // buffer and the path state the previous any-hit kernel updates
            if (ovl && i > 0) HIPCHK(c, hipStreamWaitEvent(sm, c->rev[(i - 1) % PT_RING][4], 0));
            if (sort_mat) {  // bin this bounce's paths by hit material (k_sort_*), shade in that order
                constexpr int NB = PT_SORT_BINS_MATERIAL;
                HIPCHK(c, hipMemsetAsync(c->sort_counts, 0, NB * 4, sm));
                hipLaunchKernelGGL((k_sort_count<PT_SORT_MATERIAL, NB>), gsort, dim3(256), 0, sm, cur, (const uint32_t*)in,
                                   (const float4*)c->hit, c->sort_counts, bins);
                hipLaunchKernelGGL((k_sort_scan<NB>), dim3(1), dim3(256), 0, sm, c->sort_counts);
                hipLaunchKernelGGL((k_sort_scatter<PT_SORT_MATERIAL, NB>), gsort, dim3(256), 0, sm, cur,
                                   (const uint32_t*)in, (const float4*)c->hit, c->sort_counts, c->sort_order, bins);
                R.order = c->sort_order;
            } else if (sort_sp) {  // ... by the hit point's Morton cell
                constexpr int NB = PT_SORT_BINS_SPATIAL;
                HIPCHK(c, hipMemsetAsync(c->sort_counts, 0, NB * 4, sm));
                hipLaunchKernelGGL((k_sort_count<PT_SORT_SPATIAL, NB>), gsort, dim3(256), 0, sm, cur, (const uint32_t*)in,
                                   (const float4*)c->hit, c->sort_counts, bins);
                hipLaunchKernelGGL((k_sort_scan<NB>), dim3(1), dim3(256), 0, sm, c->sort_counts);
                hipLaunchKernelGGL((k_sort_scatter<PT_SORT_SPATIAL, NB>), gsort, dim3(256), 0, sm, cur,
                                   (const uint32_t*)in, (const float4*)c->hit, c->sort_counts, c->sort_order, bins);
                R.order = c->sort_order;
            }
            if (rd->integrator == PT_INTEGRATOR_SIMPLE)
                hipLaunchKernelGGL(k_shade<PT_INTEGRATOR_SIMPLE>, gsh, dim3(PT_SHADE_BLOCK), 0, sm, R, cur,
                                   (const uint32_t*)(in + Q_NEXT), (const float4*)c->hit, nxt, c->sample_L,
                                   next_sample, c->sq, out);
            else if (rd->integrator == PT_INTEGRATOR_VOLPATH)
                hipLaunchKernelGGL(k_shade_vol, gs, dim3(256), 0, sm, R, cur, (const uint32_t*)(in + Q_NEXT),
                                   (const float4*)c->hit, nxt, c->sample_L, next_sample, (ShadowRecV*)c->sq, out);
            else {
                R.nee_jobs = c->nee_jobs;
                hipLaunchKernelGGL(k_shade<PT_INTEGRATOR_PATH>, gsh, dim3(PT_SHADE_BLOCK), 0, sm, R, cur,
                                   (const uint32_t*)(in + Q_NEXT), (const float4*)c->hit, nxt, c->sample_L,
                                   next_sample, c->sq, out);
                if (PT_SHADE_SPLIT)  // the bounce's NEE half (pt_kernels.h)
                    hipLaunchKernelGGL(k_shade_nee, gsh, dim3(PT_SHADE_BLOCK), 0, sm, R, cur,
                                       (const uint32_t*)(in + Q_NEXT), (const float4*)c->hit, c->sq, out);
            }
            if (timing || ovl) HIPCHK(c, hipEventRecord(ev[2], sm));
            if (ovl) HIPCHK(c, hipStreamWaitEvent(sa, ev[2], 0));
            if (rd->integrator == PT_INTEGRATOR_VOLPATH) {
                // transmittance along the shadow rays: one ray per lane, the grid covers the capacity
                hipLaunchKernelGGL(count ? k_shadow_tr<true> : k_shadow_tr<false>,
                                   dim3((nb + PT_TRACE_BLOCK - 1) / PT_TRACE_BLOCK), dim3(PT_TRACE_BLOCK), 0, sm,
                                   nxt, c->sample_L, (const ShadowRecV*)c->sq, (const uint32_t*)(out + Q_SHADOW),
                                   c->counters);
            } else if (rd->integrator != PT_INTEGRATOR_SIMPLE) {
                auto ks = sl ? (count ? k_shadow_sl<true> : k_shadow_sl<false>) : pick_shadow(use_pool, qn, inst, count);
                hipLaunchKernelGGL(ks, ga, dim3(PT_TRACE_BLOCK), 0, sa, nxt, c->sample_L, c->sq,
                                   (const uint32_t*)(out + Q_SHADOW), out + Q_WORDS + PT_POOL_WORDS,
                                   ovl ? c->ovf_any : c->ovf, c->counters);
            }
            HIPCHK(c, hipGetLastError());
            HIPCHK(c, hipEventRecord(ev[4], sa));
            std::swap(cur, nxt);
            ++issued;
        }
        // iterations queued past the end find zero paths; let them drain
        if (tail) {
            if (ovl && issued) HIPCHK(c, hipStreamWaitEvent(sm, c->rev[(issued - 1) % PT_RING][4], 0));
            uint32_t* in = set[issued % 3];  // the paths entering the next bounce
            const dim3 gt(std::max(1u, std::min(c->pool_blocks[0][inst][qn], (bound + PT_TRACE_BLOCK - 1) / PT_TRACE_BLOCK)));
            using TailFn = void (*)(RenderParams, PathSoA, const uint32_t*, float*, unsigned long long*);
            const TailFn kt = rd->integrator == PT_INTEGRATOR_SIMPLE
                                  ? (count ? k_tail<PT_INTEGRATOR_SIMPLE, false, true> : k_tail<PT_INTEGRATOR_SIMPLE, false, false>)
                                  : (count ? k_tail<PT_INTEGRATOR_PATH, false, true> : k_tail<PT_INTEGRATOR_PATH, false, false>);
            hipLaunchKernelGGL(kt, gt, dim3(PT_TRACE_BLOCK), 0, sm, R, cur, (const uint32_t*)in, c->sample_L, c->counters);
            HIPCHK(c, hipGetLastError());
            // its queries join rays_closest / rays_any (CNT_TAIL_*); its time only
            // the wall clock: the per-kernel times and launch counts stay the
            // wavefront kernels' own (what the roofline entries divide)
        }
        while (read < issued)
            if ((st = consume()) != PT_OK) return st;
        if (ovl && issued) HIPCHK(c, hipStreamWaitEvent(sm, c->rev[(issued - 1) % PT_RING][4], 0));

        if (stats) stats->paths += R.chunk_total;
        return PT_OK;
    };
    if ((st = drive(R, spp_local, s_chunk, trace)) != PT_OK) {
        // an error inside the overlapped loop can leave any-hit kernels queued
        // on the side stream: let them finish before the caller frees anything
        hipStreamSynchronize(c->side_stream);
        return st;
    }
    HIPCHK(c, hipStreamSynchronize(sm));
    if (stats) {
        unsigned long long hs[CNT_SHARDS * CNT_COUNT], h[CNT_COUNT] = {};
        HIPCHK(c, hipMemcpy(hs, c->counters, sizeof(hs), hipMemcpyDeviceToHost));
        for (int k = 0; k < CNT_SHARDS; k++)
            for (int j = 0; j < CNT_COUNT; j++) h[j] += hs[k * CNT_COUNT + j];
        stats->nodes_closest += h[CNT_NODES_CLOSEST];
        stats->tris_closest += h[CNT_TRIS_CLOSEST];
        stats->nodes_any += h[CNT_NODES_ANY];
        stats->rays_any += h[CNT_EXTRA_ANY];
        stats->rays_closest += h[CNT_TAIL_CLOSEST];  // the tail's queries (k_tail)
        stats->shade_hits += h[CNT_TAIL_CLOSEST];
        stats->rays_any += h[CNT_TAIL_ANY];
        stats->tris_any += h[CNT_TRIS_ANY];
        stats->ms_closest += t_cl;
        stats->ms_shade += t_sh;
        stats->ms_any += t_an;
        uint32_t drops[2] = {0, 0};
        HIPCHK(c, hipMemcpy(drops, c->stack_drops, 8, hipMemcpyDeviceToHost));
        stats->stack_overflows += drops[0];
        stats->tie_overflows += drops[1];
        stats->n_devices = 1;
    }
    return PT_OK;
}

// The fixed-SPP driver: consecutive sample chunks, each handed to on_chunk.
template <class OnChunk>
static auto fixed_chunks(OnChunk on_chunk) {
    return [on_chunk](RenderParams& R, uint32_t spp_local, uint32_t s_chunk, auto& trace) -> pt_status {
        for (uint32_t s_lo = 0; s_lo < spp_local; s_lo += s_chunk) {
            R.s_lo = s_lo;
            R.s_hi = std::min(spp_local, s_lo + s_chunk);
            if (pt_status st = trace(R)) return st;
            if (pt_status st = on_chunk(R)) return st;
        }
        return PT_OK;
    };
}

static pt_status check_render_args(pt_ctx* c, const pt_camera_desc* cam, const pt_render_desc* rd) {
    if (!c || !cam || !rd) return PT_ERR_ARG;
    if (!c->has_scene) return fail(c, PT_ERR_STATE, "no scene uploaded");
    if (cam->width <= 0 || cam->height <= 0 || (uint64_t)cam->width * cam->height > (1ull << 31))
        return fail(c, PT_ERR_ARG, "bad film size");
    if (rd->integrator > PT_INTEGRATOR_VOLPATH || rd->filter > PT_FILTER_LANCZOS)
        return fail(c, PT_ERR_ARG, "bad integrator/filter");
    if (rd->filter == PT_FILTER_LANCZOS && !(rd->filter_params[1] != 0.0 && std::isfinite(rd->filter_params[1])))
        return fail(c, PT_ERR_ARG, "Lanczos filter: filter_params[1] must hold the filter's Integral()");
    if (cam->medium < -1 || cam->medium >= (int32_t)c->n_media) return fail(c, PT_ERR_ARG, "bad camera medium");
    if (rd->filter_radius[0] <= 0 || rd->filter_radius[1] <= 0) return fail(c, PT_ERR_ARG, "bad filter radius");
    if ((rd->strata[0] || rd->strata[1]) && (uint64_t)rd->strata[0] * rd->strata[1] != rd->spp)
        return fail(c, PT_ERR_ARG, "strata %u x %u do not make the %u samples per pixel", rd->strata[0],
                    rd->strata[1], rd->spp);
    return PT_OK;
}

// Film accumulation on the device: `film_accum` itself when it is device
// memory, else a zeroed scratch film whose sum is added to the host array.
template <class Body>
static pt_status with_film(pt_ctx* c, const pt_camera_desc* cam, double* film_accum, pt_stats* S, Body body) {
    auto t0 = std::chrono::steady_clock::now();
    const uint64_t nfilm = 4ull * cam->width * cam->height;
    const bool dev = is_device_ptr(film_accum);
    double* film = film_accum;
    pt_status st;
    if (!dev) {
        if ((st = ensure(c, &c->film, c->film_cap, nfilm)) != PT_OK) return st;
        film = c->film;
        HIPCHK(c, hipMemsetAsync(film, 0, nfilm * 8, c->stream));
    }
    *S = pt_stats{};
    if ((st = body(film)) != PT_OK) return st;
    if (!dev) {
        std::vector<double> h(nfilm);
        HIPCHK(c, hipMemcpyAsync(h.data(), film, nfilm * 8, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        for (uint64_t i = 0; i < nfilm; i++) film_accum[i] += h[i];
    } else {
        HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    S->ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return PT_OK;
}

static pt_status render_adaptive_dev(pt_ctx* c, const pt_camera_desc* cam, const pt_render_desc* rd,
                                     double* film_accum, uint32_t* sample_counts, pt_stats* stats);
static pt_status render_multi(pt_ctx* c, const pt_camera_desc* cam, const pt_render_desc* rd, double* film_accum,
                              uint32_t* sample_counts, pt_stats* stats, bool adaptive);
static pt_status render_dev(pt_ctx* c, const pt_camera_desc* cam, const pt_render_desc* rd, double* film_accum,
                            pt_stats* stats);

extern "C" pt_status pt_render(pt_ctx* c, const pt_camera_desc* cam, const pt_render_desc* rd, double* film_accum,
                               pt_stats* stats) {
    pt_status st = check_render_args(c, cam, rd);
    if (st) return st;
    if (rd->flags & PT_RENDER_ADAPTIVE) return pt_render_adaptive(c, cam, rd, film_accum, nullptr, stats);
    if (!film_accum) return fail(c, PT_ERR_ARG, "film_accum is null");
    if (c->multi) return render_multi(c, cam, rd, film_accum, nullptr, stats, false);
    return render_dev(c, cam, rd, film_accum, stats);
}

// One device's fixed-SPP frame (shard rd->shard_index of rd->shard_count).
static pt_status render_dev(pt_ctx* c, const pt_camera_desc* cam, const pt_render_desc* rd, double* film_accum,
                            pt_stats* stats) {
    DeviceLock dl(c->device);
    pt_status st;
    if (!film_accum) return fail(c, PT_ERR_ARG, "film_accum is null");
    if (!(rd->pixel_begin == 0 && rd->pixel_end == 0)) return fail(c, PT_ERR_ARG, "pt_render renders whole films");
    HIPCHK(c, hipSetDevice(c->device));
    pt_stats local{};
    pt_stats* S = stats ? stats : &local;
    return with_film(c, cam, film_accum, S, [&](double* film) {
        return run(c, cam, rd, S, fixed_chunks([&](const RenderParams& R) -> pt_status {
            const uint32_t npx = (uint32_t)cam->width * cam->height;
            const int rad = std::max(R.rad_x, R.rad_y);
            const dim3 tiles((cam->width + 15) / 16, (cam->height + 15) / 16);
            // the tile gather built for the film's filter (its own code and registers only)
            auto tile = [&](auto rad_c) {
                constexpr int RAD = decltype(rad_c)::value;
                auto k = R.filter == PT_FILTER_MITCHELL ? k_gather_tile<RAD, PT_FILTER_MITCHELL>
                         : R.filter == PT_FILTER_BOX    ? k_gather_tile<RAD, PT_FILTER_BOX>
                         : R.filter == PT_FILTER_GAUSSIAN ? k_gather_tile<RAD, PT_FILTER_GAUSSIAN>
                                                          : k_gather_tile<RAD, PT_FILTER_LANCZOS>;
                hipLaunchKernelGGL(k, tiles, dim3(256), 0, c->stream, R, c->sample_L, film);
            };
            if (R.npix_work == npx && rad <= 1 && !getenv("PT_GATHER_PIXEL"))
                tile(std::integral_constant<int, 1>{});
            else if (R.npix_work == npx && rad == 2 && !getenv("PT_GATHER_PIXEL"))
                tile(std::integral_constant<int, 2>{});
            else
                hipLaunchKernelGGL(k_gather, dim3((npx + 255) / 256), dim3(256), 0, c->stream, R, c->sample_L, film);
            HIPCHK(c, hipGetLastError());
            // the chunk stays in sample_L after the frame: pt_frame_samples
            c->frame = pt_ctx::FrameRec{true, (uint32_t)cam->width, R.npix_work, R.tiled, R.tiles_x,
                                        R.s_lo, R.s_hi, R.shard_index, R.shard_count, (uint32_t)cam->height};
            return PT_OK;
        }));
    });
}

// Per-sample radiance of the last fixed-SPP frame (pt_frame_samples): the
// final sample chunk is still in sample_L, sample-major, pixels in the
// chunk's work order (8x8 tiles when R.tiled, k_fill's work_pixel).
extern "C" pt_status pt_frame_samples(pt_ctx* c, const uint32_t* pixels, const uint32_t* samples, uint32_t n,
                                      float* out_L) {
    if (!c || (n && (!pixels || !samples || !out_L))) return PT_ERR_ARG;
    const pt_ctx::FrameRec& f = c->frame;
    if (!f.valid) return fail(c, PT_ERR_STATE, "no fixed-SPP frame in the sample buffer");
    if (n == 0) return PT_OK;
    std::vector<unsigned long long> idx(n);
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t p = pixels[i], s = samples[i];
        if ((uint64_t)p >= (uint64_t)f.width * f.height) return fail(c, PT_ERR_ARG, "pixel %u outside the frame", p);
        const uint32_t x = p % f.width, y = p / f.width;
        if (s < f.shard_index || (s - f.shard_index) % f.shard_count)
            return fail(c, PT_ERR_ARG, "sample %u belongs to another shard", s);
        const uint32_t sl = (s - f.shard_index) / f.shard_count;
        if (sl < f.s_lo || sl >= f.s_hi) return fail(c, PT_ERR_ARG, "sample %u is not in the last sample chunk", s);
        const uint32_t pix_i = f.tiled ? (((y >> 3) * f.tiles_x + (x >> 3)) << 6) | ((y & 7u) << 3) | (x & 7u) : p;
        idx[i] = (unsigned long long)(sl - f.s_lo) * f.npix + pix_i;
    }
    HIPCHK(c, hipSetDevice(c->device));
    unsigned long long* di = nullptr;
    float* dout = nullptr;
    if (hipMalloc((void**)&di, 8ull * n) != hipSuccess) return fail(c, PT_ERR_OOM, "frame samples: index buffer");
    if (hipMalloc((void**)&dout, 12ull * n) != hipSuccess) {
        hipFree(di);
        return fail(c, PT_ERR_OOM, "frame samples: output buffer");
    }
    hipError_t e = hipMemcpyAsync(di, idx.data(), 8ull * n, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_frame_gather, dim3((n + 255) / 256), dim3(256), 0, c->stream, (const float*)c->sample_L,
                           (const unsigned long long*)di, n, dout);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(out_L, dout, 12ull * n, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    hipFree(di);
    hipFree(dout);
    if (e != hipSuccess) return fail(c, PT_ERR_HIP, "frame samples: %s", hipGetErrorString(e));
    return PT_OK;
}

extern "C" pt_status pt_frame_sample_range(const pt_ctx* c, uint32_t* first, uint32_t* last) {
    if (!c || !first || !last) return PT_ERR_ARG;
    const pt_ctx::FrameRec& f = c->frame;
    if (!f.valid || f.s_hi <= f.s_lo) return PT_ERR_STATE;
    *first = f.s_lo * f.shard_count + f.shard_index;
    *last = (f.s_hi - 1) * f.shard_count + f.shard_index;
    return PT_OK;
}

// TileIntegrator::Render's adaptive loop (Integrators.cpp:55-86), round by
// round over the still-active pixels (pt_kernels.hip "adaptive sampling").
// The host reads one count per round (the next round's active pixels).
extern "C" pt_status pt_render_adaptive(pt_ctx* c, const pt_camera_desc* cam, const pt_render_desc* rd,
                                        double* film_accum, uint32_t* sample_counts, pt_stats* stats) {
    pt_status st = check_render_args(c, cam, rd);
    if (st) return st;
    if (!film_accum) return fail(c, PT_ERR_ARG, "film_accum is null");
    if (rd->spp == 0) return fail(c, PT_ERR_ARG, "adaptive sampling needs spp >= 1");
    if (rd->spp > (1u << 24) / PT_ADAPT_MAX_ROUNDS) return fail(c, PT_ERR_ARG, "spp too large for 128 rounds");
    if (c->multi) return render_multi(c, cam, rd, film_accum, sample_counts, stats, true);
    return render_adaptive_dev(c, cam, rd, film_accum, sample_counts, stats);
}

// Multi-device frame: device g renders shard rd->shard_index + rd->shard_count*g
// of rd->shard_count*n (interleaved samples; 32x32 tiles when adaptive) into
// its own device film, on one host thread per device; then one grouped
// ncclReduce(ncclSum) per device sums the films (and the adaptive sample
// counts) onto the first device, whose result reaches film_accum.  This is
// the reference's Film::Merge (Film.hpp:125-132, 244-253) after
// TileIntegrator::Render's tiles (Integrators.cpp:112), over xGMI.
static pt_status render_multi(pt_ctx* c, const pt_camera_desc* cam, const pt_render_desc* rd, double* film_accum,
                              uint32_t* sample_counts, pt_stats* stats, bool adaptive) {
    auto t0 = std::chrono::steady_clock::now();
    std::vector<pt_ctx*> dv{c};
    dv.insert(dv.end(), c->peers.begin(), c->peers.end());
    const uint32_t n = (uint32_t)dv.size();
    const uint64_t npx = (uint64_t)cam->width * cam->height, nf = 4 * npx;
    for (pt_ctx* d : dv)
        if (!d->comm) return fail(c, PT_ERR_STATE, "multi-device context without communicators");
    const bool dev_film = is_device_ptr(film_accum);
    std::vector<double*> films(n);
    for (uint32_t g = 0; g < n; g++) {
        pt_ctx* d = dv[g];
        HIPCHK(c, hipSetDevice(d->device));
        if (g == 0 && dev_film) {
            films[g] = film_accum;  // accumulates in place; the reduce adds the others
            continue;
        }
        if (pt_status st = ensure(d, &d->film, d->film_cap, nf)) return fail(c, st, "device %d: %s", d->device, d->err.c_str());
        HIPCHK(c, hipMemsetAsync(d->film, 0, nf * 8, d->stream));
        films[g] = d->film;
    }
    std::vector<pt_stats> st(n);
    std::vector<pt_status> res(n, PT_OK);
    {
        std::vector<std::thread> th;
        for (uint32_t g = 0; g < n; g++)
            th.emplace_back([&, g] {
                pt_ctx* d = dv[g];
                if (hipSetDevice(d->device) != hipSuccess) {
                    res[g] = fail(d, PT_ERR_HIP, "hipSetDevice(%d)", d->device);
                    return;
                }
                pt_render_desc r = *rd;
                const uint32_t sc = rd->shard_count ? rd->shard_count : 1;
                r.shard_index = rd->shard_index + sc * g;
                r.shard_count = sc * n;
                r.flags &= ~PT_RENDER_ADAPTIVE;
                res[g] = adaptive ? render_adaptive_dev(d, cam, &r, films[g], nullptr, &st[g])
                                  : render_dev(d, cam, &r, films[g], &st[g]);
            });
        for (auto& t : th) t.join();
    }
    for (uint32_t g = 0; g < n; g++)
        if (res[g] != PT_OK) return fail(c, res[g], "device %d: %s", dv[g]->device, dv[g]->err.c_str());
    // the film (and count) reduce onto the first device, one grouped call
    ncclResult_t r = ncclGroupStart();
    for (uint32_t g = 0; g < n && r == ncclSuccess; g++) {
        r = ncclReduce(films[g], films[g], nf, ncclDouble, ncclSum, 0, dv[g]->comm, dv[g]->stream);
        if (r == ncclSuccess && adaptive)
            r = ncclReduce(dv[g]->a_counts, dv[g]->a_counts, npx, ncclUint32, ncclSum, 0, dv[g]->comm, dv[g]->stream);
    }
    const ncclResult_t r2 = ncclGroupEnd();
    if (r != ncclSuccess || r2 != ncclSuccess)
        return fail(c, PT_ERR_COMM, "film reduce: %s", ncclGetErrorString(r != ncclSuccess ? r : r2));
    for (uint32_t g = 0; g < n; g++) {
        HIPCHK(c, hipSetDevice(dv[g]->device));
        HIPCHK(c, hipStreamSynchronize(dv[g]->stream));
    }
    HIPCHK(c, hipSetDevice(c->device));
    if (!dev_film) {
        std::vector<double> h(nf);
        HIPCHK(c, hipMemcpy(h.data(), films[0], nf * 8, hipMemcpyDeviceToHost));
        for (uint64_t i = 0; i < nf; i++) film_accum[i] += h[i];
    }
    if (adaptive && sample_counts) {
        const hipMemcpyKind k = is_device_ptr(sample_counts) ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
        HIPCHK(c, hipMemcpy(sample_counts, c->a_counts, 4 * npx, k));
    }
    if (stats) {
        pt_stats S{};
        for (const pt_stats& x : st) {
            S.paths += x.paths;
            S.rays_closest += x.rays_closest;
            S.rays_any += x.rays_any;
            S.nodes_closest += x.nodes_closest;
            S.tris_closest += x.tris_closest;
            S.nodes_any += x.nodes_any;
            S.tris_any += x.tris_any;
            S.shade_hits += x.shade_hits;
            S.launches_closest += x.launches_closest;
            S.launches_any += x.launches_any;
            S.stack_overflows += x.stack_overflows;
            S.tie_overflows += x.tie_overflows;
            S.ms_closest = std::max(S.ms_closest, x.ms_closest);
            S.ms_any = std::max(S.ms_any, x.ms_any);
            S.ms_shade = std::max(S.ms_shade, x.ms_shade);
        }
        S.n_devices = n;
        S.ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        *stats = S;
    }
    return PT_OK;
}

// One device's adaptive frame (pt_render_adaptive on a one-device context).
static pt_status render_adaptive_dev(pt_ctx* c, const pt_camera_desc* cam, const pt_render_desc* rd,
                                     double* film_accum, uint32_t* sample_counts, pt_stats* stats) {
    DeviceLock dl(c->device);
    pt_status st;
    HIPCHK(c, hipSetDevice(c->device));
    const uint32_t npx = (uint32_t)cam->width * cam->height;
    if ((st = ensure(c, &c->a_est, c->a_est_cap, npx)) != PT_OK) return st;
    if ((st = ensure(c, &c->a_counts, c->a_counts_cap, npx)) != PT_OK) return st;
    if ((st = ensure(c, &c->a_map, c->a_map_cap, npx)) != PT_OK) return st;
    if ((st = ensure(c, &c->a_list, c->a_list_cap, 2ull * npx)) != PT_OK) return st;
    if ((st = ensure(c, &c->a_cnt, c->a_cnt_cap, 2 * Q_STRIDE)) != PT_OK) return st;
    const uint32_t shard_count = rd->shard_count ? rd->shard_count : 1, shard_index = rd->shard_index;
    pt_render_desc r2 = *rd;
    r2.flags |= PT_RENDER_ADAPTIVE;
    pt_stats local{};
    pt_stats* S = stats ? stats : &local;
    hipStream_t sm = c->stream;
    st = with_film(c, cam, film_accum, S, [&](double* film) {
        HIPCHK(c, hipMemsetAsync(c->a_map, 0xFF, 4ull * npx, sm));
        HIPCHK(c, hipMemsetAsync(c->a_counts, 0, 4ull * npx, sm));
        return run(c, cam, &r2, S, [&](RenderParams& R, uint32_t spp, uint32_t s_chunk, auto& trace) -> pt_status {
            uint32_t* list[2] = {c->a_list, c->a_list + npx};
            uint32_t* cnt[2] = {c->a_cnt, c->a_cnt + Q_STRIDE};
            HIPCHK(c, hipMemsetAsync(c->a_cnt, 0, 8ull * Q_STRIDE, sm));
            const uint32_t nwork = R.npix_work;
            hipLaunchKernelGGL(k_adapt_init, dim3((nwork + 255) / 256), dim3(256), 0, sm, R, shard_index, shard_count,
                               list[0], cnt[0], c->a_est, c->a_counts);
            HIPCHK(c, hipGetLastError());
            uint32_t n = 0;
            HIPCHK(c, hipMemcpyAsync(&n, cnt[0], 4, hipMemcpyDeviceToHost, sm));
            HIPCHK(c, hipStreamSynchronize(sm));
            R.tiled = 0;
            for (uint32_t round = 0; n > 0 && round < PT_ADAPT_MAX_ROUNDS; round++) {
                const uint32_t a = round & 1u;
                hipLaunchKernelGGL(k_adapt_map, dim3((n + 255) / 256), dim3(256), 0, sm, (const uint32_t*)list[a],
                                   (const uint32_t*)cnt[a], c->a_map);
                R.pix_list = list[a];
                R.npix_work = n;
                for (uint32_t s0 = 0; s0 < spp; s0 += s_chunk) {
                    R.s_lo = round * spp + s0;
                    R.s_hi = R.s_lo + std::min(s_chunk, spp - s0);
                    if (pt_status e = trace(R)) return e;
                    hipLaunchKernelGGL(k_adapt_accum, dim3((n + 255) / 256), dim3(256), 0, sm, R, (const float*)c->sample_L,
                                       c->a_est, c->a_counts);
                    hipLaunchKernelGGL(k_adapt_gather, dim3((npx + 255) / 256), dim3(256), 0, sm, R,
                                       (const int32_t*)c->a_map, (const float*)c->sample_L, film);
                    HIPCHK(c, hipGetLastError());
                }
                HIPCHK(c, hipMemsetAsync(cnt[a ^ 1u], 0, 4, sm));
                hipLaunchKernelGGL(k_adapt_decide, dim3((n + 255) / 256), dim3(256), 0, sm, (const uint32_t*)list[a],
                                   (const uint32_t*)cnt[a], (const AdaptEst*)c->a_est, (const uint32_t*)c->a_counts,
                                   PT_ADAPT_MAX_ROUNDS * spp, c->a_map, list[a ^ 1u], cnt[a ^ 1u]);
                HIPCHK(c, hipGetLastError());
                HIPCHK(c, hipMemcpyAsync(&n, cnt[a ^ 1u], 4, hipMemcpyDeviceToHost, sm));
                HIPCHK(c, hipStreamSynchronize(sm));
            }
            R.pix_list = nullptr;
            return PT_OK;
        });
    });
    if (st) return st;
    if (sample_counts) {
        const hipMemcpyKind k = is_device_ptr(sample_counts) ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
        HIPCHK(c, hipMemcpyAsync(sample_counts, c->a_counts, 4ull * npx, k, sm));
        HIPCHK(c, hipStreamSynchronize(sm));
    }
    return PT_OK;
}

extern "C" pt_status pt_render_samples(pt_ctx* c, const pt_camera_desc* cam, const pt_render_desc* rd, float* out_L,
                                       pt_stats* stats) {
    if (!c) return PT_ERR_ARG;
    DeviceLock dl(c->device);
    pt_status st = check_render_args(c, cam, rd);
    if (st) return st;
    if (!out_L) return fail(c, PT_ERR_ARG, "out_L is null");
    if (rd->shard_count > 1) return fail(c, PT_ERR_ARG, "pt_render_samples renders unsharded");
    HIPCHK(c, hipSetDevice(c->device));
    const bool ranged = !(rd->pixel_begin == 0 && rd->pixel_end == 0);
    const uint32_t pb = ranged ? rd->pixel_begin : 0;
    const uint32_t pe = ranged ? rd->pixel_end : (uint32_t)(cam->width * cam->height);
    pt_render_desc r2 = *rd;
    r2.pixel_begin = pb;
    r2.pixel_end = pe;  // always linear pixel order here
    const uint32_t npix = pe - pb;
    pt_stats local{};
    pt_stats* S = stats ? stats : &local;
    *S = pt_stats{};
    std::vector<float> h;
    r2.flags &= ~PT_RENDER_ADAPTIVE;
    return run(c, cam, &r2, S, fixed_chunks([&](const RenderParams& R) -> pt_status {
        const uint64_t n = 3ull * R.chunk_total;
        h.resize(n);
        HIPCHK(c, hipMemcpyAsync(h.data(), c->sample_L, n * 4, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        const uint32_t ns = R.s_hi - R.s_lo;
        for (uint32_t k = 0; k < ns; k++)
            for (uint32_t p = 0; p < npix; p++) {
                const float* src = &h[3ull * ((uint64_t)k * npix + p)];
                float* dst = out_L + 3ull * ((uint64_t)p * rd->spp + (R.s_lo + k));
                dst[0] = src[0];
                dst[1] = src[1];
                dst[2] = src[2];
            }
        return PT_OK;
    }));
}

extern "C" pt_status pt_film_resolve(pt_ctx* c, const double* film, int32_t width, int32_t height, uint32_t tonemap,
                                     uint8_t* rgb) {
    if (!c || !film || !rgb || width <= 0 || height <= 0 || (uint64_t)width * height > (1ull << 31) ||
        tonemap > PT_TONEMAP_ACES)
        return PT_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    const uint32_t npx = (uint32_t)width * (uint32_t)height;
    const bool fdev = is_device_ptr(film), odev = is_device_ptr(rgb);
    const double* df = film;
    uint8_t* dout = rgb;
    std::vector<void*> tmp;
    auto cleanup = [&]() {
        hipStreamSynchronize(c->stream);
        for (void* p : tmp) hipFree(p);
    };
    if (!fdev) {
        void* p = nullptr;
        if (hipMalloc(&p, 32ull * npx) != hipSuccess) return fail(c, PT_ERR_OOM, "film resolve: device film");
        tmp.push_back(p);
        df = (const double*)p;
        if (hipMemcpyAsync(p, film, 32ull * npx, hipMemcpyHostToDevice, c->stream) != hipSuccess) {
            cleanup();
            return fail(c, PT_ERR_HIP, "film resolve: upload");
        }
    }
    if (!odev) {
        void* p = nullptr;
        if (hipMalloc(&p, 3ull * npx) != hipSuccess) {
            cleanup();
            return fail(c, PT_ERR_OOM, "film resolve: device image");
        }
        tmp.push_back(p);
        dout = (uint8_t*)p;
    }
    hipLaunchKernelGGL(k_resolve, dim3((npx + 255) / 256), dim3(256), 0, c->stream, df, npx, tonemap, dout);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess && !odev) e = hipMemcpyAsync(rgb, dout, 3ull * npx, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    cleanup();
    if (e != hipSuccess) return fail(c, PT_ERR_HIP, "film resolve: %s", hipGetErrorString(e));
    return PT_OK;
}

extern "C" pt_status pt_trace(pt_ctx* c, const pt_ray* rays, uint32_t n, int any_hit, pt_hit* hits, pt_stats* stats) {
    if (!c) return PT_ERR_ARG;
    DeviceLock dl(c->device);
    if (!c || (n && (!rays || !hits))) return PT_ERR_ARG;
    if (!c->has_scene) return fail(c, PT_ERR_STATE, "no scene uploaded");
    HIPCHK(c, hipSetDevice(c->device));
    if (n == 0) return PT_OK;
    const bool rdev = is_device_ptr(rays), hdev = is_device_ptr(hits);
    pt_ray* dr = (pt_ray*)rays;
    pt_hit* dh = hits;
    std::vector<void*> tmp;
    if (!rdev) {
        HIPCHK(c, hipMalloc((void**)&dr, (size_t)n * sizeof(pt_ray)));
        tmp.push_back(dr);
        HIPCHK(c, hipMemcpyAsync(dr, rays, (size_t)n * sizeof(pt_ray), hipMemcpyHostToDevice, c->stream));
    }
    if (!hdev) {
        HIPCHK(c, hipMalloc((void**)&dh, (size_t)n * sizeof(pt_hit)));
        tmp.push_back(dh);
    }
    if (c->cap == 0 && ensure_work(c, 256) != PT_OK) return PT_ERR_OOM;
    if (pt_status bs = bind_scene(c)) return bs;
    HIPCHK(c, hipMemsetAsync(c->counters, 0, CNT_SHARDS * CNT_COUNT * 8, c->stream));
    HIPCHK(c, hipMemsetAsync(c->stack_drops, 0, 8, c->stream));  // stack and tie drops
    auto t0 = std::chrono::steady_clock::now();
    HIPCHK(c, hipEventRecord(c->ev[4], c->stream));
    uint32_t* pool = c->qcnt + 3 * SET_WORDS;
    uint32_t* n_ties = pool + PT_POOL_WORDS;
    HIPCHK(c, hipMemsetAsync(pool, 0, (PT_POOL_WORDS + Q_STRIDE) * 4, c->stream));
    uint32_t* tl = nullptr;  // rays listed for the exact re-trace (at most each once)
    HIPCHK(c, hipMalloc((void**)&tl, (size_t)n * 4));
    tmp.push_back(tl);
    // the pool traversal of the renderer: quantized nodes where the renderer
    // would use them (large scenes), unless pt_set_node_format says otherwise
    const bool qn = c->has_qnodes && (c->node_format == PT_NODES_QUANTIZED ||
                                      (c->node_format == PT_NODES_AUTO && c->n_clusters >= PT_POOL_MIN_CLUSTERS));
    const uint32_t tb = std::max(1u, std::min((n + PT_TRACE_BLOCK - 1) / PT_TRACE_BLOCK, c->trace_blocks));
    if (any_hit == 2) {  // the stackless any-hit traversal
        if (!qn || c->scene.n_instances) {
            for (void* p : tmp) hipFree(p);
            return fail(c, PT_ERR_ARG, "the stackless any-hit traversal needs quantized records and no instances");
        }
        hipLaunchKernelGGL(k_trace_rays_sl, dim3(std::max(1u, std::min((n + PT_TRACE_BLOCK - 1) / PT_TRACE_BLOCK,
                                                                        c->sl_blocks))),
                           dim3(PT_TRACE_BLOCK), 0, c->stream, (const pt_ray*)dr, n, dh, pool, c->counters);
    } else {
        hipLaunchKernelGGL(qn ? k_trace_rays<true> : k_trace_rays<false>, dim3(tb), dim3(PT_TRACE_BLOCK), 0, c->stream,
                           dr, n, any_hit, dh, pool, c->ovf, c->counters, tl, n_ties);
    }
    HIPCHK(c, hipGetLastError());
    if (!any_hit)
        hipLaunchKernelGGL(k_trace_rays_ties, dim3(std::min(64u, tb)), dim3(PT_TRACE_BLOCK), 0, c->stream,
                           (const pt_ray*)dr, dh, (const uint32_t*)tl, (const uint32_t*)n_ties, (uint32_t)n);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipEventRecord(c->ev[5], c->stream));
    if (!hdev) HIPCHK(c, hipMemcpyAsync(hits, dh, (size_t)n * sizeof(pt_hit), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (stats) {
        *stats = pt_stats{};
        unsigned long long hs[CNT_SHARDS * CNT_COUNT], h[CNT_COUNT] = {};
        HIPCHK(c, hipMemcpy(hs, c->counters, sizeof(hs), hipMemcpyDeviceToHost));
        for (int k = 0; k < CNT_SHARDS; k++)
            for (int j = 0; j < CNT_COUNT; j++) h[j] += hs[k * CNT_COUNT + j];
        float ms;
        HIPCHK(c, hipEventElapsedTime(&ms, c->ev[4], c->ev[5]));
        if (any_hit) {
            stats->rays_any = n;
            stats->nodes_any = h[CNT_NODES_ANY];
            stats->tris_any = h[CNT_TRIS_ANY];
            stats->ms_any = ms;
        } else {
            stats->rays_closest = n;
            stats->nodes_closest = h[CNT_NODES_CLOSEST];
            stats->tris_closest = h[CNT_TRIS_CLOSEST];
            stats->ms_closest = ms;
        }
        uint32_t drops[2] = {0, 0};
        HIPCHK(c, hipMemcpy(drops, c->stack_drops, 8, hipMemcpyDeviceToHost));
        stats->stack_overflows = drops[0];
        stats->tie_overflows = drops[1];
        stats->n_devices = 1;
        stats->ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    for (void* p : tmp) hipFree(p);
    return PT_OK;
}

// Copies n*in_stride floats/records to the device, runs `launch`, copies
// n*out_stride floats back (test hooks; host pointers).
template <class L>
static pt_status run_hook(pt_ctx* c, const void* in, size_t in_bytes, float* out, size_t out_bytes, L launch) {
    void* din = nullptr;
    float* dout = nullptr;
    if (hipMalloc(&din, in_bytes ? in_bytes : 1) != hipSuccess) return fail(c, PT_ERR_OOM, "hook input");
    if (hipMalloc((void**)&dout, out_bytes ? out_bytes : 4) != hipSuccess) {
        hipFree(din);
        return fail(c, PT_ERR_OOM, "hook output");
    }
    pt_status st = bind_scene(c);
    if (st == PT_OK && hipMemcpyAsync(din, in, in_bytes, hipMemcpyHostToDevice, c->stream) != hipSuccess)
        st = PT_ERR_HIP;
    if (st == PT_OK) {
        launch(din, dout);
        if (hipGetLastError() != hipSuccess) st = PT_ERR_HIP;
    }
    if (st == PT_OK && hipMemcpyAsync(out, dout, out_bytes, hipMemcpyDeviceToHost, c->stream) != hipSuccess)
        st = PT_ERR_HIP;
    if (st == PT_OK && hipStreamSynchronize(c->stream) != hipSuccess) st = PT_ERR_HIP;
    hipFree(din);
    hipFree(dout);
    return st == PT_OK ? PT_OK : fail(c, st, "hook kernel failed");
}

extern "C" pt_status pt_interact(pt_ctx* c, const pt_ray* rays, uint32_t n, float* out) {
    if (!c) return PT_ERR_ARG;
    DeviceLock dl(c->device);
    if (!c || (n && (!rays || !out))) return PT_ERR_ARG;
    if (!c->has_scene) return fail(c, PT_ERR_STATE, "no scene uploaded");
    HIPCHK(c, hipSetDevice(c->device));
    if (n == 0) return PT_OK;
    if (pt_status st = ensure_scratch(c, (uint64_t)(n + PT_TRACE_BLOCK - 1) / PT_TRACE_BLOCK * PT_TRACE_BLOCK))
        return st;
    return run_hook(c, rays, (size_t)n * sizeof(pt_ray), out, (size_t)n * 16 * sizeof(float),
                    [&](void* din, float* dout) {
                        hipLaunchKernelGGL(k_interact, dim3((n + PT_TRACE_BLOCK - 1) / PT_TRACE_BLOCK),
                                           dim3(PT_TRACE_BLOCK), 0, c->stream, (const pt_ray*)din, n, dout);
                    });
}

extern "C" pt_status pt_bsdf_cases(pt_ctx* c, int32_t material, const float* cases, uint32_t n, float* out) {
    if (!c) return PT_ERR_ARG;
    DeviceLock dl(c->device);
    if (!c || (n && (!cases || !out))) return PT_ERR_ARG;
    if (!c->has_scene) return fail(c, PT_ERR_STATE, "no scene uploaded");
    if (material < 0 || (uint32_t)material >= c->n_materials) return fail(c, PT_ERR_ARG, "bad material id");
    HIPCHK(c, hipSetDevice(c->device));
    if (n == 0) return PT_OK;
    return run_hook(c, cases, (size_t)n * 27 * sizeof(float), out, (size_t)n * 20 * sizeof(float),
                    [&](void* din, float* dout) {
                        hipLaunchKernelGGL(k_bsdf_cases, dim3((n + 127) / 128), dim3(128), 0, c->stream,
                                           (int)material, (const float*)din, n, dout);
                    });
}

extern "C" pt_status pt_light_cases(pt_ctx* c, const float* cases, uint32_t n, float* out) {
    if (!c) return PT_ERR_ARG;
    DeviceLock dl(c->device);
    if (!c || (n && (!cases || !out))) return PT_ERR_ARG;
    if (!c->has_scene) return fail(c, PT_ERR_STATE, "no scene uploaded");
    HIPCHK(c, hipSetDevice(c->device));
    const uint64_t total = (uint64_t)n * c->scene.n_lights;
    if (total == 0) return PT_OK;
    if (total > 0xFFFFFFFFull) return fail(c, PT_ERR_ARG, "too many light cases");
    return run_hook(c, cases, (size_t)n * 5 * sizeof(float), out, (size_t)total * 18 * sizeof(float),
                    [&](void* din, float* dout) {
                        hipLaunchKernelGGL(k_light_cases, dim3((uint32_t)((total + 127) / 128)), dim3(128), 0,
                                           c->stream, (const float*)din, n, dout);
                    });
}

extern "C" pt_status pt_light_picks(pt_ctx* c, const float* u, uint32_t n, int32_t* out) {
    if (!c) return PT_ERR_ARG;
    DeviceLock dl(c->device);
    if (!c || (n && (!u || !out))) return PT_ERR_ARG;
    if (!c->has_scene) return fail(c, PT_ERR_STATE, "no scene uploaded");
    HIPCHK(c, hipSetDevice(c->device));
    if (n == 0) return PT_OK;
    return run_hook(c, u, (size_t)n * sizeof(float), reinterpret_cast<float*>(out), (size_t)n * sizeof(int32_t),
                    [&](void* din, float* dout) {
                        hipLaunchKernelGGL(k_light_picks, dim3((n + 255) / 256), dim3(256), 0, c->stream,
                                           (const float*)din, n, reinterpret_cast<int32_t*>(dout));
                    });
}

// Test hook (host code, no device): the coverage mask sets pt_scene_upload
// stores for the alpha-tested triangles (pt_alpha_cov.h), per slot.
extern "C" pt_status pt_alpha_coverage(const pt_scene_desc* s, uint32_t* out) {
    if (!s || !out) return PT_ERR_ARG;
    if (pt_status st = validate_scene(nullptr, s)) return st;
    std::vector<DevGeom> geom(s->n_prims + 1);
    std::vector<DevPrimInfo> info(s->n_prims);
    slot_geometry(s, geom, info);
    alpha_records(s, geom, nullptr, nullptr, out);
    return PT_OK;
}

extern "C" pt_status pt_anim_inverse_cases(pt_ctx* c, const float* t, uint32_t n, float* out) {
    if (!c) return PT_ERR_ARG;
    DeviceLock dl(c->device);
    if (n && (!t || !out)) return PT_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    if (n == 0) return PT_OK;
    float *dt = nullptr, *dout = nullptr;
    if (hipMalloc((void**)&dt, (size_t)n * 12) != hipSuccess) return fail(c, PT_ERR_OOM, "hook input");
    if (hipMalloc((void**)&dout, (size_t)n * 64) != hipSuccess) {
        hipFree(dt);
        return fail(c, PT_ERR_OOM, "hook output");
    }
    pt_status st = PT_OK;
    if (hipMemcpyAsync(dt, t, (size_t)n * 12, hipMemcpyHostToDevice, c->stream) != hipSuccess) st = PT_ERR_HIP;
    if (st == PT_OK) {
        hipLaunchKernelGGL(k_anim_inverse, dim3((n + 255) / 256), dim3(256), 0, c->stream, (const float*)dt, n, dout);
        if (hipGetLastError() != hipSuccess) st = PT_ERR_HIP;
    }
    if (st == PT_OK && hipMemcpyAsync(out, dout, (size_t)n * 64, hipMemcpyDeviceToHost, c->stream) != hipSuccess)
        st = PT_ERR_HIP;
    if (st == PT_OK && hipStreamSynchronize(c->stream) != hipSuccess) st = PT_ERR_HIP;
    hipFree(dt);
    hipFree(dout);
    return st == PT_OK ? PT_OK : fail(c, st, "anim_inverse hook failed");
}

// Device BVH build (pt_bvh4_build_device)
#include "pt_bvh_gpu.hip"
