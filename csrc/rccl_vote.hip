// The cluster node's per-block commit vote issued from the native runtime on a communicator of its own.
//
// Every block a multi-GPU cluster node commits is preceded by one agreement (parallel/cluster.py
// CommitGate): each rank contributes 1 (ready) or 0. Through torch.distributed that is a Python call, a
// ProcessGroupNCCL work object, a host-to-device copy and a device-to-host copy per block: ~22 us of host time
// to queue in isolation and 60-70 us inside a syncing node (profiles/r5/cluster_sync_*). Here the vote is an
// ncclAllGather of one int64 from a constant device word (0 or 1; no host-to-device copy) into a small
// receive vector, the vector's copy into pinned memory and an event, queued on a dedicated stream with the
// GIL released; the outcome is collected by polling the event (a dead peer ends in a timeout, not a hang).
//
// RCCL is resolved with dlopen from the copy PyTorch already loaded (RTLD_NOLOAD first, the same SONAME), so
// the process holds one RCCL. The communicator is created once per rank from a unique id that rank 0 makes
// and the job's existing process group broadcasts (parallel/dist.py NativeVote).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <dlfcn.h>

#include <chrono>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "native.h"
#include "streams.h"

namespace upow {

namespace {

struct RcclApi {
    ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*comm_abort)(ncclComm_t) = nullptr;
    const char* (*error_string)(ncclResult_t) = nullptr;
};

const RcclApi& rccl() {
    static RcclApi api;
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);  // PyTorch's copy, when it is loaded
        if (!h) h = dlopen("librccl.so.1", RTLD_NOW);
        if (!h) h = dlopen("librccl.so", RTLD_NOW);
        if (!h) throw std::runtime_error("rccl vote: librccl not found");
        auto sym = [h](auto& fp, const char* name) {
            fp = reinterpret_cast<std::remove_reference_t<decltype(fp)>>(dlsym(h, name));
            if (!fp) throw std::runtime_error(std::string("rccl vote: missing symbol ") + name);
        };
        sym(api.get_unique_id, "ncclGetUniqueId");
        sym(api.comm_init_rank, "ncclCommInitRank");
        sym(api.all_gather, "ncclAllGather");
        sym(api.comm_destroy, "ncclCommDestroy");
        sym(api.comm_abort, "ncclCommAbort");
        sym(api.error_string, "ncclGetErrorString");
    });
    return api;
}

void nck(ncclResult_t r, const char* what) {
    if (r != ncclSuccess) throw std::runtime_error(std::string(what) + ": " + rccl().error_string(r));
}
void hck(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

struct Vote {
    ncclComm_t comm = nullptr;
    int world = 0, device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev = nullptr;
    int64_t* d_const = nullptr;  // {0, 1}
    int64_t* d_out = nullptr;    // world entries
    int64_t* h_out = nullptr;    // pinned
    bool pending = false;
    // host time of the three enqueues (all-gather, copy, event) summed over the votes: rccl_vote_stats
    double t_gather = 0, t_copy = 0, t_event = 0;
    int64_t votes = 0;
};

std::mutex g_mu;
std::vector<Vote*> g_votes;

Vote& vote_of(int64_t h) {
    if (h < 0 || size_t(h) >= g_votes.size() || !g_votes[size_t(h)]) throw std::invalid_argument("bad vote handle");
    Vote& v = *g_votes[size_t(h)];
    int cur = 0;
    hck(hipGetDevice(&cur), "hipGetDevice");
    if (cur != v.device) hck(hipSetDevice(v.device), "hipSetDevice");
    return v;
}

}  // namespace

std::string rccl_unique_id() {
    ncclUniqueId id;
    nck(rccl().get_unique_id(&id), "ncclGetUniqueId");
    return std::string(id.internal, sizeof id.internal);
}

int64_t rccl_vote_create(const std::string& uid, int world, int rank) {
    if (uid.size() != NCCL_UNIQUE_ID_BYTES) throw std::invalid_argument("rccl unique id must be 128 bytes");
    if (world < 1 || rank < 0 || rank >= world) throw std::invalid_argument("bad world / rank");
    node_device_enter();
    auto* v = new Vote();
    hck(hipGetDevice(&v->device), "hipGetDevice");
    v->world = world;
    ncclUniqueId id;
    std::memcpy(id.internal, uid.data(), sizeof id.internal);
    try {
        nck(rccl().comm_init_rank(&v->comm, world, id, rank), "ncclCommInitRank");  // collective over the ranks
        int least = 0, greatest = 0;
        hck(hipDeviceGetStreamPriorityRange(&least, &greatest), "stream priorities");
        hck(hipStreamCreateWithPriority(&v->stream, hipStreamNonBlocking, greatest), "vote stream");
        hck(hipEventCreateWithFlags(&v->ev, hipEventDisableTiming), "vote event");
        hck(hipMalloc(reinterpret_cast<void**>(&v->d_const), 2 * sizeof(int64_t)), "vote const");
        const int64_t c[2] = {0, 1};
        hck(hipMemcpy(v->d_const, c, sizeof c, hipMemcpyHostToDevice), "vote const h2d");
        hck(hipMalloc(reinterpret_cast<void**>(&v->d_out), size_t(world) * sizeof(int64_t)), "vote out");
        hck(hipHostMalloc(reinterpret_cast<void**>(&v->h_out), size_t(world) * sizeof(int64_t), hipHostMallocDefault),
            "vote pinned");
    } catch (...) {
        if (v->comm) (void)rccl().comm_abort(v->comm);
        delete v;
        throw;
    }
    std::lock_guard<std::mutex> lk(g_mu);
    g_votes.push_back(v);
    return int64_t(g_votes.size() - 1);
}

void rccl_vote_start(int64_t h, int value) {
    std::lock_guard<std::mutex> lk(g_mu);
    Vote& v = vote_of(h);
    if (v.pending) throw std::runtime_error("rccl vote: a vote is already pending");
    if (value != 0 && value != 1) throw std::invalid_argument("a vote is 0 or 1");
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    nck(rccl().all_gather(v.d_const + value, v.d_out, 1, ncclInt64, v.comm, v.stream), "ncclAllGather (vote)");
    const auto t1 = clk::now();
    hck(hipMemcpyAsync(v.h_out, v.d_out, size_t(v.world) * sizeof(int64_t), hipMemcpyDeviceToHost, v.stream), "vote d2h");
    const auto t2 = clk::now();
    hck(hipEventRecord(v.ev, v.stream), "vote event");
    const auto t3 = clk::now();
    v.t_gather += std::chrono::duration<double>(t1 - t0).count();
    v.t_copy += std::chrono::duration<double>(t2 - t1).count();
    v.t_event += std::chrono::duration<double>(t3 - t2).count();
    ++v.votes;
    v.pending = true;
}

std::vector<double> rccl_vote_stats(int64_t h) {
    std::lock_guard<std::mutex> lk(g_mu);
    Vote& v = vote_of(h);
    return {double(v.votes), v.t_gather, v.t_copy, v.t_event};
}

// the SUM of the ranks' votes, or -1 when it has not arrived within timeout_s (the caller treats that as a
// failed collective: every rank's fatal path then exits)
int64_t rccl_vote_finish(int64_t h, double timeout_s) {
    Vote* vp;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        vp = &vote_of(h);
        if (!vp->pending) throw std::runtime_error("rccl vote: nothing pending");
    }
    Vote& v = *vp;
    const auto t0 = std::chrono::steady_clock::now();
    for (int spin = 0;; ++spin) {
        const hipError_t q = hipEventQuery(v.ev);
        if (q == hipSuccess) break;
        if (q != hipErrorNotReady) hck(q, "vote event");
        if (spin > 2048) {  // ~1 us per query: a vote that is in flight arrives within the spin
            if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s) return -1;
            std::this_thread::sleep_for(std::chrono::microseconds(20));
        }
    }
    v.pending = false;
    int64_t sum = 0;
    for (int r = 0; r < v.world; ++r) sum += v.h_out[r];
    return sum;
}

void rccl_vote_destroy(int64_t h, bool abort) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (h < 0 || size_t(h) >= g_votes.size() || !g_votes[size_t(h)]) return;
    Vote* v = g_votes[size_t(h)];
    g_votes[size_t(h)] = nullptr;
    (void)hipSetDevice(v->device);
    if (v->comm) (void)(abort ? rccl().comm_abort(v->comm) : rccl().comm_destroy(v->comm));
    if (v->stream) (void)hipStreamDestroy(v->stream);
    if (v->ev) (void)hipEventDestroy(v->ev);
    if (v->d_const) (void)hipFree(v->d_const);
    if (v->d_out) (void)hipFree(v->d_out);
    if (v->h_out) (void)hipHostFree(v->h_out);
    delete v;
}

}  // namespace upow
