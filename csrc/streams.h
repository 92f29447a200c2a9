// HIP streams for sharing one MI355X between the node and a co-located miner.
//
// Every node-side launch (block verify, decompression, batched SHA-256, the UTXO table passes) goes to
// a per-device NON-BLOCKING stream created at the device's greatest priority; the PoW search goes to a
// stream at the least priority. The command processor then dispatches a waiting node kernel's
// workgroups ahead of the miner's as soon as CUs free up (there is no preemption: the miner's dispatch
// length, UPOW_POW_DISPATCH_LOG2, bounds the wait). Host copies are stream-ordered; a D2H copy is
// followed by a sync of the same stream only, never of the whole device.
// UPOW_NODE_STREAM_PRIORITY=normal puts the node stream at the default priority (A/B).
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>

namespace upow {

inline void stream_check(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

// The GPU a process's node-side work belongs to (-1: whatever the calling thread has current). A
// multi-GPU rank sets it once (``set_node_device``), so GPU calls made from its ledger worker thread
// and executor threads, which start on device 0, still land on the rank's own GPU.
inline std::atomic<int>& node_device_ref() {
    static std::atomic<int> dev{-1};
    return dev;
}
inline void set_node_device(int dev) { node_device_ref().store(dev); }
// Called at the top of every node-side GPU entry point, before any allocation or launch.
inline void node_device_enter() {
    const int want = node_device_ref().load();
    if (want < 0) return;
    int cur = 0;
    stream_check(hipGetDevice(&cur), "hipGetDevice");
    if (cur != want) stream_check(hipSetDevice(want), "hipSetDevice");
}

// Aux: background node work that must not sit in front of a block's kernels on the node stream (the
// K12 UTXO-set digest's sort and gather), at the least priority
enum class StreamRole { Node = 0, Miner = 1, Aux = 2 };

// set once this process has issued node work (UTXO passes, ECDSA, ...): a miner in the same process then
// keeps its dispatches short (csrc/pow_search.hip)
inline std::atomic<bool>& node_stream_live() {
    static std::atomic<bool> live{false};
    return live;
}

inline hipStream_t role_stream(StreamRole role) {
    constexpr int kMaxDev = 64;
    static std::mutex mu;
    static hipStream_t streams[3][kMaxDev] = {};
    int dev = 0;
    stream_check(hipGetDevice(&dev), "hipGetDevice");
    if (dev < 0 || dev >= kMaxDev) throw std::runtime_error("device ordinal out of range");
    const int r = int(role);
    std::lock_guard<std::mutex> g(mu);
    if (!streams[r][dev]) {
        int least = 0, greatest = 0;
        stream_check(hipDeviceGetStreamPriorityRange(&least, &greatest), "hipDeviceGetStreamPriorityRange");
        int prio = role == StreamRole::Node ? greatest : least;
        if (role == StreamRole::Node) {
            const char* e = std::getenv("UPOW_NODE_STREAM_PRIORITY");
            if (e && std::strcmp(e, "normal") == 0) prio = 0;
        }
        stream_check(hipStreamCreateWithPriority(&streams[r][dev], hipStreamNonBlocking, prio),
                     "hipStreamCreateWithPriority");
        if (role == StreamRole::Node) node_stream_live().store(true);
    }
    return streams[r][dev];
}

inline hipStream_t node_stream() { return role_stream(StreamRole::Node); }
inline hipStream_t miner_stream() { return role_stream(StreamRole::Miner); }
inline hipStream_t aux_stream() { return role_stream(StreamRole::Aux); }

inline void node_h2d(void* dst, const void* src, size_t n, const char* what = "h2d") {
    if (n) stream_check(hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, node_stream()), what);
}

// D2H into (pageable) host memory; returns after the data has landed
inline void node_d2h(void* dst, const void* src, size_t n, const char* what = "d2h") {
    if (!n) return;
    stream_check(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, node_stream()), what);
    stream_check(hipStreamSynchronize(node_stream()), what);
}

inline void node_memset(void* dst, int v, size_t n, const char* what = "memset") {
    if (n) stream_check(hipMemsetAsync(dst, v, n, node_stream()), what);
}

inline void node_sync(const char* what = "node stream sync") {
    stream_check(hipStreamSynchronize(node_stream()), what);
}

// Pinned staging for one node-side call's transfers (per thread, grown on demand, never returned: the
// HIP runtime may be gone when threads exit). A pageable hipMemcpyAsync is a staged, host-synchronous
// copy, and every node_d2h above ends in its own stream sync; a block's UTXO pass made five of them. With
// StagedIO the inputs are packed into pinned memory and DMA'd asynchronously, all outputs land in pinned
// memory with ONE stream sync, then are unpacked. The buffer is reused only after that sync.
struct NodeStageBuf {
    uint8_t* p = nullptr;
    size_t cap = 0;
};
inline uint8_t* node_stage(size_t n) {
    thread_local NodeStageBuf* b = new NodeStageBuf();
    if (n > b->cap) {
        if (b->p) (void)hipHostFree(b->p);  // the previous call on this thread synced its stream
        size_t c = b->cap ? b->cap : (size_t(1) << 20);
        while (c < n) c *= 2;
        b->p = nullptr;
        stream_check(hipHostMalloc(reinterpret_cast<void**>(&b->p), c, hipHostMallocDefault), "hipHostMalloc stage");
        b->cap = c;
    }
    return b->p;
}

class StagedIO {
public:
    explicit StagedIO(size_t total) : base_(node_stage(total + 64 * 16)), cap_(total + 64 * 16) {}
    void h2d(void* dst, const void* src, size_t n) {
        if (!n) return;
        uint8_t* at = take(n);
        std::memcpy(at, src, n);
        stream_check(hipMemcpyAsync(dst, at, n, hipMemcpyHostToDevice, node_stream()), "staged h2d");
    }
    // pinned space for an input the caller writes in place (no staging copy), then issued by h2d_issue
    uint8_t* h2d_take(size_t n) { return take(n); }
    void h2d_issue(void* dst, const uint8_t* at, size_t n) {
        if (n) stream_check(hipMemcpyAsync(dst, at, n, hipMemcpyHostToDevice, node_stream()), "staged h2d");
    }
    void d2h(void* dst, const void* src, size_t n) {
        if (!n) return;
        uint8_t* at = take(n);
        stream_check(hipMemcpyAsync(at, src, n, hipMemcpyDeviceToHost, node_stream()), "staged d2h");
        outs_[n_out_++] = {dst, at, n};
    }
    // one D2H of a whole device arena into pinned space; the caller unpacks it after finish()
    const uint8_t* d2h_arena(const void* src, size_t n) {
        uint8_t* at = take(n);
        if (n) stream_check(hipMemcpyAsync(at, src, n, hipMemcpyDeviceToHost, node_stream()), "staged d2h");
        return at;
    }
    // one sync for every transfer of the call, then the outputs are unpacked
    void finish(const char* what = "staged sync") {
        node_sync(what);
        for (int i = 0; i < n_out_; ++i) std::memcpy(outs_[i].dst, outs_[i].at, outs_[i].n);
        n_out_ = 0;
    }

private:
    uint8_t* take(size_t n) {
        const size_t a = (used_ + 63) & ~size_t(63);
        if (a + n > cap_) throw std::runtime_error("StagedIO: transfer plan larger than declared");
        used_ = a + n;
        return base_ + a;
    }
    struct Out {
        void* dst;
        const uint8_t* at;
        size_t n;
    };
    uint8_t* base_;
    size_t cap_, used_ = 0;
    Out outs_[16];
    int n_out_ = 0;
};

}  // namespace upow
