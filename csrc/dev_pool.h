// Caching device allocator for the per-call scratch buffers of the host wrappers (block verify,
// decompression, batched SHA-256, UTXO passes).
//
// hipMalloc + hipFree per call cost ~0.1-0.3 ms each, and hipFree synchronises the device. One 2 MB
// block makes a dozen such calls, and the ECDSA launch itself takes only ~3 ms. Buffers here are
// rounded up to a power-of-two size class and parked on a per-device free list when released, so
// the steady state makes no driver allocations at all. Reuse is safe because every node-side launch
// and copy goes to the device's node stream (csrc/streams.h) and each call synchronises that stream
// before its buffers are released: a later call's H2D copy into a recycled buffer is ordered after
// the earlier kernels that used it. Memory is never returned to the driver; the high-water mark is
// bounded by the largest batch (a few tens of MB per device).
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <mutex>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

namespace upow {

class DevPool {
public:
    static void* alloc(size_t bytes) {
        int dev = 0;
        check(hipGetDevice(&dev), "hipGetDevice");
        const int cls = size_class(bytes);
        DevPool& p = get();
        {
            std::lock_guard<std::mutex> g(p.mu_);
            auto& fl = p.free_[key(dev, cls)];
            if (!fl.empty()) {
                void* ptr = fl.back();
                fl.pop_back();
                p.live_[ptr] = key(dev, cls);
                return ptr;
            }
        }
        void* ptr = nullptr;
        check(hipMalloc(&ptr, size_t(1) << cls), "hipMalloc (pool)");
        std::lock_guard<std::mutex> g(p.mu_);
        p.live_[ptr] = key(dev, cls);
        return ptr;
    }

    static void release(void* ptr) {
        if (!ptr) return;
        DevPool& p = get();
        std::lock_guard<std::mutex> g(p.mu_);
        auto it = p.live_.find(ptr);
        if (it == p.live_.end()) return;
        p.free_[it->second].push_back(ptr);
        p.live_.erase(it);
    }

private:
    static DevPool& get() {
        static DevPool* p = new DevPool();  // never destroyed: the HIP runtime may be gone at exit
        return *p;
    }
    static int size_class(size_t bytes) {
        int c = 8;  // 256 B minimum
        while ((size_t(1) << c) < bytes) ++c;
        return c;
    }
    static long long key(int dev, int cls) { return (static_cast<long long>(dev) << 8) | cls; }
    static void check(hipError_t e, const char* what) {
        if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
    }

    std::mutex mu_;
    std::unordered_map<long long, std::vector<void*>> free_;
    std::unordered_map<void*, long long> live_;
};

// RAII scratch buffer of n elements from the pool.
template <typename T>
struct PooledBuf {
    T* p = nullptr;
    explicit PooledBuf(size_t n) { p = static_cast<T*>(DevPool::alloc(sizeof(T) * (n ? n : 1))); }
    ~PooledBuf() { DevPool::release(p); }
    PooledBuf(const PooledBuf&) = delete;
    PooledBuf& operator=(const PooledBuf&) = delete;
};

}  // namespace upow
