// ThreadSanitizer self-test of the persistent host worker pool (csrc/thread_pool.h), the one piece
// of shared-memory concurrency in the native runtime: every block decode, address pass and codec
// release runs on it. Built and run by tools/sanitize_host.sh with -fsanitize=thread.
#include <atomic>
#include <cstdio>
#include <stdexcept>
#include <thread>
#include <vector>

#include "thread_pool.h"

using upow::HostPool;

static int failures = 0;
#define CHECK(c)                                                    \
    do {                                                            \
        if (!(c)) {                                                 \
            std::fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, #c); \
            ++failures;                                             \
        }                                                           \
    } while (0)

int main() {
    // every index exactly once, for thread counts that grow and shrink between regions
    for (int threads : {1, 2, 8, 3, 16, 4, 1, 32}) {
        for (int64_t n : {0, 1, 63, 64, 1000, 8300, 100000}) {
            std::vector<int> hits(size_t(n), 0);
            HostPool::get().parallel_for(n, threads, [&](int64_t i) { hits[size_t(i)]++; });
            bool once = true;
            for (int h : hits) once &= h == 1;
            CHECK(once);
        }
    }
    // an exception in any participant stops the region and reaches the caller; the pool stays usable
    for (int rep = 0; rep < 20; ++rep) {
        bool caught = false;
        try {
            HostPool::get().parallel_for(50000, 8, [&](int64_t i) {
                if (i == 12345 + rep) throw std::runtime_error("injected");
            });
        } catch (const std::runtime_error&) {
            caught = true;
        }
        CHECK(caught);
        std::atomic<int64_t> sum{0};
        HostPool::get().parallel_for(50000, 8, [&](int64_t i) { sum += i; });
        CHECK(sum.load() == int64_t(50000) * 49999 / 2);
    }
    // two caller threads at once (the event loop and the sync decode-ahead thread): regions serialise
    std::atomic<int64_t> a{0}, b{0};
    std::thread t1([&] {
        for (int r = 0; r < 50; ++r) HostPool::get().parallel_for(4000, 8, [&](int64_t) { a++; });
    });
    std::thread t2([&] {
        for (int r = 0; r < 50; ++r) HostPool::get().parallel_for(3000, 4, [&](int64_t) { b++; });
    });
    t1.join();
    t2.join();
    CHECK(a.load() == 50 * 4000 && b.load() == 50 * 3000);
    if (failures) {
        std::fprintf(stderr, "%d failure(s)\n", failures);
        return 1;
    }
    std::printf("pool selftest: all checks passed\n");
    return 0;
}
