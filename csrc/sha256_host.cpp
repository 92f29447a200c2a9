// Host (CPU) implementations: scalar/threaded SHA-256 batch and the PoW host search used for the
// CPU fallback, the ragged tail of a GPU sweep and the exact re-check of GPU candidates.
#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <thread>
#include <vector>

#include "native.h"
#include "sha256_common.h"

namespace upow {

static uint32_t pow_h0_host(const PowJobHost& job, uint32_t v) {
    const size_t len = job.header.size();
    uint8_t hdr[138];
    std::memcpy(hdr, job.header.data(), len);
    uint32_t nonce = len == 108 ? __builtin_bswap32(v) : v;
    for (int i = 0; i < 4; ++i) hdr[len - 4 + i] = uint8_t(nonce >> (8 * i));
    uint8_t out[32];
    host_sha256(hdr, len, out);
    return load_be32(out);
}

bool pow_check_word_host(const PowJobHost& job, uint32_t v) {
    const uint32_t h0 = pow_h0_host(job, v);
    return ((h0 ^ job.tword) & job.tmask) == 0 && ((h0 >> job.frac_shift) & 0xfu) < job.frac_limit;
}

PowResult pow_search_host(const PowJobHost& job, uint64_t start, uint64_t count, int threads) {
    if (job.header.size() != 108 && job.header.size() != 138)
        throw std::invalid_argument("header must be 108 (v2) or 138 (v1) bytes");
    threads = std::max(1, threads);
    std::vector<std::vector<uint32_t>> hits(threads);
    std::vector<std::thread> pool;
    for (int t = 0; t < threads; ++t) {
        pool.emplace_back([&, t] {
            // strided partition, like the reference's worker i starting at nonce i (miner.py:139-148)
            for (uint64_t k = t; k < count; k += threads) {
                const uint32_t v = uint32_t(start + k);
                if (pow_check_word_host(job, v)) hits[t].push_back(v);
            }
        });
    }
    for (auto& th : pool) th.join();
    PowResult r;
    r.searched = count;
    for (auto& h : hits) r.words.insert(r.words.end(), h.begin(), h.end());
    std::sort(r.words.begin(), r.words.end());
    r.total_hits = uint32_t(r.words.size());
    return r;
}

std::vector<uint8_t> sha256_batch_host(const uint8_t* data, const int64_t* offsets, int64_t n, int threads) {
    std::vector<uint8_t> out(size_t(n) * 32);
    threads = std::max<int>(1, std::min<int64_t>(threads, n > 0 ? n : 1));
    auto work = [&](int t) {
        for (int64_t i = t; i < n; i += threads)
            host_sha256(data + offsets[i], size_t(offsets[i + 1] - offsets[i]), out.data() + 32 * i);
    };
    if (threads == 1) {
        work(0);
    } else {
        std::vector<std::thread> pool;
        for (int t = 0; t < threads; ++t) pool.emplace_back(work, t);
        for (auto& th : pool) th.join();
    }
    return out;
}

}  // namespace upow
