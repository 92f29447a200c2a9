// Host-side self-test of the native library's CPU paths, built with AddressSanitizer and
// UndefinedBehaviorSanitizer by tools/sanitize_host.sh ("Build the C++ with ASan/UBSan").
// Known-answer vectors: FIPS 180-2 SHA-256 "abc", RFC 6979 A.2.5 (P-256, SHA-256, "sample"),
// SEC 2 generator G; everything else is a round-trip or a cross-check between two code paths.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../csrc/native.h"
#include "../csrc/sha256_common.h"

using namespace upow;

static int failures = 0;
#define CHECK(c)                                                          \
    do {                                                                  \
        if (!(c)) {                                                       \
            std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
            ++failures;                                                   \
        }                                                                 \
    } while (0)

static std::vector<uint8_t> unhex(const char* h) {
    std::vector<uint8_t> out;
    for (size_t i = 0; h[i] && h[i + 1]; i += 2) {
        unsigned v;
        std::sscanf(h + i, "%2x", &v);
        out.push_back(uint8_t(v));
    }
    return out;
}

static std::vector<uint8_t> sha(const uint8_t* p, size_t n) {
    HostSha256 s;
    s.update(p, n);
    std::vector<uint8_t> d(32);
    s.final(d.data());
    return d;
}

static void test_sha256() {
    auto d = sha(reinterpret_cast<const uint8_t*>("abc"), 3);
    CHECK(d == unhex("ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad"));
    // batch (threaded) == scalar for lengths across the 55/56/64-byte padding boundaries
    std::mt19937 rng(7);
    std::vector<uint8_t> data;
    std::vector<int64_t> off{0};
    for (int len = 0; len < 300; ++len) {
        for (int k = 0; k < len; ++k) data.push_back(uint8_t(rng()));
        off.push_back(int64_t(data.size()));
    }
    auto b = sha256_batch_host(data.data(), off.data(), int64_t(off.size() - 1), 4);
    for (size_t i = 0; i + 1 < off.size(); ++i) {
        auto ref = sha(data.data() + off[i], size_t(off[i + 1] - off[i]));
        CHECK(std::memcmp(b.data() + 32 * i, ref.data(), 32) == 0);
    }
    // SHA-NI block function == scalar rounds (multi-block runs from random states)
    if (sha256_ni_enabled()) {
        for (int t = 0; t < 200; ++t) {
            const size_t nb = 1 + rng() % 5;
            std::vector<uint8_t> blk(64 * nb);
            for (auto& x : blk) x = uint8_t(rng());
            uint32_t a[8], c[8];
            for (int i = 0; i < 8; ++i) a[i] = c[i] = uint32_t(rng());
            sha256_ni_blocks(a, blk.data(), nb);
            for (size_t k = 0; k < nb; ++k) host_compress_scalar(c, blk.data() + 64 * k);
            CHECK(std::memcmp(a, c, sizeof(a)) == 0);
        }
    } else {
        std::printf("note: no SHA-NI on this CPU, scalar path only\n");
    }
}

static void test_base58() {
    std::mt19937 rng(11);
    for (int t = 0; t < 200; ++t) {
        std::vector<uint8_t> v(size_t(rng() % 70));
        for (auto& x : v) x = uint8_t(rng());
        for (int z = 0; z < t % 4 && z < int(v.size()); ++z) v[size_t(z)] = 0;  // leading zeros -> '1'
        CHECK(b58decode(b58encode(v.data(), v.size())) == v);
    }
    bool threw = false;
    try {
        b58decode("0OIl");
    } catch (...) {
        threw = true;
    }
    CHECK(threw);
}

static void test_p256() {
    uint8_t d[32] = {0}, pub[64];
    d[31] = 1;
    CHECK(p256_pubkey(d, pub));
    auto gx = unhex("6b17d1f2e12c4247f8bce6e563a440f277037d812deb33a0f4a13945d898c296");
    for (int i = 0; i < 32; ++i) CHECK(pub[i] == gx[31 - i]);  // little-endian x
    // RFC 6979 A.2.5, SHA-256, message "sample"
    auto dk = unhex("c9afa9d845ba75166b5c215767b1d6934e50c3db36e89b127b8a622b120f6721");
    auto e = sha(reinterpret_cast<const uint8_t*>("sample"), 6);
    uint8_t r[32], s[32];
    CHECK(p256_sign(dk.data(), e.data(), r, s));
    auto rr = unhex("efd48b2aacb6a8fd1140dd9cd45e81d69d2c877b56aaf991c34d0ea84eaf3716");
    auto ss = unhex("f7cb1c942d657c41d436c7a1b6e29f65f3e900dbb9aff4064dc4ab2f843acda8");
    for (int i = 0; i < 32; ++i) {
        CHECK(r[i] == rr[31 - i]);
        CHECK(s[i] == ss[31 - i]);
    }
    // batch verify: valid / wrong digest / off-curve key / s = 0, over several thread counts
    std::mt19937 rng(3);
    const int n = 64;
    std::vector<uint8_t> items(160 * n);
    std::vector<uint8_t> want(n);
    for (int k = 0; k < n; ++k) {
        uint8_t key[32], q[64], dig[32];
        for (auto& x : key) x = uint8_t(rng());
        key[0] &= 0x7f;
        for (auto& x : dig) x = uint8_t(rng());
        CHECK(p256_pubkey(key, q));
        CHECK(p256_sign(key, dig, r, s));
        uint8_t* it = items.data() + 160 * k;
        std::memcpy(it, q, 64);
        std::memcpy(it + 64, r, 32);
        std::memcpy(it + 96, s, 32);
        std::memcpy(it + 128, dig, 32);
        want[size_t(k)] = 1;
        if (k % 4 == 1) { it[128] ^= 1; want[size_t(k)] = 0; }
        if (k % 4 == 2) { it[32] ^= 1; want[size_t(k)] = 2; }
        if (k % 4 == 3) { std::memset(it + 96, 0, 32); want[size_t(k)] = 3; }
        if (k == 0) {  // compressed round trip through the decompressor
            uint8_t c[33], out[64], ok = 0;
            c[0] = (q[32] & 1) ? 43 : 42;
            std::memcpy(c + 1, q, 32);
            p256_decompress_host(c, 1, out, &ok);
            CHECK(ok == 1 && std::memcmp(out, q, 64) == 0);
        }
    }
    for (int threads : {1, 3, 8}) CHECK(p256_verify_host(items.data(), n, threads) == want);
}

static void test_pow_host() {
    PowJobHost job;
    job.header.assign(108, 0);
    job.header[0] = 2;
    for (int i = 1; i < 104; ++i) job.header[size_t(i)] = uint8_t(i * 37);
    job.tmask = 0xff000000u;  // 2 nibbles
    job.tword = 0x00000000u;
    PowResult res = pow_search_host(job, 0, 1u << 18, 4);
    CHECK(res.searched == (1u << 18));
    CHECK(!res.words.empty());
    for (uint32_t w : res.words) CHECK(pow_check_word_host(job, w));
}

int main() {
    test_sha256();
    test_base58();
    test_p256();
    test_pow_host();
    if (failures) {
        std::fprintf(stderr, "%d failure(s)\n", failures);
        return 1;
    }
    std::printf("host selftest: all checks passed\n");
    return 0;
}
