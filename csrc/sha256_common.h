// SHA-256 primitives shared by the host library and the gfx950 kernels.
//
// Host side: scalar SHA-256 (txids, merkle tail, PoW re-check, UTXO-set hash) used when no GPU is
// present and for the inherently sequential Merkle-Damgard tails.
// Device side: the round/schedule macros are written so that hipcc lowers them to the CDNA4 3-input
// integer ops (v_alignbit_b32 rotates, v_xor3_b32, v_add3_u32, v_bfi_b32 for Ch/Maj).
#pragma once
#include <cstddef>
#include <cstdint>
#include <cstring>

namespace upow {

static constexpr uint32_t kSha256K[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};

static constexpr uint32_t kSha256IV[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                                          0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};

inline uint32_t host_rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

inline uint32_t load_be32(const uint8_t* p) {
    return (uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | uint32_t(p[3]);
}
inline void store_be32(uint8_t* p, uint32_t v) {
    p[0] = uint8_t(v >> 24); p[1] = uint8_t(v >> 16); p[2] = uint8_t(v >> 8); p[3] = uint8_t(v);
}

// One compression of a 64-byte block given as 16 big-endian words.
inline void host_compress_words(uint32_t st[8], const uint32_t w_in[16]) {
    uint32_t w[64];
    for (int i = 0; i < 16; ++i) w[i] = w_in[i];
    for (int i = 16; i < 64; ++i) {
        uint32_t s0 = host_rotr(w[i - 15], 7) ^ host_rotr(w[i - 15], 18) ^ (w[i - 15] >> 3);
        uint32_t s1 = host_rotr(w[i - 2], 17) ^ host_rotr(w[i - 2], 19) ^ (w[i - 2] >> 10);
        w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
    for (int i = 0; i < 64; ++i) {
        uint32_t S1 = host_rotr(e, 6) ^ host_rotr(e, 11) ^ host_rotr(e, 25);
        uint32_t ch = (e & f) ^ (~e & g);
        uint32_t t1 = h + S1 + ch + kSha256K[i] + w[i];
        uint32_t S0 = host_rotr(a, 2) ^ host_rotr(a, 13) ^ host_rotr(a, 22);
        uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
        uint32_t t2 = S0 + mj;
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

// x86 SHA extensions (csrc/sha256_ni.cpp): used for every host block when the CPU has them
bool sha256_ni_enabled();
void sha256_ni_blocks(uint32_t st[8], const uint8_t* data, size_t nblocks);

inline void host_compress_scalar(uint32_t st[8], const uint8_t blk[64]) {
    uint32_t w[16];
    for (int i = 0; i < 16; ++i) w[i] = load_be32(blk + 4 * i);
    host_compress_words(st, w);
}

inline void host_compress_blocks(uint32_t st[8], const uint8_t* p, size_t nblocks) {
    static const bool ni = sha256_ni_enabled();
    if (ni) {
        sha256_ni_blocks(st, p, nblocks);
        return;
    }
    for (size_t b = 0; b < nblocks; ++b) host_compress_scalar(st, p + 64 * b);
}

inline void host_compress(uint32_t st[8], const uint8_t blk[64]) { host_compress_blocks(st, blk, 1); }

// Partial compression: run rounds [0, nrounds) of block `w` from state `st` (state NOT fed forward).
// Used to precompute the nonce-independent rounds of the PoW tail block on the host.
inline void host_rounds(uint32_t st[8], const uint32_t w[16], int nrounds) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
    for (int i = 0; i < nrounds; ++i) {
        uint32_t S1 = host_rotr(e, 6) ^ host_rotr(e, 11) ^ host_rotr(e, 25);
        uint32_t ch = (e & f) ^ (~e & g);
        uint32_t t1 = h + S1 + ch + kSha256K[i] + w[i];
        uint32_t S0 = host_rotr(a, 2) ^ host_rotr(a, 13) ^ host_rotr(a, 22);
        uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + S0 + mj;
    }
    st[0] = a; st[1] = b; st[2] = c; st[3] = d; st[4] = e; st[5] = f; st[6] = g; st[7] = h;
}

struct HostSha256 {
    uint32_t st[8];
    uint8_t buf[64];
    size_t buflen = 0;
    uint64_t total = 0;
    HostSha256() { std::memcpy(st, kSha256IV, sizeof(st)); }
    void update(const uint8_t* p, size_t n) {
        total += n;
        if (buflen) {
            size_t take = 64 - buflen < n ? 64 - buflen : n;
            std::memcpy(buf + buflen, p, take);
            buflen += take; p += take; n -= take;
            if (buflen == 64) { host_compress(st, buf); buflen = 0; }
        }
        if (n >= 64) {
            host_compress_blocks(st, p, n / 64);
            p += n & ~size_t(63);
            n &= 63;
        }
        if (n) { std::memcpy(buf, p, n); buflen = n; }
    }
    void final(uint8_t out[32]) {
        const uint64_t bits = total * 8;
        uint8_t tail[128] = {0};  // one or two padding blocks
        std::memcpy(tail, buf, buflen);
        tail[buflen] = 0x80;
        const size_t nb = buflen < 56 ? 1 : 2;
        for (int i = 0; i < 8; ++i) tail[64 * nb - 1 - i] = uint8_t(bits >> (8 * i));
        host_compress_blocks(st, tail, nb);
        buflen = 0;
        for (int i = 0; i < 8; ++i) store_be32(out + 4 * i, st[i]);
    }
};

inline void host_sha256(const uint8_t* p, size_t n, uint8_t out[32]) {
    HostSha256 h;
    h.update(p, n);
    h.final(out);
}

}  // namespace upow
