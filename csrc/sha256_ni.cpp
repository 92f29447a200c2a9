// Host SHA-256 compression on the x86 SHA extensions (SHA-NI: sha256rnds2 / sha256msg1 / sha256msg2).
//
// Every host-side hash of the node goes through host_compress (csrc/sha256_common.h): txids and
// signed-message digests of a whole block in the codec, the sequential merkle and UTXO-set tails,
// PoW re-checks of GPU candidates, the CPU miner fallback. The MI355X hosts' CPUs (and this build
// container's) implement SHA-NI, which runs a 64-byte block ~6x faster than the scalar rounds; the
// scalar path stays for CPUs without it (checked once with CPUID leaf 7, EBX bit 29).
#include <cpuid.h>
#include <immintrin.h>

#include <cstddef>
#include <cstdint>

#include "sha256_common.h"

namespace upow {

bool sha256_ni_enabled() {
    static const bool ok = [] {
        unsigned a = 0, b = 0, c = 0, d = 0;
        if (!__get_cpuid_count(7, 0, &a, &b, &c, &d)) return false;
        const bool sha = (b >> 29) & 1u;
        unsigned a1 = 0, b1 = 0, c1 = 0, d1 = 0;
        if (!__get_cpuid(1, &a1, &b1, &c1, &d1)) return false;
        const bool sse41 = (c1 >> 19) & 1u, ssse3 = (c1 >> 9) & 1u;
        return sha && sse41 && ssse3;
    }();
    return ok;
}

// `nblocks` consecutive 64-byte blocks into the state (SHA-256 word order st[0..7] = a..h).
__attribute__((target("sha,sse4.1,ssse3"))) void sha256_ni_blocks(uint32_t st[8], const uint8_t* data,
                                                                  size_t nblocks) {
    const __m128i kShuf = _mm_set_epi64x(0x0c0d0e0f08090a0bULL, 0x0405060700010203ULL);  // BE words
    // a..h -> the ABEF / CDGH register layout sha256rnds2 works on
    __m128i t = _mm_loadu_si128(reinterpret_cast<const __m128i*>(&st[0]));   // a b c d
    __m128i s1 = _mm_loadu_si128(reinterpret_cast<const __m128i*>(&st[4]));  // e f g h
    t = _mm_shuffle_epi32(t, 0xB1);                                           // b a d c
    s1 = _mm_shuffle_epi32(s1, 0x1B);                                         // h g f e
    __m128i s0 = _mm_alignr_epi8(t, s1, 8);                                   // ABEF
    s1 = _mm_blend_epi16(s1, t, 0xF0);                                        // CDGH
    while (nblocks--) {
        const __m128i abef = s0, cdgh = s1;
        __m128i m[4];
#pragma GCC unroll 16
        for (int g = 0; g < 16; ++g) {
            __m128i w;
            if (g < 4) {
                w = _mm_shuffle_epi8(_mm_loadu_si128(reinterpret_cast<const __m128i*>(data + 16 * g)), kShuf);
            } else {
                // W[4g..4g+3] = msg2(msg1(W[4g-16..], W[4g-12..]) + W[4g-7..4g-4], W[4g-4..])
                __m128i x = _mm_sha256msg1_epu32(m[(g - 4) & 3], m[(g - 3) & 3]);
                x = _mm_add_epi32(x, _mm_alignr_epi8(m[(g - 1) & 3], m[(g - 2) & 3], 4));
                w = _mm_sha256msg2_epu32(x, m[(g - 1) & 3]);
            }
            m[g & 3] = w;
            __m128i k = _mm_add_epi32(w, _mm_loadu_si128(reinterpret_cast<const __m128i*>(&kSha256K[4 * g])));
            s1 = _mm_sha256rnds2_epu32(s1, s0, k);
            k = _mm_shuffle_epi32(k, 0x0E);
            s0 = _mm_sha256rnds2_epu32(s0, s1, k);
        }
        s0 = _mm_add_epi32(s0, abef);
        s1 = _mm_add_epi32(s1, cdgh);
        data += 64;
    }
    t = _mm_shuffle_epi32(s0, 0x1B);     // F E B A
    s1 = _mm_shuffle_epi32(s1, 0xB1);    // D C H G
    s0 = _mm_blend_epi16(t, s1, 0xF0);   // D C B A -> a b c d in memory order
    s1 = _mm_alignr_epi8(s1, t, 8);      // H G F E -> e f g h
    _mm_storeu_si128(reinterpret_cast<__m128i*>(&st[0]), s0);
    _mm_storeu_si128(reinterpret_cast<__m128i*>(&st[4]), s1);
}

}  // namespace upow
