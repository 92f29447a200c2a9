// Base58 (Bitcoin alphabet) codec for the 33-byte compressed addresses (reference: the `base58`
// package used by upow/helpers.py:171-188). Host C++; the node converts addresses for every output
// it parses and every input it stores, so this sits on the block-apply path.
#include <algorithm>
#include <array>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "native.h"

namespace upow {

static const char* kB58 = "123456789ABCDEFGHJKLMNPQRSTUVWXYZabcdefghijkmnopqrstuvwxyz";

// Base conversion 2^32 -> 58^5 on 32-bit limbs: each input word is multiplied into the accumulated
// number with one 64-bit carry chain, so a 33-byte address takes ~9 x 9 limb steps instead of the
// ~33 x 45 digit steps of the schoolbook byte loop (the division is by a constant: a multiply-high).
// Allocation-free: the limbs live on the stack and the digits go to the caller's buffer. The block
// decoder calls this for every output address on all host-pool threads, and a heap vector per call
// (freed later by whichever thread reuses the workspace) serialised the pool on malloc arena locks:
// the 8,300-tx decode ran no faster on 8 threads than on 1.
static size_t b58_core(const uint8_t* data, size_t n, uint32_t* limbs, char* out) {
    constexpr uint64_t kBase = 656356768ull;  // 58^5 < 2^32
    size_t zeros = 0;
    while (zeros < n && data[zeros] == 0) ++zeros;
    const size_t m = n - zeros;
    // limbs: ceil(m * 8 / log2(58^5)) words, log2(58^5) ~ 29.29, little-endian, base 58^5
    size_t len = 0;
    const uint8_t* p = data + zeros;
    const size_t head = m % 4 ? m % 4 : 4;  // the first word takes the leading m mod 4 bytes
    for (size_t i = 0; i < m;) {
        const size_t take = i == 0 ? std::min(head, m) : 4;
        uint64_t carry = 0;
        for (size_t k = 0; k < take; ++k) carry = (carry << 8) | p[i + k];
        const unsigned shift = unsigned(8 * take);
        for (size_t j = 0; j < len; ++j) {
            carry += uint64_t(limbs[j]) << shift;
            limbs[j] = uint32_t(carry % kBase);
            carry /= kBase;
        }
        while (carry) {
            limbs[len++] = uint32_t(carry % kBase);
            carry /= kBase;
        }
        i += take;
    }
    size_t o = 0;
    for (; o < zeros; ++o) out[o] = '1';
    char buf[5];
    bool lead = true;
    for (size_t j = len; j-- > 0;) {
        uint32_t v = limbs[j];
        for (int k = 4; k >= 0; --k) {
            buf[k] = kB58[v % 58];
            v /= 58;
        }
        for (int k = 0; k < 5; ++k) {
            if (lead && buf[k] == '1') continue;  // leading zero digits of the top limb
            lead = false;
            out[o++] = buf[k];
        }
    }
    return o;
}

size_t b58encode_to(const uint8_t* data, size_t n, char* out) {
    if (n > kB58MaxInput) throw std::invalid_argument("b58encode_to: input longer than 64 bytes");
    uint32_t limbs[kB58MaxInput * 8 / 29 + 2];
    return b58_core(data, n, limbs, out);
}

std::string b58encode(const uint8_t* data, size_t n) {
    if (n <= kB58MaxInput) {
        char buf[kB58MaxOutput];
        return std::string(buf, b58encode_to(data, n, buf));
    }
    // any length (the Python binding): heap buffers, 138 digits per 100 bytes at most
    std::vector<uint32_t> limbs(n * 8 / 29 + 2);
    std::string out(n * 138 / 100 + 2, '\0');
    out.resize(b58_core(data, n, limbs.data(), &out[0]));
    return out;
}

// The inverse conversion 58^5 -> 2^32: five digits at a time are folded into 32-bit limbs with one
// 64-bit carry chain (58^5 < 2^30, so limb * 58^5 + carry stays below 2^62). The digit table is a
// function-local static, so concurrent first calls from the host pool are race-free.
std::vector<uint8_t> b58decode(const std::string& s) {
    static const std::array<int8_t, 256> map = [] {
        std::array<int8_t, 256> m{};
        m.fill(-1);
        for (int i = 0; i < 58; ++i) m[uint8_t(kB58[i])] = int8_t(i);
        return m;
    }();
    size_t end = s.size();
    while (end > 0 && (s[end - 1] == ' ' || s[end - 1] == '\n' || s[end - 1] == '\t' || s[end - 1] == '\r')) --end;
    size_t zeros = 0;
    while (zeros < end && s[zeros] == '1') ++zeros;
    const size_t m = end - zeros;
    std::vector<uint32_t> limbs(m * 6 / 32 + 2, 0);  // log2(58) < 6 bits per digit; little-endian
    size_t len = 0;
    for (size_t i = zeros; i < end;) {
        const size_t take = i == zeros && m % 5 ? m % 5 : 5;
        uint64_t carry = 0, mul = 1;
        for (size_t k = 0; k < take; ++k) {
            const int v = map[uint8_t(s[i + k])];
            if (v < 0) throw std::invalid_argument(std::string("Invalid character '") + s[i + k] + "'");
            carry = carry * 58 + uint64_t(v);
            mul *= 58;
        }
        for (size_t j = 0; j < len; ++j) {
            carry += uint64_t(limbs[j]) * mul;
            limbs[j] = uint32_t(carry);
            carry >>= 32;
        }
        while (carry) {
            limbs[len++] = uint32_t(carry);
            carry >>= 32;
        }
        i += take;
    }
    std::vector<uint8_t> out(zeros, 0);
    out.reserve(zeros + 4 * len);
    for (size_t j = len; j-- > 0;) {
        for (int k = 3; k >= 0; --k) {
            const uint8_t b = uint8_t(limbs[j] >> (8 * k));
            if (b == 0 && j == len - 1 && out.size() == zeros) continue;  // leading zero bytes of the top limb
            out.push_back(b);
        }
    }
    return out;
}

}  // namespace upow
