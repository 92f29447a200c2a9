// Base58 (Bitcoin alphabet) codec for the 33-byte compressed addresses (reference: the `base58`
// package used by upow/helpers.py:171-188). Host C++; the node converts addresses for every output
// it parses and every input it stores, so this sits on the block-apply path.
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

namespace upow {

static const char* kB58 = "123456789ABCDEFGHJKLMNPQRSTUVWXYZabcdefghijkmnopqrstuvwxyz";

std::string b58encode(const uint8_t* data, size_t n) {
    size_t zeros = 0;
    while (zeros < n && data[zeros] == 0) ++zeros;
    // big-number base conversion 256 -> 58 (log(256)/log(58) ~ 1.366)
    std::vector<uint8_t> digits((n - zeros) * 138 / 100 + 1, 0);
    size_t len = 0;
    for (size_t i = zeros; i < n; ++i) {
        uint32_t carry = data[i];
        size_t j = 0;
        for (auto it = digits.rbegin(); (carry != 0 || j < len) && it != digits.rend(); ++it, ++j) {
            carry += 256u * (*it);
            *it = uint8_t(carry % 58);
            carry /= 58;
        }
        len = j;
    }
    auto it = digits.begin() + (digits.size() - len);
    while (it != digits.end() && *it == 0) ++it;
    std::string out(zeros, '1');
    for (; it != digits.end(); ++it) out.push_back(kB58[*it]);
    return out;
}

std::vector<uint8_t> b58decode(const std::string& s_in) {
    static int8_t map[256];
    static bool init = false;
    if (!init) {
        for (int i = 0; i < 256; ++i) map[i] = -1;
        for (int i = 0; i < 58; ++i) map[uint8_t(kB58[i])] = int8_t(i);
        init = true;
    }
    std::string s = s_in;
    while (!s.empty() && (s.back() == ' ' || s.back() == '\n' || s.back() == '\t' || s.back() == '\r')) s.pop_back();
    size_t zeros = 0;
    while (zeros < s.size() && s[zeros] == '1') ++zeros;
    std::vector<uint8_t> b256((s.size() - zeros) * 733 / 1000 + 1, 0);
    size_t len = 0;
    for (size_t i = zeros; i < s.size(); ++i) {
        int v = map[uint8_t(s[i])];
        if (v < 0) throw std::invalid_argument(std::string("Invalid character '") + s[i] + "'");
        uint32_t carry = uint32_t(v);
        size_t j = 0;
        for (auto it = b256.rbegin(); (carry != 0 || j < len) && it != b256.rend(); ++it, ++j) {
            carry += 58u * (*it);
            *it = uint8_t(carry & 0xff);
            carry >>= 8;
        }
        len = j;
    }
    auto it = b256.begin() + (b256.size() - len);
    while (it != b256.end() && *it == 0) ++it;
    std::vector<uint8_t> out(zeros, 0);
    out.insert(out.end(), it, b256.end());
    return out;
}

}  // namespace upow
