// libFuzzer target (ASan + UBSan, tools/sanitize_host.sh): the node's HTTP/1.1 request framing and RFC 6455
// frame parser (csrc/http_wire.h) over arbitrary bytes cut at arbitrary points.
//
// Input: byte 0 selects the parser (bit 0: WebSocket) and byte 1 seeds the split points; the rest is the
// stream. Properties, besides "no memory error, no UB, no uncaught exception":
//  * the parse of the stream fed in pieces equals the parse of the stream fed at once: the same requests
//    (or frames) in the same order, and a protocol error in one iff in the other;
//  * every request body and frame payload respects the configured limits.
#include <cstdint>
#include <cstdlib>
#include <string>
#include <vector>

#include "../../csrc/http_wire.h"

using namespace upow::http;

namespace {

constexpr int64_t kMaxHeader = 2048, kMaxBody = 1 << 14, kMaxPayload = 1 << 12;

std::vector<size_t> pieces(size_t n, uint8_t seed) {
    std::vector<size_t> cut;
    uint32_t x = seed * 2654435761u + 1;
    for (size_t at = 0; at < n;) {
        x = x * 1664525u + 1013904223u;
        const size_t k = 1 + (x >> 16) % 97;
        cut.push_back(std::min(k, n - at));
        at += cut.back();
    }
    return cut;
}

std::string http_run(const uint8_t* p, size_t n, const std::vector<size_t>* cut, bool& failed) {
    HttpParserCore parser(kMaxHeader, kMaxBody);
    std::string log;
    failed = false;
    HttpRequest r;
    auto drain = [&] {
        while (parser.next(r)) {
            if (int64_t(r.body.size()) > kMaxBody || r.method.empty() || r.target.empty()) std::abort();
            log += r.method + ' ' + r.target + ' ' + r.version + '|' + std::to_string(r.headers.size()) + '|' +
                   std::to_string(r.body.size()) + ':' + r.body + (r.keep_alive ? "K" : "k") + (r.upgrade ? "U" : "u") +
                   '\n';
            if (r.upgrade) return false;
        }
        return true;
    };
    try {
        if (!cut) {
            parser.append(reinterpret_cast<const char*>(p), n);
            drain();
        } else {
            size_t at = 0;
            for (size_t k : *cut) {
                parser.append(reinterpret_cast<const char*>(p + at), k);
                at += k;
                if (!drain()) break;
            }
        }
    } catch (const BadRequest&) {
        failed = true;
    }
    return log;
}

std::string ws_run(const uint8_t* p, size_t n, const std::vector<size_t>* cut, bool& failed) {
    WsParserCore parser(kMaxPayload);
    std::string log;
    failed = false;
    try {
        const std::vector<size_t> one{n};
        size_t at = 0;
        for (size_t k : cut ? *cut : one) {
            for (auto& f : parser.feed(reinterpret_cast<const char*>(p + at), k)) {
                if (int64_t(f.payload.size()) > kMaxPayload || f.opcode > 10) std::abort();
                log += std::to_string(f.fin) + ',' + std::to_string(f.opcode) + ',' + f.payload + '\n';
            }
            at += k;
        }
    } catch (const WsError& e) {
        if (e.code != 1002 && e.code != 1009) std::abort();
        failed = true;
    }
    return log;
}

}  // namespace

// Built-in ASan defaults: the fuzzer runtime and the target register some header-defined globals twice
// (a spurious ODR report), and leak checking is not what these targets test.
extern "C" const char* __asan_default_options() { return "detect_odr_violation=0:detect_leaks=0"; }

extern "C" int LLVMFuzzerTestOneInput(const uint8_t* data, size_t size) {
    if (size < 2) return 0;
    const bool ws = data[0] & 1;
    const uint8_t* p = data + 2;
    const size_t n = size - 2;
    const auto cut = pieces(n, data[1]);
    bool f1 = false, f2 = false;
    const std::string a = ws ? ws_run(p, n, nullptr, f1) : http_run(p, n, nullptr, f1);
    const std::string b = ws ? ws_run(p, n, &cut, f2) : http_run(p, n, &cut, f2);
    if (f1 != f2) std::abort();
    if (f1 ? (a.compare(0, b.size(), b) != 0 && b.compare(0, a.size(), a) != 0) : a != b) std::abort();
    return 0;
}
