// HTTP/1.1 request framing and WebSocket (RFC 6455) frame parsing, pure C++ (no Python): the cores of the
// node's server protocol (csrc/http_wire.cpp binds them; upow_amd/node/http.py drives them) and of the
// libFuzzer targets (tools/fuzz_http.cpp). Everything here parses bytes from the network: every length is
// checked before it is used, and a violation throws BadRequest / WsError.
#pragma once

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <string_view>
#include <utility>
#include <vector>

namespace upow {
namespace http {

inline bool tchar(unsigned char c) {  // RFC 9110 token characters
    if (c >= '0' && c <= '9') return true;
    if ((c | 0x20) >= 'a' && (c | 0x20) <= 'z') return true;
    return std::strchr("!#$%&'*+-.^_`|~", c) != nullptr && c != 0;
}

inline std::string lower(std::string_view s) {
    std::string o(s);
    for (char& c : o)
        if (c >= 'A' && c <= 'Z') c = char(c + 32);
    return o;
}

inline std::string_view trim(std::string_view s) {
    while (!s.empty() && (s.front() == ' ' || s.front() == '\t')) s.remove_prefix(1);
    while (!s.empty() && (s.back() == ' ' || s.back() == '\t')) s.remove_suffix(1);
    return s;
}

// does a comma-separated header value list hold `token` (case-insensitive)?
inline bool has_token(std::string_view v, std::string_view token) {
    size_t at = 0;
    while (at <= v.size()) {
        size_t comma = v.find(',', at);
        if (comma == std::string_view::npos) comma = v.size();
        if (lower(trim(v.substr(at, comma - at))) == token) return true;
        at = comma + 1;
    }
    return false;
}

struct BadRequest : std::runtime_error {
    using std::runtime_error::runtime_error;
};

struct HttpRequest {
    std::string method, target, version, body, upgrade_proto;
    std::vector<std::pair<std::string, std::string>> headers;  // lower-cased names
    bool keep_alive = true, upgrade = false;
};

class HttpParserCore {
public:
    HttpParserCore(int64_t max_header, int64_t max_body) : max_header_(max_header), max_body_(max_body) {}

    // append a connection's bytes; then next() yields every complete request. An upgrade request ends
    // parsing (the bytes after it belong to the new protocol: take_rest())
    void append(const char* p, size_t n) {
        if (stopped_) throw BadRequest("parser stopped after an upgrade request");
        buf_.append(p, n);
    }
    bool next(HttpRequest& out) {
        if (stopped_) return false;
        if (!have_head_ && !parse_head()) return false;
        if (!take_body()) return false;
        emit(out);
        return true;
    }

    // the request whose headers are in but whose body is not asked for "Expect: 100-continue"
    bool need_continue() const { return have_head_ && expect_continue_ && !continued_; }
    void ack_continue() { continued_ = true; }
    std::string take_rest() {
        std::string r;
        r.swap(buf_);
        return r;
    }
    size_t buffered() const { return buf_.size(); }

private:
    bool parse_head() {
        // skip empty lines before a request line (RFC 9112 2.2)
        while (buf_.size() >= 2 && buf_[0] == '\r' && buf_[1] == '\n') buf_.erase(0, 2);
        const size_t end = buf_.find("\r\n\r\n");
        if (end == std::string::npos) {
            // no terminator yet: the head is at least size - 3 bytes long. The same verdict whatever the
            // segmentation of the stream (tools/fuzz_http.cpp checks chunked == one-shot parsing)
            if (int64_t(buf_.size()) > max_header_ + 3) throw BadRequest("request header too large");
            return false;
        }
        if (int64_t(end) > max_header_) throw BadRequest("request header too large");
        std::string_view head(buf_.data(), end);
        size_t eol = head.find("\r\n");
        std::string_view line = head.substr(0, eol);
        const size_t sp1 = line.find(' ');
        const size_t sp2 = sp1 == std::string_view::npos ? sp1 : line.find(' ', sp1 + 1);
        if (sp1 == std::string_view::npos || sp2 == std::string_view::npos || sp1 == 0)
            throw BadRequest("malformed request line");
        method_ = std::string(line.substr(0, sp1));
        for (unsigned char c : method_)
            if (!tchar(c)) throw BadRequest("invalid method");
        target_ = std::string(line.substr(sp1 + 1, sp2 - sp1 - 1));
        if (target_.empty()) throw BadRequest("empty request target");
        for (unsigned char c : target_)
            if (c <= 0x20 || c == 0x7f) throw BadRequest("invalid request target");
        const std::string_view ver = line.substr(sp2 + 1);
        if (ver == "HTTP/1.1")
            version_ = "1.1";
        else if (ver == "HTTP/1.0")
            version_ = "1.0";
        else
            throw BadRequest("unsupported HTTP version");
        headers_.clear();
        std::string_view cl, te, conn, upgrade;
        int n_cl = 0;
        expect_continue_ = false;
        size_t at = eol == std::string_view::npos ? head.size() : eol + 2;
        while (at < head.size()) {
            size_t e = head.find("\r\n", at);
            if (e == std::string_view::npos) e = head.size();
            std::string_view h = head.substr(at, e - at);
            at = e + 2;
            if (!h.empty() && (h[0] == ' ' || h[0] == '\t')) throw BadRequest("obsolete header folding");
            const size_t colon = h.find(':');
            if (colon == std::string_view::npos || colon == 0) throw BadRequest("malformed header line");
            const std::string_view name = h.substr(0, colon);
            for (unsigned char c : name)
                if (!tchar(c)) throw BadRequest("invalid header name");
            const std::string_view value = trim(h.substr(colon + 1));
            for (unsigned char c : value)
                if ((c < 0x20 && c != '\t') || c == 0x7f) throw BadRequest("invalid header value");
            std::string lname = lower(name);
            if (lname == "content-length") {
                if (n_cl++ && value != cl) throw BadRequest("conflicting content-length");
                cl = value;
            } else if (lname == "transfer-encoding") {
                te = value;
            } else if (lname == "connection") {
                conn = value;
            } else if (lname == "upgrade") {
                upgrade = value;
            } else if (lname == "expect" && lower(value) == "100-continue") {
                expect_continue_ = true;
            }
            headers_.emplace_back(std::move(lname), std::string(value));
        }
        chunked_ = false;
        body_len_ = 0;
        if (!te.empty()) {
            if (!cl.empty()) throw BadRequest("content-length with transfer-encoding");
            // the final coding must be chunked (RFC 9112 6.3)
            std::string l = lower(te);
            const size_t c = l.rfind(',');
            if (std::string(trim(std::string_view(l).substr(c == std::string::npos ? 0 : c + 1))) != "chunked")
                throw BadRequest("unsupported transfer-encoding");
            chunked_ = true;
        } else if (!cl.empty()) {
            if (cl.size() > 18) throw BadRequest("content-length too large");
            int64_t v = 0;
            for (char c : cl) {
                if (c < '0' || c > '9') throw BadRequest("invalid content-length");
                v = v * 10 + (c - '0');
            }
            if (v > max_body_) throw BadRequest("request body too large");
            body_len_ = v;
        }
        keep_alive_ = version_ == "1.1" ? !has_token(conn, "close") : has_token(conn, "keep-alive");
        upgrade_ = !upgrade.empty() && has_token(conn, "upgrade");
        upgrade_proto_ = lower(upgrade);
        buf_.erase(0, end + 4);
        have_head_ = true;
        continued_ = false;
        body_.clear();
        chunk_state_ = 0;
        return true;
    }

    // the body of the current request: true when complete (consumed from buf_)
    bool take_body() {
        if (!chunked_) {
            if (int64_t(buf_.size()) < body_len_) return false;
            body_.assign(buf_.data(), size_t(body_len_));
            buf_.erase(0, size_t(body_len_));
            return true;
        }
        for (;;) {
            if (chunk_state_ == 0) {  // chunk size line
                const size_t e = buf_.find("\r\n");
                if (e == std::string::npos) {
                    if (buf_.size() > kMaxLine + 1) throw BadRequest("chunk size line too long");
                    return false;
                }
                if (e > kMaxLine) throw BadRequest("chunk size line too long");
                std::string_view line(buf_.data(), e);
                const size_t semi = line.find(';');
                std::string_view hex = trim(line.substr(0, semi));
                if (hex.empty() || hex.size() > 15) throw BadRequest("invalid chunk size");
                int64_t v = 0;
                for (char c : hex) {
                    int d = c >= '0' && c <= '9' ? c - '0' : (c | 0x20) >= 'a' && (c | 0x20) <= 'f' ? (c | 0x20) - 'a' + 10 : -1;
                    if (d < 0) throw BadRequest("invalid chunk size");
                    v = v * 16 + d;
                }
                if (int64_t(body_.size()) + v > max_body_) throw BadRequest("request body too large");
                buf_.erase(0, e + 2);
                chunk_left_ = v;
                chunk_state_ = v == 0 ? 2 : 1;
            } else if (chunk_state_ == 1) {  // chunk data + CRLF
                if (int64_t(buf_.size()) < chunk_left_ + 2) return false;
                if (buf_[size_t(chunk_left_)] != '\r' || buf_[size_t(chunk_left_) + 1] != '\n')
                    throw BadRequest("chunk not followed by CRLF");
                body_.append(buf_.data(), size_t(chunk_left_));
                buf_.erase(0, size_t(chunk_left_) + 2);
                chunk_state_ = 0;
            } else {  // trailer section up to the empty line
                const size_t e = buf_.find("\r\n");
                if (e == std::string::npos) {
                    if (int64_t(buf_.size()) > max_header_ + 1) throw BadRequest("trailer too large");
                    return false;
                }
                if (int64_t(e) > max_header_) throw BadRequest("trailer too large");
                buf_.erase(0, e + 2);
                if (e == 0) return true;
            }
        }
    }

    void emit(HttpRequest& r) {
        r.method = method_;
        r.target = target_;
        r.version = version_;
        r.headers.swap(headers_);
        headers_.clear();
        r.body.swap(body_);
        body_.clear();
        r.keep_alive = keep_alive_;
        r.upgrade = upgrade_;
        r.upgrade_proto = upgrade_proto_;
        have_head_ = false;
        if (upgrade_) stopped_ = true;
    }

    static constexpr size_t kMaxLine = 4096;  // chunk-size line
    int64_t max_header_, max_body_;
    std::string buf_;
    bool have_head_ = false, stopped_ = false;
    std::string method_, target_, version_, body_, upgrade_proto_;
    std::vector<std::pair<std::string, std::string>> headers_;
    bool chunked_ = false, keep_alive_ = true, upgrade_ = false, expect_continue_ = false, continued_ = false;
    int64_t body_len_ = 0, chunk_left_ = 0;
    int chunk_state_ = 0;
};

// RFC 6455 frames from a client: every complete frame as (fin, opcode, payload) with the mask removed.
// Protocol errors raise with the close code to send (1002 protocol error, 1009 too big).
struct WsError : std::runtime_error {
    int code;
    WsError(const std::string& m, int c) : std::runtime_error(m), code(c) {}
};

struct WsFrame {
    bool fin = false;
    int opcode = 0;
    std::string payload;  // unmasked
};

class WsParserCore {
public:
    explicit WsParserCore(int64_t max_payload) : max_payload_(max_payload) {}

    // append a connection's bytes and return every complete frame
    std::vector<WsFrame> feed(const char* p, size_t n) {
        buf_.append(p, n);
        std::vector<WsFrame> out;
        size_t at = 0;
        for (;;) {
            const size_t avail = buf_.size() - at;
            if (avail < 2) break;
            const uint8_t b0 = uint8_t(buf_[at]), b1 = uint8_t(buf_[at + 1]);
            const bool fin = b0 & 0x80;
            const int opcode = b0 & 0x0f;
            if (b0 & 0x70) throw WsError("reserved bits set", 1002);
            if (!(b1 & 0x80)) throw WsError("client frame not masked", 1002);
            const bool control = opcode >= 8;
            if (!(opcode <= 2 || (opcode >= 8 && opcode <= 10))) throw WsError("unknown opcode", 1002);
            uint64_t len = b1 & 0x7f;
            size_t hdr = 2;
            if (len == 126) {
                if (avail < 4) break;
                len = (uint64_t(uint8_t(buf_[at + 2])) << 8) | uint8_t(buf_[at + 3]);
                hdr = 4;
            } else if (len == 127) {
                if (avail < 10) break;
                len = 0;
                for (int k = 0; k < 8; ++k) len = (len << 8) | uint8_t(buf_[at + 2 + size_t(k)]);
                hdr = 10;
                if (len >> 63) throw WsError("64-bit length with the most significant bit set", 1002);  // RFC 6455 5.2
            }
            if (control && (len > 125 || !fin)) throw WsError("invalid control frame", 1002);
            if (len > uint64_t(max_payload_)) throw WsError("frame too large", 1009);
            if (avail < hdr + 4 || avail - hdr - 4 < len) break;  // no wrap-around: len <= max_payload here
            uint8_t mask[4];
            std::memcpy(mask, buf_.data() + at + hdr, 4);
            WsFrame f;
            f.fin = fin;
            f.opcode = opcode;
            f.payload.assign(buf_.data() + at + hdr + 4, size_t(len));
            for (size_t i = 0; i < f.payload.size(); ++i) f.payload[i] = char(uint8_t(f.payload[i]) ^ mask[i & 3]);
            out.push_back(std::move(f));
            at += hdr + 4 + size_t(len);
        }
        buf_.erase(0, at);
        return out;
    }

private:
    int64_t max_payload_;
    std::string buf_;
};

}  // namespace http
}  // namespace upow
