// HTTP/1.1 request framing and WebSocket (RFC 6455) frame parsing for the node's server protocol
// (upow_amd/node/http.py).
//
// reference: the node is served by uvicorn on port 3006 (upow/node/run.py) with FastAPI routes and a
// WebSocket endpoint. At four-digit /push_tx rates the pure-Python h11 state machine was ~a third of the
// event loop's CPU per request (profiles/r3/node_soak_loop_cprofile_r3p.txt), and this image has no
// WebSocket library for uvicorn at all. Here a connection's bytes go to one native call that returns
// every COMPLETE request (method, target, version, lower-cased headers, de-chunked body, keep-alive and
// upgrade flags): one Python call per request instead of a parser callback per header. The WebSocket
// parser returns whole frames, unmasked.
#include <pybind11/pybind11.h>

#include "http_wire.h"

#include <sys/socket.h>

#include <cerrno>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <string_view>
#include <vector>

namespace py = pybind11;

namespace upow {
namespace {

// Python faces of the parser cores (csrc/http_wire.h)
class HttpParser {
public:
    HttpParser(int64_t max_header, int64_t max_body) : core_(max_header, max_body) {}

    // every complete request after appending `data`:
    // (method, target, version, [(name, value)], body, keep_alive, upgrade, upgrade_proto)
    py::list feed(py::bytes data) {
        char* p = nullptr;
        Py_ssize_t n = 0;
        PyBytes_AsStringAndSize(data.ptr(), &p, &n);
        core_.append(p, size_t(n));
        py::list out;
        http::HttpRequest r;
        while (core_.next(r)) {
            py::list hs(r.headers.size());
            for (size_t i = 0; i < r.headers.size(); ++i)
                hs[i] = py::make_tuple(py::bytes(r.headers[i].first), py::bytes(r.headers[i].second));
            out.append(py::make_tuple(r.method, py::bytes(r.target), r.version, hs, py::bytes(r.body), r.keep_alive,
                                      r.upgrade, r.upgrade_proto));
        }
        return out;
    }
    bool need_continue() const { return core_.need_continue(); }
    void ack_continue() { core_.ack_continue(); }
    py::bytes rest() { return py::bytes(core_.take_rest()); }

private:
    http::HttpParserCore core_;
};

class WsParser {
public:
    explicit WsParser(int64_t max_payload) : core_(max_payload) {}
    py::list feed(py::bytes data) {
        char* p = nullptr;
        Py_ssize_t n = 0;
        PyBytes_AsStringAndSize(data.ptr(), &p, &n);
        py::list out;
        for (auto& f : core_.feed(p, size_t(n))) out.append(py::make_tuple(f.fin, f.opcode, py::bytes(f.payload)));
        return out;
    }

private:
    http::WsParserCore core_;
};

}  // namespace

void register_http_wire(py::module_& m) {
    using http::BadRequest;
    using http::WsError;
    static py::exception<BadRequest> bad(m, "HttpBadRequest", PyExc_ValueError);
    static py::exception<WsError> wserr(m, "WsProtocolError", PyExc_ValueError);
    py::register_exception_translator([](std::exception_ptr p) {
        try {
            if (p) std::rethrow_exception(p);
        } catch (const WsError& e) {
            // args = (message, close code)
            py::tuple args = py::make_tuple(e.what(), e.code);
            PyErr_SetObject(wserr.ptr(), args.ptr());
        } catch (const BadRequest& e) {
            bad(e.what());
        }
    });
    py::class_<HttpParser>(m, "HttpParser")
        .def(py::init<int64_t, int64_t>(), py::arg("max_header") = 65536, py::arg("max_body") = int64_t(64) << 20)
        .def("feed", &HttpParser::feed,
             "complete requests: (method, target, version, [(name, value)], body, keep_alive, upgrade, upgrade_proto)")
        .def("need_continue", &HttpParser::need_continue)
        .def("ack_continue", &HttpParser::ack_continue)
        .def("rest", &HttpParser::rest);
    // One non-blocking send WITH the GIL held: a response of a few hundred bytes is one syscall of
    // microseconds, while socket.send() releases the GIL around it and the event loop then waits to get it
    // back from whichever thread took it (a wake-up on a loaded host). Returns the bytes sent (0 when the
    // socket buffer is full) or -errno; the caller hands any rest to the transport.
    m.def("send_now", [](int fd, py::buffer data) -> int64_t {
        py::buffer_info bi = data.request();
        const size_t n = size_t(bi.size * bi.itemsize);
        for (;;) {
            const ssize_t w = ::send(fd, bi.ptr, n, MSG_DONTWAIT | MSG_NOSIGNAL);
            if (w >= 0) return int64_t(w);
            if (errno == EINTR) continue;
            if (errno == EAGAIN || errno == EWOULDBLOCK) return 0;
            return -int64_t(errno);
        }
    });
    py::class_<WsParser>(m, "WsParser")
        .def(py::init<int64_t>(), py::arg("max_payload") = int64_t(16) << 20)
        .def("feed", &WsParser::feed, "complete client frames: (fin, opcode, unmasked payload)");
}

}  // namespace upow
