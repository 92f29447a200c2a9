// JSON request/response bodies with their transaction arrays left in place.
//
// A /push_block body is ~4.4 MB of JSON for a full block, almost all of it one array of tx hex strings;
// a /get_blocks page is up to 1,000 block rows, each with such an array. json.loads turns every tx into a
// Python str (5.6-8.9 ms for one full block on this image) that the native decoder then only reads.
// json_loads_spans parses the same grammar, but an array of plain ASCII strings under one of the given keys
// becomes factory(spans): spans = little-endian int64 (start, length) pairs into the body, and the decoder
// (txcodec.cpp decode_block_spans) reads the txs straight out of the body bytes.
//
// Anything outside the plain subset -- escapes are handled exactly by delegating the one string to
// json.loads, but a BOM, control characters, NaN / Infinity, invalid UTF-8, nesting past 200 levels, or
// trailing data -- raises ValueError, and the caller (upow_amd/utils/hexspans.py loads) runs json.loads on
// the whole body, which then gives the reference's exact answer or error. So this parser only has to be
// right when it succeeds. Reference behaviour: the bodies FastAPI and httpx parse for
// /root/reference/upow/node/main.py:521-652 (push_block) and main.py:97-150 (get_blocks pages).
#include <pybind11/pybind11.h>

#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

namespace py = pybind11;

namespace upow {
namespace {

// No byte < 0x20, >= 0x80 or '\\' in [p, p + len): eight bytes per step.
inline bool plain_ascii(const char* p, size_t len) {
    constexpr uint64_t ones = 0x0101010101010101ull, highs = 0x8080808080808080ull;
    size_t k = 0;
    for (; k + 8 <= len; k += 8) {
        uint64_t x;
        std::memcpy(&x, p + k, 8);
        const uint64_t bs = x ^ (ones * 0x5c);
        // high bit set, below 0x20 (x - 0x20 borrows into the high bit with x's high bit clear), or a zero byte
        // of x ^ '\\' (the same test on bs against 1)
        if ((x | ((x - ones * 0x20) & ~x) | ((bs - ones) & ~bs)) & highs) return false;
    }
    for (; k < len; ++k) {
        const unsigned char c = static_cast<unsigned char>(p[k]);
        if (c < 0x20 || c >= 0x80 || c == '\\') return false;
    }
    return true;
}

struct Parser {
    const char* s;
    size_t n;
    size_t i = 0;
    int depth = 0;
    py::object span_keys;  // a frozenset of str
    py::object factory;    // factory(spans: bytes) -> sequence
    py::object json_loads;

    [[noreturn]] void fail(const char* what) const {
        throw py::value_error(std::string("json_loads_spans: ") + what + " at byte " + std::to_string(i));
    }
    void ws() {
        while (i < n && (s[i] == ' ' || s[i] == '\t' || s[i] == '\n' || s[i] == '\r')) ++i;
    }
    bool lit(const char* w) {
        const size_t L = std::strlen(w);
        if (n - i < L || std::memcmp(s + i, w, L) != 0) return false;
        i += L;
        return true;
    }

    // A string starting at s[i] == '"'. Plain ASCII without escapes is the fast case.
    py::object string() {
        const size_t b = ++i;
        bool ascii = true, esc = false;
        while (i < n) {
            const unsigned char c = static_cast<unsigned char>(s[i]);
            if (c == '"') break;
            if (c < 0x20) fail("control character in string");
            if (c == '\\') {
                esc = true;
                i += 2;
                continue;
            }
            if (c >= 0x80) ascii = false;
            ++i;
        }
        if (i >= n) fail("unterminated string");
        const size_t e = i++;  // s[e] == '"'
        if (esc) {  // exact escape semantics: the one string through json.loads
            py::object r = json_loads(py::bytes(s + b - 1, e - b + 2));
            if (!PyUnicode_Check(r.ptr())) fail("escaped string");
            return r;
        }
        PyObject* o = ascii ? PyUnicode_DecodeASCII(s + b, Py_ssize_t(e - b), "strict")
                            : PyUnicode_DecodeUTF8(s + b, Py_ssize_t(e - b), "strict");
        if (!o) {
            PyErr_Clear();
            fail("string encoding");
        }
        return py::reinterpret_steal<py::object>(o);
    }

    py::object number() {
        const size_t b = i;
        bool is_float = false;
        if (i < n && s[i] == '-') ++i;
        if (i >= n) fail("number");
        if (s[i] == '0') {
            ++i;
        } else if (s[i] >= '1' && s[i] <= '9') {
            while (i < n && s[i] >= '0' && s[i] <= '9') ++i;
        } else {
            fail("number");  // includes -Infinity: the fallback decides
        }
        if (i < n && s[i] == '.') {
            is_float = true;
            ++i;
            const size_t d = i;
            while (i < n && s[i] >= '0' && s[i] <= '9') ++i;
            if (i == d) fail("fraction");
        }
        if (i < n && (s[i] == 'e' || s[i] == 'E')) {
            is_float = true;
            ++i;
            if (i < n && (s[i] == '+' || s[i] == '-')) ++i;
            const size_t d = i;
            while (i < n && s[i] >= '0' && s[i] <= '9') ++i;
            if (i == d) fail("exponent");
        }
        const std::string txt(s + b, i - b);
        PyObject* o;
        if (is_float) {  // float(numstr), as json.loads does
            const double v = PyOS_string_to_double(txt.c_str(), nullptr, nullptr);
            if (v == -1.0 && PyErr_Occurred()) {
                PyErr_Clear();
                fail("float");
            }
            o = PyFloat_FromDouble(v);
        } else {
            o = PyLong_FromString(txt.c_str(), nullptr, 10);  // int(numstr), incl. the digit limit
        }
        if (!o) {
            PyErr_Clear();
            fail("number value");
        }
        return py::reinterpret_steal<py::object>(o);
    }

    // An array of plain ASCII strings as (start, length) spans; false (position restored) otherwise.
    bool span_array(py::object& out) {
        const size_t b = i;  // s[i] == '['
        std::vector<int64_t> sp;
        ++i;
        ws();
        if (i < n && s[i] == ']') {
            ++i;
        } else {
            for (;;) {
                if (i >= n || s[i] != '"') {
                    i = b;
                    return false;
                }
                const size_t st = ++i;
                const char* q = static_cast<const char*>(std::memchr(s + st, '"', n - st));
                if (!q || !plain_ascii(s + st, size_t(q - s) - st)) {
                    i = b;
                    return false;
                }
                i = size_t(q - s);
                sp.push_back(int64_t(st));
                sp.push_back(int64_t(i - st));
                ++i;
                ws();
                if (i < n && s[i] == ',') {
                    ++i;
                    ws();
                    continue;
                }
                if (i < n && s[i] == ']') {
                    ++i;
                    break;
                }
                i = b;
                return false;
            }
        }
        out = factory(py::bytes(reinterpret_cast<const char*>(sp.data()), sp.size() * sizeof(int64_t)));
        return true;
    }

    py::object value(bool spannable) {
        ws();
        if (i >= n) fail("unexpected end");
        const char c = s[i];
        if (c == '"') return string();
        if (c == '{') return object();
        if (c == '[') {
            py::object r;
            if (spannable && span_array(r)) return r;
            return array();
        }
        if (c == 't' && lit("true")) return py::bool_(true);
        if (c == 'f' && lit("false")) return py::bool_(false);
        if (c == 'n' && lit("null")) return py::none();
        return number();
    }

    py::object array() {
        if (++depth > 200) fail("nesting");
        ++i;  // '['
        py::list l;
        ws();
        if (i < n && s[i] == ']') {
            ++i;
        } else {
            for (;;) {
                l.append(value(false));
                ws();
                if (i < n && s[i] == ',') {
                    ++i;
                    continue;
                }
                if (i < n && s[i] == ']') {
                    ++i;
                    break;
                }
                fail("array");
            }
        }
        --depth;
        return std::move(l);
    }

    py::object object() {
        if (++depth > 200) fail("nesting");
        ++i;  // '{'
        py::dict d;
        ws();
        if (i < n && s[i] == '}') {
            ++i;
        } else {
            for (;;) {
                ws();
                if (i >= n || s[i] != '"') fail("object key");
                py::object k = string();
                ws();
                if (i >= n || s[i] != ':') fail("colon");
                ++i;
                const int in = PySequence_Contains(span_keys.ptr(), k.ptr());
                if (in < 0) throw py::error_already_set();
                py::object v = value(in == 1);
                if (PyDict_SetItem(d.ptr(), k.ptr(), v.ptr()) != 0) throw py::error_already_set();  // last key wins
                ws();
                if (i < n && s[i] == ',') {
                    ++i;
                    continue;
                }
                if (i < n && s[i] == '}') {
                    ++i;
                    break;
                }
                fail("object");
            }
        }
        --depth;
        return std::move(d);
    }
};

py::object json_loads_spans(py::bytes body, py::object span_keys, py::object factory) {
    char* p = nullptr;
    Py_ssize_t len = 0;
    if (PyBytes_AsStringAndSize(body.ptr(), &p, &len) != 0) throw py::error_already_set();
    Parser ps{p, size_t(len)};
    // json.loads(bytes) also reads UTF-16/32 and a UTF-8 BOM: those bodies are left to it
    if (len >= 2 && (p[0] == 0 || p[1] == 0)) ps.fail("not UTF-8");
    if (len >= 3 && static_cast<unsigned char>(p[0]) == 0xef) ps.fail("BOM");
    ps.span_keys = py::reinterpret_steal<py::object>(PyFrozenSet_New(span_keys.ptr()));
    if (!ps.span_keys) throw py::error_already_set();
    ps.factory = std::move(factory);
    ps.json_loads = py::module_::import("json").attr("loads");
    py::object v = ps.value(false);
    ps.ws();
    if (ps.i != ps.n) ps.fail("trailing data");
    return v;
}

}  // namespace

void register_jsonspan(py::module_& m) {
    m.def("json_loads_spans", &json_loads_spans, py::arg("body"), py::arg("span_keys"), py::arg("factory"),
          "json.loads(body) for the plain-JSON subset, with every all-ASCII-string array under one of "
          "span_keys returned as factory(spans) (int64 (start, length) pairs into body). ValueError for "
          "anything else: the caller then runs json.loads.");
}

}  // namespace upow
