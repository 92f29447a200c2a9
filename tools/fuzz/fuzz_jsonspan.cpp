// libFuzzer target: csrc/jsonspan.cpp json_loads_spans, differential against CPython's json.loads.
//
// The span parser is the first native code to read a peer's bytes on the sync path (every /get_blocks page,
// reference /root/reference/upow/node/nodes_manager.py:79-86) and every /push_block body (reference
// upow/node/main.py:521-652). Its contract (utils/hexspans.py): when it returns, the value equals
// json.loads(body) -- with every all-ASCII string array under 'txs' / 'transactions' returned as (start,
// length) spans of the body -- and anything it does not handle raises ValueError so the caller falls back to
// json.loads. So for every input:
//   * the call either returns or raises ValueError (any other exception, or a crash / ASan / UBSan report,
//     is a finding);
//   * when it returns, json.loads(body) must succeed too, and the returned value with its spans expanded to
//     str must equal json.loads' value type-exactly (int vs float vs bool, dict key order, duplicate keys:
//     the last one wins on both sides).
// Built by tools/sanitize_host.sh with -fsanitize=fuzzer,address,undefined and an embedded interpreter
// (pybind11/embed.h, libpython3.10); the parser TU is included directly.
#include <pybind11/embed.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#include "../../csrc/jsonspan.cpp"

namespace py = pybind11;

namespace {

const char* kHelpers = R"PY(
import json, struct

class Spans:
    __slots__ = ('b',)
    def __init__(self, b):
        self.b = b

def expand(body, v):
    if isinstance(v, Spans):
        a = struct.unpack('<%dq' % (len(v.b) // 8), v.b)
        out = []
        for k in range(0, len(a), 2):
            st, ln = a[k], a[k + 1]
            assert 0 <= st and st + ln <= len(body), (st, ln, len(body))
            out.append(body[st:st + ln].decode('ascii'))
        return out
    if isinstance(v, dict):
        return {k: expand(body, x) for k, x in v.items()}
    if isinstance(v, list):
        return [expand(body, x) for x in v]
    return v

def same(a, b):
    if type(a) is not type(b):
        return False
    if isinstance(a, dict):
        return list(a.keys()) == list(b.keys()) and all(same(a[k], b[k]) for k in a)
    if isinstance(a, list):
        return len(a) == len(b) and all(same(x, y) for x, y in zip(a, b))
    if isinstance(a, float) and a != a:
        return b != b
    return a == b

def check(body, got):
    try:
        ref = json.loads(body)
    except Exception as e:
        return 'json.loads rejects what the span parser accepted: %r' % (e,)
    try:
        mine = expand(body, got)
    except Exception as e:
        return 'span expansion failed: %r' % (e,)
    if not same(mine, ref):
        return 'values differ: %r vs %r' % (mine, ref)
    return None
)PY";

py::scoped_interpreter* g_interp = nullptr;
py::object g_keys, g_factory, g_check;
py::object g_value_error;

}  // namespace

extern "C" int LLVMFuzzerInitialize(int*, char***) {
    g_interp = new py::scoped_interpreter();
    py::dict ns;
    py::exec(kHelpers, ns);
    g_factory = ns["Spans"];
    g_check = ns["check"];
    g_keys = py::make_tuple("txs", "transactions");
    g_value_error = py::module_::import("builtins").attr("ValueError");
    return 0;
}

extern "C" int LLVMFuzzerTestOneInput(const uint8_t* data, size_t size) {
    py::bytes body(reinterpret_cast<const char*>(data), size);
    py::object got;
    try {
        got = upow::json_loads_spans(body, g_keys, g_factory);
    } catch (py::value_error&) {
        return 0;  // outside the plain subset: the caller's json.loads decides
    } catch (py::error_already_set& e) {
        if (e.matches(g_value_error)) return 0;  // e.g. an escaped string json.loads itself rejected
        std::fprintf(stderr, "json_loads_spans raised a non-ValueError: %s\n", e.what());
        std::abort();
    }
    py::object msg = g_check(body, got);
    if (!msg.is_none()) {
        std::fprintf(stderr, "differential failure: %s\n", py::str(msg).cast<std::string>().c_str());
        std::abort();
    }
    return 0;
}
