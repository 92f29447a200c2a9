// Ledger journal + background SQL materialisers, on SQLite connections this layer opens and owns.
//
// reference: the block-apply writes of upow/manager.py:706-730 → upow/database.py add_block 254-270,
// add_transactions 236-252, add_transaction_outputs 524-580, remove_outputs 589-621,
// remove_pending_transactions_by_hash — asyncpg statements against PostgreSQL, issued one by one on the
// request path. Here a validated block's writes become ONE encoded batch of column-major bulk statements:
//
//   commit point   the batch is appended to an append-only journal file (CRC-framed record, write(2);
//                  fdatasync per record or per materialiser group) — together with the HBM UTXO update
//                  this is when the block is applied;
//   materialise    one background thread per database file (the UTXO table lives in a file of its own)
//                  applies queued batches to the schema.sql tables, several blocks per SQLite transaction
//                  (group commit), and records the last applied journal sequence number in that file's
//                  `upow_journal_state` inside the same transaction;
//   watermark      readers that need those tables wait until the applied sequence covers the last batch
//                  that wrote them (Python: Database._settle);
//   restart        journal records above the recorded sequence are re-applied before the ledger opens,
//                  a torn tail record is cut off.
//
// Concurrency of the commit point: a submitter reserves its sequence number and file offset under the
// journal mutex and writes its record with pwrite(2) OUTSIDE it, so a /push_tx admission never waits
// behind a block's 10 MB append; records are handed to the materialisers strictly in sequence order once
// every lower record is written (publication).
//
// Durability (sync modes): off; group (the materialisers fdatasync before applying, so no SQL file is
// ever ahead of the durable journal prefix); block (group + every BLOCK record is fdatasync'd before
// submit returns, i.e. before push_block answers and gossips); commit (every record).
//
// Undo data (a block's created and spent outpoints with their payloads) goes to an undo log of its own
// (segment files next to the journal) that journal rotation does not touch; it keeps the last `undo_keep`
// blocks so rollback over the reference's 500-block fork window never needs an index rebuild.
//
// Backpressure: a block submit waits while any materialiser has more than `max_queue_bytes` queued, so a
// sync that validates faster than SQLite materialises cannot grow memory without bound.
//
// Integrity: a statement whose expected change count is not met (a DELETE of spent outputs that did not
// find every row: the HBM index and SQL disagree) stops the writer; SQLITE_BUSY/LOCKED on a group is
// retried with backoff instead.
//
// libsqlite3 is resolved with dlopen from the copy the interpreter's _sqlite3 module already loaded.
#include <dlfcn.h>
#include <fcntl.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <dirent.h>
#include <pthread.h>
#include <sys/resource.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <sys/uio.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <climits>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <optional>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace py = pybind11;

namespace upow {
namespace {

struct sqlite3;
struct sqlite3_stmt;
typedef void (*destructor_t)(void*);
constexpr int SQLITE_OK = 0, SQLITE_BUSY = 5, SQLITE_LOCKED = 6, SQLITE_ROW = 100, SQLITE_DONE = 101,
              SQLITE_CONSTRAINT = 19;
constexpr int SQLITE_OPEN_READWRITE = 0x2, SQLITE_OPEN_CREATE = 0x4, SQLITE_OPEN_NOMUTEX = 0x8000,
              SQLITE_OPEN_URI = 0x40;

struct SqliteApi {
    int (*open_v2)(const char*, sqlite3**, int, const char*) = nullptr;
    int (*close_v2)(sqlite3*) = nullptr;
    int (*exec)(sqlite3*, const char*, void*, void*, char**) = nullptr;
    int (*busy_timeout)(sqlite3*, int) = nullptr;
    int (*prepare_v2)(sqlite3*, const char*, int, sqlite3_stmt**, const char**) = nullptr;
    int (*bind_text)(sqlite3_stmt*, int, const char*, int, destructor_t) = nullptr;
    int (*bind_int64)(sqlite3_stmt*, int, long long) = nullptr;
    int (*bind_null)(sqlite3_stmt*, int) = nullptr;
    int (*step)(sqlite3_stmt*) = nullptr;
    int (*reset)(sqlite3_stmt*) = nullptr;
    int (*clear_bindings)(sqlite3_stmt*) = nullptr;
    int (*finalize)(sqlite3_stmt*) = nullptr;
    int (*changes)(sqlite3*) = nullptr;
    long long (*column_int64)(sqlite3_stmt*, int) = nullptr;
    const char* (*errmsg)(sqlite3*) = nullptr;
    void (*free)(void*) = nullptr;
    int (*config)(int, ...) = nullptr;
    int (*initialize)() = nullptr;
    int (*shutdown)() = nullptr;
    bool ok = false;
};

const SqliteApi& api() {
    static SqliteApi a = [] {
        SqliteApi s;
        void* h = dlopen("libsqlite3.so.0", RTLD_NOW | RTLD_NOLOAD);
        if (!h) h = dlopen("libsqlite3.so.0", RTLD_NOW);
        if (!h) return s;
        auto sym = [&](auto& fn, const char* name) { fn = reinterpret_cast<std::decay_t<decltype(fn)>>(dlsym(h, name)); };
        sym(s.open_v2, "sqlite3_open_v2");
        sym(s.close_v2, "sqlite3_close_v2");
        sym(s.exec, "sqlite3_exec");
        sym(s.busy_timeout, "sqlite3_busy_timeout");
        sym(s.prepare_v2, "sqlite3_prepare_v2");
        sym(s.bind_text, "sqlite3_bind_text");
        sym(s.bind_int64, "sqlite3_bind_int64");
        sym(s.bind_null, "sqlite3_bind_null");
        sym(s.step, "sqlite3_step");
        sym(s.reset, "sqlite3_reset");
        sym(s.clear_bindings, "sqlite3_clear_bindings");
        sym(s.finalize, "sqlite3_finalize");
        sym(s.changes, "sqlite3_changes");
        sym(s.column_int64, "sqlite3_column_int64");
        sym(s.errmsg, "sqlite3_errmsg");
        sym(s.free, "sqlite3_free");
        sym(s.config, "sqlite3_config");
        sym(s.initialize, "sqlite3_initialize");
        sym(s.shutdown, "sqlite3_shutdown");
        s.ok = s.open_v2 && s.close_v2 && s.exec && s.busy_timeout && s.prepare_v2 && s.bind_text && s.bind_int64 &&
               s.bind_null && s.step && s.reset && s.clear_bindings && s.finalize && s.changes && s.column_int64 &&
               s.errmsg && s.free && s.config && s.initialize && s.shutdown;
        return s;
    }();
    if (!a.ok) throw std::runtime_error("libsqlite3.so.0 not available for the native ledger writer");
    return a;
}

// ------------------------------------------------------------------------------------------ byte codec
struct Out {
    std::string b;
    void raw(const void* p, size_t n) { b.append(static_cast<const char*>(p), n); }
    void u8(uint8_t v) { raw(&v, 1); }
    void u32(uint32_t v) { raw(&v, 4); }
    void i64(int64_t v) { raw(&v, 8); }
    void str(const std::string& s) {
        u32(uint32_t(s.size()));
        raw(s.data(), s.size());
    }
};

struct In {
    const char* p;
    const char* e;
    void need(size_t n) const {
        if (size_t(e - p) < n) throw std::runtime_error("ledger batch truncated");
    }
    template <class T>
    T get() {
        need(sizeof(T));
        T v;
        std::memcpy(&v, p, sizeof(T));
        p += sizeof(T);
        return v;
    }
    const char* take(size_t n) {
        need(n);
        const char* r = p;
        p += n;
        return r;
    }
    std::string str() {
        uint32_t n = get<uint32_t>();
        return std::string(take(n), n);
    }
};

// Column kinds of an encoded statement.
enum ColKind : uint8_t { K_NULL = 0, K_CTEXT = 1, K_CINT = 2, K_INT64 = 3, K_HEX32 = 4, K_TEXT = 5, K_HEXTEXT = 6 };

// Encode one column spec (Python side) for n rows:
//   list[str|None]                    text per row
//   ('gather', list[str], int32 buf)   text list[idx[row]]
//   ('hex32', buf, stride, offset)     lowercase hex of the 32 bytes at row*stride+offset
//   ('arena', blob, int64 offsets)     text blob[off[row]:off[row+1]] (csrc/txcodec.cpp text arenas)
//   ('hexarena', blob, int64 offsets)  lowercase hex of the bytes blob[off[row]:off[row+1]]: raw in the
//                                      journal (half the size of the text), rendered when bound
//   int64 numpy array                  integer per row
//   str / int / None                   the same value for every row
void encode_text_rows(Out& o, int64_t n, const std::vector<const char*>& ptr, const std::vector<int64_t>& len,
                      const int32_t* idx) {
    // K_TEXT: u8 has_null, [u8 null[n]], i64 off[n+1], blob
    std::vector<int64_t> off(size_t(n) + 1, 0);
    std::vector<uint8_t> nul(size_t(n), 0);
    bool any_null = false;
    for (int64_t r = 0; r < n; ++r) {
        const size_t g = idx ? size_t(idx[r]) : size_t(r);
        nul[size_t(r)] = ptr[g] == nullptr;
        any_null |= ptr[g] == nullptr;
        off[size_t(r) + 1] = off[size_t(r)] + (ptr[g] ? len[g] : 0);
    }
    o.u8(K_TEXT);
    o.u8(any_null);
    if (any_null) o.raw(nul.data(), nul.size());
    o.raw(off.data(), off.size() * 8);
    for (int64_t r = 0; r < n; ++r) {
        const size_t g = idx ? size_t(idx[r]) : size_t(r);
        if (ptr[g]) o.raw(ptr[g], size_t(len[g]));
    }
}

void utf8_list(py::list lst, std::vector<const char*>& ptr, std::vector<int64_t>& len) {
    const size_t n = lst.size();
    ptr.resize(n);
    len.resize(n);
    for (size_t i = 0; i < n; ++i) {
        PyObject* obj = PyList_GET_ITEM(lst.ptr(), i);
        if (obj == Py_None) {
            ptr[i] = nullptr;
            len[i] = 0;
            continue;
        }
        Py_ssize_t sz = 0;
        const char* s = PyUnicode_AsUTF8AndSize(obj, &sz);
        if (!s) throw py::error_already_set();
        ptr[i] = s;
        len[i] = sz;
    }
}

// a row selection int64[n] (non-negative; the caller checks the upper bound against its column)
const int64_t* row_selection(py::handle h, int64_t n) {
    py::buffer_info bi = h.cast<py::buffer>().request();
    if (bi.itemsize != 8 || bi.size != n) throw std::invalid_argument("row selection must be int64[n]");
    const int64_t* sel = static_cast<const int64_t*>(bi.ptr);
    for (int64_t r = 0; r < n; ++r)
        if (sel[r] < 0) throw std::out_of_range("row selection");
    return sel;
}

// Column copies of a block (megabytes, often on the encode pool's threads) run without the GIL so the
// HTTP event loop thread never waits for them. A /push_tx admission encodes a row or two on the loop
// thread itself: releasing there would hand the GIL to whichever thread is runnable (the ledger thread
// during a block) and make the loop wait for it back, so small columns keep it.
constexpr int64_t kNoGilRows = 256;
struct NoGilIfLarge {
    std::optional<py::gil_scoped_release> rel;
    explicit NoGilIfLarge(int64_t rows) {
        if (rows >= kNoGilRows) rel.emplace();
    }
};

void encode_col(Out& o, py::handle spec, int64_t n) {
    if (spec.is_none()) {
        o.u8(K_NULL);
    } else if (py::isinstance<py::str>(spec)) {
        o.u8(K_CTEXT);
        o.str(spec.cast<std::string>());
    } else if (py::isinstance<py::bool_>(spec) || py::isinstance<py::int_>(spec)) {
        o.u8(K_CINT);
        o.i64(spec.cast<long long>());
    } else if (py::isinstance<py::list>(spec)) {
        std::vector<const char*> ptr;
        std::vector<int64_t> len;
        utf8_list(spec.cast<py::list>(), ptr, len);
        if (int64_t(ptr.size()) != n) throw std::invalid_argument("text column length != n");
        // the row copies run without the GIL (the caller's list keeps every str alive): a block's
        // columns are megabytes, and the HTTP event loop thread must not wait for them
        NoGilIfLarge nogil(n);
        encode_text_rows(o, n, ptr, len, nullptr);
    } else if (py::isinstance<py::tuple>(spec)) {
        py::tuple t = spec.cast<py::tuple>();
        const std::string tag = t[0].cast<std::string>();
        if (tag == "gather") {
            std::vector<const char*> ptr;
            std::vector<int64_t> len;
            utf8_list(t[1].cast<py::list>(), ptr, len);
            py::buffer_info bi = t[2].cast<py::buffer>().request();
            if (bi.itemsize != 4) throw std::invalid_argument("gather index must be int32");
            if (bi.size != n) throw std::invalid_argument("gather index length != n");
            const int32_t* idx = static_cast<const int32_t*>(bi.ptr);
            for (int64_t i = 0; i < n; ++i)
                if (idx[i] < 0 || size_t(idx[i]) >= ptr.size()) throw std::out_of_range("gather index");
            NoGilIfLarge nogil(n);
            encode_text_rows(o, n, ptr, len, idx);
        } else if (tag == "hex32") {
            // ('hex32', raw, stride, offset[, sel int64[n]]): 32 raw bytes per row, optionally rows sel of raw
            py::buffer_info bi = t[1].cast<py::buffer>().request();
            const uint8_t* raw = static_cast<const uint8_t*>(bi.ptr);
            const int64_t raw_n = bi.size * bi.itemsize, stride = t[2].cast<int64_t>(), offset = t[3].cast<int64_t>();
            const int64_t* sel = t.size() > 4 ? row_selection(t[4], n) : nullptr;
            int64_t top = n - 1;
            if (sel) {
                top = -1;
                for (int64_t r = 0; r < n; ++r) top = std::max(top, sel[r]);
            }
            if (offset < 0 || stride < 0 || (n > 0 && top * stride + offset + 32 > raw_n))
                throw std::out_of_range("hex32 column out of range");
            o.u8(K_HEX32);
            NoGilIfLarge nogil(n);
            o.b.reserve(o.b.size() + size_t(n) * 32);
            for (int64_t r = 0; r < n; ++r) o.raw(raw + (sel ? sel[r] : r) * stride + offset, 32);
        } else if (tag == "arena" || tag == "hexarena") {
            // ('arena', blob, offsets int64[N + 1][, sel int64[n]]): text rows, optionally rows sel of the arena
            py::buffer_info bb = t[1].cast<py::buffer>().request(), ob = t[2].cast<py::buffer>().request();
            const int64_t* sel = t.size() > 3 ? row_selection(t[3], n) : nullptr;
            const int64_t rows = ob.size * ob.itemsize / 8 - 1;
            if (sel ? rows < 0 || ob.size * ob.itemsize % 8 : ob.size * ob.itemsize != 8 * (n + 1))
                throw std::invalid_argument("arena offsets must be int64[n + 1]");
            const char* blob = static_cast<const char*>(bb.ptr);
            const int64_t* aoff = static_cast<const int64_t*>(ob.ptr);
            const int64_t blen = bb.size * bb.itemsize;
            for (int64_t i = 0; i < (sel ? rows : n); ++i)
                if (aoff[i] < 0 || aoff[i + 1] < aoff[i] || aoff[i + 1] > blen) throw std::out_of_range("arena offsets");
            if (sel)
                for (int64_t r = 0; r < n; ++r)
                    if (sel[r] >= rows) throw std::out_of_range("arena row selection");
            if (tag == "arena") {
                o.u8(K_TEXT);
                o.u8(0);
            } else {
                o.u8(K_HEXTEXT);
            }
            NoGilIfLarge nogil(n);
            std::vector<int64_t> off(size_t(n) + 1);
            if (!sel) {
                for (int64_t i = 0; i <= n; ++i) off[size_t(i)] = aoff[i] - aoff[0];
                o.raw(off.data(), off.size() * 8);
                o.raw(blob + aoff[0], size_t(aoff[n] - aoff[0]));
            } else {
                for (int64_t r = 0; r < n; ++r) off[size_t(r) + 1] = off[size_t(r)] + aoff[sel[r] + 1] - aoff[sel[r]];
                o.raw(off.data(), off.size() * 8);
                o.b.reserve(o.b.size() + size_t(off[size_t(n)]));
                for (int64_t r = 0; r < n; ++r) o.raw(blob + aoff[sel[r]], size_t(aoff[sel[r] + 1] - aoff[sel[r]]));
            }
        } else {
            throw std::invalid_argument("unknown column tag " + tag);
        }
    } else {
        py::buffer_info bi = spec.cast<py::buffer>().request();
        if (bi.itemsize != 8 || bi.format.find_first_of("qlQL") == std::string::npos)
            throw std::invalid_argument("integer column must be int64");
        if (bi.size != n) throw std::invalid_argument("int column length != n");
        o.u8(K_INT64);
        NoGilIfLarge nogil(n);
        o.raw(bi.ptr, size_t(n) * 8);
    }
}

// Statement encoding: str sql, u32 flags (1: guard sql, 2: expected change count, bits 8..15: target
// database file), [str guard], [i64 expect],
// i64 n, u32 n_cols, cols..., u8 has_order, [i64 order[n]].
// An encoded statement owned by C++: submit() keeps the buffer itself as one part of the journal record
// (no Python bytes copy on the way out, no concatenation on the way in).
struct EncodedStmt {
    std::shared_ptr<const std::string> buf;
};

EncodedStmt encode_stmt(const std::string& sql, py::sequence cols, int64_t n, py::object order, py::object guard,
                        py::object expect, int shard, int route) {
    if (n < 0) throw std::invalid_argument("n < 0");
    if (shard < 0 || shard > 15) throw std::invalid_argument("shard must be in [0, 15]");
    if (route < 0 || route > 15 || shard + route > 16) throw std::invalid_argument("route must be in [0, 15]");
    Out o;
    o.str(sql);
    // route > 1: the rows are spread over files shard .. shard+route-1 by the first byte of column 0
    // (a tx hash), each file's materialiser applying only its own rows
    const uint32_t flags = (guard.is_none() ? 0u : 1u) | (expect.is_none() ? 0u : 2u) | (uint32_t(shard) << 8) |
                           (route > 1 ? (4u | (uint32_t(route) << 16)) : 0u);
    o.u32(flags);
    if (flags & 1) o.str(guard.cast<std::string>());
    if (flags & 2) o.i64(expect.cast<int64_t>());
    o.i64(n);
    o.u32(uint32_t(cols.size()));
    for (auto spec : cols) encode_col(o, spec, n);
    if (order.is_none()) {
        o.u8(0);
    } else if (py::isinstance<py::str>(order)) {
        // "key": rows in the order of column 0's leading 8 bytes (big-endian, stable), B-tree locality for
        // the writes; the materialiser sorts, so the block path does not
        if (order.cast<std::string>() != "key") throw std::invalid_argument("order must be int64[n] or 'key'");
        o.u8(2);
    } else {
        py::buffer_info bi = order.cast<py::buffer>().request();
        if (bi.itemsize != 8 || bi.size != n) throw std::invalid_argument("order must be int64[n]");
        const int64_t* ord = static_cast<const int64_t*>(bi.ptr);
        for (int64_t i = 0; i < n; ++i)
            if (ord[i] < 0 || ord[i] >= n) throw std::out_of_range("order");
        o.u8(1);
        o.raw(ord, size_t(n) * 8);
    }
    return EncodedStmt{std::make_shared<const std::string>(std::move(o.b))};
}

// Decoded view of one column inside a batch buffer.
struct ColView {
    uint8_t kind = K_NULL;
    std::string ctext;
    long long cint = 0;
    const char* data = nullptr;  // INT64 / HEX32 rows, TEXT blob
    const uint8_t* nul = nullptr;
    const char* off = nullptr;  // TEXT offsets (i64[n+1], unaligned)
};

int64_t ld64(const char* p) {
    int64_t v;
    std::memcpy(&v, p, 8);
    return v;
}

uint32_t hex_nibble(char c) {
    if (c >= '0' && c <= '9') return uint32_t(c - '0');
    if (c >= 'a' && c <= 'f') return uint32_t(c - 'a' + 10);
    if (c >= 'A' && c <= 'F') return uint32_t(c - 'A' + 10);
    return 0;
}

// First byte of row r's tx hash in column c (raw hex32 rows, or hex text): the routing key of a
// statement spread over several files.
uint32_t route_byte(const ColView& c, int64_t r) {
    if (c.kind == K_HEX32) return uint8_t(c.data[32 * r]);
    if (c.kind == K_HEXTEXT) {
        const int64_t o0 = ld64(c.off + 8 * r), o1 = ld64(c.off + 8 * (r + 1));
        return o1 > o0 ? uint8_t(c.data[o0]) : 0u;
    }
    if (c.kind == K_TEXT && !(c.nul && c.nul[r])) {
        const int64_t o0 = ld64(c.off + 8 * r), o1 = ld64(c.off + 8 * (r + 1));
        if (o1 - o0 >= 2) return (hex_nibble(c.data[o0]) << 4) | hex_nibble(c.data[o0 + 1]);
    }
    if (c.kind == K_CTEXT && c.ctext.size() >= 2) return (hex_nibble(c.ctext[0]) << 4) | hex_nibble(c.ctext[1]);
    return 0;
}

const char kHex[] = "0123456789abcdef";

struct SqlError : std::runtime_error {
    int rc;
    SqlError(const std::string& m, int c) : std::runtime_error(m), rc(c) {}
};

// A statement changed a different number of rows than its batch declared (ledger/index divergence).
struct MismatchError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

// ------------------------------------------------------------------------------------------ journal
constexpr uint32_t kMagic = 0x314a5055;  // "UPJ1"
// records at least this large (a block's) are written in kWriteChunk slices with the checksum computed alongside
constexpr size_t kSplitWriteBytes = size_t(1) << 20;
constexpr size_t kWriteChunk = size_t(1) << 20;
struct RecHeader {
    uint32_t magic;
    uint32_t crc;       // CRC-32C over seq, block_id, meta_len, payload_len and both sections
    uint64_t seq;
    int64_t block_id;   // -1: not a block
    uint64_t meta_len;
    uint64_t payload_len;
};
static_assert(sizeof(RecHeader) == 40, "journal record header layout");

uint32_t crc32c_sw(uint32_t crc, const uint8_t* p, size_t n) {
    static uint32_t table[8][256];
    static bool init = [] {
        for (uint32_t i = 0; i < 256; ++i) {
            uint32_t c = i;
            for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
            table[0][i] = c;
        }
        for (uint32_t i = 0; i < 256; ++i)
            for (int t = 1; t < 8; ++t) table[t][i] = (table[t - 1][i] >> 8) ^ table[0][table[t - 1][i] & 0xff];
        return true;
    }();
    (void)init;
    crc = ~crc;
    while (n >= 8) {
        uint64_t v;
        std::memcpy(&v, p, 8);
        v ^= crc;
        crc = table[7][v & 0xff] ^ table[6][(v >> 8) & 0xff] ^ table[5][(v >> 16) & 0xff] ^
              table[4][(v >> 24) & 0xff] ^ table[3][(v >> 32) & 0xff] ^ table[2][(v >> 40) & 0xff] ^
              table[1][(v >> 48) & 0xff] ^ table[0][v >> 56];
        p += 8;
        n -= 8;
    }
    while (n--) crc = (crc >> 8) ^ table[0][(crc ^ *p++) & 0xff];
    return ~crc;
}

__attribute__((target("sse4.2"))) uint32_t crc32c_hw(uint32_t crc, const uint8_t* p, size_t n) {
    uint64_t c = ~crc;
    while (n >= 8) {
        uint64_t v;
        std::memcpy(&v, p, 8);
        c = __builtin_ia32_crc32di(c, v);
        p += 8;
        n -= 8;
    }
    uint32_t c32 = uint32_t(c);
    while (n--) c32 = __builtin_ia32_crc32qi(c32, *p++);
    return ~c32;
}

// Three interleaved streams of the crc32 instruction (latency 3, throughput 1 per cycle: one stream uses a
// third of the unit). Each 3L-byte step runs the three L-byte thirds from registers (c, 0, 0) and joins them
// with the zero-extension operators of the raw register, which are linear: after the step the register is
// M_2L(a) ^ M_L(b) ^ d. M_L and M_2L are applied as four 256-entry byte tables each, built once from the
// images of the 32 basis vectors. A block's 9 MB journal record is checksummed ~3x faster than one stream.
struct Crc3Tables {
    static constexpr size_t L = 8192;
    uint32_t ml[4][256], m2l[4][256];
    __attribute__((target("sse4.2"))) Crc3Tables() {
        uint32_t basis[32];
        for (int i = 0; i < 32; ++i) {
            uint64_t r = uint64_t(1) << i;
            for (size_t k = 0; k < L / 8; ++k) r = __builtin_ia32_crc32di(r, 0);
            basis[i] = uint32_t(r);
        }
        fill(ml, basis);
        uint32_t basis2[32];
        for (int i = 0; i < 32; ++i) basis2[i] = apply(ml, basis[i]);
        fill(m2l, basis2);
    }
    static void fill(uint32_t t[4][256], const uint32_t* basis) {
        for (int k = 0; k < 4; ++k)
            for (uint32_t v = 0; v < 256; ++v) {
                uint32_t r = 0;
                for (int b = 0; b < 8; ++b)
                    if (v >> b & 1u) r ^= basis[8 * k + b];
                t[k][v] = r;
            }
    }
    static uint32_t apply(const uint32_t t[4][256], uint32_t x) {
        return t[0][x & 0xff] ^ t[1][(x >> 8) & 0xff] ^ t[2][(x >> 16) & 0xff] ^ t[3][x >> 24];
    }
};

__attribute__((target("sse4.2"))) uint32_t crc32c_hw3(uint32_t crc, const uint8_t* p, size_t n) {
    constexpr size_t L = Crc3Tables::L;
    if (n < 3 * L) return crc32c_hw(crc, p, n);
    static const Crc3Tables tab;
    uint32_t c = ~crc;
    while (n >= 3 * L) {
        uint64_t a = c, b = 0, d = 0;
        for (size_t k = 0; k < L; k += 8) {
            uint64_t x, y, z;
            std::memcpy(&x, p + k, 8);
            std::memcpy(&y, p + L + k, 8);
            std::memcpy(&z, p + 2 * L + k, 8);
            a = __builtin_ia32_crc32di(a, x);
            b = __builtin_ia32_crc32di(b, y);
            d = __builtin_ia32_crc32di(d, z);
        }
        c = Crc3Tables::apply(tab.m2l, uint32_t(a)) ^ Crc3Tables::apply(tab.ml, uint32_t(b)) ^ uint32_t(d);
        p += 3 * L;
        n -= 3 * L;
    }
    return crc32c_hw(~c, p, n);
}

uint32_t crc32c(uint32_t crc, const void* p, size_t n) {
    static const bool hw = __builtin_cpu_supports("sse4.2");
    return hw ? crc32c_hw3(crc, static_cast<const uint8_t*>(p), n) : crc32c_sw(crc, static_cast<const uint8_t*>(p), n);
}

uint32_t record_crc(const RecHeader& h, const char* meta, const char* payload) {
    uint32_t c = crc32c(0, &h.seq, sizeof(RecHeader) - 8);
    c = crc32c(c, meta, h.meta_len);
    return crc32c(c, payload, h.payload_len);
}

using Part = std::shared_ptr<const std::string>;

// the same checksum over a payload held as consecutive parts (no meta section)
uint32_t record_crc_parts(const RecHeader& h, const std::vector<Part>& parts) {
    uint32_t c = crc32c(0, &h.seq, sizeof(RecHeader) - 8);
    for (auto& pt : parts) c = crc32c(c, pt->data(), pt->size());
    return c;
}

// one record = header + parts, written with as few pwritev(2) calls as the iovec limit allows
void pwritev_all(int fd, const RecHeader& h, const std::vector<Part>& parts, off_t at) {
    std::vector<iovec> iov;
    iov.reserve(parts.size() + 1);
    iov.push_back({const_cast<RecHeader*>(&h), sizeof h});
    for (auto& pt : parts)
        if (!pt->empty()) iov.push_back({const_cast<char*>(pt->data()), pt->size()});
    size_t i = 0;
    while (i < iov.size()) {
        const int cnt = int(std::min<size_t>(iov.size() - i, IOV_MAX));
        ssize_t w = ::pwritev(fd, &iov[i], cnt, at);
        if (w < 0) {
            if (errno == EINTR) continue;
            throw std::runtime_error(std::string("journal write failed: ") + strerror(errno));
        }
        at += w;
        while (w > 0 && i < iov.size()) {  // consume what was written (a short write resumes mid-iovec)
            if (size_t(w) >= iov[i].iov_len) {
                w -= ssize_t(iov[i].iov_len);
                ++i;
            } else {
                iov[i].iov_base = static_cast<char*>(iov[i].iov_base) + w;
                iov[i].iov_len -= size_t(w);
                w = 0;
            }
        }
    }
}

// The body of a record (its parts, without the header) from `at`, in slices of about `chunk` bytes; with
// `writeback`, each slice's writeback to the device is started as soon as it is in the page cache
// (sync_file_range WRITE: no wait), so the commit's fdatasync finds most of the record already on its way.
void pwrite_body_chunked(int fd, const std::vector<Part>& parts, off_t at, size_t chunk, bool writeback) {
    std::vector<iovec> iov;
    size_t pi = 0, po = 0;  // next part, offset inside it
    while (pi < parts.size()) {
        iov.clear();
        size_t n = 0;
        while (pi < parts.size() && n < chunk && iov.size() < size_t(IOV_MAX)) {
            const std::string& pt = *parts[pi];
            const size_t take = std::min(pt.size() - po, chunk - n);
            if (take) iov.push_back({const_cast<char*>(pt.data() + po), take});
            n += take;
            po += take;
            if (po == pt.size()) {
                ++pi;
                po = 0;
            }
        }
        const off_t start = at;
        size_t i = 0;
        while (i < iov.size()) {
            ssize_t w = ::pwritev(fd, &iov[i], int(iov.size() - i), at);
            if (w < 0) {
                if (errno == EINTR) continue;
                throw std::runtime_error(std::string("journal write failed: ") + strerror(errno));
            }
            at += w;
            while (w > 0 && i < iov.size()) {
                if (size_t(w) >= iov[i].iov_len) {
                    w -= ssize_t(iov[i].iov_len);
                    ++i;
                } else {
                    iov[i].iov_base = static_cast<char*>(iov[i].iov_base) + w;
                    iov[i].iov_len -= size_t(w);
                    w = 0;
                }
            }
        }
        if (writeback && at > start) ::sync_file_range(fd, start, at - start, SYNC_FILE_RANGE_WRITE);
    }
}

void pwrite_all(int fd, const char* p, size_t n, off_t at) {
    while (n) {
        ssize_t w = ::pwrite(fd, p, n, at);
        if (w < 0) {
            if (errno == EINTR) continue;
            throw std::runtime_error(std::string("journal write failed: ") + strerror(errno));
        }
        p += w;
        at += w;
        n -= size_t(w);
    }
}

bool read_exact(int fd, char* p, size_t n, off_t at) {
    while (n) {
        ssize_t r = ::pread(fd, p, n, at);
        if (r < 0 && errno == EINTR) continue;
        if (r <= 0) return false;
        p += r;
        n -= size_t(r);
        at += r;
    }
    return true;
}

// The distribution's libsqlite3 is built with OMIT_LOOKASIDE (every small allocation goes to malloc) and
// the default MEMSTATUS=1, which wraps each malloc/free in one process-wide mutex: two materialiser
// threads on two files then serialise on that mutex. Allocation statistics can only be switched off before
// the library is initialised, so this runs when the extension loads (before any connection exists):
// returns the sqlite3_config result (0 = applied, 21 = library already initialised).
int sqlite_disable_memstatus() {
    const SqliteApi& a = api();
    constexpr int SQLITE_CONFIG_MEMSTATUS = 9;
    return a.config(SQLITE_CONFIG_MEMSTATUS, 0);
}

// ------------------------------------------------------------------------------------------ undo log
// A block's undo data lives in segment files `<prefix>.<n>` (n = 0, 1, ...), each holding up to
// `seg_blocks` records: {magic, crc, block_id, len} + body. A negative block_id is a tombstone ("forget
// blocks >= -(block_id + 1)", written on rollback so a restart does not resurrect rolled-back blocks).
// Whole segments whose newest block is older than the retention window are unlinked: no compaction copy.
constexpr uint32_t kUndoMagic = 0x31445055;  // "UPD1"
struct UndoHeader {
    uint32_t magic;
    uint32_t crc;  // CRC-32C over block_id, len and the body
    int64_t block_id;
    uint64_t len;
};
static_assert(sizeof(UndoHeader) == 24, "undo record header layout");

class UndoLog {
   public:
    UndoLog(std::string prefix, int64_t keep, int64_t seg_blocks)
        : prefix_(std::move(prefix)), keep_(std::max<int64_t>(1, keep)), seg_blocks_(std::max<int64_t>(1, seg_blocks)) {}

    ~UndoLog() {
        for (auto& kv : segs_)
            if (kv.second.fd >= 0) ::close(kv.second.fd);
    }

    void open() {
        std::lock_guard<std::mutex> lk(mu_);
        const size_t slash = prefix_.rfind('/');
        const std::string dir = slash == std::string::npos ? "." : prefix_.substr(0, slash);
        const std::string base = (slash == std::string::npos ? prefix_ : prefix_.substr(slash + 1)) + ".";
        std::vector<int64_t> found;
        if (DIR* d = ::opendir(dir.c_str())) {
            while (dirent* e = ::readdir(d)) {
                const std::string name = e->d_name;
                if (name.size() <= base.size() || name.compare(0, base.size(), base) != 0) continue;
                const std::string num = name.substr(base.size());
                if (num.find_first_not_of("0123456789") != std::string::npos) continue;
                found.push_back(std::stoll(num));
            }
            ::closedir(d);
        }
        std::sort(found.begin(), found.end());
        for (int64_t no : found) {
            Seg& sg = segs_[no];
            sg.fd = ::open(path(no).c_str(), O_RDWR | O_CLOEXEC);
            if (sg.fd < 0) throw std::runtime_error("undo log: cannot open " + path(no) + ": " + strerror(errno));
            scan(no, sg, no == found.back());
        }
        if (segs_.empty()) new_segment(0);
    }

    void put(int64_t block_id, const std::string& body) {
        std::lock_guard<std::mutex> lk(mu_);
        append(block_id, body);
        index_max_ = std::max(index_max_, block_id);
        prune();
    }

    void forget_from(int64_t block_id) {
        std::lock_guard<std::mutex> lk(mu_);
        index_.erase(index_.lower_bound(block_id), index_.end());
        append(-(block_id + 1), std::string());
        index_max_ = index_.empty() ? -1 : index_.rbegin()->first;
    }

    bool get(int64_t block_id, std::string& out) {
        std::lock_guard<std::mutex> lk(mu_);
        auto it = index_.find(block_id);
        if (it == index_.end()) return false;
        auto sg = segs_.find(it->second.first);
        if (sg == segs_.end()) return false;
        UndoHeader h;
        if (!read_exact(sg->second.fd, reinterpret_cast<char*>(&h), sizeof h, it->second.second) ||
            h.magic != kUndoMagic || h.block_id != block_id)
            return false;
        out.assign(h.len, '\0');
        if (!read_exact(sg->second.fd, out.data(), out.size(), it->second.second + off_t(sizeof h))) return false;
        return crc(h, out.data()) == h.crc;
    }

    void fill_stats(py::dict& d) {
        std::lock_guard<std::mutex> lk(mu_);
        int64_t bytes = 0;
        for (auto& kv : segs_) bytes += kv.second.size;
        d["undo_segments"] = int64_t(segs_.size());
        d["undo_blocks"] = int64_t(index_.size());
        d["undo_bytes"] = bytes;
        d["undo_first_block"] = index_.empty() ? int64_t(-1) : index_.begin()->first;
        d["undo_pruned_segments"] = pruned_;
    }

   private:
    struct Seg {
        int fd = -1;
        off_t size = 0;
        int64_t records = 0;
        int64_t max_block = -1;
    };

    std::string path(int64_t no) const { return prefix_ + "." + std::to_string(no); }

    static uint32_t crc(const UndoHeader& h, const char* body) {
        uint32_t c = crc32c(0, &h.block_id, sizeof(UndoHeader) - 8);
        return crc32c(c, body, h.len);
    }

    void new_segment(int64_t no) {
        Seg& sg = segs_[no];
        sg.fd = ::open(path(no).c_str(), O_RDWR | O_CREAT | O_CLOEXEC, 0644);
        if (sg.fd < 0) throw std::runtime_error("undo log: cannot create " + path(no) + ": " + strerror(errno));
    }

    void scan(int64_t no, Seg& sg, bool last) {
        const off_t end = ::lseek(sg.fd, 0, SEEK_END);
        off_t at = 0;
        while (at + off_t(sizeof(UndoHeader)) <= end) {
            UndoHeader h;
            if (!read_exact(sg.fd, reinterpret_cast<char*>(&h), sizeof h, at) || h.magic != kUndoMagic) break;
            if (h.len > uint64_t(end) || at + off_t(sizeof h + h.len) > end) break;
            std::string body(h.len, '\0');
            if (!read_exact(sg.fd, body.data(), body.size(), at + off_t(sizeof h)) || crc(h, body.data()) != h.crc) break;
            if (h.block_id >= 0) {
                index_[h.block_id] = {no, at};
                sg.max_block = std::max(sg.max_block, h.block_id);
            } else {
                index_.erase(index_.lower_bound(-(h.block_id + 1)), index_.end());
            }
            ++sg.records;
            at += off_t(sizeof h + h.len);
        }
        if (at != end && last && ::ftruncate(sg.fd, at) != 0) throw std::runtime_error("undo log truncate failed");
        sg.size = at;
        index_max_ = index_.empty() ? -1 : index_.rbegin()->first;
    }

    void append(int64_t block_id, const std::string& body) {
        auto cur = std::prev(segs_.end());
        if (cur->second.records >= seg_blocks_) {
            new_segment(cur->first + 1);
            cur = std::prev(segs_.end());
        }
        Seg& sg = cur->second;
        UndoHeader h{kUndoMagic, 0, block_id, body.size()};
        h.crc = crc(h, body.data());
        pwrite_all(sg.fd, reinterpret_cast<const char*>(&h), sizeof h, sg.size);
        pwrite_all(sg.fd, body.data(), body.size(), sg.size + off_t(sizeof h));
        if (block_id >= 0) {
            index_[block_id] = {cur->first, sg.size};
            sg.max_block = std::max(sg.max_block, block_id);
        }
        sg.size += off_t(sizeof h + body.size());
        ++sg.records;
    }

    void prune() {
        // unlink whole segments (never the current one) whose newest block is outside the window
        const int64_t floor_id = index_max_ - keep_;
        for (auto it = segs_.begin(); it != segs_.end() && std::next(it) != segs_.end();) {
            if (it->second.max_block >= floor_id) {
                ++it;
                continue;
            }
            for (auto ix = index_.begin(); ix != index_.end();)
                ix = ix->second.first == it->first ? index_.erase(ix) : std::next(ix);
            ::close(it->second.fd);
            ::unlink(path(it->first).c_str());
            ++pruned_;
            it = segs_.erase(it);
        }
    }

    std::string prefix_;
    int64_t keep_, seg_blocks_;
    std::mutex mu_;
    std::map<int64_t, Seg> segs_;
    std::map<int64_t, std::pair<int64_t, off_t>> index_;  // block id -> (segment, offset)
    int64_t index_max_ = -1;
    int64_t pruned_ = 0;
};

// ------------------------------------------------------------------------------------------ writer
// One journal, several database files ("shards"): each statement names the file it writes (flags bits
// 8..15) and every file has its own materialiser thread and connection, so the UTXO table and the
// block/tx tables are brought up to date in parallel. Each file records the last journal sequence it
// applied (upow_journal_state, updated in the same transaction as the rows).
enum SyncMode { SYNC_OFF = 0, SYNC_GROUP = 1, SYNC_COMMIT = 2, SYNC_BLOCK = 3 };

struct Batch {
    uint64_t seq;
    // u32 n_stmts + statements, as consecutive parts: a submitted batch keeps its encoded statements as
    // they came (no concatenated copy), a replayed record is one part. A statement never spans two parts.
    std::vector<Part> parts;
    size_t size = 0;
    off_t end = 0;  // journal offset just past the record
};

struct Shard {
    std::string path;
    sqlite3* db = nullptr;
    std::unordered_map<std::string, sqlite3_stmt*> stmts;  // shard thread only
    std::deque<Batch> queue;
    size_t queued_bytes = 0;
    uint64_t applied = 0;
    int64_t groups = 0, replayed = 0, apply_ns = 0, commit_ns = 0, sync_ns = 0;
    std::thread thread;
};

class LedgerWriter {
   public:
    LedgerWriter(const std::vector<std::string>& db_paths, const std::string& journal_path, int sync_mode,
                 int64_t cache_mb, int group_max, int64_t journal_max_bytes, int64_t undo_keep,
                 int64_t max_queue_bytes, double throttle_timeout_s, int busy_timeout_ms)
        : journal_path_(journal_path), sync_(sync_mode), group_max_(std::max(1, group_max)),
          journal_max_(journal_max_bytes), max_queue_bytes_(max_queue_bytes), throttle_timeout_s_(throttle_timeout_s),
          busy_timeout_ms_(std::max(1, busy_timeout_ms)), undo_(journal_path + ".undo", undo_keep, 64) {
        if (db_paths.empty() || db_paths.size() > 16) throw std::invalid_argument("1..16 database files");
        if (sync_ < SYNC_OFF || sync_ > SYNC_BLOCK) throw std::invalid_argument("sync mode must be 0..3");
        for (auto& p : db_paths) {
            shards_.emplace_back(new Shard());
            Shard& sh = *shards_.back();
            sh.path = p;
            open_shard(sh, cache_mb);
        }
        fd_ = ::open(journal_path.c_str(), O_RDWR | O_CREAT | O_CLOEXEC, 0644);
        if (fd_ < 0) throw std::runtime_error("ledger writer: cannot open journal " + journal_path + ": " + strerror(errno));
        undo_.open();
        recover();
        for (size_t i = 0; i < shards_.size(); ++i) shards_[i]->thread = std::thread([this, i] { run(i); });
        io_thread_ = std::thread([this] { io_run(); });
    }

    ~LedgerWriter() { close(); }

    void close() {
        {
            std::unique_lock<std::mutex> lk(mu_);
            if (closed_) return;
        }
        {
            // deferred records still in the I/O queue are written (and published) before the shards stop
            std::lock_guard<std::mutex> g(io_mu_);
            io_stop_ = true;
        }
        io_cv_.notify_all();
        if (io_thread_.joinable()) io_thread_.join();
        {
            std::unique_lock<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        cv_done_.notify_all();
        for (auto& sh : shards_)
            if (sh->thread.joinable()) sh->thread.join();
        {
            std::lock_guard<std::mutex> jl(jmu_);
            if (fd_ >= 0) {
                ::fdatasync(fd_);
                ::close(fd_);
                fd_ = -1;
            }
        }
        for (auto& sh : shards_) {
            for (auto& kv : sh->stmts) api().finalize(kv.second);
            sh->stmts.clear();
            if (sh->db) api().close_v2(sh->db);
            sh->db = nullptr;
        }
        std::lock_guard<std::mutex> lk(mu_);
        closed_ = true;
    }

    // Commit point: reserve (seq, offset), write the record outside the journal mutex, publish it to the
    // materialisers in sequence order, make it durable as the sync mode asks. Returns the sequence number.
    // ``sync`` false (a block whose caller overlaps the journal with its own work): the record is handed to
    // the journal I/O thread right after its reservation, which checksums it, writes it, stores the block's
    // undo data, publishes it and fdatasyncs it; durable(seq) waits for all of that. The sequence number
    // (the commit order) is fixed before submit returns either way.
    // ``group`` (deferred records only): the I/O thread does not fdatasync this block record on its own; the
    // caller's later durable(seq) makes the whole prefix durable with one fdatasync (group commit of a sync
    // page: a crash loses at most the page's unsynced tail, which the node fetches again).
    uint64_t submit(std::vector<Part> stmts, std::string meta, int64_t block_id, bool sync = true, bool group = false) {
        Batch b;
        const uint32_t ns = uint32_t(stmts.size());
        b.parts.reserve(stmts.size() + 1);
        b.parts.push_back(std::make_shared<const std::string>(reinterpret_cast<const char*>(&ns), 4));
        b.size = 4;
        for (auto& st : stmts) {
            b.size += st->size();
            b.parts.push_back(std::move(st));
        }
        if (block_id >= 0) throttle();
        const size_t rec = sizeof(RecHeader) + b.size;
        off_t at;
        {
            std::lock_guard<std::mutex> jl(jmu_);
            {
                std::lock_guard<std::mutex> lk(mu_);
                if (failed_) throw std::runtime_error("ledger writer stopped after an error: " + error_);
                if (closed_ || stop_) throw std::runtime_error("ledger writer is closed");
            }
            b.seq = next_seq_++;
            at = journal_size_;
            journal_size_ += off_t(rec);
            bytes_written_ += int64_t(rec);
            ++inflight_;
            b.end = at + off_t(rec);
            if (!sync) {
                // queued under the reservation lock: the I/O thread sees deferred records in sequence order
                const uint64_t seq = b.seq;
                {
                    std::lock_guard<std::mutex> g(io_mu_);
                    io_q_.push_back(IoJob{std::move(b), at, block_id, std::move(meta), group});
                    ++io_pending_;
                }
                io_cv_.notify_one();
                return seq;
            }
        }
        const uint64_t seq = b.seq;
        std::string werr = write_record(b, at, block_id);
        if (!werr.empty()) throw std::runtime_error(werr);
        if (sync_ == SYNC_COMMIT || (sync_ == SYNC_BLOCK && block_id >= 0)) make_durable(seq);
        if (block_id >= 0 && !meta.empty()) undo_.put(block_id, meta);
        return seq;
    }

    // checksum + write one reserved record, then publish it (in sequence order); returns the write error
    // (`before_publish`: a helper thread joined after the write and before the record is published)
    std::string write_record(Batch& b, off_t at, int64_t block_id, std::thread* before_publish = nullptr) {
        RecHeader h{kMagic, 0, b.seq, block_id, 0, b.size};
        const auto t0 = std::chrono::steady_clock::now();
        std::string werr;
        auto t1 = t0;
        if (b.size >= kSplitWriteBytes) {
            // a block-sized record: the checksum (a pass over the whole body) runs on a helper thread while
            // this one writes the body slice by slice, starting each slice's writeback; the header (with the
            // checksum) goes last. Recovery reads header + body and checks the sum, as for any record.
            uint32_t crc = 0;
            std::thread sum([&] { crc = record_crc_parts(h, b.parts); });
            try {
                pwrite_body_chunked(fd_, b.parts, at + off_t(sizeof h), kWriteChunk, early_writeback_ && sync_ != SYNC_OFF);
            } catch (const std::exception& e) {
                werr = e.what();
            }
            t1 = std::chrono::steady_clock::now();
            sum.join();
            h.crc = crc;
            if (werr.empty()) {
                try {
                    pwrite_all(fd_, reinterpret_cast<const char*>(&h), sizeof h, at);
                } catch (const std::exception& e) {
                    werr = e.what();
                }
            }
        } else {
            h.crc = record_crc_parts(h, b.parts);
            t1 = std::chrono::steady_clock::now();
            try {
                pwritev_all(fd_, h, b.parts, at);
            } catch (const std::exception& e) {
                werr = e.what();
            }
        }
        const auto t2 = std::chrono::steady_clock::now();
        if (before_publish && before_publish->joinable()) before_publish->join();
        const auto t3 = std::chrono::steady_clock::now();
        auto ns = [](auto a, auto b) { return std::chrono::duration_cast<std::chrono::nanoseconds>(b - a).count(); };
        const bool split = b.size >= kSplitWriteBytes;  // split: t0..t1 the body write, t1..t2 the rest of the sum
        io_crc_ns_ += split ? ns(t1, t2) : ns(t0, t1);
        io_write_ns_ += split ? ns(t0, t1) : ns(t1, t2);
        io_undo_wait_ns_ += ns(t2, t3);
        {
            std::lock_guard<std::mutex> jl(jmu_);
            --inflight_;
        }
        {
            std::lock_guard<std::mutex> lk(mu_);
            if (!werr.empty() && !failed_) {
                failed_ = true;
                error_ = werr;
            }
            written_.emplace(b.seq, std::move(b));
            publish_locked();
        }
        cv_.notify_all();
        cv_done_.notify_all();
        return werr;
    }

    struct IoJob {
        Batch batch;
        off_t at;
        int64_t block_id;
        std::string meta;
        bool group = false;  // group commit: no per-record fdatasync (durable() syncs the prefix)
        std::chrono::steady_clock::time_point queued = std::chrono::steady_clock::now();
    };

    // The journal I/O thread: deferred (block) records in submission order. The undo data is stored before
    // the record is published, so a published block always has its undo record; the fdatasync follows.
    void io_run() {
        pthread_setname_np(pthread_self(), "upow-wr-io");
        for (;;) {
            IoJob job;
            {
                std::unique_lock<std::mutex> lk(io_mu_);
                io_cv_.wait(lk, [&] { return io_stop_ || !io_q_.empty(); });
                if (io_q_.empty()) return;  // stopping and drained
                job = std::move(io_q_.front());
                io_q_.pop_front();
            }
            io_queue_ns_ += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() -
                                                                                 job.queued).count();
            ++io_records_;
            const uint64_t seq = job.batch.seq;
            std::string err;
            // the undo record (its own file) is written alongside the journal record; both finish before
            // the block is published
            std::thread undo;
            if (job.block_id >= 0 && !job.meta.empty()) {
                undo = std::thread([&] {
                    try {
                        undo_.put(job.block_id, job.meta);
                    } catch (const std::exception& e) {
                        err = e.what();
                    }
                });
            }
            std::string werr = write_record(job.batch, job.at, job.block_id, &undo);
            if (werr.empty() && !err.empty()) {
                std::lock_guard<std::mutex> lk(mu_);
                if (!failed_) {
                    failed_ = true;
                    error_ = "undo log: " + err;
                }
            }
            // block records: durable before durable(seq) returns (any mode but off); other deferred
            // records only in commit mode (the materialisers' group sync covers them otherwise)
            const bool want_sync = sync_ == SYNC_COMMIT || (sync_ != SYNC_OFF && job.block_id >= 0 && !job.group);
            if (job.group) ++group_records_;
            if (werr.empty() && err.empty() && want_sync) {
                try {
                    make_durable(seq);
                } catch (const std::exception&) {
                }
            }
            {
                std::lock_guard<std::mutex> g(io_mu_);
                --io_pending_;
                io_done_ = std::max(io_done_, seq);
            }
            io_done_cv_.notify_all();
        }
    }

    // Fault injection (tests): hold queued batches back from SQL.
    void set_paused(bool p) {
        {
            std::lock_guard<std::mutex> lk(mu_);
            paused_ = p;
        }
        cv_.notify_all();
        cv_done_.notify_all();
    }

    uint64_t applied(int shard) {
        std::lock_guard<std::mutex> lk(mu_);
        return applied_locked(shard);
    }

    // Block until every record with sequence <= seq is in the SQL tables of `shard` (-1: all files).
    void wait(uint64_t seq, int shard, double timeout_s) {
        std::unique_lock<std::mutex> lk(mu_);
        auto pred = [&] { return applied_locked(shard) >= seq || failed_; };
        if (timeout_s > 0) {
            if (!cv_done_.wait_for(lk, std::chrono::duration<double>(timeout_s), pred))
                throw std::runtime_error("ledger writer: timed out waiting for the SQL materialiser");
        } else {
            cv_done_.wait(lk, pred);
        }
        if (failed_ && applied_locked(shard) < seq) throw std::runtime_error("ledger writer failed: " + error_);
    }

    // Every record with sequence <= seq durable on disk (fdatasync'd journal prefix).
    void durable(uint64_t seq) {
        {
            // a deferred record: its I/O job (write, undo data, publication, fdatasync) has to be done
            std::unique_lock<std::mutex> g(io_mu_);
            io_done_cv_.wait(g, [&] { return io_pending_ == 0 || io_done_ >= seq; });
        }
        {
            std::lock_guard<std::mutex> lk(mu_);
            if (failed_ && next_pub_ <= seq) throw std::runtime_error("ledger writer failed: " + error_);
        }
        if (sync_ == SYNC_OFF) return;
        make_durable(seq);
        std::lock_guard<std::mutex> lk(mu_);
        if (failed_ && synced_.load() < seq) throw std::runtime_error("ledger writer failed: " + error_);
    }

    py::object journal_meta(int64_t block_id) {
        std::string out;
        if (!undo_.get(block_id, out)) return py::none();
        return py::bytes(out);
    }

    // Drop the undo data of blocks >= block_id (they were rolled back).
    void forget_blocks_from(int64_t block_id) { undo_.forget_from(block_id); }

    py::dict stats() {
        py::dict d;
        {
            std::lock_guard<std::mutex> jl(jmu_);
            std::lock_guard<std::mutex> lk(mu_);
            d["submitted"] = submitted_;
            d["applied"] = applied_locked(-1);
            size_t queued = 0, qbytes = 0;
            int64_t groups = 0, replayed = 0;
            double apply_s = 0, commit_s = 0, sync_s = 0;
            py::list per;
            for (auto& sh : shards_) {
                queued = std::max(queued, sh->queue.size());
                qbytes = std::max(qbytes, sh->queued_bytes);
                groups += sh->groups;
                replayed = std::max(replayed, sh->replayed);
                apply_s = std::max(apply_s, sh->apply_ns / 1e9);
                commit_s = std::max(commit_s, sh->commit_ns / 1e9);
                sync_s = std::max(sync_s, sh->sync_ns / 1e9);
                py::dict x;
                x["applied"] = sh->applied;
                x["groups"] = sh->groups;
                x["apply_s"] = sh->apply_ns / 1e9;
                x["commit_s"] = sh->commit_ns / 1e9;
                x["replayed"] = sh->replayed;
                x["queued"] = sh->queue.size();
                x["queued_bytes"] = sh->queued_bytes;
                per.append(x);
            }
            d["queued"] = queued;
            d["queued_bytes"] = qbytes;
            d["max_queue_bytes"] = max_queue_bytes_;
            d["throttle_waits"] = throttle_waits_;
            d["throttle_s"] = throttle_ns_ / 1e9;
            d["busy_retries"] = busy_retries_;
            d["groups"] = groups;
            d["journal_bytes"] = int64_t(journal_size_);
            d["bytes_written"] = bytes_written_;
            d["apply_s"] = apply_s;  // the slowest file
            d["commit_s"] = commit_s;
            d["sync_s"] = sync_s;
            d["replayed"] = replayed;
            d["rotations"] = rotations_;
            d["failed"] = failed_;
            d["error"] = error_;
            d["change_mismatches"] = mismatches_;
            d["sync_mode"] = sync_;
            d["synced"] = synced_.load();
            d["synced_bytes"] = synced_bytes_.load();
            d["fdatasyncs"] = syncs_.load();
            d["group_records"] = group_records_.load();
            d["fdatasync_s"] = sync_total_ns_.load() / 1e9;
            // the journal I/O thread's deferred records: wait in its queue, checksum, write, wait for the undo
            // record's writer (block records)
            d["io_records"] = io_records_.load();
            d["io_queue_s"] = io_queue_ns_.load() / 1e9;
            d["io_crc_s"] = io_crc_ns_.load() / 1e9;
            d["io_write_s"] = io_write_ns_.load() / 1e9;
            d["io_undo_wait_s"] = io_undo_wait_ns_.load() / 1e9;
            d["shards"] = per;
            py::dict st;
            for (auto& kv : stmt_stats_) st[py::str(kv.first)] = py::make_tuple(kv.second.first / 1e9, kv.second.second);
            d["statements"] = st;
        }
        undo_.fill_stats(d);
        return d;
    }

   private:
    uint64_t applied_locked(int shard) const {
        if (shard >= 0) return shards_.at(size_t(shard))->applied;
        uint64_t m = ~uint64_t(0);
        for (auto& sh : shards_) m = std::min(m, sh->applied);
        return m;
    }

    // caller holds mu_: queue every written record that continues the published prefix
    void publish_locked() {
        while (!written_.empty() && written_.begin()->first == next_pub_) {
            Batch b = std::move(written_.begin()->second);
            written_.erase(written_.begin());
            for (auto& sh : shards_) {
                sh->queue.push_back(b);
                sh->queued_bytes += b.size;
            }
            submitted_ = b.seq;
            pub_end_ = b.end;
            ++next_pub_;
        }
    }

    size_t max_queued_bytes_locked() const {
        size_t m = 0;
        for (auto& sh : shards_) m = std::max(m, sh->queued_bytes);
        return m;
    }

    void throttle() {
        if (max_queue_bytes_ <= 0) return;
        std::unique_lock<std::mutex> lk(mu_);
        auto ok = [&] { return max_queued_bytes_locked() < size_t(max_queue_bytes_) || failed_ || stop_ || paused_; };
        if (ok()) return;
        const auto t0 = std::chrono::steady_clock::now();
        ++throttle_waits_;
        cv_done_.wait_for(lk, std::chrono::duration<double>(throttle_timeout_s_), ok);
        throttle_ns_ += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
    }

    void make_durable(uint64_t seq) {
        {
            // the record and every lower one written (published), so one sync covers a contiguous prefix
            std::unique_lock<std::mutex> lk(mu_);
            cv_done_.wait(lk, [&] { return next_pub_ > seq || failed_ || stop_; });
        }
        ensure_synced(seq);
    }

    void ensure_synced(uint64_t seq) {
        if (synced_.load() >= seq) return;
        std::lock_guard<std::mutex> sl(sync_mu_);
        if (synced_.load() >= seq) return;
        uint64_t upto;
        off_t upto_end;
        {
            std::lock_guard<std::mutex> lk(mu_);
            upto = next_pub_ - 1;
            upto_end = pub_end_;
        }
        const auto t0 = std::chrono::steady_clock::now();
        ::fdatasync(fd_);
        sync_total_ns_ += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
        ++syncs_;
        if (upto > synced_.load()) {
            synced_.store(upto);
            synced_bytes_.store(int64_t(upto_end));
        }
    }

    void open_shard(Shard& sh, int64_t cache_mb) {
        const SqliteApi& a = api();
        int rc = a.open_v2(sh.path.c_str(), &sh.db,
                           SQLITE_OPEN_READWRITE | SQLITE_OPEN_CREATE | SQLITE_OPEN_NOMUTEX | SQLITE_OPEN_URI, nullptr);
        if (rc != SQLITE_OK) {
            std::string m = sh.db ? a.errmsg(sh.db) : "open failed";
            if (sh.db) a.close_v2(sh.db);
            sh.db = nullptr;
            throw std::runtime_error("ledger writer: cannot open " + sh.path + ": " + m);
        }
        // short per-attempt wait: a group that still finds the file locked is retried (run()), so a long
        // Python-side transaction delays materialisation but never stops the writer
        a.busy_timeout(sh.db, busy_timeout_ms_);
        // the journal is the durability point: SQL commits never need to reach the disk on their own
        exec(sh.db, "PRAGMA journal_mode = WAL");
        exec(sh.db, "PRAGMA synchronous = OFF");
        exec(sh.db, "PRAGMA foreign_keys = OFF");
        exec(sh.db, "PRAGMA secure_delete = OFF");  // the distribution build defaults to zero-filling freed cells
        exec(sh.db, "PRAGMA cache_size = -" + std::to_string(std::max<int64_t>(16, cache_mb) * 1024));
        // memory-mapped reads (UPOW_SQLITE_MMAP_MB): B-tree pages a materialiser misses in its page cache
        // are read from the mapping instead of copied out of the OS page cache
        if (const char* mm = std::getenv("UPOW_SQLITE_MMAP_MB"))
            exec(sh.db, "PRAGMA mmap_size = " + std::to_string(std::max<int64_t>(0, std::atoll(mm)) << 20));
        exec(sh.db, "PRAGMA wal_autocheckpoint = 0");
        exec(sh.db, "CREATE TABLE IF NOT EXISTS upow_journal_state (k INTEGER PRIMARY KEY CHECK (k = 0), seq INTEGER NOT NULL)");
        exec(sh.db, "INSERT OR IGNORE INTO upow_journal_state (k, seq) VALUES (0, 0)");
        sh.applied = uint64_t(query_int(sh.db, "SELECT seq FROM upow_journal_state WHERE k = 0"));
    }

    static void exec(sqlite3* db, const std::string& sql) {
        char* err = nullptr;
        int rc = api().exec(db, sql.c_str(), nullptr, nullptr, &err);
        if (rc != SQLITE_OK) {
            std::string m = err ? err : api().errmsg(db);
            if (err) api().free(err);
            throw SqlError("ledger writer: " + m + " [" + sql.substr(0, 120) + "]", rc);
        }
    }

    static void rollback(sqlite3* db) {
        char* e = nullptr;
        api().exec(db, "ROLLBACK", nullptr, nullptr, &e);
        if (e) api().free(e);
    }

    static int64_t query_int(sqlite3* db, const std::string& sql) {
        const SqliteApi& a = api();
        sqlite3_stmt* st = nullptr;
        int rc = a.prepare_v2(db, sql.c_str(), int(sql.size()), &st, nullptr);
        if (rc != SQLITE_OK) throw SqlError(std::string("ledger writer: ") + a.errmsg(db), rc);
        int64_t v = 0;
        rc = a.step(st);
        if (rc == SQLITE_ROW) v = a.column_int64(st, 0);
        a.finalize(st);
        if (rc != SQLITE_ROW && rc != SQLITE_DONE) throw SqlError(std::string("ledger writer: ") + a.errmsg(db), rc);
        return v;
    }

    static sqlite3_stmt* prepared(Shard& sh, const std::string& sql) {
        auto it = sh.stmts.find(sql);
        if (it != sh.stmts.end()) return it->second;
        sqlite3_stmt* st = nullptr;
        int rc = api().prepare_v2(sh.db, sql.c_str(), int(sql.size()), &st, nullptr);
        if (rc != SQLITE_OK) throw SqlError(std::string("ledger writer: ") + api().errmsg(sh.db) + " [" + sql + "]", rc);
        if (sh.stmts.size() > 256) {
            for (auto& kv : sh.stmts) api().finalize(kv.second);
            sh.stmts.clear();
        }
        sh.stmts[sql] = st;
        return st;
    }

    // Apply the statements of one encoded batch that belong to `shard`, inside its open transaction.
    void apply_batch(size_t shard, const std::vector<Part>& parts, bool strict) {
        const SqliteApi& a = api();
        Shard& sh = *shards_[shard];
        if (parts.empty()) throw std::runtime_error("ledger batch: empty");
        size_t pi = 0;
        In in{parts[0]->data(), parts[0]->data() + parts[0]->size()};
        const uint32_t ns = in.get<uint32_t>();
        for (uint32_t s = 0; s < ns; ++s) {
            while (in.p == in.e && pi + 1 < parts.size()) {  // the next statement starts the next part
                ++pi;
                in = In{parts[pi]->data(), parts[pi]->data() + parts[pi]->size()};
            }
            const std::string sql = in.str();
            const uint32_t flags = in.get<uint32_t>();
            std::string guard;
            int64_t expect = -1;
            if (flags & 1) guard = in.str();
            if (flags & 2) expect = in.get<int64_t>();
            const size_t target = (flags >> 8) & 0xffu;
            const int64_t n = in.get<int64_t>();
            const uint32_t nc = in.get<uint32_t>();
            std::vector<ColView> cols(nc);
            for (auto& c : cols) {
                c.kind = in.get<uint8_t>();
                switch (c.kind) {
                    case K_NULL: break;
                    case K_CTEXT: c.ctext = in.str(); break;
                    case K_CINT: c.cint = in.get<int64_t>(); break;
                    case K_INT64: c.data = in.take(size_t(n) * 8); break;
                    case K_HEX32: c.data = in.take(size_t(n) * 32); break;
                    case K_TEXT:
                    case K_HEXTEXT: {
                        const uint8_t has_null = c.kind == K_TEXT ? in.get<uint8_t>() : 0;
                        if (has_null) c.nul = reinterpret_cast<const uint8_t*>(in.take(size_t(n)));
                        c.off = in.take(size_t(n + 1) * 8);
                        const int64_t blen = ld64(c.off + 8 * n);
                        c.data = in.take(size_t(blen));
                        break;
                    }
                    default: throw std::runtime_error("ledger batch: bad column kind");
                }
            }
            const char* order = nullptr;
            const uint8_t order_kind = in.get<uint8_t>();
            if (order_kind == 1) order = in.take(size_t(n) * 8);
            const size_t route = (flags & 4) ? ((flags >> 16) & 0xffu) : 1;
            if (target + route > shards_.size()) throw std::runtime_error("ledger batch: statement for an unknown file");
            if (shard < target || shard >= target + route) continue;
            std::vector<int64_t> key_order;
            if (order_kind == 2) {
                if (nc == 0 || cols[0].kind != K_HEX32) throw std::runtime_error("ledger batch: key order needs hex32 column 0");
                std::vector<std::pair<uint64_t, int64_t>> kv{static_cast<size_t>(n)};
                for (int64_t r = 0; r < n; ++r) {
                    uint64_t k = 0;
                    for (int b = 0; b < 8; ++b) k = (k << 8) | uint8_t(cols[0].data[32 * r + b]);
                    kv[size_t(r)] = {k, r};
                }
                std::sort(kv.begin(), kv.end());  // (key, row): equal keys keep row order
                key_order.resize(size_t(n));
                for (int64_t r = 0; r < n; ++r) key_order[size_t(r)] = kv[size_t(r)].second;
                order = reinterpret_cast<const char*>(key_order.data());
            }
            if (!guard.empty() && query_int(sh.db, guard) == 0) continue;
            // routed statement: which rows belong to this file (first byte of the column-0 tx hash)
            std::vector<uint8_t> mine;
            if (route > 1) {
                if (nc == 0) throw std::runtime_error("ledger batch: routed statement without columns");
                mine.assign(size_t(n), 0);
                int64_t cnt = 0;
                for (int64_t r = 0; r < n; ++r) {
                    const uint32_t b = route_byte(cols[0], r);
                    mine[size_t(r)] = uint8_t((b * route) >> 8) == uint8_t(shard - target);
                    cnt += mine[size_t(r)];
                }
                if (expect == n) expect = cnt;  // "every row changes" holds per file
            }
            const auto ts0 = std::chrono::steady_clock::now();
            sqlite3_stmt* st = prepared(sh, sql);
            int64_t changes = 0;
            char hexbuf[8][64];
            std::vector<std::string> hextext(nc);  // rendered K_HEXTEXT values (bound as static text)
            for (int64_t k = 0; k < n; ++k) {
                const int64_t r = order ? ld64(order + 8 * k) : k;
                if (!mine.empty() && !mine[size_t(r)]) continue;
                int hb = 0;
                for (uint32_t j = 0; j < nc; ++j) {
                    const ColView& c = cols[j];
                    const int p = int(j) + 1;
                    switch (c.kind) {
                        case K_NULL: a.bind_null(st, p); break;
                        case K_CTEXT: a.bind_text(st, p, c.ctext.data(), int(c.ctext.size()), nullptr); break;
                        case K_CINT: a.bind_int64(st, p, c.cint); break;
                        case K_INT64: a.bind_int64(st, p, ld64(c.data + 8 * r)); break;
                        case K_HEX32: {
                            if (hb >= 8) throw std::runtime_error("at most 8 hex32 columns");
                            char* out = hexbuf[hb++];
                            const uint8_t* src = reinterpret_cast<const uint8_t*>(c.data) + 32 * r;
                            for (int b = 0; b < 32; ++b) {
                                out[2 * b] = kHex[src[b] >> 4];
                                out[2 * b + 1] = kHex[src[b] & 15];
                            }
                            a.bind_text(st, p, out, 64, nullptr);
                            break;
                        }
                        case K_HEXTEXT: {
                            const int64_t o0 = ld64(c.off + 8 * r), o1 = ld64(c.off + 8 * (r + 1));
                            std::string& h = hextext[j];
                            h.resize(size_t(2 * (o1 - o0)));
                            const uint8_t* src = reinterpret_cast<const uint8_t*>(c.data) + o0;
                            for (int64_t b = 0; b < o1 - o0; ++b) {
                                h[size_t(2 * b)] = kHex[src[b] >> 4];
                                h[size_t(2 * b + 1)] = kHex[src[b] & 15];
                            }
                            a.bind_text(st, p, h.data(), int(h.size()), nullptr);
                            break;
                        }
                        case K_TEXT: {
                            if (c.nul && c.nul[r]) {
                                a.bind_null(st, p);
                            } else {
                                const int64_t o0 = ld64(c.off + 8 * r), o1 = ld64(c.off + 8 * (r + 1));
                                a.bind_text(st, p, c.data + o0, int(o1 - o0), nullptr);
                            }
                            break;
                        }
                    }
                }
                int rc = a.step(st);
                if (rc != SQLITE_DONE && rc != SQLITE_ROW) {
                    std::string m = a.errmsg(sh.db);
                    a.reset(st);
                    throw SqlError("ledger writer: " + m + " [" + sql.substr(0, 120) + "]", rc);
                }
                changes += a.changes(sh.db);
                a.reset(st);
            }
            a.clear_bindings(st);
            const int64_t ns_used =
                std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - ts0).count();
            std::lock_guard<std::mutex> lk(mu_);
            auto& acc = stmt_stats_[sql.substr(0, 48)];
            acc.first += ns_used;
            acc.second += n;
            if (expect >= 0 && changes != expect) {
                ++mismatches_;
                // the journaled block said every one of these rows exists (validated against the HBM
                // index): SQL and the index have diverged. Stop before materialising anything further.
                if (strict)
                    throw MismatchError("ledger writer: " + std::to_string(changes) + " of " + std::to_string(expect) +
                                        " rows changed [" + sql.substr(0, 120) + "]");
            }
        }
    }

    // Start-up: re-apply, per file, every intact record above that file's recorded sequence; cut off a
    // torn tail record.
    void recover() {
        off_t at = 0;
        const off_t end = ::lseek(fd_, 0, SEEK_END);
        std::vector<std::pair<uint64_t, std::vector<Part>>> records;
        uint64_t max_seq = 0;
        uint64_t min_applied = ~uint64_t(0);
        for (auto& sh : shards_) {
            max_seq = std::max(max_seq, sh->applied);
            min_applied = std::min(min_applied, sh->applied);
        }
        while (at + off_t(sizeof(RecHeader)) <= end) {
            RecHeader h;
            if (!read_exact(fd_, reinterpret_cast<char*>(&h), sizeof h, at) || h.magic != kMagic) break;
            const off_t body = at + off_t(sizeof h);
            if (h.meta_len > uint64_t(end) || h.payload_len > uint64_t(end) ||
                body + off_t(h.meta_len + h.payload_len) > end)
                break;
            std::string meta(h.meta_len, '\0');
            auto payload = std::make_shared<std::string>(h.payload_len, '\0');
            if (!read_exact(fd_, meta.data(), meta.size(), body) ||
                !read_exact(fd_, payload->data(), payload->size(), body + off_t(h.meta_len)))
                break;
            if (record_crc(h, meta.data(), payload->data()) != h.crc) break;
            if (h.seq > min_applied) records.emplace_back(h.seq, std::vector<Part>{payload});
            max_seq = std::max<uint64_t>(max_seq, h.seq);
            at = body + off_t(h.meta_len + h.payload_len);
        }
        if (at != end) {
            if (::ftruncate(fd_, at) != 0) throw std::runtime_error("journal truncate failed");
            ::fdatasync(fd_);
        }
        journal_size_ = at;
        ::lseek(fd_, at, SEEK_SET);
        next_seq_ = max_seq + 1;
        next_pub_ = next_seq_;
        pub_end_ = at;
        synced_.store(max_seq);
        synced_bytes_.store(int64_t(at));
        for (size_t i = 0; i < shards_.size(); ++i) {
            Shard& sh = *shards_[i];
            uint64_t last = 0;
            int64_t n = 0;
            exec(sh.db, "BEGIN IMMEDIATE");
            try {
                for (auto& r : records) {
                    if (r.first <= sh.applied) continue;
                    apply_batch(i, r.second, false);
                    last = r.first;
                    ++n;
                }
                if (n) exec(sh.db, "UPDATE upow_journal_state SET seq = " + std::to_string(last) + " WHERE k = 0");
                exec(sh.db, "COMMIT");
            } catch (...) {
                rollback(sh.db);
                throw;
            }
            if (n) sh.applied = last;
            sh.replayed = n;
        }
        submitted_ = applied_locked(-1);
        for (auto& sh : shards_) submitted_ = std::max(submitted_, sh->applied);
    }

    void maybe_rotate() {
        // every record is in every file: make the SQL side durable, then start an empty journal
        std::lock_guard<std::mutex> jl(jmu_);
        if (inflight_ != 0) return;  // a reserved record is still being written
        {
            std::lock_guard<std::mutex> lk(mu_);
            if (!written_.empty()) return;
            for (auto& sh : shards_)
                if (!sh->queue.empty() || sh->applied != submitted_) return;
        }
        if (journal_max_ <= 0 || journal_size_ < journal_max_) return;
        for (auto& sh : shards_) {
            exec(sh->db, "PRAGMA synchronous = FULL");
            exec(sh->db, "UPDATE upow_journal_state SET seq = seq WHERE k = 0");
            exec(sh->db, "PRAGMA wal_checkpoint(PASSIVE)");
            exec(sh->db, "PRAGMA synchronous = OFF");
        }
        if (::ftruncate(fd_, 0) != 0) throw std::runtime_error("journal truncate failed");
        ::fdatasync(fd_);
        ::lseek(fd_, 0, SEEK_SET);
        journal_size_ = 0;
        {
            std::lock_guard<std::mutex> lk(mu_);
            pub_end_ = 0;
        }
        synced_bytes_.store(0);
        ++rotations_;  // the undo log is separate: rollback keeps working across rotations
    }

    void run(size_t i) {
        Shard& sh = *shards_[i];
        pthread_setname_np(pthread_self(), ("upow-wr-" + std::to_string(i)).c_str());
        // materialising is background work: below the block path and the HTTP loop in the CPU share the
        // process gets (GPU boxes run a node under a CPU quota far below the core count). Ten materialisers
        // keep ~10 cores busy behind a stream of 2 MB blocks; at nice 19 (CFS weight 15 against the block
        // path's 1024) they take what the block path leaves: the verify bench ran at 732-820 k tx/s against
        // 638-730 k at nice 5 in three interleaved pairs on one box (profiles/r6/writer_nice/). The writer's
        // queue bound (UPOW_WRITER_MAX_QUEUE_MB) still holds blocks back if they fall too far behind.
        int nice_level = 19;
        if (const char* nv = std::getenv("UPOW_WRITER_NICE")) nice_level = std::atoi(nv);
        if (nice_level > 0) setpriority(PRIO_PROCESS, pid_t(syscall(SYS_gettid)), std::min(nice_level, 19));
        for (;;) {
            std::vector<Batch> group;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_ || (!sh.queue.empty() && !failed_ && !paused_); });
                if (sh.queue.empty() || failed_) {
                    if (stop_) return;
                    continue;
                }
                if (paused_ && !stop_) continue;
                while (!sh.queue.empty() && int(group.size()) < group_max_) {
                    group.push_back(std::move(sh.queue.front()));
                    sh.queue.pop_front();
                }
            }
            auto t0 = std::chrono::steady_clock::now();
            try {
                // no SQL file may get ahead of the durable journal prefix: every materialiser makes sure the
                // group's records are synced (one fdatasync serves all files; free when already synced)
                if (sync_ != SYNC_OFF) ensure_synced(group.back().seq);
                auto t1 = std::chrono::steady_clock::now();
                std::chrono::steady_clock::time_point t2;
                for (int attempt = 0;; ++attempt) {
                    try {
                        exec(sh.db, "BEGIN IMMEDIATE");
                        try {
                            for (auto& b : group) apply_batch(i, b.parts, true);
                            exec(sh.db, "UPDATE upow_journal_state SET seq = " + std::to_string(group.back().seq) +
                                            " WHERE k = 0");
                            t2 = std::chrono::steady_clock::now();
                            exec(sh.db, "COMMIT");
                        } catch (...) {
                            rollback(sh.db);
                            throw;
                        }
                        break;
                    } catch (const SqlError& e) {
                        // another connection holds the file's write lock (a long Python-side transaction):
                        // back off and retry the whole group instead of stopping the ledger
                        const int rc = e.rc & 0xff;
                        bool stopping;
                        {
                            std::lock_guard<std::mutex> lk(mu_);
                            stopping = stop_;
                            if (rc == SQLITE_BUSY || rc == SQLITE_LOCKED) ++busy_retries_;
                        }
                        if ((rc != SQLITE_BUSY && rc != SQLITE_LOCKED) || stopping) throw;
                        std::this_thread::sleep_for(std::chrono::milliseconds(std::min(1000, 5 << std::min(attempt, 8))));
                    }
                }
                auto t3 = std::chrono::steady_clock::now();
                {
                    std::lock_guard<std::mutex> lk(mu_);
                    sh.applied = group.back().seq;
                    for (auto& b : group) sh.queued_bytes -= b.size;
                    ++sh.groups;
                    sh.sync_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count();
                    sh.apply_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(t2 - t1).count();
                    sh.commit_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(t3 - t2).count();
                }
                cv_done_.notify_all();
                maybe_rotate();
            } catch (const std::exception& e) {
                {
                    std::lock_guard<std::mutex> lk(mu_);
                    failed_ = true;
                    error_ = sh.path + ": " + e.what();
                }
                cv_done_.notify_all();
                cv_.notify_all();
            }
        }
    }

    std::string journal_path_;
    int sync_;
    int group_max_;
    int64_t journal_max_;
    std::vector<std::unique_ptr<Shard>> shards_;
    int64_t max_queue_bytes_;
    double throttle_timeout_s_;
    int busy_timeout_ms_;
    UndoLog undo_;
    int fd_ = -1;
    off_t journal_size_ = 0;
    std::mutex jmu_;  // reservations: next_seq_, journal_size_, inflight_
    uint64_t next_seq_ = 1;
    int64_t inflight_ = 0;  // reserved records not yet written
    int64_t bytes_written_ = 0;
    std::mutex mu_;  // publication, queues, watermarks, statistics
    std::condition_variable cv_, cv_done_;
    std::map<uint64_t, Batch> written_;  // written but not yet published (a lower record still in flight)
    uint64_t next_pub_ = 1;
    off_t pub_end_ = 0;       // journal offset past the last published record
    uint64_t submitted_ = 0;  // last published sequence
    bool stop_ = false, closed_ = false, failed_ = false, paused_ = false;
    std::string error_;
    int64_t rotations_ = 0, mismatches_ = 0, busy_retries_ = 0, throttle_waits_ = 0, throttle_ns_ = 0;
    std::mutex sync_mu_;
    std::atomic<uint64_t> synced_{0};
    std::atomic<int64_t> synced_bytes_{0};
    std::atomic<int64_t> syncs_{0}, sync_total_ns_{0}, group_records_{0};
    // UPOW_JOURNAL_EARLY_WRITEBACK=0: block records written without starting their writeback slice by slice
    const bool early_writeback_ = [] {
        const char* v = std::getenv("UPOW_JOURNAL_EARLY_WRITEBACK");
        return !(v && std::string(v) == "0");
    }();
    std::atomic<int64_t> io_records_{0}, io_queue_ns_{0}, io_crc_ns_{0}, io_write_ns_{0}, io_undo_wait_ns_{0};
    std::map<std::string, std::pair<int64_t, int64_t>> stmt_stats_;  // sql prefix -> (ns, rows)
    // journal I/O thread (deferred block records)
    std::mutex io_mu_;
    std::condition_variable io_cv_, io_done_cv_;
    std::deque<IoJob> io_q_;
    int64_t io_pending_ = 0;
    uint64_t io_done_ = 0;
    bool io_stop_ = false;
    std::thread io_thread_;
};

}  // namespace

void register_ledger_writer(py::module_& m) {
    static const int memstatus_rc = sqlite_disable_memstatus();
    m.attr("sqlite_memstatus_config_rc") = memstatus_rc;
    py::class_<EncodedStmt>(m, "EncodedStmt")
        .def("__len__", [](const EncodedStmt& e) { return e.buf->size(); })
        .def("tobytes", [](const EncodedStmt& e) { return py::bytes(*e.buf); });
    m.def("ledger_encode_stmt", &encode_stmt, py::arg("sql"), py::arg("cols"), py::arg("n"),
          py::arg("order") = py::none(), py::arg("guard") = py::none(), py::arg("expect") = py::none(),
          py::arg("shard") = 0, py::arg("route") = 1, "encode one column-major bulk statement for LedgerWriter.submit");
    m.def("crc32c", [](py::buffer b) {
        py::buffer_info bi = b.request();
        return crc32c(0, bi.ptr, size_t(bi.size * bi.itemsize));
    });
    py::class_<LedgerWriter>(m, "LedgerWriter")
        .def(py::init([](std::vector<std::string> dbs, const std::string& journal, int sync, int64_t cache_mb,
                         int group_max, int64_t journal_max, int64_t undo_keep, int64_t max_queue_bytes,
                         double throttle_timeout_s, int busy_timeout_ms) {
                 py::gil_scoped_release nogil;
                 return new LedgerWriter(dbs, journal, sync, cache_mb, group_max, journal_max, undo_keep,
                                         max_queue_bytes, throttle_timeout_s, busy_timeout_ms);
             }),
             py::arg("db_paths"), py::arg("journal_path"), py::arg("sync_mode") = 1, py::arg("cache_mb") = 256,
             py::arg("group_max") = 8, py::arg("journal_max_bytes") = int64_t(1) << 30, py::arg("undo_keep") = 600,
             py::arg("max_queue_bytes") = int64_t(512) << 20, py::arg("throttle_timeout_s") = 300.0,
             py::arg("busy_timeout_ms") = 5000)
        .def("submit",
             [](LedgerWriter& w, py::list stmts, py::object meta, int64_t block_id, bool sync, bool group) {
                 // encoded statements are taken as they are (shared buffers); plain bytes are copied
                 std::vector<Part> v;
                 v.reserve(stmts.size());
                 for (auto x : stmts) {
                     if (py::isinstance<EncodedStmt>(x)) {
                         v.push_back(x.cast<const EncodedStmt&>().buf);
                     } else if (PyBytes_Check(x.ptr())) {
                         v.push_back(std::make_shared<const std::string>(PyBytes_AS_STRING(x.ptr()),
                                                                         size_t(PyBytes_GET_SIZE(x.ptr()))));
                     } else {
                         throw std::invalid_argument("statements must be encoded statements or bytes");
                     }
                 }
                 // meta (the block's undo data): bytes, or a list of buffers joined here in one copy
                 std::vector<std::pair<const char*, size_t>> mparts;
                 std::vector<py::buffer_info> keep;
                 if (py::isinstance<py::list>(meta)) {
                     for (auto x : meta.cast<py::list>()) {
                         keep.push_back(x.cast<py::buffer>().request());
                         mparts.emplace_back(static_cast<const char*>(keep.back().ptr),
                                             size_t(keep.back().size * keep.back().itemsize));
                     }
                 } else {
                     keep.push_back(meta.cast<py::buffer>().request());
                     mparts.emplace_back(static_cast<const char*>(keep.back().ptr),
                                         size_t(keep.back().size * keep.back().itemsize));
                 }
                 size_t total = 0;
                 for (auto& pr : mparts) total += pr.second;
                 // a write-behind mempool record only reserves a sequence number and queues: keep the GIL
                 // (see NoGilIfLarge); a block record may wait for writer backpressure and a synced one
                 // for its write, both without the GIL
                 std::optional<py::gil_scoped_release> nogil;
                 if (sync || block_id >= 0 || total >= (size_t(1) << 16)) nogil.emplace();
                 std::string m;
                 m.reserve(total);
                 for (auto& pr : mparts) m.append(pr.first, pr.second);
                 return w.submit(std::move(v), std::move(m), block_id, sync, group);
             },
             py::arg("stmts"), py::arg("meta") = py::bytes(""), py::arg("block_id") = -1, py::arg("sync") = true,
             py::arg("group") = false)
        .def("applied", &LedgerWriter::applied, py::arg("shard") = -1)
        .def("set_paused", &LedgerWriter::set_paused)
        .def("wait", &LedgerWriter::wait, py::arg("seq"), py::arg("shard") = -1, py::arg("timeout_s") = 0.0,
             py::call_guard<py::gil_scoped_release>())
        .def("durable", &LedgerWriter::durable, py::arg("seq"), py::call_guard<py::gil_scoped_release>())
        .def("journal_meta", &LedgerWriter::journal_meta)
        .def("forget_blocks_from", &LedgerWriter::forget_blocks_from)
        .def("stats", &LedgerWriter::stats)
        .def("close", &LedgerWriter::close, py::call_guard<py::gil_scoped_release>());
}

}  // namespace upow
