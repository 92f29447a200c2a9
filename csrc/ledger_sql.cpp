// Native bulk ledger writes: column-major `executemany` on the ledger's own SQLite connection.
//
// reference: the block-apply writes of upow/database.py (add_transactions 236-252,
// add_transaction_outputs 524-580, remove_outputs 589-621, remove_pending_transactions_by_hash) —
// asyncpg row-by-row INSERT/DELETE against PostgreSQL. Here the embedded ledger (SQLite, schema.sql
// layout) is written from whole-block arrays: Python's sqlite3.executemany needs one tuple of Python
// objects per row and re-binds every parameter through the object layer; this binds straight from
// the block codec's buffers (64-hex tx hashes rendered from raw 32-byte digests, int64 columns from
// numpy arrays, text columns from the codec's string lists) and steps one prepared statement with
// the GIL released.
//
// The statements run on the SAME sqlite3* handle as the Python connection (so they are part of the
// block's single BEGIN ... COMMIT transaction, and ':memory:' ledgers work): the handle is read from
// the CPython 3.10 `pysqlite_Connection` object (first field after PyObject_HEAD) and validated by
// Database (filename + total_changes must match what the Python connection reports) before use.
// libsqlite3 is resolved with dlopen(RTLD_NOLOAD) from the copy _sqlite3 already loaded, so both
// sides use the same library instance.
#include <dlfcn.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <numeric>
#include <stdexcept>
#include <string>
#include <vector>

namespace py = pybind11;

namespace upow {
namespace {

struct sqlite3;
struct sqlite3_stmt;
typedef void (*destructor_t)(void*);
constexpr int SQLITE_OK = 0, SQLITE_ROW = 100, SQLITE_DONE = 101, SQLITE_CONSTRAINT = 19;

struct SqliteApi {
    int (*prepare_v2)(sqlite3*, const char*, int, sqlite3_stmt**, const char**) = nullptr;
    int (*bind_text)(sqlite3_stmt*, int, const char*, int, destructor_t) = nullptr;
    int (*bind_int64)(sqlite3_stmt*, int, long long) = nullptr;
    int (*bind_null)(sqlite3_stmt*, int) = nullptr;
    int (*step)(sqlite3_stmt*) = nullptr;
    int (*reset)(sqlite3_stmt*) = nullptr;
    int (*finalize)(sqlite3_stmt*) = nullptr;
    int (*changes)(sqlite3*) = nullptr;
    int (*total_changes)(sqlite3*) = nullptr;
    int (*get_autocommit)(sqlite3*) = nullptr;
    const char* (*errmsg)(sqlite3*) = nullptr;
    const char* (*db_filename)(sqlite3*, const char*) = nullptr;
    bool ok = false;
};

const SqliteApi& api() {
    static SqliteApi a = [] {
        SqliteApi s;
        void* h = dlopen("libsqlite3.so.0", RTLD_NOW | RTLD_NOLOAD);
        if (!h) h = dlopen("libsqlite3.so.0", RTLD_NOW);
        if (!h) return s;
        auto sym = [&](auto& fn, const char* name) { fn = reinterpret_cast<std::decay_t<decltype(fn)>>(dlsym(h, name)); };
        sym(s.prepare_v2, "sqlite3_prepare_v2");
        sym(s.bind_text, "sqlite3_bind_text");
        sym(s.bind_int64, "sqlite3_bind_int64");
        sym(s.bind_null, "sqlite3_bind_null");
        sym(s.step, "sqlite3_step");
        sym(s.reset, "sqlite3_reset");
        sym(s.finalize, "sqlite3_finalize");
        sym(s.changes, "sqlite3_changes");
        sym(s.total_changes, "sqlite3_total_changes");
        sym(s.get_autocommit, "sqlite3_get_autocommit");
        sym(s.errmsg, "sqlite3_errmsg");
        sym(s.db_filename, "sqlite3_db_filename");
        s.ok = s.prepare_v2 && s.bind_text && s.bind_int64 && s.bind_null && s.step && s.reset && s.finalize &&
               s.changes && s.total_changes && s.get_autocommit && s.errmsg && s.db_filename;
        return s;
    }();
    if (!a.ok) throw std::runtime_error("libsqlite3.so.0 not available for the native ledger writer");
    return a;
}

sqlite3* handle_of(py::handle conn) {
    // only ever reinterpret a real sqlite3.Connection (or a subclass of it)
    static PyObject* conn_type = py::module_::import("sqlite3").attr("Connection").ptr();
    if (PyObject_IsInstance(conn.ptr(), conn_type) != 1) throw py::type_error("expected a sqlite3.Connection");
    // CPython 3.10 Modules/_sqlite/connection.h: struct { PyObject_HEAD; sqlite3 *db; ... }
    sqlite3* db = *reinterpret_cast<sqlite3**>(reinterpret_cast<char*>(conn.ptr()) + sizeof(PyObject));
    if (!db) throw std::runtime_error("sqlite3 connection is closed");
    return db;
}

// One bound column of a bulk statement.
struct Col {
    enum Kind { TEXT_LIST, GATHER, HEX32, INT64, CONST_TEXT, CONST_INT, NUL, ARENA } kind = NUL;
    std::vector<const char*> ptr;  // TEXT_LIST / GATHER: UTF-8 views (nullptr = NULL)
    std::vector<int> len;
    const int32_t* idx = nullptr;  // GATHER
    int64_t idx_n = 0;
    const uint8_t* raw = nullptr;  // HEX32
    int64_t stride = 0, offset = 0, raw_n = 0;
    const char* blob = nullptr;     // ARENA: concatenated text + offsets[n + 1]
    const int64_t* aoff = nullptr;
    const int64_t* ival = nullptr;  // INT64
    int64_t ival_n = 0;
    std::string ctext;
    long long cint = 0;
};

void utf8_list(py::list lst, Col& c) {
    const size_t n = lst.size();
    c.ptr.resize(n);
    c.len.resize(n);
    for (size_t i = 0; i < n; ++i) {
        PyObject* o = PyList_GET_ITEM(lst.ptr(), i);
        if (o == Py_None) {
            c.ptr[i] = nullptr;
            c.len[i] = 0;
            continue;
        }
        Py_ssize_t sz = 0;
        const char* s = PyUnicode_AsUTF8AndSize(o, &sz);
        if (!s) throw py::error_already_set();
        c.ptr[i] = s;
        c.len[i] = int(sz);
    }
}

// Column specs (Python side):
//   list[str|None]                   text per row
//   ('gather', list[str], int32 buf)  text list[idx[row]]
//   ('hex32', buf, stride, offset)    lowercase hex of the 32 bytes at row*stride+offset
//   ('arena', blob, int64 offsets)    text blob[off[row]:off[row+1]] (csrc/txcodec.cpp text arenas)
//   int64 numpy array                 integer per row
//   str / int / None                  the same value for every row
Col parse_col(py::handle spec, int64_t n) {
    Col c;
    if (spec.is_none()) {
        c.kind = Col::NUL;
    } else if (py::isinstance<py::str>(spec)) {
        c.kind = Col::CONST_TEXT;
        c.ctext = spec.cast<std::string>();
    } else if (py::isinstance<py::int_>(spec)) {
        c.kind = Col::CONST_INT;
        c.cint = spec.cast<long long>();
    } else if (py::isinstance<py::list>(spec)) {
        c.kind = Col::TEXT_LIST;
        utf8_list(spec.cast<py::list>(), c);
        if (int64_t(c.ptr.size()) != n) throw std::invalid_argument("text column length != n");
    } else if (py::isinstance<py::tuple>(spec)) {
        py::tuple t = spec.cast<py::tuple>();
        const std::string tag = t[0].cast<std::string>();
        if (tag == "gather") {
            c.kind = Col::GATHER;
            utf8_list(t[1].cast<py::list>(), c);
            py::buffer_info bi = t[2].cast<py::buffer>().request();
            if (bi.itemsize != 4) throw std::invalid_argument("gather index must be int32");
            c.idx = static_cast<const int32_t*>(bi.ptr);
            c.idx_n = bi.size;
            if (c.idx_n != n) throw std::invalid_argument("gather index length != n");
            for (int64_t i = 0; i < n; ++i)
                if (c.idx[i] < 0 || size_t(c.idx[i]) >= c.ptr.size()) throw std::out_of_range("gather index");
        } else if (tag == "hex32") {
            c.kind = Col::HEX32;
            py::buffer_info bi = t[1].cast<py::buffer>().request();
            c.raw = static_cast<const uint8_t*>(bi.ptr);
            c.raw_n = bi.size * bi.itemsize;
            c.stride = t[2].cast<int64_t>();
            c.offset = t[3].cast<int64_t>();
            if (n > 0 && ((n - 1) * c.stride + c.offset + 32 > c.raw_n || c.offset < 0 || c.stride < 0))
                throw std::out_of_range("hex32 column out of range");
        } else if (tag == "arena") {
            c.kind = Col::ARENA;
            py::buffer_info bb = t[1].cast<py::buffer>().request(), ob = t[2].cast<py::buffer>().request();
            // offsets arrive as raw bytes (txcodec) or an int64 array: only the byte size is checked
            if (ob.size * ob.itemsize != 8 * (n + 1)) throw std::invalid_argument("arena offsets must be int64[n + 1]");
            c.blob = static_cast<const char*>(bb.ptr);
            c.aoff = static_cast<const int64_t*>(ob.ptr);
            const int64_t blen = bb.size * bb.itemsize;
            for (int64_t i = 0; i < n; ++i)
                if (c.aoff[i] < 0 || c.aoff[i + 1] < c.aoff[i] || c.aoff[i + 1] > blen)
                    throw std::out_of_range("arena offsets");
        } else {
            throw std::invalid_argument("unknown column tag " + tag);
        }
    } else {
        py::buffer_info bi = spec.cast<py::buffer>().request();
        if (bi.itemsize != 8 || bi.format.find_first_of("qlQL") == std::string::npos)
            throw std::invalid_argument("integer column must be int64");
        c.kind = Col::INT64;
        c.ival = static_cast<const int64_t*>(bi.ptr);
        c.ival_n = bi.size;
        if (c.ival_n != n) throw std::invalid_argument("int column length != n");
    }
    return c;
}

const char kHex[] = "0123456789abcdef";

[[noreturn]] void raise_sql(const SqliteApi& a, sqlite3* db, int rc) {
    std::string msg = a.errmsg(db);
    py::gil_scoped_acquire g;
    if ((rc & 0xff) == SQLITE_CONSTRAINT) {
        PyErr_SetString(py::module_::import("sqlite3").attr("IntegrityError").ptr(), msg.c_str());
    } else {
        PyErr_SetString(py::module_::import("sqlite3").attr("OperationalError").ptr(), msg.c_str());
    }
    throw py::error_already_set();
}

// Execute `sql` once per row with the given column bindings; rows run in `order` when given.
// Returns the summed sqlite3_changes() (rows inserted/deleted).
int64_t executemany(py::object conn, const std::string& sql, py::sequence cols, int64_t n, py::object order_obj) {
    const SqliteApi& a = api();
    sqlite3* db = handle_of(conn);
    std::vector<Col> cs;
    cs.reserve(cols.size());
    for (auto spec : cols) cs.push_back(parse_col(spec, n));
    std::vector<int64_t> order;
    if (!order_obj.is_none()) {
        py::buffer_info bi = order_obj.cast<py::buffer>().request();
        if (bi.itemsize != 8 || bi.size != n) throw std::invalid_argument("order must be int64[n]");
        const int64_t* o = static_cast<const int64_t*>(bi.ptr);
        order.assign(o, o + n);
        for (int64_t v : order)
            if (v < 0 || v >= n) throw std::out_of_range("order");
    }
    int64_t total = 0;
    {
        py::gil_scoped_release nogil;
        sqlite3_stmt* st = nullptr;
        int rc = a.prepare_v2(db, sql.c_str(), int(sql.size()), &st, nullptr);
        if (rc != SQLITE_OK) raise_sql(a, db, rc);
        char hexbuf[8][64];
        for (int64_t k = 0; k < n; ++k) {
            const int64_t r = order.empty() ? k : order[size_t(k)];
            int hb = 0;
            for (size_t j = 0; j < cs.size(); ++j) {
                const Col& c = cs[j];
                const int p = int(j) + 1;
                switch (c.kind) {
                    case Col::NUL: a.bind_null(st, p); break;
                    case Col::CONST_TEXT: a.bind_text(st, p, c.ctext.data(), int(c.ctext.size()), nullptr); break;
                    case Col::CONST_INT: a.bind_int64(st, p, c.cint); break;
                    case Col::INT64: a.bind_int64(st, p, c.ival[r]); break;
                    case Col::TEXT_LIST:
                        if (c.ptr[size_t(r)]) a.bind_text(st, p, c.ptr[size_t(r)], c.len[size_t(r)], nullptr);
                        else a.bind_null(st, p);
                        break;
                    case Col::GATHER: {
                        const size_t g = size_t(c.idx[r]);
                        if (c.ptr[g]) a.bind_text(st, p, c.ptr[g], c.len[g], nullptr);
                        else a.bind_null(st, p);
                        break;
                    }
                    case Col::ARENA:
                        a.bind_text(st, p, c.blob + c.aoff[r], int(c.aoff[r + 1] - c.aoff[r]), nullptr);
                        break;
                    case Col::HEX32: {
                        if (hb >= 8) {
                            a.finalize(st);
                            throw std::invalid_argument("at most 8 hex32 columns");
                        }
                        char* out = hexbuf[hb++];
                        const uint8_t* src = c.raw + r * c.stride + c.offset;
                        for (int b = 0; b < 32; ++b) {
                            out[2 * b] = kHex[src[b] >> 4];
                            out[2 * b + 1] = kHex[src[b] & 15];
                        }
                        a.bind_text(st, p, out, 64, nullptr);
                        break;
                    }
                }
            }
            rc = a.step(st);
            if (rc != SQLITE_DONE && rc != SQLITE_ROW) {
                a.reset(st);
                a.finalize(st);
                raise_sql(a, db, rc);
            }
            total += a.changes(db);
            a.reset(st);
        }
        a.finalize(st);
    }
    return total;
}

}  // namespace

void register_ledger_sql(py::module_& m) {
    m.def("sql_probe", [](py::object conn) {
        const SqliteApi& a = api();
        sqlite3* db = handle_of(conn);
        const char* fn = a.db_filename(db, "main");
        return py::make_tuple(std::string(fn ? fn : ""), a.total_changes(db), a.get_autocommit(db));
    }, "(filename, total_changes, autocommit) as seen through the native handle of a sqlite3.Connection");
    m.def("sql_executemany", &executemany, py::arg("conn"), py::arg("sql"), py::arg("cols"), py::arg("n"),
          py::arg("order") = py::none(),
          "column-major executemany on the connection's own handle; returns the summed row changes");
}

}  // namespace upow
