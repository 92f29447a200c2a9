// pybind11 module `upow_amd._native`: the MI355X-native core (host C++ + gfx950 HIP kernels).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>
#include <malloc.h>
#include <stdexcept>

#include "native.h"
#include "sha256_common.h"
#include "thread_pool.h"

namespace py = pybind11;
using namespace upow;

namespace upow {
void register_txcodec(py::module_& m);  // txcodec.cpp
void register_ledger_writer(py::module_& m);  // ledger_writer.cpp
void register_gov_index(py::module_& m);  // gov_index.cpp
void register_stall_probe(py::module_& m);  // stall_probe.cpp
void register_log_appender(py::module_& m);  // log_appender.cpp
void register_http_wire(py::module_& m);  // http_wire.cpp
void register_mempool_index(py::module_& m);  // mempool_index.cpp
void register_jsonspan(py::module_& m);  // jsonspan.cpp
void register_utxo_host(py::module_& m);  // utxo_host.cpp
}

static PowJobHost make_job(py::bytes header, uint32_t tmask, uint32_t tword, uint32_t frac_shift,
                           uint32_t frac_limit) {
    PowJobHost j;
    std::string h = header;
    j.header.assign(h.begin(), h.end());
    j.tmask = tmask;
    j.tword = tword;
    j.frac_shift = frac_shift;
    j.frac_limit = frac_limit;
    return j;
}

static py::tuple pow_result_tuple(const PowResult& r) {
    return py::make_tuple(r.searched, r.total_hits, r.words);
}

static void packed_args(py::buffer data, py::buffer offsets, const uint8_t*& d, const int64_t*& o, int64_t& n,
                        int64_t& nbytes) {
    py::buffer_info di = data.request(), oi = offsets.request();
    if (oi.itemsize != 8 || oi.ndim != 1) throw std::invalid_argument("offsets must be a 1-D int64 buffer");
    d = static_cast<const uint8_t*>(di.ptr);
    o = static_cast<const int64_t*>(oi.ptr);
    n = oi.shape[0] - 1;
    nbytes = di.size * di.itemsize;
    if (n < 0) throw std::invalid_argument("offsets must have n+1 entries");
    for (int64_t i = 0; i < n; ++i)
        if (o[i] < 0 || o[i + 1] < o[i] || o[i + 1] > nbytes) throw std::out_of_range("bad offsets");
}

PYBIND11_MODULE(_native, m) {
    m.doc() = "upow_amd native core: host C++ crypto + gfx950 HIP kernels";
    register_txcodec(m);
    register_ledger_writer(m);
    register_gov_index(m);
    register_stall_probe(m);
    register_log_appender(m);
    register_http_wire(m);
    register_mempool_index(m);
    register_jsonspan(m);
    register_utxo_host(m);

    // glibc allocator thresholds (mallopt): every 2 MB block's columns are fresh multi-megabyte Python bytes;
    // above the (dynamic) mmap threshold each one is a new mapping whose pages fault in on first write, and
    // a trimmed heap top faults in again next block. A fixed threshold/trim size keeps those pages mapped and
    // reused (utils/cpus.py tune_malloc, called by the node and bench entry points). Returns success.
    m.def("malloc_tune", [](int64_t mmap_threshold, int64_t trim_threshold) {
        bool ok = true;
        if (mmap_threshold > 0) ok &= mallopt(M_MMAP_THRESHOLD, int(std::min<int64_t>(mmap_threshold, INT32_MAX))) == 1;
        if (trim_threshold > 0) ok &= mallopt(M_TRIM_THRESHOLD, int(std::min<int64_t>(trim_threshold, INT32_MAX))) == 1;
        return ok;
    });

    m.def("sha256", [](py::bytes msg) {
        std::string s = msg;
        uint8_t out[32];
        host_sha256(reinterpret_cast<const uint8_t*>(s.data()), s.size(), out);
        return py::bytes(reinterpret_cast<const char*>(out), 32);
    });

    m.def("sha256_batch_host", [](py::buffer data, py::buffer offsets, int threads) {
        const uint8_t* d; const int64_t* o; int64_t n, nb;
        packed_args(data, offsets, d, o, n, nb);
        std::vector<uint8_t> out;
        {
            py::gil_scoped_release rel;
            out = sha256_batch_host(d, o, n, threads);
        }
        return py::bytes(reinterpret_cast<const char*>(out.data()), out.size());
    }, py::arg("data"), py::arg("offsets"), py::arg("threads") = 1);

    // SHA-256 of the first nchars[k] characters of hexes[idx[k]] (the ASCII text itself, not the bytes it
    // encodes): the reference's second verify attempt hashes the signed prefix of the tx hex string
    // (transaction_input.py:84-120). Zero-copy views of the str objects, hashed on the host pool.
    m.def("sha256_hex_prefixes", [](py::list hexes, py::array_t<int64_t, py::array::c_style | py::array::forcecast> idx,
                                   py::array_t<int64_t, py::array::c_style | py::array::forcecast> nchars, int threads) {
        const int64_t n = int64_t(idx.size());
        if (int64_t(nchars.size()) != n) throw py::value_error("sha256_hex_prefixes: idx and nchars differ in length");
        const int64_t* ix = idx.data();
        const int64_t* nc = nchars.data();
        std::vector<const char*> src(static_cast<size_t>(n));
        std::vector<py::object> keep;  // the str objects stay alive while the GIL is released, whatever the list does
        keep.reserve(static_cast<size_t>(n));
        const int64_t n_hex = int64_t(hexes.size());
        for (int64_t k = 0; k < n; ++k) {
            if (ix[k] < 0 || ix[k] >= n_hex) throw py::index_error("sha256_hex_prefixes: tx index out of range");
            PyObject* o = PyList_GET_ITEM(hexes.ptr(), Py_ssize_t(ix[k]));
            keep.push_back(py::reinterpret_borrow<py::object>(o));
            if (!PyUnicode_Check(o)) throw py::type_error("transaction hex must be str");
            Py_ssize_t sz = 0;
            const char* p = PyUnicode_AsUTF8AndSize(o, &sz);
            if (!p) throw py::error_already_set();
            if (nc[k] < 0 || nc[k] > int64_t(sz)) throw py::value_error("sha256_hex_prefixes: prefix longer than the hex");
            src[size_t(k)] = p;
        }
        std::string out(size_t(n) * 32, '\0');
        {
            py::gil_scoped_release rel;
            HostPool::get().parallel_for(n, threads, [&](int64_t k) {
                host_sha256(reinterpret_cast<const uint8_t*>(src[size_t(k)]), size_t(nc[k]),
                            reinterpret_cast<uint8_t*>(&out[size_t(k) * 32]));
            });
        }
        return py::bytes(out);
    }, py::arg("hexes"), py::arg("idx"), py::arg("nchars"), py::arg("threads") = 1);

    m.def("sha256_batch_gpu", [](py::buffer data, py::buffer offsets) {
        const uint8_t* d; const int64_t* o; int64_t n, nb;
        packed_args(data, offsets, d, o, n, nb);
        std::vector<uint8_t> out;
        {
            py::gil_scoped_release rel;
            out = sha256_batch_gpu(d, nb, o, n);
        }
        return py::bytes(reinterpret_cast<const char*>(out.data()), out.size());
    });

    m.def("pow_check_word", [](py::bytes header, uint32_t tmask, uint32_t tword, uint32_t fs, uint32_t fl,
                               uint32_t v) { return pow_check_word_host(make_job(header, tmask, tword, fs, fl), v); });

    m.def("pow_search_host", [](py::bytes header, uint32_t tmask, uint32_t tword, uint32_t fs, uint32_t fl,
                                uint64_t start, uint64_t count, int threads) {
        PowJobHost j = make_job(header, tmask, tword, fs, fl);
        PowResult r;
        {
            py::gil_scoped_release rel;
            r = pow_search_host(j, start, count, threads);
        }
        return pow_result_tuple(r);
    });

    m.def("pow_search_gpu", [](py::bytes header, uint32_t tmask, uint32_t tword, uint32_t fs, uint32_t fl,
                               uint64_t start, uint64_t count, int grid_blocks, uint32_t chunk_iters, uint32_t cap, int variant) {
        PowJobHost j = make_job(header, tmask, tword, fs, fl);
        PowResult r;
        {
            py::gil_scoped_release rel;
            r = pow_search_gpu(j, start, count, grid_blocks, chunk_iters, cap, variant);
        }
        return pow_result_tuple(r);
    }, py::arg("header"), py::arg("tmask"), py::arg("tword"), py::arg("frac_shift"), py::arg("frac_limit"),
       py::arg("start"), py::arg("count"), py::arg("grid_blocks") = 0, py::arg("chunk_iters") = 0,
       py::arg("cap") = 1 << 16, py::arg("variant") = 0);

    m.def("set_node_device", [](int dev) { set_node_device_native(dev); }, py::arg("device"),
          "pin node-side GPU work (verify, decompress, batched SHA-256) to this device from every thread");
    m.def("pow_kernel_info", [](int variant) {
        PowKernelInfo k = pow_kernel_info(variant);
        return py::dict(py::arg("cus") = k.cus, py::arg("blocks_per_cu") = k.blocks_per_cu,
                        py::arg("resident_blocks") = k.resident_blocks);
    }, py::arg("variant") = 0);
    m.def("p256_verify", [](py::buffer items, bool gpu, int threads) {
        py::buffer_info bi = items.request();
        const int64_t nbytes = bi.size * bi.itemsize;
        if (nbytes % 160) throw std::invalid_argument("items must be n x 160 bytes");
        const int64_t n = nbytes / 160;
        const uint8_t* p = static_cast<const uint8_t*>(bi.ptr);
        std::vector<uint8_t> st;
        {
            py::gil_scoped_release rel;
            st = gpu ? p256_verify_gpu(p, n) : p256_verify_host(p, n, threads);
        }
        return py::bytes(reinterpret_cast<const char*>(st.data()), st.size());
    }, py::arg("items"), py::arg("gpu") = false, py::arg("threads") = 1);

    m.def("p256_decompress", [](py::buffer in, bool gpu) {
        py::buffer_info bi = in.request();
        const int64_t nbytes = bi.size * bi.itemsize;
        if (nbytes % 33) throw std::invalid_argument("input must be n x 33 bytes");
        const int64_t n = nbytes / 33;
        std::vector<uint8_t> out(static_cast<size_t>(n) * 64), ok(static_cast<size_t>(n));
        {
            py::gil_scoped_release rel;
            if (gpu) p256_decompress_gpu(static_cast<const uint8_t*>(bi.ptr), n, out.data(), ok.data());
            else p256_decompress_host(static_cast<const uint8_t*>(bi.ptr), n, out.data(), ok.data());
        }
        return py::make_tuple(py::bytes(reinterpret_cast<const char*>(out.data()), out.size()),
                              py::bytes(reinterpret_cast<const char*>(ok.data()), ok.size()));
    }, py::arg("data"), py::arg("gpu") = false);

    m.def("p256_on_curve", [](py::buffer in, bool gpu, int threads) {
        py::buffer_info bi = in.request();
        const int64_t nbytes = bi.size * bi.itemsize;
        if (nbytes % 64) throw std::invalid_argument("input must be n x 64 bytes (x LE | y LE)");
        const int64_t n = nbytes / 64;
        std::string ok(static_cast<size_t>(n), '\0');
        {
            py::gil_scoped_release rel;
            auto* o = reinterpret_cast<uint8_t*>(&ok[0]);
            if (gpu) p256_on_curve_gpu(static_cast<const uint8_t*>(bi.ptr), n, o);
            else p256_on_curve_host(static_cast<const uint8_t*>(bi.ptr), n, o, threads);
        }
        return py::bytes(ok);
    }, py::arg("data"), py::arg("gpu") = false, py::arg("threads") = 8);

    m.def("p256_pubkey", [](py::bytes d_be) -> py::object {
        std::string d = d_be;
        if (d.size() != 32) throw std::invalid_argument("private key must be 32 bytes big-endian");
        uint8_t out[64];
        if (!p256_pubkey(reinterpret_cast<const uint8_t*>(d.data()), out)) return py::none();
        return py::bytes(reinterpret_cast<const char*>(out), 64);
    });

    // s^-1 * 2^256 mod n (32 bytes little-endian in and out, s in [1, n)): the verifier's divsteps inverse,
    // exposed for its differential test against Python's pow
    m.def("p256_scalar_inv_mont", [](py::bytes s_le) -> py::bytes {
        const std::string s = s_le;
        if (s.size() != 32) throw std::invalid_argument("need 32 bytes little-endian");
        uint64_t in[4], out[4];
        std::memcpy(in, s.data(), 32);
        p256_scalar_inv_mont_host(out, in);
        return py::bytes(reinterpret_cast<const char*>(out), 32);
    });

    // the kernels' field arithmetic on the host, for its differential test against Python integers
    m.def("p256_fe_ops", [](py::bytes a_le, py::bytes b_le) -> py::bytes {
        const std::string a = a_le, b = b_le;
        if (a.size() != 32 || b.size() != 32) throw std::invalid_argument("need 32-byte little-endian a, b");
        uint32_t x[8], y[8], out[32];
        std::memcpy(x, a.data(), 32);
        std::memcpy(y, b.data(), 32);
        p256_fe_ops_host(x, y, out);
        return py::bytes(reinterpret_cast<const char*>(out), sizeof out);
    });
    m.def("rccl_unique_id", []() { return py::bytes(rccl_unique_id()); });
    m.def("rccl_vote_create", [](py::bytes uid, int world, int rank) {
        const std::string u = uid;
        py::gil_scoped_release rel;  // collective: waits for every rank
        return rccl_vote_create(u, world, rank);
    });
    // queueing a vote takes a few microseconds: done holding the GIL (releasing it would let another
    // thread take it for up to a switch interval before this one gets it back)
    m.def("rccl_vote_start", [](int64_t h, int value) { rccl_vote_start(h, value); });
    m.def("rccl_vote_finish", [](int64_t h, double timeout_s) {
        py::gil_scoped_release rel;
        return rccl_vote_finish(h, timeout_s);
    });
    m.def("rccl_vote_stats", [](int64_t h) { return rccl_vote_stats(h); });
    m.def("rccl_vote_destroy", [](int64_t h, bool abort) {
        py::gil_scoped_release rel;
        rccl_vote_destroy(h, abort);
    }, py::arg("h"), py::arg("abort") = false);
    m.def("p256_g16_entries", [](int64_t first, int64_t count) -> py::bytes {
        std::vector<uint8_t> o;
        { py::gil_scoped_release rel; o = p256_g16_entries(first, count); }
        return py::bytes(reinterpret_cast<const char*>(o.data()), o.size());
    });
    m.def("p256_fe_reduce", [](py::bytes c_le) -> py::bytes {
        const std::string c = c_le;
        if (c.size() != 64) throw std::invalid_argument("need 64 bytes little-endian");
        uint32_t x[16], out[8];
        std::memcpy(x, c.data(), 64);
        p256_fe_reduce_host(x, out);
        return py::bytes(reinterpret_cast<const char*>(out), sizeof out);
    });

    m.def("p256_sign", [](py::bytes d_be, py::bytes digest) -> py::object {
        std::string d = d_be, h = digest;
        if (d.size() != 32 || h.size() != 32) throw std::invalid_argument("need 32-byte key and digest");
        uint8_t r[32], s[32];
        if (!p256_sign(reinterpret_cast<const uint8_t*>(d.data()), reinterpret_cast<const uint8_t*>(h.data()), r, s))
            return py::none();
        return py::make_tuple(py::bytes(reinterpret_cast<const char*>(r), 32),
                              py::bytes(reinterpret_cast<const char*>(s), 32));
    });

    // Batch forms for wallets and synthetic-chain setup (bench_verify distinct keys): n keys / n (key,
    // digest) pairs on the host pool without the GIL. A key outside [1, n-1] leaves its 64 output bytes zero.
    m.def("p256_pubkey_batch", [](py::bytes keys_be, int threads) -> py::bytes {
        const std::string d = keys_be;
        if (d.size() % 32) throw std::invalid_argument("keys must be n x 32 bytes big-endian");
        const int64_t n = int64_t(d.size() / 32);
        std::string out(size_t(n) * 64, '\0');
        {
            py::gil_scoped_release rel;
            HostPool::get().parallel_for(n, threads, [&](int64_t i) {
                uint8_t q[64];
                if (p256_pubkey(reinterpret_cast<const uint8_t*>(d.data()) + 32 * i, q)) std::memcpy(&out[size_t(64 * i)], q, 64);
            });
        }
        return py::bytes(out);
    }, py::arg("keys_be"), py::arg("threads") = 8);

    m.def("p256_sign_batch", [](py::bytes keys_be, py::bytes digests, int threads) -> py::bytes {
        const std::string d = keys_be, h = digests;
        if (d.size() % 32 || h.size() != d.size()) throw std::invalid_argument("need n x 32-byte keys and digests");
        const int64_t n = int64_t(d.size() / 32);
        std::string out(size_t(n) * 64, '\0');
        {
            py::gil_scoped_release rel;
            HostPool::get().parallel_for(n, threads, [&](int64_t i) {
                uint8_t r[32], s[32];
                const auto* kp = reinterpret_cast<const uint8_t*>(d.data()) + 32 * i;
                const auto* hp = reinterpret_cast<const uint8_t*>(h.data()) + 32 * i;
                if (p256_sign(kp, hp, r, s)) {
                    std::memcpy(&out[size_t(64 * i)], r, 32);
                    std::memcpy(&out[size_t(64 * i + 32)], s, 32);
                }
            });
        }
        return py::bytes(out);
    }, py::arg("keys_be"), py::arg("digests"), py::arg("threads") = 8);

    auto recs_arg = [](py::buffer b, int64_t& n) {
        py::buffer_info bi = b.request();
        const int64_t nb = bi.size * bi.itemsize;
        if (nb % 40) throw std::invalid_argument("utxo key records must be n x 40 bytes");
        n = nb / 40;
        return static_cast<const uint8_t*>(bi.ptr);
    };
    m.def("utxo_create", &utxo_create);
    m.def("utxo_destroy", &utxo_destroy);
    m.def("utxo_capacity", &utxo_capacity);
    m.def("utxo_rehash", [](int64_t h, uint32_t log2_cap) {
        uint64_t r;
        { py::gil_scoped_release rel; r = utxo_rehash(h, log2_cap); }
        return py::make_tuple(uint32_t(r), uint32_t(r >> 32));  // (entries moved, no free slot)
    });
    m.def("utxo_insert", [recs_arg](int64_t h, py::buffer recs, py::object payload) {
        int64_t n; const uint8_t* p = recs_arg(recs, n);
        const uint8_t* pp = nullptr;
        py::buffer_info pi;
        if (!payload.is_none()) {
            pi = payload.cast<py::buffer>().request();
            if (pi.size * pi.itemsize != n * 80) throw std::invalid_argument("payload must be n x 80 bytes");
            pp = static_cast<const uint8_t*>(pi.ptr);
        }
        uint64_t r;
        { py::gil_scoped_release rel; r = utxo_insert(h, p, n, pp); }
        return py::make_tuple(uint32_t(r), uint32_t(r >> 32));  // (no free slot, duplicates skipped)
    }, py::arg("h"), py::arg("recs"), py::arg("payload") = py::none());
    m.def("utxo_lookup", [recs_arg](int64_t h, py::buffer recs) {
        int64_t n; const uint8_t* p = recs_arg(recs, n);
        std::vector<uint8_t> o, pay;
        { py::gil_scoped_release rel; o = utxo_lookup(h, p, n, pay); }
        return py::make_tuple(py::bytes(reinterpret_cast<const char*>(o.data()), o.size()),
                              py::bytes(reinterpret_cast<const char*>(pay.data()), pay.size()));
    });
    m.def("utxo_probe", [recs_arg](int64_t h, py::buffer recs) {
        int64_t n; const uint8_t* p = recs_arg(recs, n);
        std::vector<uint8_t> o;
        { py::gil_scoped_release rel; o = utxo_probe(h, p, n); }
        return py::bytes(reinterpret_cast<const char*>(o.data()), o.size());
    });
    m.def("utxo_erase", [recs_arg](int64_t h, py::buffer recs) {
        int64_t n; const uint8_t* p = recs_arg(recs, n);
        std::vector<uint8_t> o;
        { py::gil_scoped_release rel; o = utxo_erase(h, p, n); }
        return py::bytes(reinterpret_cast<const char*>(o.data()), o.size());
    });
    // ins: a list of (records n x 40, payloads n x 80 or None) groups; all groups carry payloads or none do
    m.def("utxo_apply_async", [recs_arg](int64_t h, py::list ins, py::buffer dels) {
        int64_t n_del;
        const uint8_t* pd = recs_arg(dels, n_del);
        std::vector<UtxoSeg> segs;
        std::vector<py::buffer_info> keep;
        keep.reserve(2 * ins.size());
        int with_pay = -1;
        for (py::handle item : ins) {
            py::tuple t = item.cast<py::tuple>();
            int64_t n;
            const uint8_t* pr = recs_arg(t[0].cast<py::buffer>(), n);
            const uint8_t* pp = nullptr;
            if (!t[1].is_none()) {
                keep.push_back(t[1].cast<py::buffer>().request());
                if (keep.back().size * keep.back().itemsize != n * 80) throw std::invalid_argument("payload must be n x 80 bytes");
                pp = static_cast<const uint8_t*>(keep.back().ptr);
            }
            if (n && with_pay >= 0 && with_pay != (pp != nullptr)) throw std::invalid_argument("payloads for all groups or none");
            if (n) with_pay = pp != nullptr;
            segs.push_back(UtxoSeg{pr, pp, n});
        }
        uint32_t prev[3];
        bool had;
        { py::gil_scoped_release rel; had = utxo_apply_async(h, segs, with_pay == 1, pd, n_del, prev); }
        return py::make_tuple(had, prev[0], prev[1], prev[2]);
    }, py::arg("h"), py::arg("ins"), py::arg("dels"));
    m.def("utxo_apply_wait", [](int64_t h) {
        uint32_t r[3];
        bool had;
        { py::gil_scoped_release rel; had = utxo_apply_wait(h, r); }
        return py::make_tuple(had, r[0], r[1], r[2]);  // (pending, no free slot, duplicates, erased)
    });
    m.def("utxo_dump", [](int64_t h) {
        std::vector<uint8_t> o;
        { py::gil_scoped_release rel; o = utxo_dump(h, nullptr); }
        return py::bytes(reinterpret_cast<const char*>(o.data()), o.size());
    });
    // The whole-block input pass: reads the segment arrays in place (any buffer: the codec's bytes or numpy
    // arrays) and returns numpy arrays the pass wrote straight out of its pinned staging (one copy each).
    m.def("utxo_block_inputs", [recs_arg](int64_t h, py::buffer keys, py::buffer in_start, py::buffer out_amount,
                                          py::buffer out_start, uint32_t want_tag) {
        int64_t n_in; const uint8_t* kp = recs_arg(keys, n_in);
        py::buffer_info bi = in_start.request(), bo = out_start.request(), ba = out_amount.request();
        const size_t is_n = size_t(bi.size * bi.itemsize), os_n = size_t(bo.size * bo.itemsize);
        const size_t oa_n = size_t(ba.size * ba.itemsize);
        if (is_n % 4 || is_n < 4 || os_n != is_n || oa_n % 8) throw std::invalid_argument("bad segment arrays");
        const int64_t n_tx = int64_t(is_n / 4) - 1;
        const int32_t* isp = static_cast<const int32_t*>(bi.ptr);
        const int32_t* osp = static_cast<const int32_t*>(bo.ptr);
        const uint64_t* oap = static_cast<const uint64_t*>(ba.ptr);
        const int64_t n_out = int64_t(oa_n / 8);
        for (int64_t t = 0; t < n_tx; ++t)  // the kernels index with these: validate them on the host
            if (isp[t] < 0 || isp[t + 1] < isp[t] || osp[t] < 0 || osp[t + 1] < osp[t])
                throw std::invalid_argument("segment offsets must be non-decreasing");
        if (isp[n_tx] != n_in || osp[n_tx] != n_out || isp[0] != 0 || osp[0] != 0)
            throw std::invalid_argument("segment offsets do not cover the arrays");
        py::array_t<uint8_t> tags(n_in), pay(n_in * 80);
        py::array_t<uint32_t> dup(n_in), miss(std::max<int64_t>(n_tx, 0));
        py::array_t<int64_t> fee(std::max<int64_t>(n_tx, 0));
        BlockInputsOut r{tags.mutable_data(), pay.mutable_data(), dup.mutable_data(), fee.mutable_data(),
                         miss.mutable_data()};
        {
            py::gil_scoped_release rel;
            utxo_block_inputs(h, kp, n_in, isp, oap, n_out, osp, n_tx, want_tag, r);
        }
        return py::make_tuple(tags, pay, dup, fee, miss, r.n_dup);
    });
    m.def("utxo_set_hash", [](int64_t h, uint32_t tag) {
        std::vector<uint8_t> d;
        uint64_t n = 0;
        { py::gil_scoped_release rel; d = utxo_set_hash(h, tag, &n); }
        return py::make_tuple(py::bytes(reinterpret_cast<const char*>(d.data()), d.size()), n);
    });
    m.def("utxo_k12_snapshot", [](int64_t h, uint32_t tag) {
        py::gil_scoped_release rel;
        return utxo_k12_snapshot(h, tag);
    });
    m.def("utxo_k12_digest", [](int64_t id) {
        uint64_t n = 0;
        std::vector<uint8_t> d;
        { py::gil_scoped_release rel; d = utxo_k12_digest(id, &n); }
        return py::make_tuple(py::bytes(reinterpret_cast<const char*>(d.data()), d.size()), n);
    });
    m.def("utxo_set_message", [](int64_t h, uint32_t tag) {
        auto* v = new std::vector<uint8_t>();
        uint64_t n = 0;
        { py::gil_scoped_release rel; *v = utxo_set_message(h, tag, &n); }
        py::capsule own(v, [](void* p) { delete static_cast<std::vector<uint8_t>*>(p); });
        return py::array_t<uint8_t>({py::ssize_t(v->size())}, {py::ssize_t(1)}, v->data(), own);
    });
    m.def("utxo_address_scan", [](int64_t h, py::bytes addr, uint32_t tag_mask, uint32_t stake_sel) {
        std::string a = addr;
        std::vector<uint8_t> o, pay;
        uint64_t total = 0;
        {
            py::gil_scoped_release rel;
            o = utxo_address_scan(h, reinterpret_cast<const uint8_t*>(a.data()), uint32_t(a.size()), tag_mask,
                                  stake_sel, pay, &total);
        }
        return py::make_tuple(py::bytes(reinterpret_cast<const char*>(o.data()), o.size()),
                              py::bytes(reinterpret_cast<const char*>(pay.data()), pay.size()), total);
    }, py::arg("h"), py::arg("addr"), py::arg("tag_mask"), py::arg("stake_sel") = 0);
    m.def("utxo_dump_payload", [](int64_t h) {
        std::vector<uint8_t> o, pay;
        { py::gil_scoped_release rel; o = utxo_dump(h, &pay); }
        return py::make_tuple(py::bytes(reinterpret_cast<const char*>(o.data()), o.size()),
                              py::bytes(reinterpret_cast<const char*>(pay.data()), pay.size()));
    });

    m.def("b58encode", [](py::bytes b) {
        std::string s = b;
        return b58encode(reinterpret_cast<const uint8_t*>(s.data()), s.size());
    });
    m.def("b58decode", [](const std::string& s) {
        std::vector<uint8_t> v;
        try {
            v = b58decode(s);
        } catch (const std::invalid_argument& e) {
            throw py::value_error(e.what());
        }
        return py::bytes(reinterpret_cast<const char*>(v.data()), v.size());
    });

    m.def("gpu_device_count", &gpu_device_count);
    m.def("gpu_arch_name", &gpu_arch_name);
}
