// pybind11 module `upow_amd._native`: the MI355X-native core (host C++ + gfx950 HIP kernels).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>
#include <stdexcept>

#include "native.h"
#include "sha256_common.h"

namespace py = pybind11;
using namespace upow;

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
       py::arg("start"), py::arg("count"), py::arg("grid_blocks") = 0, py::arg("chunk_iters") = 256,
       py::arg("cap") = 1 << 16, py::arg("variant") = 0);

    m.def("gpu_device_count", &gpu_device_count);
    m.def("gpu_arch_name", &gpu_arch_name);
}
