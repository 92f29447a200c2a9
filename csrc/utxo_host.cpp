// The UTXO index on the host (UPOW_UTXO_BACKEND=host, and every node without a GPU): the same record-level
// contract as the HBM table of csrc/utxo_table.hip — 40-byte key records {txid, u32 index, u32 tag}, 80-byte
// payloads {u64 amount, u32 addr_len, u32 flags, addr[64]}, tags 0xff = absent / any — as a C++ hash map
// with an owner-address index for K14, so a CPU node (the test suite, a gloo cluster rehearsal) applies a
// block's index writes in one native call instead of a Python dict walk per outpoint.
//
// Reference: the seven output tables of upow/database.py (unspent_outputs and the governance tables) and their
// lookups (database.py:788-837), balance queries by address (database.py:909-937, 1138-1205).
//
// Keys compare on (txid, index & 0xff), as the device table does (an outpoint index is one byte on the wire).
// Inserts of a live outpoint are refused and counted (a ledger bug if it ever happens); erases honour a tag.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace py = pybind11;

namespace upow {
namespace {

struct Rec {  // 40 bytes
    uint8_t txid[32];
    uint32_t index;
    uint32_t tag;
};
struct Pay {  // 80 bytes
    uint64_t amount;
    uint32_t addr_len;
    uint32_t flags;
    uint8_t addr[64];
};
static_assert(sizeof(Rec) == 40 && sizeof(Pay) == 80, "record layouts");

struct Key {
    uint64_t w[4];
    uint32_t idx;
    bool operator==(const Key& o) const {
        return w[0] == o.w[0] && w[1] == o.w[1] && w[2] == o.w[2] && w[3] == o.w[3] && idx == o.idx;
    }
};
struct KeyHash {
    size_t operator()(const Key& k) const {
        uint64_t h = k.w[0] ^ (uint64_t(k.idx) * 0x9E3779B97F4A7C15ull);
        h ^= h >> 29;
        h *= 0xBF58476D1CE4E5B9ull;
        return size_t(h ^ (h >> 32));
    }
};
inline Key key_of(const Rec& r) {
    Key k;
    std::memcpy(k.w, r.txid, 32);
    k.idx = r.index & 0xffu;
    return k;
}
struct Entry {
    uint32_t tag;
    Pay pay;
};

class HostUtxo {
   public:
    // returns the outpoints already live (left untouched)
    uint64_t insert(const Rec* r, const Pay* p, int64_t n) {
        std::lock_guard<std::mutex> lk(mu_);
        uint64_t dups = 0;
        map_.reserve(map_.size() + size_t(n));
        for (int64_t i = 0; i < n; ++i) {
            const Key k = key_of(r[i]);
            Entry e;
            e.tag = r[i].tag & 0xffu;
            if (p)
                e.pay = p[i];
            else
                std::memset(&e.pay, 0, sizeof(Pay));
            auto ins = map_.emplace(k, e);
            if (!ins.second) {
                ++dups;
                continue;
            }
            if (e.pay.addr_len) by_addr_[addr_key(e.pay)].insert(k);
        }
        return dups;
    }

    void lookup(const Rec* r, int64_t n, uint8_t* tags, Pay* pay) const {
        std::lock_guard<std::mutex> lk(mu_);
        for (int64_t i = 0; i < n; ++i) {
            auto it = map_.find(key_of(r[i]));
            if (it == map_.end()) {
                tags[i] = 0xff;
                if (pay) std::memset(&pay[i], 0, sizeof(Pay));
            } else {
                tags[i] = uint8_t(it->second.tag);
                if (pay) pay[i] = it->second.pay;
            }
        }
    }

    // erased[i] = 1 when removed: only an entry whose tag equals r[i].tag (0xff: any)
    uint64_t erase(const Rec* r, int64_t n, uint8_t* erased) {
        std::lock_guard<std::mutex> lk(mu_);
        uint64_t count = 0;
        for (int64_t i = 0; i < n; ++i) {
            const Key k = key_of(r[i]);
            const uint32_t want = r[i].tag & 0xffu;
            auto it = map_.find(k);
            uint8_t res = 0;
            if (it != map_.end() && (want == 0xffu || it->second.tag == want)) {
                if (it->second.pay.addr_len) {
                    auto a = by_addr_.find(addr_key(it->second.pay));
                    if (a != by_addr_.end()) {
                        a->second.erase(k);
                        if (a->second.empty()) by_addr_.erase(a);
                    }
                }
                map_.erase(it);
                res = 1;
                ++count;
            }
            erased[i] = res;
        }
        return count;
    }

    void clear() {
        std::lock_guard<std::mutex> lk(mu_);
        map_.clear();
        by_addr_.clear();
    }

    size_t size() const {
        std::lock_guard<std::mutex> lk(mu_);
        return map_.size();
    }

    void dump(std::vector<Rec>& recs, std::vector<Pay>* pays) const {
        std::lock_guard<std::mutex> lk(mu_);
        recs.resize(map_.size());
        if (pays) pays->resize(map_.size());
        size_t o = 0;
        for (const auto& kv : map_) {
            put(kv.first, kv.second.tag, recs[o]);
            if (pays) (*pays)[o] = kv.second.pay;
            ++o;
        }
    }

    // K14: live outpoints owned by `addr` in the tables of `tag_mask`; stake_sel 0 any, 1 not staked, 2 staked
    // (only unspent_outputs rows carry the stake flag)
    void address_scan(const std::string& addr, uint32_t tag_mask, uint32_t stake_sel, std::vector<Rec>& recs,
                      std::vector<Pay>& pays) const {
        std::lock_guard<std::mutex> lk(mu_);
        auto a = by_addr_.find(addr);
        if (a == by_addr_.end()) return;
        for (const Key& k : a->second) {
            const Entry& e = map_.at(k);
            if (e.tag >= 32u || !((tag_mask >> e.tag) & 1u)) continue;
            const bool staked = e.tag == 0u && (e.pay.flags & 1u);
            if (stake_sel != 0u && staked != (stake_sel == 2u)) continue;
            Rec r;
            put(k, e.tag, r);
            recs.push_back(r);
            pays.push_back(e.pay);
        }
    }

   private:
    static std::string addr_key(const Pay& p) {
        return std::string(reinterpret_cast<const char*>(p.addr), std::min<uint32_t>(p.addr_len, 64));
    }
    static void put(const Key& k, uint32_t tag, Rec& r) {
        std::memcpy(r.txid, k.w, 32);
        r.index = k.idx;
        r.tag = tag;
    }

    mutable std::mutex mu_;
    std::unordered_map<Key, Entry, KeyHash> map_;
    std::unordered_map<std::string, std::unordered_set<Key, KeyHash>> by_addr_;
};

const Rec* recs_of(const py::buffer& b, int64_t& n, py::buffer_info& keep) {
    keep = b.request();
    const int64_t nb = keep.size * keep.itemsize;
    if (nb % 40) throw std::invalid_argument("utxo key records must be n x 40 bytes");
    n = nb / 40;
    return static_cast<const Rec*>(keep.ptr);
}

template <class T>
py::array_t<uint8_t> as_bytes_array(const std::vector<T>& v) {
    py::array_t<uint8_t> out(int64_t(v.size() * sizeof(T)));
    if (!v.empty()) std::memcpy(out.mutable_data(), v.data(), v.size() * sizeof(T));
    return out;
}

}  // namespace

void register_utxo_host(py::module_& m) {
    py::class_<HostUtxo, std::shared_ptr<HostUtxo>>(m, "HostUtxo")
        .def(py::init<>())
        .def("__len__", &HostUtxo::size)
        .def("clear", &HostUtxo::clear)
        .def("insert", [](HostUtxo& t, py::buffer recs, py::object payload) {
            int64_t n;
            py::buffer_info ki, pi;
            const Rec* r = recs_of(recs, n, ki);
            const Pay* p = nullptr;
            if (!payload.is_none()) {
                pi = py::buffer(payload).request();
                if (pi.size * pi.itemsize != n * 80) throw std::invalid_argument("payload must be n x 80 bytes");
                p = static_cast<const Pay*>(pi.ptr);
            }
            py::gil_scoped_release rel;
            return t.insert(r, p, n);
        }, py::arg("recs"), py::arg("payload") = py::none(), "insert key records (+ payloads); returns duplicates")
        .def("lookup", [](const HostUtxo& t, py::buffer recs) {
            int64_t n;
            py::buffer_info ki;
            const Rec* r = recs_of(recs, n, ki);
            py::array_t<uint8_t> tags(n), pay(n * 80);
            uint8_t* tp = tags.mutable_data();
            Pay* pp = reinterpret_cast<Pay*>(pay.mutable_data());
            {
                py::gil_scoped_release rel;
                t.lookup(r, n, tp, pp);
            }
            return py::make_tuple(tags, pay);
        }, "(tags u8[n], payloads u8[n*80]) of the records' outpoints (0xff / zeros when absent)")
        .def("probe", [](const HostUtxo& t, py::buffer recs) {
            int64_t n;
            py::buffer_info ki;
            const Rec* r = recs_of(recs, n, ki);
            py::array_t<uint8_t> tags(n);
            uint8_t* tp = tags.mutable_data();
            {
                py::gil_scoped_release rel;
                t.lookup(r, n, tp, nullptr);
            }
            return tags;
        })
        .def("erase", [](HostUtxo& t, py::buffer recs) {
            int64_t n;
            py::buffer_info ki;
            const Rec* r = recs_of(recs, n, ki);
            py::array_t<uint8_t> out(n);
            uint8_t* op = out.mutable_data();
            {
                py::gil_scoped_release rel;
                t.erase(r, n, op);
            }
            return out;
        }, "erase the records' outpoints whose tag matches the record's (0xff: any); u8 flags")
        .def("dump", [](const HostUtxo& t, bool with_payload) {
            std::vector<Rec> recs;
            std::vector<Pay> pays;
            {
                py::gil_scoped_release rel;
                t.dump(recs, with_payload ? &pays : nullptr);
            }
            return py::make_tuple(as_bytes_array(recs), as_bytes_array(pays));
        }, py::arg("with_payload") = true)
        .def("address_scan", [](const HostUtxo& t, py::bytes addr, uint32_t tag_mask, uint32_t stake_sel) {
            std::vector<Rec> recs;
            std::vector<Pay> pays;
            t.address_scan(std::string(addr), tag_mask, stake_sel, recs, pays);
            return py::make_tuple(as_bytes_array(recs), as_bytes_array(pays));
        });
}

}  // namespace upow
