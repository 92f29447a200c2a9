// Host mempool index (upow_amd/ledger/mempool.py wraps it): pending tx hashes with their propagation time,
// journal sequence and block-template key, and the outpoints they spend.
//
// reference: add_pending_transaction / get_pending_spent_outputs / the template query
// ``ORDER BY fees / LENGTH(tx_hex) DESC, LENGTH(tx_hex), tx_hex`` (upow/database.py:93-115, 173-174,
// 832-838). A committed block removes its txs and inputs from this index on the ledger thread; with a
// Python dict and set that was a few milliseconds of GIL-holding work per 8k-tx block (bytes objects per
// row, dict pops, set differences), competing with the HTTP loop. Here the block's raw txid and outpoint
// arrays are consumed as they are, without the GIL, and admissions are one hash-map probe per key.
//
// Locking: every method takes the index's own reader/writer lock, so a lookup on the HTTP loop (spent_of,
// has_tx) can never walk a hash node that a block's confirm_raw, running GIL-free on the ledger thread, is
// erasing. Rule that keeps it deadlock-free against the GIL: nobody blocks on the lock while holding the GIL
// (a contended acquire first releases the GIL, see `Shared`/`Exclusive`), and the GIL-free sections
// re-acquire the GIL only after dropping the lock.
//
// Template order: the reference divides ``fees`` (a NUMERIC with <= 8 decimals) by the hex length; two
// distinct ratios of such values differ by far more than a 28-digit quotient resolves, so comparing
// fee_a * len_b with fee_b * len_a exactly gives the same order (ties: length, then the hex string).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <array>
#include <cstdint>
#include <cstring>
#include <condition_variable>
#include <mutex>
#include <shared_mutex>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace py = pybind11;

namespace upow {
namespace {

using H32 = std::array<uint8_t, 32>;
using Op36 = std::array<uint8_t, 36>;

struct HHash {
    template <class A>
    size_t operator()(const A& a) const noexcept {
        uint64_t x, y;
        std::memcpy(&x, a.data(), 8);
        std::memcpy(&y, a.data() + a.size() - 8, 8);
        return size_t(x ^ (y * 0x9E3779B97F4A7C15ull));
    }
};

int hexv(char c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
}

H32 h32_hex(const std::string& s) {
    if (s.size() != 64) throw std::invalid_argument("tx hash must be 64 hex digits");
    H32 h;
    for (size_t i = 0; i < 32; ++i) {
        const int a = hexv(s[2 * i]), b = hexv(s[2 * i + 1]);
        if (a < 0 || b < 0) throw std::invalid_argument("tx hash must be hex");
        h[i] = uint8_t(a << 4 | b);
    }
    return h;
}

Op36 op_key(const std::string& hash, int64_t index) {
    const H32 h = h32_hex(hash);
    Op36 k;
    std::memcpy(k.data(), h.data(), 32);
    const uint32_t i = uint32_t(index);
    std::memcpy(k.data() + 32, &i, 4);
    return k;
}

// a decimal string ("0.000010", "12", "1e-5" is not produced by numeric()) in 1e-8 units
int64_t fee_units(const std::string& s) {
    int64_t whole = 0, frac = 0;
    int nfrac = 0;
    bool dot = false, neg = false;
    size_t i = 0;
    if (i < s.size() && (s[i] == '-' || s[i] == '+')) neg = s[i++] == '-';
    for (; i < s.size(); ++i) {
        const char c = s[i];
        if (c == '.') {
            if (dot) throw std::invalid_argument("bad fee");
            dot = true;
        } else if (c >= '0' && c <= '9') {
            if (!dot) {
                whole = whole * 10 + (c - '0');
                if (whole > (int64_t(1) << 40)) throw std::invalid_argument("fee too large");
            } else if (nfrac < 8) {
                frac = frac * 10 + (c - '0');
                ++nfrac;
            } else if (c != '0') {
                throw std::invalid_argument("fee with more than 8 decimals");
            }
        } else {
            throw std::invalid_argument("bad fee");
        }
    }
    while (nfrac < 8) {
        frac *= 10;
        ++nfrac;
    }
    const int64_t v = whole * 100000000 + frac;
    return neg ? -v : v;
}

// Writer-preferring reader/writer lock (std::shared_mutex is glibc's reader-preferring rwlock: a steady
// stream of overlapping lookups could starve a block's confirm). A waiting writer stops new readers.
class RwLock {
public:
    bool try_lock_shared() {
        std::lock_guard<std::mutex> g(m_);
        if (writer_ || waiting_) return false;
        ++readers_;
        return true;
    }
    void lock_shared() {
        std::unique_lock<std::mutex> g(m_);
        cv_.wait(g, [&] { return !writer_ && !waiting_; });
        ++readers_;
    }
    void unlock_shared() {
        std::lock_guard<std::mutex> g(m_);
        if (--readers_ == 0) cv_.notify_all();
    }
    bool try_lock() {
        std::lock_guard<std::mutex> g(m_);
        if (writer_ || readers_) return false;
        writer_ = true;
        return true;
    }
    void lock() {
        std::unique_lock<std::mutex> g(m_);
        ++waiting_;
        cv_.wait(g, [&] { return !writer_ && readers_ == 0; });
        --waiting_;
        writer_ = true;
    }
    void unlock() {
        std::lock_guard<std::mutex> g(m_);
        writer_ = false;
        cv_.notify_all();
    }

private:
    std::mutex m_;
    std::condition_variable cv_;
    int readers_ = 0, waiting_ = 0;
    bool writer_ = false;
};

// Acquire the index lock from a thread that holds the GIL: an uncontended acquire keeps the GIL; a
// contended one waits with the GIL released (the holder may need the GIL to finish).
template <class Lock>
struct GilSafe {
    Lock lk;
    explicit GilSafe(RwLock& m) : lk(m, std::try_to_lock) {
        if (!lk.owns_lock()) {
            py::gil_scoped_release nogil;
            lk.lock();
        }
    }
};
using Shared = GilSafe<std::shared_lock<RwLock>>;
using Exclusive = GilSafe<std::unique_lock<RwLock>>;

struct Entry {
    int64_t ptime = 0;
    int64_t seq = 0;    // journal sequence of the admission's batch (0: loaded from SQL)
    uint64_t order = 0;  // admission order (the table's row order)
    int64_t fee = 0;     // 1e-8 units
    py::object hex;      // the tx hex str (kept as the object the caller gave: no copy out)
    const char* hp = nullptr;  // its UTF-8 bytes (owned by `hex`): ordering reads them without the GIL
    int64_t len = 0;
};

class MempoolIndex {
public:
    MempoolIndex() = default;
    ~MempoolIndex() {
        py::gil_scoped_acquire g;  // entries hold Python references
        txs_.clear();
    }

    void load(py::list tx_rows, py::list spent_rows) {
        Exclusive g(mu_);
        for (auto r : tx_rows) {
            py::tuple t = r.cast<py::tuple>();
            add_entry(h32_hex(t[0].cast<std::string>()), t[1].cast<int64_t>(), t[2], py::str(t[3]).cast<std::string>(), 0);
        }
        for (auto r : spent_rows) {
            py::tuple t = r.cast<py::tuple>();
            spent_.insert(op_key(t[0].cast<std::string>(), t[1].cast<int64_t>()));
        }
    }

    bool empty() const {
        Shared g(mu_);
        return txs_.empty() && spent_.empty();
    }
    size_t size() const {
        Shared g(mu_);
        return txs_.size();
    }
    size_t spent_size() const {
        Shared g(mu_);
        return spent_.size();
    }
    bool has_tx(const std::string& h) const {
        const H32 k = h32_hex(h);
        Shared g(mu_);
        return txs_.count(k) != 0;
    }

    py::list spent_of(py::iterable outputs) const {
        // keys parsed first (Python objects, GIL), then one probe pass under the lock
        std::vector<std::pair<py::object, int64_t>> items;
        std::vector<Op36> keys;
        std::unordered_set<Op36, HHash> seen;
        for (auto o : outputs) {
            py::tuple t = o.cast<py::tuple>();
            const int64_t i = t[1].cast<int64_t>();
            const Op36 k = op_key(t[0].cast<std::string>(), i);
            if (!seen.insert(k).second) continue;
            items.emplace_back(py::reinterpret_borrow<py::object>(t[0]), i);
            keys.push_back(k);
        }
        std::vector<char> hit(keys.size(), 0);
        {
            Shared g(mu_);
            for (size_t j = 0; j < keys.size(); ++j) hit[j] = spent_.count(keys[j]) != 0;
        }
        py::list out;
        for (size_t j = 0; j < keys.size(); ++j)
            if (hit[j]) out.append(py::make_tuple(items[j].first, items[j].second));
        return out;
    }

    // (tx hex, raw hash) in block-template order, up to `limit` hex characters in total
    py::list ordered(int64_t limit) const {
        std::vector<std::pair<const H32*, const Entry*>> v;
        py::gil_scoped_release nogil;
        std::shared_lock<RwLock> g(mu_);  // held until the result is built: entries stay put
        v = select(limit);
        py::gil_scoped_acquire gil;
        py::list out;
        for (auto& p : v)
            out.append(py::make_tuple(p.second->hex, py::bytes(reinterpret_cast<const char*>(p.first->data()), 32)));
        return out;
    }

    // the mining template of /get_mining_info and the new-block event (reference main.py:675-695): the
    // selected txs re-sorted by hex string; returns (first `head` hexes, all tx hashes as hex strs, the
    // same hashes as one JSON array body `"h0","h1",...` for the response, count). Selection, sorts and
    // text run without the GIL under the shared lock; only the result objects need the GIL.
    py::tuple mining_template(int64_t limit, int64_t head) const {
        std::vector<std::pair<const H32*, const Entry*>> v;
        std::string frag, hx;
        py::gil_scoped_release nogil;
        std::shared_lock<RwLock> g(mu_);  // held until the result is built: entries stay put
        {
            v = select(limit);
            std::sort(v.begin(), v.end(), [](const auto& a, const auto& b) { return hex_less(*a.second, *b.second); });
            static const char* digits = "0123456789abcdef";
            hx.resize(v.size() * 64);
            frag.reserve(v.size() * 67);
            for (size_t k = 0; k < v.size(); ++k) {
                const uint8_t* d = v[k].first->data();
                char* h = &hx[k * 64];
                for (int j = 0; j < 32; ++j) {
                    h[2 * j] = digits[d[j] >> 4];
                    h[2 * j + 1] = digits[d[j] & 15];
                }
                if (k) frag.push_back(',');
                frag.push_back('"');
                frag.append(h, 64);
                frag.push_back('"');
            }
        }
        py::gil_scoped_acquire gil;
        py::list first, hashes;
        for (size_t k = 0; k < v.size(); ++k) {
            if (int64_t(k) < head) first.append(v[k].second->hex);
            hashes.append(py::str(hx.data() + k * 64, 64));
        }
        return py::make_tuple(first, hashes, py::bytes(frag), v.size());
    }

    // tx hex of the pending txs among `hashes` (hex strings; malformed ones ignored), in admission order
    py::list hex_in_order(py::iterable hashes) const {
        std::vector<const Entry*> hit;
        std::vector<H32> keys;
        std::unordered_set<H32, HHash> seen;
        for (auto h : hashes) {
            H32 k;
            try {
                k = h32_hex(h.cast<std::string>());
            } catch (const std::exception&) {
                continue;
            }
            if (seen.insert(k).second) keys.push_back(k);
        }
        Shared g(mu_);
        for (auto& k : keys) {
            auto it = txs_.find(k);
            if (it != txs_.end()) hit.push_back(&it->second);
        }
        std::sort(hit.begin(), hit.end(), [](const Entry* a, const Entry* b) { return a->order < b->order; });
        py::list out;
        for (auto* e : hit) out.append(e->hex);
        return out;
    }

    // reserve a tx and its inputs: None, 'duplicate' or 'double spend'
    py::object try_add(const std::string& tx_hash, int64_t ptime, py::list inputs, py::object tx_hex, py::object fees) {
        const H32 h = h32_hex(tx_hash);
        std::vector<Op36> keys;
        keys.reserve(inputs.size());
        for (auto in : inputs) {
            py::tuple t = in.cast<py::tuple>();
            keys.push_back(op_key(t[0].cast<std::string>(), t[1].cast<int64_t>()));
        }
        const std::string fee_text = py::str(fees).cast<std::string>();
        Exclusive g(mu_);
        if (txs_.count(h)) return py::str("duplicate");
        for (auto& k : keys)
            if (spent_.count(k)) return py::str("double spend");
        add_entry(h, ptime, tx_hex, fee_text, 0);
        for (auto& k : keys) spent_.insert(k);
        return py::none();
    }

    void set_seq(const std::string& tx_hash, py::list inputs, int64_t seq) {
        const H32 h = h32_hex(tx_hash);
        std::vector<Op36> keys;
        for (auto in : inputs) {
            py::tuple t = in.cast<py::tuple>();
            keys.push_back(op_key(t[0].cast<std::string>(), t[1].cast<int64_t>()));
        }
        Exclusive g(mu_);
        auto it = txs_.find(h);
        if (it != txs_.end()) it->second.seq = seq;
        for (auto& k : keys) spent_seq_[k] = seq;
    }

    // a committed block's txs (n x 32 raw) and spent outpoints (n x >= 36 records) leave the index; returns
    // the hits (raw bytes) and those whose admission was journaled after sequence `after` (None: none late)
    py::tuple confirm_raw(py::buffer txids_b, py::buffer in_keys_b, py::object after) {
        const py::buffer_info ti = txids_b.request(), ki = in_keys_b.request();
        const size_t tbytes = size_t(ti.size * ti.itemsize), kbytes = size_t(ki.size * ki.itemsize);
        const size_t kw = ki.ndim == 2 ? size_t(ki.shape[1]) * size_t(ki.itemsize) : 40;
        if (tbytes % 32) throw std::invalid_argument("txids must be n x 32 bytes");
        if (kw < 36 || (kbytes && kbytes % kw)) throw std::invalid_argument("input keys must be n x >= 36 bytes");
        const uint8_t* tp = static_cast<const uint8_t*>(ti.ptr);
        const uint8_t* kp = static_cast<const uint8_t*>(ki.ptr);
        const size_t nt = tbytes / 32, nk = kw ? kbytes / kw : 0;
        const bool have_after = !after.is_none();
        const int64_t aft = have_after ? after.cast<int64_t>() : 0;
        std::vector<H32> hit_tx, late_tx;
        std::vector<Op36> hit_in, late_in;
        std::vector<py::object> dropped;  // Python refs released with the GIL held
        {
            py::gil_scoped_release nogil;
            std::unique_lock<RwLock> g(mu_);  // dropped before the GIL is taken back
            if (!txs_.empty()) {
                for (size_t i = 0; i < nt; ++i) {
                    H32 k;
                    std::memcpy(k.data(), tp + 32 * i, 32);
                    auto it = txs_.find(k);
                    if (it == txs_.end()) continue;
                    hit_tx.push_back(k);
                    if (have_after && it->second.seq > aft) late_tx.push_back(k);
                    dropped.push_back(std::move(it->second.hex));
                    txs_.erase(it);
                }
            }
            if (!spent_.empty()) {
                for (size_t i = 0; i < nk; ++i) {
                    Op36 k;
                    std::memcpy(k.data(), kp + kw * i, 36);
                    if (!spent_.erase(k)) continue;
                    hit_in.push_back(k);
                    auto s = spent_seq_.find(k);
                    const int64_t sq = s == spent_seq_.end() ? 0 : s->second;
                    if (s != spent_seq_.end()) spent_seq_.erase(s);
                    if (have_after && sq > aft) late_in.push_back(k);
                }
            }
            if (txs_.empty()) min_ptime_valid_ = false;
        }
        dropped.clear();
        return py::make_tuple(rows(hit_tx), rows(hit_in), rows(late_tx), rows(late_in));
    }

    bool maybe_stale(int64_t now, int64_t delta) {
        Exclusive g(mu_);
        if (!min_ptime_valid_ || now - min_ptime_ <= delta) return false;
        recompute_min();
        return min_ptime_valid_ && now - min_ptime_ > delta;
    }

private:
    // block-template order: fee density (exact cross-multiplication), then length, then hex; cut at `limit`
    std::vector<std::pair<const H32*, const Entry*>> select(int64_t limit) const {
        std::vector<std::pair<const H32*, const Entry*>> v;
        v.reserve(txs_.size());
        for (auto& kv : txs_) v.emplace_back(&kv.first, &kv.second);
        std::sort(v.begin(), v.end(), [](const auto& a, const auto& b) {
            const Entry& x = *a.second;
            const Entry& y = *b.second;
            const __int128 l = __int128(x.fee) * y.len, r = __int128(y.fee) * x.len;
            if (l != r) return l > r;  // higher fee density first
            if (x.len != y.len) return x.len < y.len;
            return hex_less(x, y);
        });
        int64_t size = 0;
        size_t n = 0;
        for (; n < v.size(); ++n) {
            if (size + v[n].second->len > limit) break;
            size += v[n].second->len;
        }
        v.resize(n);
        return v;
    }

    // tx hex strings are ASCII: UTF-8 length == character length
    static bool hex_less(const Entry& a, const Entry& b) {
        const int c = std::memcmp(a.hp, b.hp, size_t(std::min(a.len, b.len)));
        return c < 0 || (c == 0 && a.len < b.len);
    }

    void add_entry(const H32& h, int64_t ptime, py::object hex, const std::string& fees, int64_t seq) {
        Entry e;
        e.ptime = ptime;
        e.seq = seq;
        e.order = next_order_++;
        e.fee = fee_units(fees);
        Py_ssize_t n = 0;
        const char* hp = PyUnicode_Check(hex.ptr()) ? PyUnicode_AsUTF8AndSize(hex.ptr(), &n) : nullptr;
        if (!hp) throw std::invalid_argument("tx hex must be str");
        e.hp = hp;
        e.len = int64_t(PyUnicode_GET_LENGTH(hex.ptr()));
        e.hex = std::move(hex);
        txs_[h] = std::move(e);
        if (!min_ptime_valid_ || ptime < min_ptime_) {
            min_ptime_ = ptime;
            min_ptime_valid_ = true;
        }
    }

    void recompute_min() {
        min_ptime_valid_ = !txs_.empty();
        if (!min_ptime_valid_) return;
        min_ptime_ = INT64_MAX;
        for (auto& kv : txs_) min_ptime_ = std::min(min_ptime_, kv.second.ptime);
    }

    template <class K>
    static py::list rows(const std::vector<K>& v) {
        py::list out(v.size());
        for (size_t i = 0; i < v.size(); ++i) out[i] = py::bytes(reinterpret_cast<const char*>(v[i].data()), v[i].size());
        return out;
    }

    mutable RwLock mu_;
    std::unordered_map<H32, Entry, HHash> txs_;
    std::unordered_set<Op36, HHash> spent_;
    std::unordered_map<Op36, int64_t, HHash> spent_seq_;
    uint64_t next_order_ = 0;
    int64_t min_ptime_ = 0;
    bool min_ptime_valid_ = false;
};

}  // namespace

void register_mempool_index(py::module_& m) {
    py::class_<MempoolIndex>(m, "MempoolIndexCore")
        .def(py::init<>())
        .def("load", &MempoolIndex::load)
        .def("empty", &MempoolIndex::empty)
        .def("__len__", &MempoolIndex::size)
        .def("spent_count", &MempoolIndex::spent_size)
        .def("has_tx", &MempoolIndex::has_tx)
        .def("spent_of", &MempoolIndex::spent_of)
        .def("ordered", &MempoolIndex::ordered)
        .def("hex_in_order", &MempoolIndex::hex_in_order)
        .def("mining_template", &MempoolIndex::mining_template)
        .def("try_add", &MempoolIndex::try_add)
        .def("set_seq", &MempoolIndex::set_seq)
        .def("confirm_raw", &MempoolIndex::confirm_raw, py::arg("txids"), py::arg("in_keys"), py::arg("after") = py::none())
        .def("maybe_stale", &MempoolIndex::maybe_stale);
}

}  // namespace upow
