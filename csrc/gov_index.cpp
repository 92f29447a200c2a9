// Governance store: the six governance tables and the staked rows of unspent_outputs in host memory, the
// emission cascade as exact decimal running sums, and the native block path's governance rule check and
// apply.
//
// reference: every governance question is SQL against PostgreSQL — registrations, stakes, voting power and
// ballots (upow/database.py:939-1436), the nine per-tx rule checks of upow/upow_transactions/transaction.py
// :240-479, and the per-block emission cascade get_active_inodes -> inode power -> validator stake ->
// delegate stake (database.py:1127-1136, 1189-1205, 1377-1426), recomputed from scratch for every block.
// Here (driven by upow_amd/ledger/governance.py and ledger/govcheck.py):
//
//   tables     rows keyed by the 36-byte outpoint (txid || u32 index) with the columns the reference's
//              joins read: address, amount (outputs_amounts[index]), voter (inputs_addresses[index]) and the
//              block timestamp; indexed by address string, voter string, and by the POINT an address denotes
//              (33-byte normalised compressed key: both string forms of an address at once, no sqrt)
//   cascade    stake(D) = sum amount/1e8; vstake(V) = round_up(sum vote*stake(voter)/10);
//              ipower(I) = round_up(sum vote*vstake(voter)/10) — running sums over exact 28-digit decimals
//              (int128 coefficient + exponent) that reproduce Python's Decimal values AND exponents, updated
//              per row change along the dependency edges; anything that would round is reported as
//              "unknown" and the caller recomputes it sequentially the reference's way
//   check      one call validates every governance tx of a block against the pre-block state
//   apply      one call inserts a block's governance/stake outputs and removes its governance spends
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <map>
#include <optional>
#include <string>
#include <string_view>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "native.h"

namespace py = pybind11;

namespace upow {
namespace {

using Key = std::array<uint8_t, 36>;
using Pt = std::array<uint8_t, 33>;

struct KHash {
    size_t operator()(const Key& k) const noexcept {
        uint64_t a, b;
        std::memcpy(&a, k.data(), 8);
        std::memcpy(&b, k.data() + 28, 8);
        return size_t(a ^ (b * 0x9E3779B97F4A7C15ull));
    }
};
struct PHash {
    size_t operator()(const Pt& k) const noexcept {
        uint64_t a, b;
        std::memcpy(&a, k.data() + 1, 8);
        std::memcpy(&b, k.data() + 25, 8);
        return size_t(a ^ (b * 0x9E3779B97F4A7C15ull) ^ k[0]);
    }
};

const Pt kNoPt{};  // "no point" (an unparseable address): Python's point_key None

// table ids: governance.GOV_TABLES order, then the staked rows of unspent_outputs
enum Tid { INODE = 0, VALIDATOR = 1, VVP = 2, DVP = 3, VBALLOT = 4, IBALLOT = 5, STAKE = 6, NT = 7 };
enum : uint8_t { HAS_ADDR = 1, HAS_AMOUNT = 2, HAS_VOTER = 4, HAS_TS = 8 };

struct Row {
    std::string addr, voter;
    int64_t amount = 0, ts = 0;
    uint64_t seq = 0;
    Pt pt{}, vpt{};
    uint8_t f = 0;
    uint8_t term = 0;  // ballots: 0 no term in its receiver's sum, 1 unknown (sum marked bad), 2 term_c/term_e
    int8_t term_e = 0;
    __int128 term_c = 0;
};

using KeySet = std::unordered_set<Key, KHash>;

struct Table {
    std::unordered_map<Key, Row, KHash> rows;
    std::unordered_map<std::string, KeySet> by_addr, by_voter;
    std::unordered_map<Pt, KeySet, PHash> by_pt, by_vpt;
    uint64_t next_seq = 0;
};

// ------------------------------------------------------------------------------------------ exact decimal
typedef __int128 i128;

i128 p10(int k) {
    static const std::array<i128, 39> t = [] {
        std::array<i128, 39> a{};
        a[0] = 1;
        for (int i = 1; i < 39; ++i) a[i] = a[i - 1] * 10;
        return a;
    }();
    return t[size_t(k)];
}
inline i128 iabs(i128 x) { return x < 0 ? -x : x; }
const int kPrec = 28;

// division and remainder by a positive power of ten: 64-bit instructions when both fit (the common case
// for amounts and votes), the 128-bit library routine otherwise
inline bool small(i128 x) { return x >= INT64_MIN && x <= INT64_MAX; }
inline i128 qdiv(i128 a, i128 m) { return small(a) && small(m) ? i128(int64_t(a) / int64_t(m)) : a / m; }
inline i128 qmod(i128 a, i128 m) { return small(a) && small(m) ? i128(int64_t(a) % int64_t(m)) : a % m; }

struct Dec {
    i128 c = 0;
    int e = 0;
};
inline bool fits(i128 c) { return iabs(c) < p10(kPrec); }
// c * 10^k still within 28 digits (checked before multiplying: no 128-bit overflow)
inline bool scale_fits(i128 c, int k) { return k >= 0 && k <= kPrec && iabs(c) < p10(kPrec - k); }

// Decimal(amount) / SMALLEST (1e8): the exact quotient at the exponent closest to the ideal 0
Dec from_amount(int64_t a) {
    if (a == 0) return Dec{0, 0};
    int64_t c = a;
    int t = 0;
    while (t < 8 && c % 10 == 0) {
        c /= 10;
        ++t;
    }
    return Dec{i128(c), -(8 - t)};
}

bool mul(const Dec& a, const Dec& b, Dec& out) {
    i128 c;
    if (__builtin_mul_overflow(a.c, b.c, &c) || !fits(c)) return false;  // more than 28 digits: Python rounds
    out = {c, a.e + b.e};
    return true;
}

// x / 10 (Decimal(10)): exact, at the ideal exponent x.e when the coefficient allows
Dec div10(const Dec& a) { return qmod(a.c, 10) == 0 ? Dec{qdiv(a.c, 10), a.e} : Dec{a.c, a.e - 1}; }

bool add(const Dec& a, const Dec& b, int sign, Dec& out) {
    const int e = std::min(a.e, b.e);
    const int da = a.e - e, db = b.e - e;
    if (!scale_fits(a.c, da) || !scale_fits(b.c, db)) return false;
    const i128 ac = a.c * p10(da), bc = b.c * p10(db);
    const i128 c = sign > 0 ? ac + bc : ac - bc;
    if (!fits(c)) return false;
    out = {c, e};
    return true;
}

bool quantize_exact(const Dec& a, int e, Dec& out) {
    if (e < a.e) {
        if (!scale_fits(a.c, a.e - e)) return false;
        out = {a.c * p10(a.e - e), e};
        return true;
    }
    if (e - a.e > 38) return false;
    const i128 m = p10(e - a.e);
    if (qmod(a.c, m) != 0) return false;
    out = {qdiv(a.c, m), e};
    return true;
}

// round_up_decimal (helpers.py:147-157): quantize to 1e-8 (ROUND_HALF_EVEN) only when digits lie beyond it
Dec round_up(const Dec& d) {
    if (d.e >= -8) return d;
    const int k = -8 - d.e;
    if (k > 38) return Dec{0, -8};
    const i128 m = p10(k);
    const i128 r = qmod(d.c, m);
    if (r == 0) return d;
    i128 q = qdiv(d.c, m);
    const i128 twice = 2 * iabs(r);
    if (twice > m || (twice == m && (q % 2 != 0))) q += d.c < 0 ? -1 : 1;
    return Dec{q, -8};
}

py::object dec_py(const Dec& d) {
    // (sign, digits, exponent) for decimal.Decimal(tuple): value and exponent preserved exactly
    i128 c = iabs(d.c);
    std::string digits;
    if (c == 0) digits = "0";
    while (c) {
        digits.push_back(char('0' + int(c % 10)));
        c /= 10;
    }
    std::reverse(digits.begin(), digits.end());
    py::tuple dt(digits.size());
    for (size_t i = 0; i < digits.size(); ++i) dt[i] = py::int_(digits[i] - '0');
    return py::make_tuple(d.c < 0 ? 1 : 0, dt, d.e);
}

struct XSum {  // sum(terms, Decimal(0)) under additions and removals, exact or not ok
    static constexpr int kLo = -56, kN = 64;  // term exponents kept: [-56, 7]
    Dec v;
    int32_t cnt[kN] = {};  // live terms per exponent (the result's exponent is min(0, smallest live one))
    bool ok = true;
    void update(const Dec& t, int sign) {
        if (!ok) return;
        Dec r;
        if (t.e < kLo || t.e >= kLo + kN || !add(v, t, sign, r)) {
            ok = false;
            return;
        }
        v = r;
        cnt[t.e - kLo] += sign;
    }
    bool result(Dec& out) const {
        if (!ok) return false;
        for (int i = 0; i < kN; ++i)
            if (cnt[i]) return quantize_exact(v, std::min(0, i + kLo), out);
        out = Dec{0, 0};
        return true;
    }
};

// ------------------------------------------------------------------------------------------ address codec
std::string hex_of(const uint8_t* p, size_t n) {
    static const char* hx = "0123456789abcdef";
    std::string s(2 * n, '0');
    for (size_t i = 0; i < n; ++i) {
        s[2 * i] = hx[p[i] >> 4];
        s[2 * i + 1] = hx[p[i] & 15];
    }
    return s;
}

bool point_key(const uint8_t* raw, size_t len, Pt& out) {
    if (len == 33) {
        out[0] = raw[0] == 43 ? 43 : 42;
        std::memcpy(out.data() + 1, raw + 1, 32);
        return true;
    }
    if (len == 64) {
        out[0] = (raw[32] & 1) ? 43 : 42;
        std::memcpy(out.data() + 1, raw, 32);
        return true;
    }
    return false;
}

int hexv(char c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
}

// string_to_bytes (helpers.py:183-188): hex first, then base58; false when only Python can say
bool string_to_bytes(const std::string& s, std::vector<uint8_t>& out) {
    bool hex = s.size() % 2 == 0;
    for (char c : s) {
        if (c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\v' || c == '\f') return false;
        if (hexv(c) < 0) hex = false;
    }
    out.clear();
    if (hex) {
        for (size_t i = 0; i < s.size(); i += 2) out.push_back(uint8_t(hexv(s[i]) << 4 | hexv(s[i + 1])));
        return true;
    }
    try {
        out = b58decode(s);
    } catch (...) {
        return false;
    }
    return true;
}

std::string b58_of_pt(const Pt& p) { return b58encode(p.data(), 33); }

// bytes_to_string (helpers.py:160-168): 64 B -> hex, 33 B -> base58 of the normalised prefix || x
std::string bytes_to_string(const uint8_t* raw, size_t len) {
    if (len == 64) return hex_of(raw, 64);
    uint8_t b[33];
    b[0] = raw[0] == 43 ? 43 : 42;
    std::memcpy(b + 1, raw + 1, 32);
    return b58encode(b, 33);
}

Key key_of(const uint8_t* txid32, uint32_t index) {
    Key k;
    std::memcpy(k.data(), txid32, 32);
    std::memcpy(k.data() + 32, &index, 4);
    return k;
}

template <class T>
const T* buf(const py::buffer& b, size_t n, const char* what) {
    py::buffer_info bi = b.request();
    if (size_t(bi.size * bi.itemsize) < n * sizeof(T)) throw std::invalid_argument(std::string("short buffer: ") + what);
    return static_cast<const T*>(bi.ptr);
}

constexpr int64_t S = 100000000;

// ------------------------------------------------------------------------------------------ store
class GovStore {
   public:
    GovStore() { build(); }

    // ---- rows
    // empty tables, cascade off until build() (bulk loads then build once)
    void clear() {
        for (auto& t : tabs_) t = Table();
        astake_.clear();
        vsum_.clear();
        isum_.clear();
        vval_.clear();
        bad_v_.clear();
        bad_i_.clear();
        pending_v_.clear();
        live_ = false;
    }

    // rows: list of (key36 bytes, address|None, amount|None, voter|None, ts|None, pt bytes|None, vpt bytes|None)
    void add_rows(int tid, py::list rows) {
        for (auto item : rows) {
            py::tuple r = item.cast<py::tuple>();
            std::string kb = r[0].cast<std::string>();
            if (kb.size() != 36) throw std::invalid_argument("key must be 36 bytes");
            Key k;
            std::memcpy(k.data(), kb.data(), 36);
            Row row;
            if (!r[1].is_none()) row.addr = r[1].cast<std::string>(), row.f |= HAS_ADDR;
            if (!r[2].is_none()) row.amount = r[2].cast<int64_t>(), row.f |= HAS_AMOUNT;
            if (!r[3].is_none()) row.voter = r[3].cast<std::string>(), row.f |= HAS_VOTER;
            if (!r[4].is_none()) row.ts = r[4].cast<int64_t>(), row.f |= HAS_TS;
            row.pt = pt_arg(r[5]);
            row.vpt = pt_arg(r[6]);
            insert(tid, k, std::move(row));
        }
    }

    int64_t remove_keys(int tid, py::bytes keys36) {
        std::string s = keys36;
        int64_t n = 0;
        for (size_t o = 0; o + 36 <= s.size(); o += 36) {
            Key k;
            std::memcpy(k.data(), s.data() + o, 36);
            n += erase(tid, k);
        }
        return n;
    }

    size_t count(int tid) const { return tabs_.at(size_t(tid)).rows.size(); }

    py::object row_py(const Key& k, const Row& r) const {
        return py::make_tuple(py::bytes(reinterpret_cast<const char*>(k.data()), 36),
                              (r.f & HAS_ADDR) ? py::object(py::str(r.addr)) : py::none(),
                              (r.f & HAS_AMOUNT) ? py::object(py::int_(r.amount)) : py::none(),
                              (r.f & HAS_VOTER) ? py::object(py::str(r.voter)) : py::none(),
                              (r.f & HAS_TS) ? py::object(py::int_(r.ts)) : py::none());
    }

    py::object get(int tid, py::bytes key36) const {
        std::string s = key36;
        if (s.size() != 36) return py::none();
        Key k;
        std::memcpy(k.data(), s.data(), 36);
        const Table& t = tabs_.at(size_t(tid));
        auto it = t.rows.find(k);
        return it == t.rows.end() ? py::none() : row_py(it->first, it->second);
    }

    // rows in insertion (rowid) order; ``keys``: None = the whole table
    py::list rows(int tid) const {
        const Table& t = tabs_.at(size_t(tid));
        std::vector<const std::pair<const Key, Row>*> v;
        v.reserve(t.rows.size());
        for (auto& kv : t.rows) v.push_back(&kv);
        std::sort(v.begin(), v.end(), [](auto* a, auto* b) { return a->second.seq < b->second.seq; });
        py::list out;
        for (auto* kv : v) out.append(row_py(kv->first, kv->second));
        return out;
    }

    // rows whose address (voter) string is one of ``values``, in rowid order
    py::list rows_by(int tid, py::list values, bool voter) const {
        const Table& t = tabs_.at(size_t(tid));
        const auto& idx = voter ? t.by_voter : t.by_addr;
        std::vector<const std::pair<const Key, Row>*> v;
        std::unordered_set<Key, KHash> seen;
        for (auto val : values) {
            if (val.is_none()) continue;
            auto it = idx.find(val.cast<std::string>());
            if (it == idx.end()) continue;
            for (auto& k : it->second)
                if (seen.insert(k).second) v.push_back(&*t.rows.find(k));
        }
        std::sort(v.begin(), v.end(), [](auto* a, auto* b) { return a->second.seq < b->second.seq; });
        py::list out;
        for (auto* kv : v) out.append(row_py(kv->first, kv->second));
        return out;
    }

    // keys (36 B each, concatenated) of rows whose address (voter) denotes point ``pt``
    py::bytes keys_by_point(int tid, py::bytes pt33, bool voter) const {
        Pt p = pt_arg(pt33);
        const Table& t = tabs_.at(size_t(tid));
        const auto& idx = voter ? t.by_vpt : t.by_pt;
        auto it = idx.find(p);
        std::string out;
        if (it != idx.end())
            for (auto& k : it->second) out.append(reinterpret_cast<const char*>(k.data()), 36);
        return py::bytes(out);
    }

    // ---- cascade results (None: recompute sequentially)
    py::object stake_py(py::object pt) {
        Dec d;
        if (!stake(pt_arg(pt), d)) return py::none();
        return dec_py(d);
    }
    py::object validator_stake_py(py::object pt) {
        flush();
        Dec d;
        if (!vstake(pt_arg(pt), d)) return py::none();
        return dec_py(d);
    }
    py::object inode_power_py(py::object pt) {
        flush();
        Pt p = pt_arg(pt);
        if (bad_i_.count(p)) return py::none();
        Dec d{0, 0};
        auto it = isum_.find(p);
        if (it != isum_.end() && !it->second.result(d)) return py::none();
        return dec_py(round_up(d));
    }

    void build() {
        astake_.clear();
        vsum_.clear();
        isum_.clear();
        vval_.clear();
        bad_v_.clear();
        bad_i_.clear();
        pending_v_.clear();
        live_ = false;
        for (auto& kv : tabs_[STAKE].rows) stake_row(kv.second, 1, false);
        for (auto* t : {&tabs_[VBALLOT], &tabs_[IBALLOT]})
            for (auto& kv : t->rows) kv.second.term = 0;
        for (auto& kv : tabs_[VBALLOT].rows) vballot(kv.second, 1, false);
        vval_.clear();
        for (auto& kv : tabs_[IBALLOT].rows) iballot(kv.second, 1);
        live_ = true;
    }

    // ---- block rule check (ledger/govcheck.py): 0 pass, 1 fail (object path), 2 needs the active inode
    //      lists (call again with them)
    py::tuple check_block(py::buffer tx_type_b, py::buffer out_type_b, py::buffer out_amount_b, py::buffer out_addr_b,
                          py::buffer out_len_b, py::buffer out_start_b, py::buffer in_start_b, py::buffer in_keys_b,
                          py::buffer pay_b, py::buffer txid_b, py::buffer gov_b, int64_t n, double now, bool syncing,
                          py::bytes pending_keys, py::set pending_stake_addrs, int64_t pending_votes,
                          py::object active_false, py::object active_true_count, int64_t max_inodes) {
        const uint8_t* tt = buf<uint8_t>(tx_type_b, size_t(n), "tx_type");
        const int32_t* os = buf<int32_t>(out_start_b, size_t(n) + 1, "out_start");
        const int32_t* is = buf<int32_t>(in_start_b, size_t(n) + 1, "in_start");
        const int64_t n_out = os[n], n_in = is[n];
        const uint8_t* ot = buf<uint8_t>(out_type_b, size_t(n_out), "out_type");
        const uint64_t* oa = buf<uint64_t>(out_amount_b, size_t(n_out), "out_amount");
        const uint8_t* oaddr = buf<uint8_t>(out_addr_b, size_t(n_out) * 64, "out_addr");
        const uint8_t* olen = buf<uint8_t>(out_len_b, size_t(n_out), "out_len");
        const uint8_t* ik = buf<uint8_t>(in_keys_b, size_t(n_in) * 40, "in_keys");
        const uint8_t* pay = buf<uint8_t>(pay_b, size_t(n_in) * 80, "payload");
        const uint8_t* txid = buf<uint8_t>(txid_b, size_t(n) * 32, "txid");
        const uint8_t* gov = buf<uint8_t>(gov_b, size_t(n), "gov mask");
        KeySet pend;
        {
            std::string s = pending_keys;
            for (size_t o = 0; o + 36 <= s.size(); o += 36) {
                Key k;
                std::memcpy(k.data(), s.data() + o, 36);
                pend.insert(k);
            }
        }
        std::unordered_set<std::string> pstake;
        for (auto a : pending_stake_addrs) pstake.insert(a.cast<std::string>());
        std::unordered_set<std::string> active_f;
        const bool have_active = !active_false.is_none();
        if (have_active)
            for (auto a : active_false.cast<py::list>()) active_f.insert(a.cast<std::string>());
        const int64_t active_t = active_true_count.is_none() ? -1 : active_true_count.cast<int64_t>();
        auto live = [&](int tid, const Pt& p, bool cp, bool voter) {
            const Table& t = tabs_[size_t(tid)];
            const auto& idx = voter ? t.by_vpt : t.by_pt;
            auto it = idx.find(p);
            if (it == idx.end() || it->second.empty()) return false;
            if (!cp || pend.empty()) return true;
            for (auto& k : it->second)
                if (!pend.count(k)) return true;
            return false;
        };
        auto delegate_power = [&](const Pt& p) { return live(DVP, p, false, false) || live(VBALLOT, p, false, true); };
        auto in_pay = [&](int64_t j, const uint8_t*& raw, uint32_t& len) {
            raw = pay + 80 * j + 16;
            std::memcpy(&len, pay + 80 * j + 8, 4);
        };
        py::dict signers;
        bool need_active = false;
        static const std::string kUnstakeException = "8befeb253bc6eddd8501f5b27a02b195f5c06a51ccf788213cbedafe7cc49c53";
        for (int64_t k = 0; k < n; ++k) {
            if (!gov[k]) continue;
            const int t = tt[k];
            const int64_t j0 = is[k];
            if (j0 >= is[k + 1]) return py::make_tuple(1, signers);
            const uint8_t* raw0;
            uint32_t len0;
            in_pay(j0, raw0, len0);
            Pt pt0;
            if (!point_key(raw0, len0, pt0)) return py::make_tuple(1, signers);
            int64_t sum[10] = {0}, cnt[10] = {0}, last[10];
            for (int q = 0; q < 10; ++q) last[q] = -1;
            for (int64_t o = os[k]; o < os[k + 1]; ++o) {
                const int ty = ot[o];
                if (ty > 9) return py::make_tuple(1, signers);
                sum[ty] += int64_t(oa[o]);
                ++cnt[ty];
                last[ty] = o;
            }
            auto out_pt = [&](int64_t o, Pt& p) { return o >= 0 && point_key(oaddr + 64 * o, olen[o], p); };
            if (cnt[1]) {  // stake (transaction.py:434-465)
                if (live(STAKE, pt0, false, false) && !syncing) return py::make_tuple(1, signers);
                if (pstake.count(bytes_to_string(raw0, len0))) return py::make_tuple(1, signers);
                if (sum[9] > 0) {
                    if (sum[9] != 10 * S || delegate_power(pt0)) return py::make_tuple(1, signers);
                } else if (!delegate_power(pt0)) {
                    return py::make_tuple(1, signers);
                }
            }
            if (cnt[2]) {  // unstake (transaction.py:467-479)
                if (live(VBALLOT, pt0, false, true) && hex_of(txid + 32 * k, 32) != kUnstakeException)
                    return py::make_tuple(1, signers);
                if (pending_votes) return py::make_tuple(1, signers);
            }
            if (t == 7) {  // vote as delegate (transaction.py:292-316; block validation: stake without mempool)
                Pt rp;
                if (sum[7] > 10 * S || sum[7] <= 0 || live(INODE, pt0, true, false) || !live(STAKE, pt0, false, false) ||
                    !out_pt(last[7], rp) || !live(VALIDATOR, rp, true, false))
                    return py::make_tuple(1, signers);
                continue;  // votes: no further rule applies (transaction.py verify order)
            } else if (t == 6) {  // vote as validator (transaction.py:258-290)
                Pt rp;
                if (sum[6] > 10 * S || sum[6] <= 0 || live(INODE, pt0, true, false) || !live(VALIDATOR, pt0, true, false) ||
                    !out_pt(last[6], rp) || !live(INODE, rp, true, false))
                    return py::make_tuple(1, signers);
                continue;
            } else if (t == 5) {  // validator registration (transaction.py:371-398)
                if (!live(STAKE, pt0, false, false) || live(VALIDATOR, pt0, true, false) || live(INODE, pt0, true, false) ||
                    sum[5] != 100 * S || cnt[8] != 1 || int64_t(oa[last[8]]) != 10 * S)
                    return py::make_tuple(1, signers);
            } else if (t == 8 || t == 9) {  // revokes (transaction.py:400-432): signed by each ballot's voter
                const Table& bt = tabs_[t == 8 ? IBALLOT : VBALLOT];
                bool valid = false;
                std::vector<uint8_t> vraw, first;
                for (int64_t j = is[k]; j < is[k + 1]; ++j) {
                    uint32_t idx;
                    std::memcpy(&idx, ik + 40 * j + 32, 4);
                    auto it = bt.rows.find(key_of(ik + 40 * j, idx));
                    if (it == bt.rows.end() || idx != 0 || !(it->second.f & HAS_VOTER) || !(it->second.f & HAS_TS))
                        return py::make_tuple(1, signers);
                    if (!string_to_bytes(it->second.voter, vraw) || (vraw.size() != 33 && vraw.size() != 64))
                        return py::make_tuple(1, signers);
                    signers[py::int_(j)] = py::bytes(reinterpret_cast<const char*>(vraw.data()), vraw.size());
                    if (j == is[k]) first = vraw;
                    valid = valid || now - double(it->second.ts) >= 48.0 * 3600.0;
                }
                Pt vp;
                if (!point_key(first.data(), first.size(), vp)) return py::make_tuple(1, signers);
                if (t == 8 && !live(VALIDATOR, vp, true, false)) return py::make_tuple(1, signers);
                if (!live(STAKE, vp, false, false) || !valid) return py::make_tuple(1, signers);
            }
            if (t == 4 || cnt[3]) {  // inode de-registration / registration: need the active inode lists
                if (!have_active || active_t < 0) {
                    need_active = true;
                    continue;
                }
                const std::string address = bytes_to_string(raw0, len0);
                if (t == 4) {
                    if (!live(INODE, pt0, false, false) || active_f.count(address)) return py::make_tuple(1, signers);
                }
                if (cnt[3]) {
                    if (sum[3] != 1000 * S || !live(STAKE, pt0, false, false) || live(INODE, pt0, true, false) ||
                        live(VALIDATOR, pt0, true, false) || active_t >= max_inodes || active_f.count(address))
                        return py::make_tuple(1, signers);
                }
            }
        }
        return py::make_tuple(need_active ? 2 : 0, signers);
    }

    // ---- block apply (native path): governance/stake outputs in, governance spends out
    // ``in_str``/``in_off``: each input's owner as the tx row's inputs_addresses column holds it (compressed
    // base58 of the spent output's address; txcodec input_address_strings(per_input=True))
    py::dict apply_block(py::buffer out_type_b, py::buffer txid_b, py::buffer out_tx_b, py::buffer out_start_b,
                         py::buffer out_amount_b, py::buffer out_addr_b, py::buffer out_len_b, py::buffer addr_blob,
                         py::buffer addr_off_b, py::buffer in_start_b, py::buffer pay_b, py::buffer in_keys_b,
                         py::buffer in_tag_b, py::buffer in_str, py::buffer in_off_b, int64_t n, int64_t block_ts) {
        const int32_t* os = buf<int32_t>(out_start_b, size_t(n) + 1, "out_start");
        const int32_t* is = buf<int32_t>(in_start_b, size_t(n) + 1, "in_start");
        const int64_t n_out = os[n], n_in = is[n];
        const uint8_t* ot = buf<uint8_t>(out_type_b, size_t(n_out), "out_type");
        const uint8_t* txid = buf<uint8_t>(txid_b, size_t(n) * 32, "txid");
        const int32_t* otx = buf<int32_t>(out_tx_b, size_t(n_out), "out_tx");
        const uint64_t* oa = buf<uint64_t>(out_amount_b, size_t(n_out), "out_amount");
        const uint8_t* oaddr = buf<uint8_t>(out_addr_b, size_t(n_out) * 64, "out_addr");
        const uint8_t* olen = buf<uint8_t>(out_len_b, size_t(n_out), "out_len");
        const int64_t* aoff = buf<int64_t>(addr_off_b, size_t(n_out) + 1, "address offsets");
        const uint8_t* pay = buf<uint8_t>(pay_b, size_t(n_in) * 80, "payload");
        const uint8_t* ik = buf<uint8_t>(in_keys_b, size_t(n_in) * 40, "in_keys");
        const uint8_t* itag = buf<uint8_t>(in_tag_b, size_t(n_in), "in_tag");
        const int64_t* ioff = buf<int64_t>(in_off_b, size_t(n_in) + 1, "input string offsets");
        const py::buffer_info bbi = addr_blob.request(), sbi = in_str.request();
        const std::string_view blob(static_cast<const char*>(bbi.ptr), size_t(bbi.size * bbi.itemsize));
        const std::string_view istr(static_cast<const char*>(sbi.ptr), size_t(sbi.size * sbi.itemsize));
        if (ioff[n_in] > int64_t(istr.size())) throw std::invalid_argument("input strings: offsets past the blob");
        if (n_out && aoff[n_out] > int64_t(blob.size())) throw std::invalid_argument("addresses: offsets past the blob");
        // pure C++ from here (the caller holds the index lock; the buffers stay alive for the call)
        std::optional<py::gil_scoped_release> nogil;
        nogil.emplace();
        // spends leave their tables (UTXO tags: 0 unspent_outputs -> staked rows, 1..6 governance tables)
        static const int kTagTid[7] = {STAKE, INODE, VALIDATOR, VVP, DVP, VBALLOT, IBALLOT};
        int64_t removed = 0, added = 0;
        for (int64_t j = 0; j < n_in; ++j) {
            const int tag = itag[j];
            if (tag > 6) continue;
            uint32_t flags;
            std::memcpy(&flags, pay + 80 * j + 12, 4);
            if (tag == 0 && !(flags & 1)) continue;  // an unstaked output: not in the stake table
            uint32_t idx;
            std::memcpy(&idx, ik + 40 * j + 32, 4);
            removed += erase(kTagTid[tag], key_of(ik + 40 * j, idx));
        }
        // outputs land in their tables (output type -> table), in block order (= rowid order)
        static const int kTypeTid[10] = {-1, STAKE, -1, INODE, -1, VALIDATOR, IBALLOT, VBALLOT, VVP, DVP};
        for (int64_t o = 0; o < n_out; ++o) {
            const int ty = ot[o];
            const int tid = ty < 10 ? kTypeTid[ty] : -1;
            if (tid < 0) continue;
            const int64_t k = otx[o];
            const uint32_t index = uint32_t(o - os[k]);
            Row row;
            row.addr.assign(blob.data() + aoff[o], size_t(aoff[o + 1] - aoff[o]));
            row.f |= HAS_ADDR | HAS_AMOUNT | HAS_TS;
            row.amount = int64_t(oa[o]);
            row.ts = block_ts;
            if (!point_key(oaddr + 64 * o, olen[o], row.pt)) row.pt = kNoPt;
            // voter = inputs_addresses[index] of the creating tx (the reference's subscript): the compressed
            // base58 of that input's spent-output owner, as the tx row's inputs_addresses column holds it
            const int64_t j = is[k] + int64_t(index);
            if (j < is[k + 1]) {
                uint32_t len;
                std::memcpy(&len, pay + 80 * j + 8, 4);
                Pt vp;
                if (point_key(pay + 80 * j + 16, len, vp)) {
                    row.vpt = vp;
                    row.voter.assign(istr.data() + ioff[j], size_t(ioff[j + 1] - ioff[j]));
                    row.f |= HAS_VOTER;
                }
            }
            insert(tid, key_of(txid + 32 * k, index), std::move(row));
            ++added;
        }
        nogil.reset();
        py::dict d;
        d["removed"] = removed;
        d["added"] = added;
        return d;
    }

   private:
    static Pt pt_arg(py::handle h) {
        if (h.is_none()) return kNoPt;
        std::string s = h.cast<std::string>();
        Pt p = kNoPt;
        if (s.size() == 33) std::memcpy(p.data(), s.data(), 33);
        return p;
    }

    void index_add(Table& t, const Key& k, const Row& r) {
        if (r.f & HAS_ADDR) t.by_addr[r.addr].insert(k);
        if (r.f & HAS_VOTER) t.by_voter[r.voter].insert(k);
        t.by_pt[r.pt].insert(k);
        t.by_vpt[r.vpt].insert(k);
    }

    template <class M, class K>
    static void index_del(M& m, const K& key, const Key& k) {
        auto it = m.find(key);
        if (it == m.end()) return;
        it->second.erase(k);
        if (it->second.empty()) m.erase(it);
    }

    void insert(int tid, const Key& k, Row&& row) {
        Table& t = tabs_.at(size_t(tid));
        if (t.rows.count(k)) erase(tid, k);
        row.seq = t.next_seq++;
        auto& ref = t.rows.emplace(k, std::move(row)).first->second;
        index_add(t, k, ref);
        if (live_) changed(tid, ref, 1);
    }

    int erase(int tid, const Key& k) {
        Table& t = tabs_.at(size_t(tid));
        auto it = t.rows.find(k);
        if (it == t.rows.end()) return 0;
        if (live_) changed(tid, it->second, -1);
        const Row& r = it->second;
        if (r.f & HAS_ADDR) index_del(t.by_addr, r.addr, k);
        if (r.f & HAS_VOTER) index_del(t.by_voter, r.voter, k);
        index_del(t.by_pt, r.pt, k);
        index_del(t.by_vpt, r.vpt, k);
        t.rows.erase(it);
        return 1;
    }

    // ---- cascade
    bool stake(const Pt& p, Dec& out) const {
        auto it = astake_.find(p);
        if (it == astake_.end()) {
            out = Dec{0, 0};
            return true;
        }
        return it->second.result(out);
    }

    bool vstake(const Pt& p, Dec& out) {
        if (bad_v_.count(p)) return false;
        auto c = vval_.find(p);
        if (c != vval_.end()) {
            out = c->second;
            return true;
        }
        Dec r{0, 0};
        auto it = vsum_.find(p);
        if (it != vsum_.end() && !it->second.result(r)) return false;
        out = vval_[p] = round_up(r);
        return true;
    }

    // a ballot's term vote * stake(voter) / 10 enters (sign > 0) or leaves its receiver's sum; the term is
    // kept on the row (the receiver is the row's own point, which never changes)
    static void set_term(Row& row, bool ok, const Dec& t) {
        row.term = ok ? 2 : 1;
        row.term_c = t.c;
        row.term_e = int8_t(t.e);
    }

    void vballot(Row& row, int sign, bool propagate) {
        const Pt& recv = row.pt;
        if (sign > 0) {
            Dec st, prod;
            bool ok = (row.f & HAS_AMOUNT) && (row.f & HAS_VOTER) && row.vpt != kNoPt && stake(row.vpt, st) &&
                      mul(from_amount(row.amount), st, prod);
            if (!ok) {
                bad_v_.insert(recv);
                set_term(row, false, Dec{});
            } else {
                const Dec term = div10(prod);
                vsum_[recv].update(term, 1);
                set_term(row, true, term);
            }
        } else if (row.term) {
            if (row.term == 2) vsum_[recv].update(Dec{row.term_c, row.term_e}, -1);
            row.term = 0;
        }
        if (propagate) {
            pending_v_.insert(recv);
            vval_.erase(recv);
        }
    }

    void iballot(Row& row, int sign) {
        const Pt& recv = row.pt;
        if (sign > 0) {
            Dec vs, prod;
            bool ok = (row.f & HAS_AMOUNT) && (row.f & HAS_VOTER) && row.vpt != kNoPt && vstake(row.vpt, vs) &&
                      mul(from_amount(row.amount), vs, prod);
            if (!ok) {
                bad_i_.insert(recv);
                set_term(row, false, Dec{});
            } else {
                const Dec term = div10(prod);
                isum_[recv].update(term, 1);
                set_term(row, true, term);
            }
        } else if (row.term) {
            if (row.term == 2) isum_[recv].update(Dec{row.term_c, row.term_e}, -1);
            row.term = 0;
        }
    }

    void stake_row(const Row& row, int sign, bool propagate) {
        XSum& s = astake_[row.pt];
        if (!(row.f & HAS_AMOUNT))
            s.ok = false;
        else
            s.update(from_amount(row.amount), sign);
        if (propagate) {  // re-term every ballot this delegate cast
            auto it = tabs_[VBALLOT].by_vpt.find(row.pt);
            if (it == tabs_[VBALLOT].by_vpt.end()) return;
            std::vector<Key> ks(it->second.begin(), it->second.end());
            for (auto& k : ks) {
                Row& r = tabs_[VBALLOT].rows.at(k);
                vballot(r, -1, false);
                vballot(r, 1, true);
            }
        }
    }

    void flush() {  // re-term the inode ballots of validators whose stake may have changed
        while (!pending_v_.empty()) {
            Pt p = *pending_v_.begin();
            pending_v_.erase(pending_v_.begin());
            auto it = tabs_[IBALLOT].by_vpt.find(p);
            if (it == tabs_[IBALLOT].by_vpt.end()) continue;
            std::vector<Key> ks(it->second.begin(), it->second.end());
            for (auto& k : ks) {
                Row& r = tabs_[IBALLOT].rows.at(k);
                iballot(r, -1);
                iballot(r, 1);
            }
        }
    }

    void changed(int tid, Row& row, int sign) {
        if (tid == STAKE)
            stake_row(row, sign, true);
        else if (tid == VBALLOT)
            vballot(row, sign, true);
        else if (tid == IBALLOT)
            iballot(row, sign);
    }

    std::array<Table, NT> tabs_;
    bool live_ = false;
    std::unordered_map<Pt, XSum, PHash> astake_, vsum_, isum_;
    std::unordered_map<Pt, Dec, PHash> vval_;
    std::unordered_set<Pt, PHash> bad_v_, bad_i_, pending_v_;
};

// ------------------------------------------------------------------------------- block column prep
constexpr uint8_t kOutValidatorVotingPower = 8, kOutDelegateVotingPower = 9;  // OutputType (helpers.py)
// The per-block column work of ledger/govcheck.py BlockGovernance on the native path, one pass each
// (numpy took ~0.5 ms per 2 MB block in unique/gather/compare/reduceat temporaries on the ledger thread).

// gov[t] = tx t is governance-relevant: a non-REGULAR tx type, or any output of a non-REGULAR type
py::tuple gov_block_mask(py::buffer tx_type_b, py::buffer out_type_b, py::buffer out_tx_b, int64_t n, int64_t n_out) {
    const uint8_t* tt = buf<uint8_t>(tx_type_b, size_t(n), "tx_type");
    const uint8_t* ot = buf<uint8_t>(out_type_b, size_t(n_out), "out_type");
    const int32_t* otx = buf<int32_t>(out_tx_b, size_t(n_out), "out_tx");
    std::string gov(size_t(n), '\0');
    bool any = false;
    for (int64_t t = 0; t < n; ++t)
        if (tt[t]) gov[size_t(t)] = 1, any = true;
    for (int64_t o = 0; o < n_out; ++o)
        if (ot[o]) {
            const int32_t t = otx[o];
            if (t < 0 || t >= n) throw std::invalid_argument("out_tx out of range");
            gov[size_t(t)] = 1;
            any = true;
        }
    return py::make_tuple(py::bytes(gov), any);
}

// After the UTXO pass: each input's expected table tag (spend_lut[tx type]), whether any input is not live in
// that table (tag mismatch or no payload), and get_fees (transaction.py:499-518): REGULAR txs keep
// inputs - outputs + their voting-power outputs, every other tx type has fee 0.
py::tuple gov_block_inputs(py::buffer tx_type_b, py::buffer in_tx_b, py::buffer tags_b, py::buffer pay_b,
                           py::buffer spend_lut_b, py::buffer out_type_b, py::buffer out_start_b, py::buffer out_amount_b,
                           py::buffer fee_b, int64_t n, int64_t n_in, int64_t n_out) {
    const uint8_t* tt = buf<uint8_t>(tx_type_b, size_t(n), "tx_type");
    const int32_t* itx = buf<int32_t>(in_tx_b, size_t(n_in), "in_tx");
    const uint8_t* tags = buf<uint8_t>(tags_b, size_t(n_in), "tags");
    const uint8_t* pay = buf<uint8_t>(pay_b, size_t(n_in) * 80, "payload");
    const uint8_t* lut = buf<uint8_t>(spend_lut_b, 256, "spend_lut");
    const uint8_t* ot = buf<uint8_t>(out_type_b, size_t(n_out), "out_type");
    const int32_t* os = buf<int32_t>(out_start_b, size_t(n) + 1, "out_start");
    const uint64_t* oa = buf<uint64_t>(out_amount_b, size_t(n_out), "out_amount");
    const int64_t* fee = buf<int64_t>(fee_b, size_t(n), "fee");
    if (os[n] != n_out) throw std::invalid_argument("out_start does not end at n_out");
    std::string in_tag(size_t(n_in), '\0');
    bool bad = false;
    for (int64_t j = 0; j < n_in; ++j) {
        const int32_t t = itx[j];
        if (t < 0 || t >= n) throw std::invalid_argument("in_tx out of range");
        const uint8_t want = lut[tt[t]];
        in_tag[size_t(j)] = char(want);
        uint32_t len;
        std::memcpy(&len, pay + 80 * j + 8, 4);
        bad |= tags[j] != want || len == 0;
    }
    std::string fout(size_t(n) * 8, '\0');
    int64_t* f = reinterpret_cast<int64_t*>(&fout[0]);
    for (int64_t t = 0; t < n; ++t) {
        if (tt[t]) {
            f[t] = 0;
            continue;
        }
        int64_t v = fee[t];
        for (int32_t o = os[t]; o < os[t + 1]; ++o)
            if (ot[o] == kOutValidatorVotingPower || ot[o] == kOutDelegateVotingPower) v += int64_t(oa[o]);
        f[t] = v;
    }
    return py::make_tuple(py::bytes(in_tag), bad, py::bytes(fout));
}

}  // namespace

void register_gov_index(py::module_& m) {
    py::class_<GovStore>(m, "GovStore")
        .def(py::init<>())
        .def("clear", &GovStore::clear)
        .def("add_rows", &GovStore::add_rows)
        .def("remove_keys", &GovStore::remove_keys)
        .def("count", &GovStore::count)
        .def("get", &GovStore::get)
        .def("rows", &GovStore::rows)
        .def("rows_by", &GovStore::rows_by, py::arg("tid"), py::arg("values"), py::arg("voter") = false)
        .def("keys_by_point", &GovStore::keys_by_point, py::arg("tid"), py::arg("pt"), py::arg("voter") = false)
        .def("stake", &GovStore::stake_py)
        .def("validator_stake", &GovStore::validator_stake_py)
        .def("inode_power", &GovStore::inode_power_py)
        .def("build", &GovStore::build)
        .def("check_block", &GovStore::check_block)
        .def("apply_block", &GovStore::apply_block);
    m.def("gov_block_mask", &gov_block_mask);
    m.def("gov_block_inputs", &gov_block_inputs);
}

}  // namespace upow
