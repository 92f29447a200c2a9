// Transaction decoder core, pure C++ (no Python): hex -> fields -> canonical bytes, txid, signed-message
// digest, address strings and JSON columns for ONE transaction (the reading rules of the reference parser,
// upow/upow_transactions/transaction.py:520-592). csrc/txcodec.cpp runs it over a block's txs on the host
// pool; tools/fuzz_txdecode.cpp feeds it mutated bytes under ASan + UBSan. Every read is bounds-checked
// (`need`); anything the fast path does not decide is flagged for the Python parser instead.
#pragma once

#include <array>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "native.h"
#include "sha256_common.h"

namespace upow {

enum TxFlag : uint8_t {
    TX_FAST = 0,      // fully decoded, regular outputs, 1-or-n signatures
    TX_GENERAL = 1,   // valid encoding the fast path does not handle
    TX_MALFORMED = 2,  // the Python parser has to see it (it raises or reads it leniently)
    TX_COINBASE = 3    // specifier 36 (sync pages carry the block's coinbase among its txs)
};

struct DecIn {
    uint8_t txid[32];
    uint8_t index, type;
    int32_t sig;  // index into the tx's unique-signature list
};
struct DecOut {
    uint8_t addr[64];
    uint8_t len;
    uint8_t type;
    uint64_t amount;
};
struct DecTx {
    uint8_t flag = TX_MALFORMED;
    uint8_t version = 0;
    bool canonical = false;
    bool upper_hex = false;  // the input used A-F digits (the stored hex must be re-rendered)
    bool grouped = false;    // 1 < k < n signatures: input i's signature is its owner key's group (ins[].sig = -1)
    int32_t msg_off = -1, msg_len = 0;  // into canon bytes
    uint8_t tx_type = 0;                // TransactionType from the message; kTypeAsk: Python decides
    int32_t signed_len = 0;             // hex(False) byte length (a prefix of canon)
    std::vector<DecIn> ins;
    std::vector<DecOut> outs;
    std::vector<uint8_t> sigs;  // unique signatures, 64 B each (r LE | s LE)
    std::vector<uint8_t> canon;
    uint8_t txid[32];
    uint8_t digest[32];
    std::vector<std::string> out_addr;  // bytes_to_string form; the first outs.size() entries are live
    std::string out_addr_json, out_amount_json;
    // back to the freshly-constructed state while keeping every buffer's capacity: a workspace's DecTx
    // objects are reused block after block, so the steady state decodes without touching malloc
    void reset() {
        flag = TX_MALFORMED;
        version = 0;
        canonical = upper_hex = grouped = false;
        msg_off = -1;
        msg_len = 0;
        tx_type = 0;
        signed_len = 0;
        ins.clear();
        outs.clear();
        sigs.clear();
        canon.clear();
        out_addr_json.clear();
        out_amount_json.clear();
    }
};

static inline int hexval(char c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
}

static const char kHex[] = "0123456789abcdef";

static void hex32(const uint8_t* b, char* out) {
    static const char hx[] = "0123456789abcdef";
    for (int i = 0; i < 32; ++i) {
        out[2 * i] = hx[b[i] >> 4];
        out[2 * i + 1] = hx[b[i] & 15];
    }
}

static std::string to_hex(const uint8_t* p, size_t n) {
    std::string s(2 * n, '0');
    for (size_t i = 0; i < n; ++i) {
        s[2 * i] = kHex[p[i] >> 4];
        s[2 * i + 1] = kHex[p[i] & 15];
    }
    return s;
}

// base58 of a 33-byte compressed address, memoised per thread in a direct-mapped table (blocks pay the
// same few addresses over and over: change outputs, exchanges, pools). Fixed-size slots: a lookup hashes
// the key's x bytes (uniform for curve points) and never allocates.
struct B58Slot {
    uint8_t key[33];
    uint8_t len = 0;  // 0 = empty
    char s[46];
};
static void b58_33(const uint8_t b[33], std::string& out) {
    constexpr size_t kSlots = 1u << 13;
    thread_local std::vector<B58Slot> cache(kSlots);
    uint64_t h;
    std::memcpy(&h, b + 1, 8);
    B58Slot& e = cache[size_t((h ^ b[0]) * 0x9E3779B97F4A7C15ull >> 51)];
    if (e.len && std::memcmp(e.key, b, 33) == 0) {
        out.assign(e.s, e.len);
        return;
    }
    char buf[kB58MaxOutput];
    const size_t len = b58encode_to(b, 33, buf);
    out.assign(buf, len);  // reuses the workspace string's buffer: no allocation per output
    if (len <= sizeof(e.s)) {
        std::memcpy(e.key, b, 33);
        std::memcpy(e.s, buf, len);
        e.len = uint8_t(len);
    }
}

// bytes_to_string (codec.py): 64 B -> hex, 33 B -> base58 of normalised prefix || x
static void addr_string(const uint8_t* a, int len, std::string& out) {
    if (len == 64) {
        out.resize(128);
        for (int i = 0; i < 64; ++i) {
            out[size_t(2 * i)] = kHex[a[i] >> 4];
            out[size_t(2 * i + 1)] = kHex[a[i] & 15];
        }
        return;
    }
    uint8_t b[33];
    b[0] = a[0] == 43 ? 43 : 42;
    std::memcpy(b + 1, a + 1, 32);
    b58_33(b, out);
}

// True when string_to_bytes(s) would take the bytes.fromhex branch (an all-hex base58 string of even
// length): the Python path would then misread the address, so leave such outputs to it.
static bool hex_ambiguous(const std::string& s) {
    if (s.size() % 2) return false;
    for (char c : s)
        if (hexval(c) < 0) return false;
    return true;
}

constexpr uint8_t kTypeAsk = 255;

// get_transaction_type_from_message (helpers.py:97-112): int(message.decode()) looked up among the
// TransactionType values 4-9, REGULAR otherwise. Decided here for the unambiguous encodings: all ASCII
// digits (leading zeros allowed), or ASCII without any digit (int() fails). A message that is not valid
// UTF-8 is rendered as hex first, whose integer value is never 4-9 (a byte >= 0x80 contributes an 8x/9x
// digit pair or an a-f digit). Anything else (signs, whitespace, underscores, non-ASCII digits...) is left
// to Python's int().
static uint8_t message_tx_type(const uint8_t* m, size_t n) {
    bool ascii = true, digits = n > 0, any_digit = false;
    for (size_t i = 0; i < n; ++i) {
        ascii &= m[i] < 0x80;
        const bool d = m[i] >= '0' && m[i] <= '9';
        digits &= d;
        any_digit |= d;
    }
    if (!ascii) {
        // valid UTF-8 with non-ASCII characters may hold Unicode digits: ask Python
        size_t i = 0;
        while (i < n) {
            const uint8_t c = m[i];
            const int len = c < 0x80 ? 1 : (c >> 5) == 6 ? 2 : (c >> 4) == 14 ? 3 : (c >> 3) == 30 ? 4 : 0;
            if (!len || i + size_t(len) > n) return 0;  // invalid UTF-8 -> hex rendering -> REGULAR
            for (int k = 1; k < len; ++k)
                if ((m[i + size_t(k)] >> 6) != 2) return 0;
            i += size_t(len);
        }
        return kTypeAsk;
    }
    if (digits) {
        uint32_t v = 0;
        for (size_t i = 0; i < n; ++i) {
            v = v * 10 + uint32_t(m[i] - '0');
            if (v > 1000) return 0;
        }
        return (v >= 4 && v <= 9) ? uint8_t(v) : 0;
    }
    return any_digit ? kTypeAsk : 0;
}

// Hex digit table: low nibble = value, 0x10 = upper-case A-F, 0x80 = not a hex digit. Random hex has no
// predictable digit/letter pattern, so the branchy hexval() costs ~2 mispredicts per byte; the table
// decodes a 214-byte tx in a few hundred cycles with all error checks folded into one OR at the end.
static const std::array<uint8_t, 256> kHexTab = [] {
    std::array<uint8_t, 256> t{};
    t.fill(0x80);
    for (int c = 0; c < 10; ++c) t[size_t('0' + c)] = uint8_t(c);
    for (int c = 0; c < 6; ++c) {
        t[size_t('a' + c)] = uint8_t(10 + c);
        t[size_t('A' + c)] = uint8_t(0x10 | (10 + c));
    }
    return t;
}();

static void decode_one(const char* hx, size_t hlen, DecTx& t) {
    t.reset();
    if (hlen % 2) return;
    thread_local std::vector<uint8_t> b;  // per-thread scratch: no allocation per tx
    b.resize(hlen / 2);
    {
        const uint8_t* h = reinterpret_cast<const uint8_t*>(hx);
        uint8_t acc = 0;
        for (size_t i = 0; i < b.size(); ++i) {
            const uint8_t hi = kHexTab[h[2 * i]], lo = kHexTab[h[2 * i + 1]];
            acc |= hi | lo;
            b[i] = uint8_t(hi << 4 | (lo & 15));
        }
        if (acc & 0x80) return;  // whitespace etc.: bytes.fromhex semantics are the parser's business
        t.upper_hex = (acc & 0x10) != 0;
    }
    const size_t n = b.size();
    size_t p = 0;
    auto need = [&](size_t k) { return p + k <= n; };
    if (!need(2)) return;
    t.version = b[p++];
    if (t.version > 3) return;  // NotImplementedError in the parser
    const int n_in = b[p++];
    t.ins.resize(static_cast<size_t>(n_in));
    for (auto& in : t.ins) {
        if (!need(34)) return;
        std::memcpy(in.txid, &b[p], 32);
        in.index = b[p + 32];
        in.type = b[p + 33];
        p += 34;
        if (in.type != 0 && in.type != 10) return;  // InputType(..) raises
    }
    if (!need(1)) return;
    const int n_out = b[p++];
    t.outs.resize(size_t(n_out));
    bool general = false;
    const int alen = t.version == 1 ? 64 : 33;
    for (auto& o : t.outs) {
        if (!need(size_t(alen) + 1)) return;
        std::memcpy(o.addr, &b[p], size_t(alen));
        o.len = uint8_t(alen);
        p += size_t(alen);
        const int amount_len = b[p++];
        if (!need(size_t(amount_len) + 1)) return;
        uint64_t amount = 0;
        for (int k = 0; k < amount_len; ++k) {
            if (k >= 8) {
                if (b[p + size_t(k)]) general = true;  // wider than 64 bits
                continue;
            }
            amount |= uint64_t(b[p + size_t(k)]) << (8 * k);
        }
        o.amount = amount;
        p += size_t(amount_len);
        o.type = b[p++];
        if (o.type > 9 || o.type == 4) return;  // OutputType(..) raises (values 0-3, 5-9)
    }
    if (!need(1)) return;
    const uint8_t spec = b[p++];
    const uint8_t* msg = nullptr;
    size_t mlen = 0;
    bool has_msg = false;
    if (spec == 36) {  // coinbase inside the tx list
        t.flag = TX_COINBASE;
        return;
    }
    if (spec == 1) {
        const int lbytes = t.version <= 2 ? 1 : 2;
        if (!need(size_t(lbytes))) return;
        mlen = b[p] | (lbytes == 2 ? size_t(b[p + 1]) << 8 : 0);
        p += size_t(lbytes);
        if (!need(mlen)) return;
        msg = &b[p];
        p += mlen;
        has_msg = true;
        t.tx_type = message_tx_type(msg, mlen);
    } else if (spec != 0) {
        return;  // AssertionError in the parser
    }
    // signatures: 64-byte (r, s) pairs up to the end; a zero r or a ragged tail is parser territory
    if ((n - p) % 64) return;
    const size_t n_sig = (n - p) / 64;
    thread_local std::vector<const uint8_t*> sig_ptr, in_sig;
    sig_ptr.resize(n_sig);
    for (size_t k = 0; k < n_sig; ++k) {
        const uint8_t* s = &b[p + 64 * k];
        bool rz = true;
        for (int q = 0; q < 32; ++q) rz &= s[q] == 0;
        if (rz) return;
        sig_ptr[k] = s;
    }
    // signature -> input assignment (transaction.py:566-590)
    in_sig.resize(static_cast<size_t>(n_in));
    if (n_sig == 1) {
        for (auto& s : in_sig) s = sig_ptr[0];
    } else if (n_sig == size_t(n_in)) {
        for (size_t k = 0; k < n_sig; ++k) in_sig[k] = sig_ptr[k];
    } else if (n_sig > 1 && n_sig < size_t(n_in)) {
        // grouped by the inputs' owner keys in order of first appearance, signature g for group g: the
        // owners come from the UTXO pass (upow_amd/ledger/fastpath.py resolves the groups). Repeated
        // signatures would shrink the canonical list: the Python parser takes those
        for (size_t a = 0; a < n_sig; ++a)
            for (size_t z = a + 1; z < n_sig; ++z)
                if (std::memcmp(sig_ptr[a], sig_ptr[z], 64) == 0) {
                    t.flag = TX_GENERAL;
                    return;
                }
        t.grouped = true;
    } else {
        t.flag = TX_GENERAL;  // more signatures than inputs, or none: the parser's exception / unsigned inputs
        return;
    }
    if (n_in == 0 || n_out == 0) general = true;
    // canonical re-serialisation (Transaction.hex)
    std::vector<uint8_t>& c = t.canon;
    c.reserve(n + 16);
    c.push_back(t.version);
    c.push_back(uint8_t(n_in));
    for (auto& in : t.ins) {
        c.insert(c.end(), in.txid, in.txid + 32);
        c.push_back(in.index);
        c.push_back(in.type);
    }
    c.push_back(uint8_t(n_out));
    for (auto& o : t.outs) {
        if (o.len == 33) {
            c.push_back(o.addr[0] == 43 ? 43 : 42);
            c.insert(c.end(), o.addr + 1, o.addr + 33);
        } else {
            c.insert(c.end(), o.addr, o.addr + 64);
        }
        int bl = 0;
        for (uint64_t a = o.amount; a; a >>= 8) ++bl;
        c.push_back(uint8_t(bl));
        for (int k = 0; k < bl; ++k) c.push_back(uint8_t(o.amount >> (8 * k)));
        c.push_back(o.type);
    }
    t.signed_len = int32_t(c.size());
    if (has_msg) {
        c.push_back(1);
        if (t.version <= 2) {
            c.push_back(uint8_t(mlen));
        } else {
            c.push_back(uint8_t(mlen));
            c.push_back(uint8_t(mlen >> 8));
        }
        t.msg_off = int32_t(c.size());
        t.msg_len = int32_t(mlen);
        c.insert(c.end(), msg, msg + mlen);
        if (t.version >= 3) t.signed_len = int32_t(c.size());
    } else {
        c.push_back(0);
    }
    if (t.grouped) {  // every signature once, in order (= order of first use once the groups are resolved)
        for (size_t k = 0; k < n_sig; ++k) {
            t.sigs.insert(t.sigs.end(), sig_ptr[k], sig_ptr[k] + 64);
            c.insert(c.end(), sig_ptr[k], sig_ptr[k] + 64);
        }
        for (auto& in : t.ins) in.sig = -1;
    }
    for (size_t i = 0; i < (t.grouped ? size_t(0) : size_t(n_in)); ++i) {
        int found = -1;
        const size_t ns = t.sigs.size() / 64;
        for (size_t k = 0; k < ns; ++k)
            if (std::memcmp(&t.sigs[64 * k], in_sig[i], 64) == 0) {
                found = int(k);
                break;
            }
        if (found < 0) {
            found = int(ns);
            t.sigs.insert(t.sigs.end(), in_sig[i], in_sig[i] + 64);
            c.insert(c.end(), in_sig[i], in_sig[i] + 64);
        }
        t.ins[i].sig = found;
    }
    t.canonical = c.size() == n && std::memcmp(c.data(), b.data(), n) == 0;
    host_sha256(c.data(), c.size(), t.txid);
    host_sha256(c.data(), size_t(t.signed_len), t.digest);
    // output address strings + JSON columns (database.add_transactions)
    if (t.out_addr.size() < t.outs.size()) t.out_addr.resize(t.outs.size());
    t.out_addr_json = "[";
    t.out_amount_json = "[";
    for (size_t k = 0; k < t.outs.size(); ++k) {
        std::string& s = t.out_addr[k];
        addr_string(t.outs[k].addr, t.outs[k].len, s);
        if (t.outs[k].len == 33 && hex_ambiguous(s)) general = true;
        if (k) {
            t.out_addr_json += ',';
            t.out_amount_json += ',';
        }
        t.out_addr_json += '"';
        t.out_addr_json += s;
        t.out_addr_json += '"';
        char num[24];
        char* e = num + sizeof(num);
        char* q = e;
        uint64_t v = t.outs[k].amount;
        do {
            *--q = char('0' + v % 10);
            v /= 10;
        } while (v);
        t.out_amount_json.append(q, size_t(e - q));
    }
    t.out_addr_json += ']';
    t.out_amount_json += ']';
    t.flag = general ? TX_GENERAL : TX_FAST;
}


}  // namespace upow
