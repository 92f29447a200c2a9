// libFuzzer target (ASan + UBSan, tools/sanitize_host.sh): the block codec's per-transaction decoder
// (csrc/txdecode.h) on arbitrary input. Every pushed tx and every block from a peer goes through it.
//
// Input: byte 0 selects how the rest becomes the tx hex string: 0 lower-case hex of the bytes, 1 upper-case
// hex, 2 the bytes themselves as the "hex" text (odd lengths, non-hex characters, whitespace). Properties,
// besides "no memory error, no UB":
//  * a decoded tx (TX_FAST) is internally consistent: signature indices, the message window and the signed
//    prefix lie inside the canonical bytes, txid = SHA-256(canonical bytes), digest = SHA-256(signed prefix);
//  * canonical form is a fixed point: decoding the canonical bytes again gives the same canonical bytes,
//    txid, flag and columns, and reports them canonical (except n signatures for n inputs with repeats:
//    the canonical bytes keep each signature once, which reads back as the grouped form).
#include <cstdint>
#include <cstdlib>
#include <string>

#include "../../csrc/txdecode.h"

using namespace upow;

#include <cstdio>

#define check(c)                                                                   \
    do {                                                                           \
        if (!(c)) {                                                                \
            std::fprintf(stderr, "fuzz_txdecode: property failed at line %d: %s\n", __LINE__, #c); \
            std::abort();                                                          \
        }                                                                          \
    } while (0)

// Built-in ASan defaults: the fuzzer runtime and the target register some header-defined globals twice
// (a spurious ODR report), and leak checking is not what these targets test.
extern "C" const char* __asan_default_options() { return "detect_odr_violation=0:detect_leaks=0"; }

extern "C" int LLVMFuzzerTestOneInput(const uint8_t* data, size_t size) {
    if (size < 1) return 0;
    const int mode = data[0] % 3;
    const uint8_t* p = data + 1;
    const size_t n = size - 1;
    std::string hx;
    if (mode == 2) {
        hx.assign(reinterpret_cast<const char*>(p), n);
    } else {
        hx = to_hex(p, n);
        if (mode == 1)
            for (char& c : hx)
                if (c >= 'a' && c <= 'f') c = char(c - 32);
    }
    DecTx t;
    decode_one(hx.data(), hx.size(), t);
    check(t.flag <= TX_COINBASE);
    if (t.flag != TX_FAST) return 0;
    const size_t cn = t.canon.size();
    check(t.signed_len > 0 && size_t(t.signed_len) <= cn);
    check(t.msg_off < 0 || size_t(t.msg_off) + size_t(t.msg_len) <= cn);
    check(t.ins.size() <= 255 && t.outs.size() <= 255 && !t.ins.empty() && !t.outs.empty());
    check(t.sigs.size() % 64 == 0 && !t.sigs.empty());
    for (auto& in : t.ins) check(t.grouped ? in.sig == -1 : (in.sig >= 0 && size_t(in.sig) < t.sigs.size() / 64));
    if (t.grouped) check(t.sigs.size() / 64 > 1 && t.sigs.size() / 64 < t.ins.size());
    for (size_t k = 0; k < t.outs.size(); ++k) check(t.outs[k].len == 33 || t.outs[k].len == 64);
    uint8_t d[32];
    host_sha256(t.canon.data(), cn, d);
    check(std::memcmp(d, t.txid, 32) == 0);
    host_sha256(t.canon.data(), size_t(t.signed_len), d);
    check(std::memcmp(d, t.digest, 32) == 0);
    if (mode != 2) check(t.canonical == (cn == n && std::memcmp(t.canon.data(), p, n) == 0));
    DecTx u;
    const std::string ch = to_hex(t.canon.data(), cn);
    decode_one(ch.data(), ch.size(), u);
    const size_t uniq = t.sigs.size() / 64;
    if (!t.grouped && uniq != 1 && uniq != t.ins.size()) {
        // n signatures for n inputs with repeats: the canonical bytes keep each signature once
        // (transaction.py:76-81), and k < n signatures read back as the grouped-by-key form
        check(u.flag == TX_GENERAL);
        return 0;
    }
    check(u.flag == TX_FAST && u.canonical && u.canon == t.canon && u.grouped == t.grouped);
    check(std::memcmp(u.txid, t.txid, 32) == 0 && u.signed_len == t.signed_len && u.tx_type == t.tx_type);
    check(u.out_addr_json == t.out_addr_json && u.out_amount_json == t.out_amount_json);
    return 0;
}
