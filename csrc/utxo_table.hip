// K7/K8/K9: HBM-resident UTXO set (outpoint -> output-table tag, amount, owner address) for gfx950.
//
// reference: the seven per-type output tables queried/inserted/deleted with
// `(tx_hash, index) = ANY($1::tx_output[])` (upow/database.py:439-825, used by upow/manager.py:531-543
// and upow/upow_transactions/transaction.py:99-124).
//
// Open addressing with linear probing over 48-byte slots {txid words[8], meta, pad[3]}; meta packs
// state (empty/full/tombstone/busy), the output index and the table tag. A block's inputs/outputs
// are applied as whole batches (one lane per outpoint): probe, insert and erase kernels. Batches of
// different kinds are separate launches, so no op races a different op; inserts claim a slot with a
// CAS on its meta word and publish it with an atomic exchange after the key words.
// The table lives in HBM for the life of the node (288 GB leaves room for ~10^9 outpoints); the
// txid's first word is already uniformly random, so it is the hash.
//
// Each slot has an 80-byte payload in a parallel array {amount u64, address length u32, pad,
// address bytes[64]} — what block validation needs from a spent output (fees, signature key,
// inputs_addresses) without touching the SQL tables. Probing scans only the compact 48-byte key
// slots; the payload line is read once, on a hit.
#include <hip/hip_runtime.h>

#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "native.h"

namespace upow {

struct alignas(16) UtxoSlot {
    uint32_t k[8];
    uint32_t meta;
    uint32_t pad[3];
};
static_assert(sizeof(UtxoSlot) == 48, "slot size");

enum : uint32_t { ST_EMPTY = 0, ST_FULL = 1, ST_TOMB = 2, ST_BUSY = 3 };

struct UtxoKeyRec {  // 40 bytes: txid (raw bytes), index, tag
    uint8_t txid[32];
    uint32_t index;
    uint32_t tag;
};
static_assert(sizeof(UtxoKeyRec) == 40, "key record");

struct alignas(16) UtxoPayload {  // 80 bytes
    uint64_t amount;
    uint32_t addr_len;
    uint32_t pad;
    uint8_t addr[64];
};
static_assert(sizeof(UtxoPayload) == 80, "payload");

__device__ __forceinline__ uint32_t ld_u32(const uint8_t* p) {
    return uint32_t(p[0]) | (uint32_t(p[1]) << 8) | (uint32_t(p[2]) << 16) | (uint32_t(p[3]) << 24);
}
__device__ __forceinline__ uint32_t slot_hash(const uint32_t k[8], uint32_t idx) {
    uint32_t h = k[0] ^ (idx * 0x9E3779B1u);
    h ^= h >> 15;
    h *= 0x2c1b3c6du;
    h ^= h >> 12;
    return h;
}
__device__ __forceinline__ void load_key(const UtxoKeyRec& r, uint32_t k[8]) {
#pragma unroll
    for (int i = 0; i < 8; ++i) k[i] = ld_u32(r.txid + 4 * i);
}
__device__ __forceinline__ bool key_eq(const UtxoSlot& s, const uint32_t k[8]) {
    uint32_t d = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) d |= s.k[i] ^ k[i];
    return d == 0;
}

__global__ __launch_bounds__(256) void utxo_insert_kernel(UtxoSlot* __restrict__ tab, UtxoPayload* __restrict__ pay,
                                                          uint32_t mask, const UtxoKeyRec* __restrict__ recs,
                                                          const UtxoPayload* __restrict__ in_pay, int64_t n,
                                                          uint32_t* __restrict__ failed) {
    const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t k[8];
    load_key(recs[i], k);
    const uint32_t idx = recs[i].index & 0xffu, tag = recs[i].tag & 0xffu;
    uint32_t s = slot_hash(k, idx) & mask;
    for (uint32_t probe = 0; probe <= mask; ++probe) {
        uint32_t* mp = &tab[s].meta;
        const uint32_t m = __hip_atomic_load(mp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t st = m & 3u;
        if (st == ST_EMPTY || st == ST_TOMB) {
            if (atomicCAS(mp, m, ST_BUSY) == m) {
#pragma unroll
                for (int w = 0; w < 8; ++w) tab[s].k[w] = k[w];
                if (in_pay) {
                    pay[s] = in_pay[i];
                } else {
                    pay[s].amount = 0;
                    pay[s].addr_len = 0;
                }
                __threadfence();
                atomicExch(mp, ST_FULL | (idx << 8) | (tag << 16));
                return;
            }
            --probe;  // lost the race for this slot: look at it again
            continue;
        }
        s = (s + 1) & mask;
    }
    atomicAdd(failed, 1u);
}

// tags_out[i] = tag of the outpoint, 0xff when absent
__global__ __launch_bounds__(256) void utxo_probe_kernel(const UtxoSlot* __restrict__ tab, uint32_t mask,
                                                         const UtxoKeyRec* __restrict__ recs, int64_t n,
                                                         uint8_t* __restrict__ tags_out) {
    const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t k[8];
    load_key(recs[i], k);
    const uint32_t idx = recs[i].index & 0xffu;
    uint32_t s = slot_hash(k, idx) & mask;
    uint8_t res = 0xff;
    for (uint32_t probe = 0; probe <= mask; ++probe) {
        const uint32_t m = tab[s].meta;
        const uint32_t st = m & 3u;
        if (st == ST_EMPTY) break;
        if (st == ST_FULL && ((m >> 8) & 0xffu) == idx && key_eq(tab[s], k)) {
            res = uint8_t((m >> 16) & 0xffu);
            break;
        }
        s = (s + 1) & mask;
    }
    tags_out[i] = res;
}

// lookup = probe + payload gather (payload zeroed when absent)
__global__ __launch_bounds__(256) void utxo_lookup_kernel(const UtxoSlot* __restrict__ tab,
                                                          const UtxoPayload* __restrict__ pay, uint32_t mask,
                                                          const UtxoKeyRec* __restrict__ recs, int64_t n,
                                                          uint8_t* __restrict__ tags_out,
                                                          UtxoPayload* __restrict__ pay_out) {
    const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t k[8];
    load_key(recs[i], k);
    const uint32_t idx = recs[i].index & 0xffu;
    uint32_t s = slot_hash(k, idx) & mask;
    uint8_t res = 0xff;
    int64_t hit = -1;
    for (uint32_t probe = 0; probe <= mask; ++probe) {
        const uint32_t m = tab[s].meta;
        const uint32_t st = m & 3u;
        if (st == ST_EMPTY) break;
        if (st == ST_FULL && ((m >> 8) & 0xffu) == idx && key_eq(tab[s], k)) {
            res = uint8_t((m >> 16) & 0xffu);
            hit = s;
            break;
        }
        s = (s + 1) & mask;
    }
    tags_out[i] = res;
    if (hit >= 0) {
        pay_out[i] = pay[hit];
    } else {
        UtxoPayload z{};
        pay_out[i] = z;
    }
}

// erase: only entries whose tag matches recs[i].tag (0xff = any); erased[i] = 1 when removed
__global__ __launch_bounds__(256) void utxo_erase_kernel(UtxoSlot* __restrict__ tab, uint32_t mask,
                                                         const UtxoKeyRec* __restrict__ recs, int64_t n,
                                                         uint8_t* __restrict__ erased, uint32_t* __restrict__ count) {
    const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t k[8];
    load_key(recs[i], k);
    const uint32_t idx = recs[i].index & 0xffu, want = recs[i].tag & 0xffu;
    uint32_t s = slot_hash(k, idx) & mask;
    uint8_t res = 0;
    for (uint32_t probe = 0; probe <= mask; ++probe) {
        uint32_t* mp = &tab[s].meta;
        const uint32_t m = __hip_atomic_load(mp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t st = m & 3u;
        if (st == ST_EMPTY) break;
        if (st == ST_FULL && ((m >> 8) & 0xffu) == idx && key_eq(tab[s], k)) {
            if (want == 0xffu || ((m >> 16) & 0xffu) == want) {
                if (atomicCAS(mp, m, (m & ~3u) | ST_TOMB) == m) {
                    res = 1;
                    atomicAdd(count, 1u);
                }
            }
            break;
        }
        s = (s + 1) & mask;
    }
    erased[i] = res;
}

__global__ __launch_bounds__(256) void utxo_dump_kernel(const UtxoSlot* __restrict__ tab,
                                                        const UtxoPayload* __restrict__ pay, uint32_t cap,
                                                        UtxoKeyRec* __restrict__ out, UtxoPayload* __restrict__ pay_out,
                                                        uint32_t* __restrict__ count) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= cap) return;
    const uint32_t m = tab[s].meta;
    if ((m & 3u) != ST_FULL) return;
    const uint32_t o = atomicAdd(count, 1u);
    UtxoKeyRec r;
#pragma unroll
    for (int w = 0; w < 8; ++w) {
        r.txid[4 * w] = uint8_t(tab[s].k[w]);
        r.txid[4 * w + 1] = uint8_t(tab[s].k[w] >> 8);
        r.txid[4 * w + 2] = uint8_t(tab[s].k[w] >> 16);
        r.txid[4 * w + 3] = uint8_t(tab[s].k[w] >> 24);
    }
    r.index = (m >> 8) & 0xffu;
    r.tag = (m >> 16) & 0xffu;
    out[o] = r;
    if (pay_out) pay_out[o] = pay[s];
}

// ------------------------------------------------------------------------------------------------
static void uck(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

struct UtxoTableDev {
    int device = 0;
    UtxoSlot* tab = nullptr;
    UtxoPayload* pay = nullptr;
    uint32_t cap = 0;
    uint32_t* d_counter = nullptr;
};

static std::mutex g_ut_mu;
static std::unordered_map<int64_t, UtxoTableDev> g_tables;
static int64_t g_next_handle = 1;

static UtxoTableDev& table(int64_t h) {
    auto it = g_tables.find(h);
    if (it == g_tables.end()) throw std::invalid_argument("bad utxo table handle");
    int dev = 0;
    uck(hipGetDevice(&dev), "hipGetDevice");
    if (dev != it->second.device) uck(hipSetDevice(it->second.device), "hipSetDevice");
    return it->second;
}

int64_t utxo_create(uint32_t log2_cap) {
    if (log2_cap < 8 || log2_cap > 31) throw std::invalid_argument("log2 capacity must be in [8, 31]");
    UtxoTableDev t;
    uck(hipGetDevice(&t.device), "hipGetDevice");
    t.cap = 1u << log2_cap;
    uck(hipMalloc(&t.tab, sizeof(UtxoSlot) * size_t(t.cap)), "hipMalloc utxo table");
    uck(hipMemset(t.tab, 0, sizeof(UtxoSlot) * size_t(t.cap)), "memset utxo table");
    uck(hipMalloc(&t.pay, sizeof(UtxoPayload) * size_t(t.cap)), "hipMalloc utxo payload");
    uck(hipMalloc(&t.d_counter, sizeof(uint32_t)), "hipMalloc counter");
    std::lock_guard<std::mutex> lk(g_ut_mu);
    const int64_t h = g_next_handle++;
    g_tables[h] = t;
    return h;
}

void utxo_destroy(int64_t h) {
    std::lock_guard<std::mutex> lk(g_ut_mu);
    auto it = g_tables.find(h);
    if (it == g_tables.end()) return;
    (void)hipFree(it->second.tab);
    (void)hipFree(it->second.pay);
    (void)hipFree(it->second.d_counter);
    g_tables.erase(it);
}

uint32_t utxo_capacity(int64_t h) {
    std::lock_guard<std::mutex> lk(g_ut_mu);
    return table(h).cap;
}

template <typename T>
struct DevBuf {
    T* p = nullptr;
    explicit DevBuf(size_t n) { uck(hipMalloc(&p, sizeof(T) * (n ? n : 1)), "hipMalloc"); }
    ~DevBuf() { (void)hipFree(p); }
};

uint32_t utxo_insert(int64_t h, const uint8_t* recs, int64_t n, const uint8_t* payload) {
    std::lock_guard<std::mutex> lk(g_ut_mu);
    UtxoTableDev& t = table(h);
    if (n == 0) return 0;
    DevBuf<UtxoKeyRec> d(n);
    uck(hipMemcpy(d.p, recs, sizeof(UtxoKeyRec) * n, hipMemcpyHostToDevice), "h2d recs");
    DevBuf<UtxoPayload> dp(payload ? n : 0);
    if (payload) uck(hipMemcpy(dp.p, payload, sizeof(UtxoPayload) * n, hipMemcpyHostToDevice), "h2d payload");
    uck(hipMemset(t.d_counter, 0, sizeof(uint32_t)), "memset");
    hipLaunchKernelGGL(utxo_insert_kernel, dim3(int((n + 255) / 256)), dim3(256), 0, 0, t.tab, t.pay, t.cap - 1, d.p,
                       payload ? dp.p : nullptr, n, t.d_counter);
    uck(hipGetLastError(), "utxo_insert_kernel");
    uint32_t failed = 0;
    uck(hipMemcpy(&failed, t.d_counter, sizeof(uint32_t), hipMemcpyDeviceToHost), "d2h failed");
    return failed;
}

std::vector<uint8_t> utxo_lookup(int64_t h, const uint8_t* recs, int64_t n, std::vector<uint8_t>& payload_out) {
    std::lock_guard<std::mutex> lk(g_ut_mu);
    UtxoTableDev& t = table(h);
    std::vector<uint8_t> out(static_cast<size_t>(n));
    payload_out.assign(static_cast<size_t>(n) * sizeof(UtxoPayload), 0);
    if (n == 0) return out;
    DevBuf<UtxoKeyRec> d(n);
    DevBuf<uint8_t> o(n);
    DevBuf<UtxoPayload> po(n);
    uck(hipMemcpy(d.p, recs, sizeof(UtxoKeyRec) * n, hipMemcpyHostToDevice), "h2d recs");
    hipLaunchKernelGGL(utxo_lookup_kernel, dim3(int((n + 255) / 256)), dim3(256), 0, 0, t.tab, t.pay, t.cap - 1, d.p, n,
                       o.p, po.p);
    uck(hipGetLastError(), "utxo_lookup_kernel");
    uck(hipMemcpy(out.data(), o.p, size_t(n), hipMemcpyDeviceToHost), "d2h tags");
    uck(hipMemcpy(payload_out.data(), po.p, payload_out.size(), hipMemcpyDeviceToHost), "d2h payload");
    return out;
}

std::vector<uint8_t> utxo_probe(int64_t h, const uint8_t* recs, int64_t n) {
    std::lock_guard<std::mutex> lk(g_ut_mu);
    UtxoTableDev& t = table(h);
    std::vector<uint8_t> out(static_cast<size_t>(n));
    if (n == 0) return out;
    DevBuf<UtxoKeyRec> d(n);
    DevBuf<uint8_t> o(n);
    uck(hipMemcpy(d.p, recs, sizeof(UtxoKeyRec) * n, hipMemcpyHostToDevice), "h2d recs");
    hipLaunchKernelGGL(utxo_probe_kernel, dim3(int((n + 255) / 256)), dim3(256), 0, 0, t.tab, t.cap - 1, d.p, n, o.p);
    uck(hipGetLastError(), "utxo_probe_kernel");
    uck(hipMemcpy(out.data(), o.p, size_t(n), hipMemcpyDeviceToHost), "d2h tags");
    return out;
}

std::vector<uint8_t> utxo_erase(int64_t h, const uint8_t* recs, int64_t n) {
    std::lock_guard<std::mutex> lk(g_ut_mu);
    UtxoTableDev& t = table(h);
    std::vector<uint8_t> out(static_cast<size_t>(n));
    if (n == 0) return out;
    DevBuf<UtxoKeyRec> d(n);
    DevBuf<uint8_t> o(n);
    uck(hipMemcpy(d.p, recs, sizeof(UtxoKeyRec) * n, hipMemcpyHostToDevice), "h2d recs");
    uck(hipMemset(t.d_counter, 0, sizeof(uint32_t)), "memset");
    hipLaunchKernelGGL(utxo_erase_kernel, dim3(int((n + 255) / 256)), dim3(256), 0, 0, t.tab, t.cap - 1, d.p, n, o.p,
                       t.d_counter);
    uck(hipGetLastError(), "utxo_erase_kernel");
    uck(hipMemcpy(out.data(), o.p, size_t(n), hipMemcpyDeviceToHost), "d2h erased");
    return out;
}

std::vector<uint8_t> utxo_dump(int64_t h, std::vector<uint8_t>* payload_out) {
    std::lock_guard<std::mutex> lk(g_ut_mu);
    UtxoTableDev& t = table(h);
    DevBuf<UtxoKeyRec> d(t.cap);
    DevBuf<UtxoPayload> dp(payload_out ? t.cap : 0);
    uck(hipMemset(t.d_counter, 0, sizeof(uint32_t)), "memset");
    hipLaunchKernelGGL(utxo_dump_kernel, dim3(int((t.cap + 255) / 256)), dim3(256), 0, 0, t.tab, t.pay, t.cap, d.p,
                       payload_out ? dp.p : nullptr, t.d_counter);
    uck(hipGetLastError(), "utxo_dump_kernel");
    uint32_t n = 0;
    uck(hipMemcpy(&n, t.d_counter, sizeof(uint32_t), hipMemcpyDeviceToHost), "d2h n");
    std::vector<uint8_t> out(size_t(n) * sizeof(UtxoKeyRec));
    if (n) uck(hipMemcpy(out.data(), d.p, out.size(), hipMemcpyDeviceToHost), "d2h dump");
    if (payload_out) {
        payload_out->assign(size_t(n) * sizeof(UtxoPayload), 0);
        if (n) uck(hipMemcpy(payload_out->data(), dp.p, payload_out->size(), hipMemcpyDeviceToHost), "d2h payload");
    }
    return out;
}

}  // namespace upow
