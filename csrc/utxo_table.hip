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
#include <hipcub/device/device_radix_sort.hpp>

#include <algorithm>
#include <cstddef>
#include <cstring>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "dev_pool.h"
#include "native.h"
#include "streams.h"
#include "sha256_common.h"

namespace upow {

struct alignas(16) UtxoSlot {
    uint32_t k[8];
    uint32_t meta;
    uint32_t pad[3];
};
static_assert(sizeof(UtxoSlot) == 48, "slot size");
static_assert(offsetof(UtxoSlot, meta) == 32 && offsetof(UtxoSlot, pad) == 36, "meta + fingerprint are one aligned 16-byte word");

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
    uint32_t flags;  // bit 0: is_stake (unspent_outputs.is_stake = 1)
    uint8_t addr[64];
};
constexpr uint32_t PAY_STAKE = 1u;
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

// Owner fingerprint kept in the key slot (pad[0]): address bytes 1..4 (after the 42/43 parity prefix of
// a compressed key these are x-coordinate bytes, i.e. uniformly random), so the K14 address scan can
// reject a slot from the 48-byte key line alone and touch the 80-byte payload line only on a likely hit.
__device__ __forceinline__ uint32_t addr_fingerprint(const uint8_t* addr) { return ld_u32(addr + 1); }

// Insert: walk the probe chain to its first EMPTY slot remembering the first reusable (EMPTY or
// tombstone) slot; a live entry with the same outpoint already in the chain is a duplicate and is not
// inserted again (counter[1]). The remembered slot is claimed with a CAS; a lane that loses the race
// walks the chain again. counter[0] counts entries that found no slot (table full).
// Lanes of one launch never insert the same outpoint twice (block validation rejects duplicate inputs,
// hence duplicate txids), so the chain walk only has to see entries published by earlier launches.
// one entry into the table (the insert kernel's lane body, shared with the rehash): `p` = its payload or
// nullptr, `fp` = its owner fingerprint
__device__ __forceinline__ void insert_one(UtxoSlot* __restrict__ tab, UtxoPayload* __restrict__ pay, uint32_t mask,
                                           const uint32_t k[8], uint32_t idx, uint32_t tag,
                                           const UtxoPayload* __restrict__ p, uint32_t fp,
                                           uint32_t* __restrict__ counter) {
    const uint32_t home = slot_hash(k, idx) & mask;
    for (int attempt = 0; attempt < 64; ++attempt) {
        uint32_t s = home, free_slot = 0xffffffffu, free_meta = 0;
        for (uint32_t probe = 0; probe <= mask; ++probe) {
            const uint32_t m = __hip_atomic_load(&tab[s].meta, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint32_t st = m & 3u;
            if (st == ST_FULL && ((m >> 8) & 0xffu) == idx && key_eq(tab[s], k)) {
                atomicAdd(counter + 1, 1u);
                return;
            }
            if ((st == ST_EMPTY || st == ST_TOMB) && free_slot == 0xffffffffu) {
                free_slot = s;
                free_meta = m;
            }
            if (st == ST_EMPTY) break;
            s = (s + 1) & mask;
        }
        if (free_slot == 0xffffffffu) break;
        uint32_t* mp = &tab[free_slot].meta;
        if (atomicCAS(mp, free_meta, ST_BUSY) != free_meta) continue;  // lost the race: walk again
#pragma unroll
        for (int w = 0; w < 8; ++w) tab[free_slot].k[w] = k[w];
        if (p) {
            pay[free_slot] = *p;
        } else {
            UtxoPayload z{};
            pay[free_slot] = z;
        }
        tab[free_slot].pad[0] = fp;
        __threadfence();
        atomicExch(mp, ST_FULL | (idx << 8) | (tag << 16));
        return;
    }
    atomicAdd(counter, 1u);
}

__global__ __launch_bounds__(256) void utxo_insert_kernel(UtxoSlot* __restrict__ tab, UtxoPayload* __restrict__ pay,
                                                          uint32_t mask, const UtxoKeyRec* __restrict__ recs,
                                                          const UtxoPayload* __restrict__ in_pay, int64_t n,
                                                          uint32_t* __restrict__ counter) {
    const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t k[8];
    load_key(recs[i], k);
    const uint32_t idx = recs[i].index & 0xffu, tag = recs[i].tag & 0xffu;
    insert_one(tab, pay, mask, k, idx, tag, in_pay ? &in_pay[i] : nullptr, in_pay ? addr_fingerprint(in_pay[i].addr) : 0u,
               counter);
}

// Rehash: one lane per slot of the old table; a live entry goes into the new table with its payload and its
// owner fingerprint as they are (tombstones and empty slots are dropped)
__global__ __launch_bounds__(256) void utxo_migrate_kernel(const UtxoSlot* __restrict__ old_tab,
                                                           const UtxoPayload* __restrict__ old_pay, uint32_t old_cap,
                                                           UtxoSlot* __restrict__ tab, UtxoPayload* __restrict__ pay,
                                                           uint32_t mask, uint32_t* __restrict__ counter) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= old_cap) return;
    const uint32_t m = old_tab[s].meta;
    if ((m & 3u) != ST_FULL) return;
    uint32_t k[8];
#pragma unroll
    for (int w = 0; w < 8; ++w) k[w] = old_tab[s].k[w];
    insert_one(tab, pay, mask, k, (m >> 8) & 0xffu, (m >> 16) & 0xffu, &old_pay[s], old_tab[s].pad[0], counter);
    atomicAdd(counter + 2, 1u);
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


// K14: outputs owned by one address (reference `database.py:909-937,1138-1205`: balance / spendable
// outputs by address). One lane per slot streams the key metas and, for live slots whose tag is in
// `tag_mask`, the 80-byte payload line; the address is compared as four 16-byte vectors held in SGPRs
// (the query is uniform). The slot's owner fingerprint is checked first, so the payload line is read
// only for likely hits. Matches are rare, so they are compacted with one atomic each; the amount sum
// is a wave reduction + one 64-bit atomic per wave that found anything.
__global__ __launch_bounds__(256) void utxo_address_scan_kernel(const UtxoSlot* __restrict__ tab,
                                                                const UtxoPayload* __restrict__ pay, uint32_t cap,
                                                                uint4 q0, uint4 q1, uint4 q2, uint4 q3, uint32_t qlen,
                                                                uint32_t qfp, uint32_t tag_mask, uint32_t stake_sel,
                                                                uint32_t max_out,
                                                                UtxoKeyRec* __restrict__ out,
                                                                UtxoPayload* __restrict__ pay_out,
                                                                uint32_t* __restrict__ count,
                                                                unsigned long long* __restrict__ total) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t amt = 0;
    if (s < cap) {
        // meta and fingerprint in one 16-byte load (slot bytes 32..47, 16-byte aligned)
        const uint4 mw = *reinterpret_cast<const uint4*>(&tab[s].meta);
        const uint32_t m = mw.x;
        const uint32_t tag = (m >> 16) & 0xffu;
        // stake_sel: 0 any output, 1 only is_stake = 0 (spendable), 2 only is_stake = 1
        const uint32_t stake = tag == 0u ? (pay[s].flags & PAY_STAKE) : 0u;
        if ((m & 3u) == ST_FULL && tag < 32u && ((tag_mask >> tag) & 1u) && mw.y == qfp &&
            pay[s].addr_len == qlen && (stake_sel == 0u || (stake_sel == 1u) == (stake == 0u))) {
            const uint4* a = reinterpret_cast<const uint4*>(pay[s].addr);
            const uint4 a0 = a[0], a1 = a[1], a2 = a[2], a3 = a[3];
            const uint32_t d = (a0.x ^ q0.x) | (a0.y ^ q0.y) | (a0.z ^ q0.z) | (a0.w ^ q0.w) | (a1.x ^ q1.x) |
                               (a1.y ^ q1.y) | (a1.z ^ q1.z) | (a1.w ^ q1.w) | (a2.x ^ q2.x) | (a2.y ^ q2.y) |
                               (a2.z ^ q2.z) | (a2.w ^ q2.w) | (a3.x ^ q3.x) | (a3.y ^ q3.y) | (a3.z ^ q3.z) |
                               (a3.w ^ q3.w);
            if (d == 0) {
                amt = pay[s].amount;
                const uint32_t o = atomicAdd(count, 1u);
                if (o < max_out) {
                    UtxoKeyRec r;
#pragma unroll
                    for (int w = 0; w < 8; ++w) {
                        r.txid[4 * w] = uint8_t(tab[s].k[w]);
                        r.txid[4 * w + 1] = uint8_t(tab[s].k[w] >> 8);
                        r.txid[4 * w + 2] = uint8_t(tab[s].k[w] >> 16);
                        r.txid[4 * w + 3] = uint8_t(tab[s].k[w] >> 24);
                    }
                    r.index = (m >> 8) & 0xffu;
                    r.tag = tag;
                    out[o] = r;
                    pay_out[o] = pay[s];
                }
            }
        }
    }
    // wave64 sum: amounts are < 2^63 in total (MAX_SUPPLY in smallest units fits in 2^51)
    for (int off = 32; off > 0; off >>= 1) amt += __shfl_down(amt, off, 64);
    if ((threadIdx.x & 63u) == 0 && amt) atomicAdd(total, static_cast<unsigned long long>(amt));
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
    node_memset(t.tab, 0, sizeof(UtxoSlot) * size_t(t.cap), "memset utxo table");
    uck(hipMalloc(&t.pay, sizeof(UtxoPayload) * size_t(t.cap)), "hipMalloc utxo payload");
    node_memset(t.pay, 0, sizeof(UtxoPayload) * size_t(t.cap), "memset utxo payload");
    node_sync("utxo_create");
    uck(hipMalloc(&t.d_counter, 2 * sizeof(uint32_t)), "hipMalloc counter");
    std::lock_guard<std::mutex> lk(g_ut_mu);
    const int64_t h = g_next_handle++;
    g_tables[h] = t;
    return h;
}

// Asynchronous index update of one committed block (the block path's last GPU step): the inputs are
// packed into pinned memory owned by the table, ONE H2D copy, the insert and the erase launch and a D2H
// of their three counters are queued on the node stream and an event is recorded; the call returns
// without waiting. Every later pass on the table is queued behind it on the same stream, so it reads the
// updated table with no host round trip in between; the counters are collected (event sync) by
// utxo_apply_wait, or by the next utxo_apply_async before it reuses the buffers.
struct AsyncApply {
    hipEvent_t ev = nullptr;
    uint8_t* host = nullptr;
    size_t host_cap = 0;
    uint8_t* dev = nullptr;
    size_t dev_cap = 0;
    const uint32_t* res = nullptr;  // pinned: (entries with no free slot, duplicates skipped, erased)
    bool live = false;
};
static std::unordered_map<int64_t, AsyncApply> g_async;  // by table handle, under g_ut_mu

static bool async_collect(AsyncApply& a, uint32_t out[3]) {
    out[0] = out[1] = out[2] = 0;
    if (!a.live) return false;
    a.live = false;
    uck(hipEventSynchronize(a.ev), "utxo async apply");
    out[0] = a.res[0];
    out[1] = a.res[1];
    out[2] = a.res[2];
    return true;
}

static void async_release(int64_t h) {  // under g_ut_mu
    auto it = g_async.find(h);
    if (it == g_async.end()) return;
    uint32_t r[3];
    try {
        async_collect(it->second, r);
    } catch (...) {
    }
    if (it->second.ev) (void)hipEventDestroy(it->second.ev);
    if (it->second.host) (void)hipHostFree(it->second.host);
    if (it->second.dev) (void)hipFree(it->second.dev);
    g_async.erase(it);
}

static size_t align256(size_t n) { return (n + 255) & ~size_t(255); }

bool utxo_apply_async(int64_t h, const std::vector<UtxoSeg>& ins, bool with_pay, const uint8_t* del, int64_t n_del,
                      uint32_t prev[3]) {
    int64_t n_ins = 0;
    for (const UtxoSeg& g : ins) n_ins += g.n;
    const bool ins_pay = with_pay && n_ins > 0;
    std::lock_guard<std::mutex> lk(g_ut_mu);
    UtxoTableDev& t = table(h);
    AsyncApply& a = g_async[h];
    const bool had = async_collect(a, prev);
    const size_t off_pay = align256(size_t(n_ins) * sizeof(UtxoKeyRec));
    const size_t off_del = off_pay + align256(ins_pay ? size_t(n_ins) * sizeof(UtxoPayload) : 0);
    const size_t off_cnt = off_del + align256(size_t(n_del) * sizeof(UtxoKeyRec));
    const size_t off_st = off_cnt + 256;  // erase status bytes (device only)
    const size_t dev_need = off_st + align256(size_t(n_del));
    if (!a.ev) uck(hipEventCreateWithFlags(&a.ev, hipEventDisableTiming), "hipEventCreate");
    if (off_cnt + 256 > a.host_cap) {
        if (a.host) uck(hipHostFree(a.host), "hipHostFree");  // the previous apply was collected above
        a.host = nullptr;
        a.host_cap = std::max<size_t>(off_cnt + 256, size_t(4) << 20) * 2;
        uck(hipHostMalloc(reinterpret_cast<void**>(&a.host), a.host_cap, hipHostMallocDefault), "hipHostMalloc");
    }
    if (dev_need > a.dev_cap) {
        if (a.dev) {
            node_sync("utxo async regrow");
            uck(hipFree(a.dev), "hipFree");
        }
        a.dev = nullptr;
        a.dev_cap = std::max<size_t>(dev_need, size_t(4) << 20) * 2;
        uck(hipMalloc(reinterpret_cast<void**>(&a.dev), a.dev_cap), "hipMalloc");
    }
    size_t at = 0;  // the groups land back to back: no concatenation on the caller's side
    for (const UtxoSeg& g : ins) {
        if (!g.n) continue;
        std::memcpy(a.host + at * sizeof(UtxoKeyRec), g.recs, size_t(g.n) * sizeof(UtxoKeyRec));
        if (ins_pay) std::memcpy(a.host + off_pay + at * sizeof(UtxoPayload), g.pay, size_t(g.n) * sizeof(UtxoPayload));
        at += size_t(g.n);
    }
    if (n_del) std::memcpy(a.host + off_del, del, size_t(n_del) * sizeof(UtxoKeyRec));
    hipStream_t st = node_stream();
    uck(hipMemcpyAsync(a.dev, a.host, off_cnt, hipMemcpyHostToDevice, st), "async apply h2d");
    uint32_t* cnt = reinterpret_cast<uint32_t*>(a.dev + off_cnt);
    uck(hipMemsetAsync(cnt, 0, 16, st), "async apply memset");
    if (n_ins) {
        hipLaunchKernelGGL(utxo_insert_kernel, dim3(int((n_ins + 255) / 256)), dim3(256), 0, st, t.tab, t.pay, t.cap - 1,
                           reinterpret_cast<const UtxoKeyRec*>(a.dev),
                           ins_pay ? reinterpret_cast<const UtxoPayload*>(a.dev + off_pay) : nullptr, n_ins, cnt);
        uck(hipGetLastError(), "utxo_insert_kernel (async)");
    }
    if (n_del) {
        hipLaunchKernelGGL(utxo_erase_kernel, dim3(int((n_del + 255) / 256)), dim3(256), 0, st, t.tab, t.cap - 1,
                           reinterpret_cast<const UtxoKeyRec*>(a.dev + off_del), n_del, a.dev + off_st, cnt + 2);
        uck(hipGetLastError(), "utxo_erase_kernel (async)");
    }
    uint32_t* res = reinterpret_cast<uint32_t*>(a.host + off_cnt);
    uck(hipMemcpyAsync(res, cnt, 3 * sizeof(uint32_t), hipMemcpyDeviceToHost, st), "async apply d2h");
    uck(hipEventRecord(a.ev, st), "hipEventRecord");
    a.res = res;
    a.live = true;
    return had;
}

bool utxo_apply_wait(int64_t h, uint32_t out[3]) {
    std::lock_guard<std::mutex> lk(g_ut_mu);
    (void)table(h);
    auto it = g_async.find(h);
    if (it == g_async.end()) {
        out[0] = out[1] = out[2] = 0;
        return false;
    }
    return async_collect(it->second, out);
}

void utxo_destroy(int64_t h) {
    std::lock_guard<std::mutex> lk(g_ut_mu);
    async_release(h);
    auto it = g_tables.find(h);
    if (it == g_tables.end()) return;
    (void)hipFree(it->second.tab);
    (void)hipFree(it->second.pay);
    (void)hipFree(it->second.d_counter);
    g_tables.erase(it);
}

// Rebuild the table at capacity 2^log2_cap on the device (growth, or the same size to drop tombstones): the
// live entries move from the old arrays into fresh ones in one launch, no host round trip (the dump + host
// re-insert it replaces moved the whole set over PCIe twice: ~0.5 GB at 5 M outpoints). Queued on the node
// stream behind any pending async apply, so the handle stays valid throughout. Returns (live entries moved) |
// (entries that found no slot << 32).
uint64_t utxo_rehash(int64_t h, uint32_t log2_cap) {
    if (log2_cap < 8 || log2_cap > 31) throw std::invalid_argument("log2 capacity must be in [8, 31]");
    std::lock_guard<std::mutex> lk(g_ut_mu);
    UtxoTableDev& t = table(h);
    const uint32_t cap = 1u << log2_cap;
    UtxoSlot* tab = nullptr;
    UtxoPayload* pay = nullptr;
    uck(hipMalloc(&tab, sizeof(UtxoSlot) * size_t(cap)), "hipMalloc utxo table (rehash)");
    try {
        uck(hipMalloc(&pay, sizeof(UtxoPayload) * size_t(cap)), "hipMalloc utxo payload (rehash)");
    } catch (...) {
        (void)hipFree(tab);
        throw;
    }
    node_memset(tab, 0, sizeof(UtxoSlot) * size_t(cap), "memset utxo table (rehash)");
    node_memset(pay, 0, sizeof(UtxoPayload) * size_t(cap), "memset utxo payload (rehash)");
    PooledBuf<uint32_t> cnt(4);
    node_memset(cnt.p, 0, 4 * sizeof(uint32_t), "memset");
    hipLaunchKernelGGL(utxo_migrate_kernel, dim3(int((t.cap + 255) / 256)), dim3(256), 0, node_stream(), t.tab, t.pay,
                       t.cap, tab, pay, cap - 1, cnt.p);
    uck(hipGetLastError(), "utxo_migrate_kernel");
    uint32_t c[4] = {0, 0, 0, 0};
    node_d2h(c, cnt.p, sizeof c, "d2h rehash counters");  // synchronises the node stream: the old arrays are idle
    (void)hipFree(t.tab);
    (void)hipFree(t.pay);
    t.tab = tab;
    t.pay = pay;
    t.cap = cap;
    return uint64_t(c[2] - c[0]) | (uint64_t(c[0]) << 32);
}

uint32_t utxo_capacity(int64_t h) {
    std::lock_guard<std::mutex> lk(g_ut_mu);
    return table(h).cap;
}

// per-call scratch comes from the caching pool (csrc/dev_pool.h): no hipMalloc/hipFree per block
template <typename T>
using DevBuf = PooledBuf<T>;

uint64_t utxo_insert(int64_t h, const uint8_t* recs, int64_t n, const uint8_t* payload) {
    std::lock_guard<std::mutex> lk(g_ut_mu);
    UtxoTableDev& t = table(h);
    if (n == 0) return 0;
    DevBuf<UtxoKeyRec> d(n);
    node_h2d(d.p, recs, sizeof(UtxoKeyRec) * n, "h2d recs");
    DevBuf<UtxoPayload> dp(payload ? n : 0);
    if (payload) node_h2d(dp.p, payload, sizeof(UtxoPayload) * n, "h2d payload");
    node_memset(t.d_counter, 0, 2 * sizeof(uint32_t), "memset");
    hipLaunchKernelGGL(utxo_insert_kernel, dim3(int((n + 255) / 256)), dim3(256), 0, node_stream(), t.tab, t.pay, t.cap - 1, d.p,
                       payload ? dp.p : nullptr, n, t.d_counter);
    uck(hipGetLastError(), "utxo_insert_kernel");
    uint32_t c[2] = {0, 0};
    node_d2h(c, t.d_counter, sizeof c, "d2h failed");
    return uint64_t(c[0]) | (uint64_t(c[1]) << 32);  // (table full) | (duplicates << 32)
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
    node_h2d(d.p, recs, sizeof(UtxoKeyRec) * n, "h2d recs");
    hipLaunchKernelGGL(utxo_lookup_kernel, dim3(int((n + 255) / 256)), dim3(256), 0, node_stream(), t.tab, t.pay, t.cap - 1, d.p, n,
                       o.p, po.p);
    uck(hipGetLastError(), "utxo_lookup_kernel");
    node_d2h(out.data(), o.p, size_t(n), "d2h tags");
    node_d2h(payload_out.data(), po.p, payload_out.size(), "d2h payload");
    return out;
}

std::vector<uint8_t> utxo_probe(int64_t h, const uint8_t* recs, int64_t n) {
    std::lock_guard<std::mutex> lk(g_ut_mu);
    UtxoTableDev& t = table(h);
    std::vector<uint8_t> out(static_cast<size_t>(n));
    if (n == 0) return out;
    DevBuf<UtxoKeyRec> d(n);
    DevBuf<uint8_t> o(n);
    node_h2d(d.p, recs, sizeof(UtxoKeyRec) * n, "h2d recs");
    hipLaunchKernelGGL(utxo_probe_kernel, dim3(int((n + 255) / 256)), dim3(256), 0, node_stream(), t.tab, t.cap - 1, d.p, n, o.p);
    uck(hipGetLastError(), "utxo_probe_kernel");
    node_d2h(out.data(), o.p, size_t(n), "d2h tags");
    return out;
}

std::vector<uint8_t> utxo_erase(int64_t h, const uint8_t* recs, int64_t n) {
    std::lock_guard<std::mutex> lk(g_ut_mu);
    UtxoTableDev& t = table(h);
    std::vector<uint8_t> out(static_cast<size_t>(n));
    if (n == 0) return out;
    DevBuf<UtxoKeyRec> d(n);
    DevBuf<uint8_t> o(n);
    node_h2d(d.p, recs, sizeof(UtxoKeyRec) * n, "h2d recs");
    node_memset(t.d_counter, 0, sizeof(uint32_t), "memset");
    hipLaunchKernelGGL(utxo_erase_kernel, dim3(int((n + 255) / 256)), dim3(256), 0, node_stream(), t.tab, t.cap - 1, d.p, n, o.p,
                       t.d_counter);
    uck(hipGetLastError(), "utxo_erase_kernel");
    node_d2h(out.data(), o.p, size_t(n), "d2h erased");
    return out;
}

std::vector<uint8_t> utxo_address_scan(int64_t h, const uint8_t* addr, uint32_t len, uint32_t tag_mask,
                                       uint32_t stake_sel, std::vector<uint8_t>& payload_out, uint64_t* total_out) {
    if (len > 64) throw std::invalid_argument("address is at most 64 bytes");
    std::lock_guard<std::mutex> lk(g_ut_mu);
    UtxoTableDev& t = table(h);
    uint4 q[4];
    std::memset(q, 0, sizeof(q));
    std::memcpy(q, addr, len);  // payload addresses are zero-padded to 64 bytes
    uint32_t qfp = 0;           // same bytes as addr_fingerprint() on the zero-padded query
    std::memcpy(&qfp, reinterpret_cast<const uint8_t*>(q) + 1, 4);
    // first pass sizes the output; a second pass runs only if more matches than the guess came back
    uint32_t cap_out = 4096, n = 0;
    DevBuf<unsigned long long> dt(1);
    for (int pass = 0; pass < 2; ++pass) {
        DevBuf<UtxoKeyRec> d(cap_out);
        DevBuf<UtxoPayload> dp(cap_out);
        node_memset(t.d_counter, 0, sizeof(uint32_t), "memset");
        node_memset(dt.p, 0, sizeof(unsigned long long), "memset");
        hipLaunchKernelGGL(utxo_address_scan_kernel, dim3(int((t.cap + 255) / 256)), dim3(256), 0, node_stream(), t.tab, t.pay,
                           t.cap, q[0], q[1], q[2], q[3], len, qfp, tag_mask, stake_sel, cap_out, d.p, dp.p, t.d_counter, dt.p);
        uck(hipGetLastError(), "utxo_address_scan_kernel");
        node_d2h(&n, t.d_counter, sizeof(uint32_t), "d2h n");
        if (n <= cap_out) {
            unsigned long long tot = 0;
            node_d2h(&tot, dt.p, sizeof(tot), "d2h total");
            *total_out = tot;
            std::vector<uint8_t> out(size_t(n) * sizeof(UtxoKeyRec));
            payload_out.assign(size_t(n) * sizeof(UtxoPayload), 0);
            if (n) {
                node_d2h(out.data(), d.p, out.size(), "d2h recs");
                node_d2h(payload_out.data(), dp.p, payload_out.size(), "d2h payload");
            }
            return out;
        }
        cap_out = n;
    }
    throw std::runtime_error("utxo_address_scan: table changed between passes");
}

std::vector<uint8_t> utxo_dump(int64_t h, std::vector<uint8_t>* payload_out) {
    std::lock_guard<std::mutex> lk(g_ut_mu);
    UtxoTableDev& t = table(h);
    DevBuf<UtxoKeyRec> d(t.cap);
    DevBuf<UtxoPayload> dp(payload_out ? t.cap : 0);
    node_memset(t.d_counter, 0, sizeof(uint32_t), "memset");
    hipLaunchKernelGGL(utxo_dump_kernel, dim3(int((t.cap + 255) / 256)), dim3(256), 0, node_stream(), t.tab, t.pay, t.cap, d.p,
                       payload_out ? dp.p : nullptr, t.d_counter);
    uck(hipGetLastError(), "utxo_dump_kernel");
    uint32_t n = 0;
    node_d2h(&n, t.d_counter, sizeof(uint32_t), "d2h n");
    std::vector<uint8_t> out(size_t(n) * sizeof(UtxoKeyRec));
    if (n) node_d2h(out.data(), d.p, out.size(), "d2h dump");
    if (payload_out) {
        payload_out->assign(size_t(n) * sizeof(UtxoPayload), 0);
        if (n) node_d2h(payload_out->data(), dp.p, payload_out->size(), "d2h payload");
    }
    return out;
}

// ================================================================================================
// Whole-block input pass (K7 + K10 + K11 in one round trip) and the sorted UTXO-set hash (K12).
// ================================================================================================

// K10: duplicate outpoints within a block. One 64-bit CAS per lane into a scratch table whose word
// packs a 40-bit fingerprint of (txid, index) with the lane id of the first inserter; a lane that
// meets its own fingerprint reports that lane (dup_of = winner + 1). The host confirms candidates
// against the full 36-byte keys, so a fingerprint collision can never fail a valid block.
__device__ __forceinline__ uint64_t outpoint_fp(const uint32_t k[8], uint32_t idx) {
    uint64_t h = (uint64_t(k[0]) << 32 | k[1]) ^ (uint64_t(k[2]) << 17) ^ (uint64_t(k[3]) * 0x9E3779B97F4A7C15ull) ^
                 (uint64_t(k[4]) << 7) ^ (uint64_t(k[5]) << 29) ^ k[6] ^ (uint64_t(k[7]) << 41) ^
                 (uint64_t(idx) * 0xC2B2AE3D27D4EB4Full);
    h ^= h >> 31;
    h *= 0xBF58476D1CE4E5B9ull;
    h ^= h >> 29;
    return h;
}

__global__ __launch_bounds__(256) void block_dup_kernel(const UtxoKeyRec* __restrict__ recs, int64_t n,
                                                        unsigned long long* __restrict__ scratch, uint32_t mask,
                                                        uint32_t* __restrict__ dup_of) {
    const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t k[8];
    load_key(recs[i], k);
    const uint64_t fp = outpoint_fp(k, recs[i].index & 0xffu);
    const unsigned long long mine = (fp & ~0xFFFFFFull) | (uint64_t(i) & 0xFFFFFFull);
    const unsigned long long want = fp & ~0xFFFFFFull;
    uint32_t s = uint32_t(fp) & mask;
    uint32_t res = 0;
    for (uint32_t probe = 0; probe <= mask; ++probe) {
        const unsigned long long prev = atomicCAS(&scratch[s], 0ull, mine);
        if (prev == 0ull) break;  // claimed: first occurrence
        if ((prev & ~0xFFFFFFull) == want) {
            res = uint32_t(prev & 0xFFFFFFull) + 1u;
            break;
        }
        s = (s + 1) & mask;
    }
    dup_of[i] = res;
}

// K11: per-tx fee = sum(spent amounts) - sum(output amounts), int64 smallest units; missing[t] counts
// inputs not found with the wanted tag.
__global__ __launch_bounds__(256) void block_fee_kernel(const uint8_t* __restrict__ tags,
                                                        const UtxoPayload* __restrict__ pay,
                                                        const int32_t* __restrict__ in_start,
                                                        const uint64_t* __restrict__ out_amount,
                                                        const int32_t* __restrict__ out_start, int64_t n_tx,
                                                        uint32_t want_tag, int64_t* __restrict__ fee,
                                                        uint32_t* __restrict__ missing) {
    const int64_t t = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (t >= n_tx) return;
    int64_t acc = 0;
    uint32_t miss = 0;
    for (int32_t k = in_start[t]; k < in_start[t + 1]; ++k) {
        if (tags[k] != want_tag || pay[k].addr_len == 0) ++miss;
        acc += int64_t(pay[k].amount);
    }
    for (int32_t k = out_start[t]; k < out_start[t + 1]; ++k) acc -= int64_t(out_amount[k]);
    fee[t] = acc;
    missing[t] = miss;
}

void utxo_block_inputs(int64_t h, const uint8_t* keys, int64_t n_in, const int32_t* in_start,
                       const uint64_t* out_amount, int64_t n_out, const int32_t* out_start, int64_t n_tx,
                       uint32_t want_tag, BlockInputsOut& r) {
    std::lock_guard<std::mutex> lk(g_ut_mu);
    UtxoTableDev& t = table(h);
    r.n_dup = 0;
    if (n_tx == 0) {  // no tx, so no input either: nothing to write
        return;
    }
    if (n_in >= (int64_t(1) << 24)) throw std::invalid_argument("too many inputs for one block pass");
    uint32_t log2 = 8;
    while ((int64_t(1) << log2) < 2 * n_in) ++log2;
    const uint32_t scap = 1u << log2;
    // Two arenas, one transfer each: the four inputs are packed into one pinned region laid out as the
    // device arena (one H2D), the five outputs are written into one device arena (one D2H), instead of
    // a copy call per array (each hipMemcpyAsync is ~5 us of host time on the block path).
    size_t in_off[5] = {0}, out_off[6] = {0};
    {
        const size_t in_n[4] = {sizeof(UtxoKeyRec) * size_t(n_in), 8 * size_t(n_out), 4 * size_t(n_tx + 1),
                                4 * size_t(n_tx + 1)};
        for (int i = 0; i < 4; ++i) in_off[i + 1] = ((in_off[i] + in_n[i]) + 255) & ~size_t(255);
        const size_t out_n[5] = {size_t(n_in), sizeof(UtxoPayload) * size_t(n_in), 4 * size_t(n_in),
                                 8 * size_t(n_tx), 4 * size_t(n_tx)};
        for (int i = 0; i < 5; ++i) out_off[i + 1] = ((out_off[i] + out_n[i]) + 255) & ~size_t(255);
    }
    DevBuf<uint8_t> d_in(in_off[4]), d_outa(out_off[5]);
    DevBuf<unsigned long long> d_scratch(scap);
    auto* d_keys = reinterpret_cast<UtxoKeyRec*>(d_in.p + in_off[0]);
    auto* d_out = reinterpret_cast<uint64_t*>(d_in.p + in_off[1]);
    auto* d_in_start = reinterpret_cast<int32_t*>(d_in.p + in_off[2]);
    auto* d_out_start = reinterpret_cast<int32_t*>(d_in.p + in_off[3]);
    auto* d_tags = d_outa.p + out_off[0];
    auto* d_pay = reinterpret_cast<UtxoPayload*>(d_outa.p + out_off[1]);
    auto* d_dup = reinterpret_cast<uint32_t*>(d_outa.p + out_off[2]);
    auto* d_fee = reinterpret_cast<int64_t*>(d_outa.p + out_off[3]);
    auto* d_miss = reinterpret_cast<uint32_t*>(d_outa.p + out_off[4]);
    StagedIO io(in_off[4] + out_off[5]);
    uint8_t* hin = io.h2d_take(in_off[4]);
    auto put = [&](int i, const void* src, size_t n) {  // (an empty input array's pointer may be null)
        if (n) std::memcpy(hin + in_off[i], src, n);
    };
    put(0, keys, sizeof(UtxoKeyRec) * size_t(n_in));
    put(1, out_amount, 8 * size_t(n_out));
    put(2, in_start, 4 * size_t(n_tx + 1));
    put(3, out_start, 4 * size_t(n_tx + 1));
    io.h2d_issue(d_in.p, hin, in_off[4]);
    node_memset(d_scratch.p, 0, sizeof(unsigned long long) * scap, "memset scratch");
    if (n_in) {
        const dim3 g(unsigned((n_in + 255) / 256));
        hipLaunchKernelGGL(utxo_lookup_kernel, g, dim3(256), 0, node_stream(), t.tab, t.pay, t.cap - 1, d_keys, n_in, d_tags,
                           d_pay);
        uck(hipGetLastError(), "utxo_lookup_kernel");
        hipLaunchKernelGGL(block_dup_kernel, g, dim3(256), 0, node_stream(), d_keys, n_in, d_scratch.p, scap - 1, d_dup);
        uck(hipGetLastError(), "block_dup_kernel");
    }
    hipLaunchKernelGGL(block_fee_kernel, dim3(unsigned((n_tx + 255) / 256)), dim3(256), 0, node_stream(), d_tags, d_pay,
                       d_in_start, d_out, d_out_start, n_tx, want_tag, d_fee, d_miss);
    uck(hipGetLastError(), "block_fee_kernel");
    const uint8_t* hout = io.d2h_arena(d_outa.p, out_off[5]);
    io.finish("block inputs");  // one sync, then each output copied once out of the pinned staging
    if (n_in) {  // (an empty numpy array's data pointer may be null)
        std::memcpy(r.tags, hout + out_off[0], size_t(n_in));
        std::memcpy(r.payload, hout + out_off[1], sizeof(UtxoPayload) * size_t(n_in));
        std::memcpy(r.dup_of, hout + out_off[2], 4 * size_t(n_in));
    }
    std::memcpy(r.fee, hout + out_off[3], 8 * size_t(n_tx));
    std::memcpy(r.missing, hout + out_off[4], 4 * size_t(n_tx));
    // exact confirmation of duplicate candidates (full 36-byte key compare)
    const UtxoKeyRec* kr = reinterpret_cast<const UtxoKeyRec*>(keys);
    for (int64_t i = 0; i < n_in; ++i) {
        if (!r.dup_of[i]) continue;
        const uint32_t w = r.dup_of[i] - 1;
        if (std::memcmp(kr[i].txid, kr[w].txid, 32) != 0 || (kr[i].index & 0xffu) != (kr[w].index & 0xffu))
            r.dup_of[i] = 0;  // fingerprint collision, not a duplicate
        else
            ++r.n_dup;
    }
}

// K12: SHA-256 over (txid || index byte) of every entry with `tag`, sorted by (txid, index).
// Stable LSD radix sort on the device (hipCUB): index, then the txid's four 64-bit big-endian words
// from least to most significant; the message is gathered on the device and hashed on the host
// (Merkle–Damgard is sequential).
__global__ __launch_bounds__(256) void set_compact_kernel(const UtxoSlot* __restrict__ tab, uint32_t cap,
                                                          uint32_t tag, UtxoKeyRec* __restrict__ out,
                                                          uint32_t* __restrict__ count) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= cap) return;
    const uint32_t m = tab[s].meta;
    if ((m & 3u) != ST_FULL || ((m >> 16) & 0xffu) != tag) return;
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
    r.tag = tag;
    out[o] = r;
}

// column c of the sort: 0 = index, 1..4 = big-endian txid word (4 - c), gathered through perm
__global__ __launch_bounds__(256) void sort_column_kernel(const UtxoKeyRec* __restrict__ recs,
                                                          const uint32_t* __restrict__ perm, uint32_t n, int c,
                                                          uint64_t* __restrict__ col) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const UtxoKeyRec& r = recs[perm[i]];
    if (c == 0) {
        col[i] = r.index & 0xffu;
        return;
    }
    const uint8_t* b = r.txid + 8 * (4 - c);
    uint64_t v = 0;
#pragma unroll
    for (int q = 0; q < 8; ++q) v = (v << 8) | b[q];
    col[i] = v;
}

__global__ __launch_bounds__(256) void iota_kernel(uint32_t* __restrict__ p, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = i;
}

__global__ __launch_bounds__(256) void set_message_kernel(const UtxoKeyRec* __restrict__ recs,
                                                          const uint32_t* __restrict__ perm, uint32_t n,
                                                          uint8_t* __restrict__ msg) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const UtxoKeyRec& r = recs[perm[i]];
    uint8_t* o = msg + size_t(i) * 33;
#pragma unroll
    for (int q = 0; q < 32; ++q) o[q] = r.txid[q];
    o[32] = uint8_t(r.index);
}

std::vector<uint8_t> utxo_set_message(int64_t h, uint32_t tag, uint64_t* count_out) {
    std::lock_guard<std::mutex> lk(g_ut_mu);
    UtxoTableDev& t = table(h);
    DevBuf<UtxoKeyRec> recs(t.cap);
    node_memset(t.d_counter, 0, sizeof(uint32_t), "memset");
    hipLaunchKernelGGL(set_compact_kernel, dim3((t.cap + 255) / 256), dim3(256), 0, node_stream(), t.tab, t.cap, tag, recs.p,
                       t.d_counter);
    uck(hipGetLastError(), "set_compact_kernel");
    uint32_t n = 0;
    node_d2h(&n, t.d_counter, sizeof(uint32_t), "d2h n");
    if (count_out) *count_out = n;
    std::vector<uint8_t> msg(size_t(n) * 33);
    if (n) {
        DevBuf<uint32_t> perm_a(n), perm_b(n);
        DevBuf<uint64_t> col_a(n), col_b(n);
        const dim3 g((n + 255) / 256);
        hipLaunchKernelGGL(iota_kernel, g, dim3(256), 0, node_stream(), perm_a.p, n);
        size_t temp_bytes = 0;
        uck(hipcub::DeviceRadixSort::SortPairs(nullptr, temp_bytes, col_a.p, col_b.p, perm_a.p, perm_b.p, n, 0, 64,
                                               node_stream()),
            "radix sort sizing");
        DevBuf<uint8_t> temp(temp_bytes);
        for (int c = 0; c <= 4; ++c) {  // least significant column first; radix sort is stable
            hipLaunchKernelGGL(sort_column_kernel, g, dim3(256), 0, node_stream(), recs.p, perm_a.p, n, c, col_a.p);
            uck(hipGetLastError(), "sort_column_kernel");
            uck(hipcub::DeviceRadixSort::SortPairs(temp.p, temp_bytes, col_a.p, col_b.p, perm_a.p, perm_b.p, n,
                                                   0, c == 0 ? 8 : 64, node_stream()),
                "radix sort");
            std::swap(perm_a.p, perm_b.p);
        }
        DevBuf<uint8_t> d_msg(size_t(n) * 33);
        hipLaunchKernelGGL(set_message_kernel, g, dim3(256), 0, node_stream(), recs.p, perm_a.p, n, d_msg.p);
        uck(hipGetLastError(), "set_message_kernel");
        node_d2h(msg.data(), d_msg.p, msg.size(), "d2h message");
    }
    return msg;
}

// ---- K12 off the block path: the block thread takes a snapshot (one compaction launch on the node stream,
// so it sees exactly this block's table; no host sync), a worker thread turns it into the digest (sort and
// gather on the aux stream, chunked D2H into pinned buffers overlapped with the host SHA-256). The next
// block's kernels never queue behind the sort, and the 33-byte-per-UTXO message never becomes one host
// allocation (165 MB at 5 M UTXOs).
struct K12Snap {
    int device = 0;
    uint32_t cap = 0;
    PooledBuf<UtxoKeyRec> recs;
    PooledBuf<uint32_t> count;
    hipEvent_t ready = nullptr;
    K12Snap(uint32_t c) : cap(c), recs(c), count(1) {}
};
static std::mutex g_k12_mu;
static std::unordered_map<int64_t, std::unique_ptr<K12Snap>> g_k12;
static int64_t g_k12_next = 1;

int64_t utxo_k12_snapshot(int64_t h, uint32_t tag) {
    std::unique_ptr<K12Snap> s;
    {
        std::lock_guard<std::mutex> lk(g_ut_mu);
        UtxoTableDev& t = table(h);
        s = std::make_unique<K12Snap>(t.cap);
        s->device = t.device;
        node_memset(s->count.p, 0, sizeof(uint32_t), "memset k12 count");
        hipLaunchKernelGGL(set_compact_kernel, dim3((t.cap + 255) / 256), dim3(256), 0, node_stream(), t.tab, t.cap,
                           tag, s->recs.p, s->count.p);
        uck(hipGetLastError(), "set_compact_kernel");
        uck(hipEventCreateWithFlags(&s->ready, hipEventDisableTiming), "hipEventCreate");
        uck(hipEventRecord(s->ready, node_stream()), "hipEventRecord");
    }
    std::lock_guard<std::mutex> g(g_k12_mu);
    const int64_t id = g_k12_next++;
    g_k12[id] = std::move(s);
    return id;
}

std::vector<uint8_t> utxo_k12_digest(int64_t id, uint64_t* count_out) {
    std::unique_ptr<K12Snap> s;
    {
        std::lock_guard<std::mutex> g(g_k12_mu);
        auto it = g_k12.find(id);
        if (it == g_k12.end()) throw std::invalid_argument("bad K12 snapshot id");
        s = std::move(it->second);
        g_k12.erase(it);
    }
    uck(hipSetDevice(s->device), "hipSetDevice");
    hipStream_t st = aux_stream();
    uck(hipStreamWaitEvent(st, s->ready, 0), "hipStreamWaitEvent");
    uint32_t n = 0;
    uck(hipMemcpyAsync(&n, s->count.p, sizeof(uint32_t), hipMemcpyDeviceToHost, st), "d2h k12 count");
    uck(hipStreamSynchronize(st), "k12 count sync");
    if (count_out) *count_out = n;
    HostSha256 sha;
    if (n) {
        PooledBuf<uint32_t> perm_a(n), perm_b(n);
        PooledBuf<uint64_t> col_a(n), col_b(n);
        const dim3 g((n + 255) / 256);
        hipLaunchKernelGGL(iota_kernel, g, dim3(256), 0, st, perm_a.p, n);
        size_t temp_bytes = 0;
        uck(hipcub::DeviceRadixSort::SortPairs(nullptr, temp_bytes, col_a.p, col_b.p, perm_a.p, perm_b.p, n, 0, 64, st),
            "radix sort sizing");
        PooledBuf<uint8_t> temp(temp_bytes);
        uint32_t* pa = perm_a.p;
        uint32_t* pb = perm_b.p;
        for (int c = 0; c <= 4; ++c) {  // least significant column first; radix sort is stable
            hipLaunchKernelGGL(sort_column_kernel, g, dim3(256), 0, st, s->recs.p, pa, n, c, col_a.p);
            uck(hipGetLastError(), "sort_column_kernel");
            uck(hipcub::DeviceRadixSort::SortPairs(temp.p, temp_bytes, col_a.p, col_b.p, pa, pb, n, 0, c == 0 ? 8 : 64,
                                                   st),
                "radix sort");
            std::swap(pa, pb);
        }
        PooledBuf<uint8_t> d_msg(size_t(n) * 33);
        hipLaunchKernelGGL(set_message_kernel, g, dim3(256), 0, st, s->recs.p, pa, n, d_msg.p);
        uck(hipGetLastError(), "set_message_kernel");
        // two pinned staging buffers: chunk k+1 is copied while chunk k is hashed
        constexpr size_t kChunk = size_t(16) << 20;
        static uint8_t* pinned[2] = {nullptr, nullptr};
        static std::mutex pin_mu;
        std::lock_guard<std::mutex> pl(pin_mu);
        for (auto& b : pinned)
            if (!b) uck(hipHostMalloc(reinterpret_cast<void**>(&b), kChunk, hipHostMallocDefault), "hipHostMalloc");
        hipEvent_t ev[2];
        for (auto& e : ev) uck(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
        const size_t total = size_t(n) * 33;
        auto issue = [&](size_t off, int b) {
            const size_t len = std::min(kChunk, total - off);
            uck(hipMemcpyAsync(pinned[b], d_msg.p + off, len, hipMemcpyDeviceToHost, st), "d2h k12 chunk");
            uck(hipEventRecord(ev[b], st), "hipEventRecord");
            return len;
        };
        size_t off = 0;
        int b = 0;
        size_t len = issue(0, 0);
        while (len) {
            uck(hipEventSynchronize(ev[b]), "k12 chunk sync");
            const size_t next = off + len;
            size_t next_len = 0;
            if (next < total) next_len = issue(next, 1 - b);
            sha.update(pinned[b], len);
            off = next;
            len = next_len;
            b = 1 - b;
        }
        uck(hipStreamSynchronize(st), "k12 sync");  // the pooled buffers may be reused after this
        for (auto& e : ev) (void)hipEventDestroy(e);
    }
    (void)hipEventDestroy(s->ready);
    std::vector<uint8_t> digest(32);
    sha.final(digest.data());
    return digest;
}

// the sequential SHA-256 tail runs without the table lock: block application is not held up by it
std::vector<uint8_t> utxo_set_hash(int64_t h, uint32_t tag, uint64_t* count_out) {
    const std::vector<uint8_t> msg = utxo_set_message(h, tag, count_out);
    std::vector<uint8_t> digest(32);
    host_sha256(msg.data(), msg.size(), digest.data());
    return digest;
}

}  // namespace upow
