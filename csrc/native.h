// Declarations shared between the pybind11 bindings (bindings.cpp, host C++) and the HIP
// translation units (*.hip). Only plain host types cross this boundary.
#pragma once
#include <cstdint>
#include <functional>
#include <string>
#include <vector>

namespace upow {

// ---------------------------------------------------------------- PoW (K1)
struct PowJobHost {
    std::vector<uint8_t> header;  // full 108-byte (v2) or 138-byte (v1) header; nonce bytes ignored
    uint32_t tmask = 0, tword = 0, frac_shift = 0, frac_limit = 16;
};

struct PowResult {
    uint64_t searched = 0;
    uint32_t total_hits = 0;
    std::vector<uint32_t> words;  // candidate nonce words (v2: bswap(nonce), v1: nonce)
};

struct PowKernelInfo {
    int cus = 0, blocks_per_cu = 0, resident_blocks = 0;
};
PowKernelInfo pow_kernel_info(int variant);

bool pow_check_word_host(const PowJobHost& job, uint32_t v);
PowResult pow_search_host(const PowJobHost& job, uint64_t start, uint64_t count, int threads);
PowResult pow_search_gpu(const PowJobHost& job, uint64_t start, uint64_t count, int grid_blocks,
                         uint32_t chunk_iters, uint32_t cap, int variant);

// ---------------------------------------------------------------- batched SHA-256 (K3/K4/K12)
// messages packed back to back in `data`, message i = data[offsets[i] .. offsets[i+1])
std::vector<uint8_t> sha256_batch_host(const uint8_t* data, const int64_t* offsets, int64_t n, int threads);
std::vector<uint8_t> sha256_batch_gpu(const uint8_t* data, int64_t nbytes, const int64_t* offsets, int64_t n);

// ---------------------------------------------------------------- P-256 (K5/K6/K15)
// verify items: 160-byte records {qx LE, qy LE, r LE, s LE, e = SHA-256 digest BE}
// status: 1 valid, 0 invalid, 2 key off-curve, 3 r/s out of range
std::vector<uint8_t> p256_verify_host(const uint8_t* items, int64_t n, int threads);
// one 160-byte VerifyItem on 64-bit limbs (csrc/p256_host.cpp); status as p256_verify_host
uint8_t p256_verify_one_host64(const uint8_t* item);
// p256.hip's fixed-base table: 32 x 256 affine points, each x[8] y[8] little-endian u32 words
const void* p256_g_table_host();
// s^-1 * 2^256 mod n for s in [1, n) (little-endian 64-bit limbs): the divsteps inverse of p256_field.h
void p256_scalar_inv_mont_host(uint64_t out[4], const uint64_t s[4]);
// a*b, a^2, a+b, a-b mod p (8 little-endian 32-bit limbs each, canonical inputs); c (16 limbs) mod p
void p256_fe_ops_host(const uint32_t a[8], const uint32_t b[8], uint32_t out[32]);
void p256_fe_reduce_host(const uint32_t c[16], uint32_t out[8]);
// the cluster's per-block commit vote on a native RCCL communicator of its own (csrc/rccl_vote.hip)
// one-lane-per-signature batch verify launch (csrc/p256_batch.hip): VerifyItem items, 16-bit G table,
// 16 window-table entries of scratch per signature, status bytes
void p256_batch_launch(char variant, const void* items, int64_t n, const void* gtab16, void* scratch, uint8_t* status,
                       int spw, void* stream);
std::string rccl_unique_id();
int64_t rccl_vote_create(const std::string& uid, int world, int rank);
void rccl_vote_start(int64_t h, int value);
int64_t rccl_vote_finish(int64_t h, double timeout_s);  // SUM of the votes, -1 on timeout
void rccl_vote_destroy(int64_t h, bool abort);
std::vector<double> rccl_vote_stats(int64_t h);  // votes, then seconds in the all-gather, copy, event enqueues
// entries [first, first + count) of the device's 16-bit fixed-base window table (x, y little-endian each)
std::vector<uint8_t> p256_g16_entries(int64_t first, int64_t count);
std::vector<uint8_t> p256_verify_gpu(const uint8_t* items, int64_t n);
void p256_decompress_host(const uint8_t* in33, int64_t n, uint8_t* out64, uint8_t* ok);
void p256_decompress_gpu(const uint8_t* in33, int64_t n, uint8_t* out64, uint8_t* ok);
// signer keys decompressed into verify items on the device, output addresses curve-checked, signatures
// verified: one stream order, one sync (p256.hip); fill(jobkeys33, sigdig96, outkeys33) packs the inputs
void p256_verify_fused_gpu(int64_t n_jobs, int64_t n_out, const std::function<void(uint8_t*, uint8_t*, uint8_t*)>& fill,
                           uint8_t* st, uint8_t* out_ok, std::vector<uint8_t>* items_out);
// on-curve check of 64-byte (version-1) addresses x LE | y LE: ok[i] = 1 iff x, y < p and y^2 = x^3 - 3x + b
void p256_on_curve_host(const uint8_t* xy64, int64_t n, uint8_t* ok, int threads);
void p256_on_curve_gpu(const uint8_t* xy64, int64_t n, uint8_t* ok);
// pin node-side GPU work of this process to one device (csrc/streams.h node_device_enter); -1 = unpinned
void set_node_device_native(int dev);
bool p256_pubkey(const uint8_t d_be[32], uint8_t out_le[64]);
bool p256_sign(const uint8_t d_be[32], const uint8_t digest[32], uint8_t r_le[32], uint8_t s_le[32]);

// ---------------------------------------------------------------- HBM UTXO index (K7/K8/K9)
// key records: 40 bytes {txid[32] raw, uint32 index, uint32 tag}
int64_t utxo_create(uint32_t log2_cap);
void utxo_destroy(int64_t h);
uint32_t utxo_capacity(int64_t h);
uint64_t utxo_rehash(int64_t h, uint32_t log2_cap);  // #moved | (#no slot << 32)
// payload records: 80 bytes {u64 amount, u32 address length, u32 pad, address[64]} (nullptr = zeros)
uint64_t utxo_insert(int64_t h, const uint8_t* recs, int64_t n, const uint8_t* payload);  // #full | (#duplicates << 32)
std::vector<uint8_t> utxo_probe(int64_t h, const uint8_t* recs, int64_t n);  // tag or 0xff
std::vector<uint8_t> utxo_lookup(int64_t h, const uint8_t* recs, int64_t n, std::vector<uint8_t>& payload_out);
std::vector<uint8_t> utxo_erase(int64_t h, const uint8_t* recs, int64_t n);  // 1 if erased
// queue one block's inserts + erases on the node stream and return; prev = the previous async apply's
// (no free slot, duplicates, erased) counters, collected first (returns whether there was one)
struct UtxoSeg { const uint8_t* recs; const uint8_t* pay; int64_t n; };  // n x 40 records, n x 80 payloads
bool utxo_apply_async(int64_t h, const std::vector<UtxoSeg>& ins, bool with_pay, const uint8_t* del, int64_t n_del,
                      uint32_t prev[3]);
bool utxo_apply_wait(int64_t h, uint32_t out[3]);  // collect the pending async apply's counters
std::vector<uint8_t> utxo_dump(int64_t h, std::vector<uint8_t>* payload_out);
// K14: live outputs whose payload address equals addr[0:len] and whose tag is in tag_mask
std::vector<uint8_t> utxo_address_scan(int64_t h, const uint8_t* addr, uint32_t len, uint32_t tag_mask,
                                       uint32_t stake_sel, std::vector<uint8_t>& payload_out, uint64_t* total_out);

// whole-block input pass: lookup (K7) + duplicate candidates (K10) + per-tx fees (K11) in one round trip
// Outputs of the whole-block input pass, written in place (the caller's arrays: no intermediate copies)
struct BlockInputsOut {
    uint8_t* tags;      // per input: table tag (0xff absent)
    uint8_t* payload;   // per input: 80-byte payload
    uint32_t* dup_of;   // per input: 1 + index of the earlier identical input, else 0
    int64_t* fee;       // per tx: sum(spent) - sum(outputs), smallest units
    uint32_t* missing;  // per tx: inputs not found with want_tag (or without payload)
    uint32_t n_dup = 0;
};
void utxo_block_inputs(int64_t h, const uint8_t* keys, int64_t n_in, const int32_t* in_start,
                       const uint64_t* out_amount, int64_t n_out, const int32_t* out_start, int64_t n_tx,
                       uint32_t want_tag, BlockInputsOut& r);
// K12: SHA-256 over (txid || index byte) of the entries with `tag`, sorted by (txid, index)
std::vector<uint8_t> utxo_set_hash(int64_t h, uint32_t tag, uint64_t* count_out);
// the (txid || index byte) message of table `tag` sorted by (txid, index): K12 without its hash tail
std::vector<uint8_t> utxo_set_message(int64_t h, uint32_t tag, uint64_t* count_out);
int64_t utxo_k12_snapshot(int64_t h, uint32_t tag);
std::vector<uint8_t> utxo_k12_digest(int64_t id, uint64_t* count_out);

// ---------------------------------------------------------------- base58
std::string b58encode(const uint8_t* data, size_t n);  // n <= kB58MaxInput
// allocation-free form: writes at most kB58MaxOutput characters to out, returns how many
constexpr size_t kB58MaxInput = 64, kB58MaxOutput = 88;  // 64 bytes -> at most 88 digits
size_t b58encode_to(const uint8_t* data, size_t n, char* out);
std::vector<uint8_t> b58decode(const std::string& s);

// ---------------------------------------------------------------- device info
int gpu_device_count();
std::string gpu_arch_name(int device);

}  // namespace upow
