// K5/K6/K15: P-256 ECDSA batch verify, point decompression, keygen and RFC 6979 signing.
//
// reference: fastecdsa ecdsa.verify / ecdsa.sign / keys.get_public_key / util.mod_sqrt, called one
// signature at a time from upow/upow_transactions/transaction_input.py:84-120,
// upow/upow_transactions/transaction.py:148-180,484-497 and upow/helpers.py:58-62,135-144.
//
// GPU design (gfx950, one signature per lane):
//  * u1*G uses a fixed-base byte-window table T[j][b] = b*256^j*G (32 x 255 affine points, 522 KB,
//    L2/Infinity-Cache resident) -> 32 mixed additions and no doublings;
//  * u2*Q uses a 4-bit fixed window over a per-lane table {1..15}Q kept in global scratch
//    ([lane][k] 96-byte Jacobian entries) because 1.4 KB per lane does not fit LDS at useful
//    occupancy -> 256 doublings + 64 additions;
//  * no field inversion: x(R) == r is tested as X == r*Z^2 (and (r+n)*Z^2 when r+n < p);
//  * s^-1 mod n by a Montgomery-domain fixed-window exponentiation;
//  * status per item: 1 valid, 0 invalid, 2 public key not on curve, 3 r/s out of [1, n]
//    (fastecdsa raises for 2/3; the Python layer turns them into EcdsaError).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "dev_pool.h"
#include "native.h"
#include "streams.h"
#include "p256_field.h"
#include "sha256_common.h"

namespace upow {
using namespace p256;

// ------------------------------------------------------------------------------------------------
// fixed-base table (host-built once, uploaded once per device)
// ------------------------------------------------------------------------------------------------
static constexpr int kGWin = 32;   // byte windows
static constexpr int kGEnt = 256;  // entry 0 unused

static std::once_flag g_tab_once;
static std::vector<aff> g_tab;  // [kGWin][kGEnt]

static void build_g_table() {
    std::vector<jac> jt(size_t(kGWin) * kGEnt);
    jac base = jac_from_aff(aff{fe{P256_GX}, fe{P256_GY}});
    for (int j = 0; j < kGWin; ++j) {
        jac acc = jac_inf();
        for (int b = 1; b < kGEnt; ++b) {
            acc = jac_add(acc, base);
            jt[size_t(j) * kGEnt + b] = acc;
        }
        // base <- 256 * base
        jac nb = base;
        for (int k = 0; k < 8; ++k) nb = jac_dbl(nb);
        base = nb;
    }
    // batch-normalise (Montgomery's trick) skipping entry 0
    std::vector<fe> pref(jt.size());
    fe run = fe_one();
    for (size_t i = 0; i < jt.size(); ++i) {
        if (i % kGEnt == 0) { pref[i] = run; continue; }
        pref[i] = run;
        run = fe_mul(run, jt[i].z);
    }
    fe inv = fe_inv(run);
    g_tab.assign(jt.size(), aff{fe_zero(), fe_zero()});
    for (size_t ii = jt.size(); ii-- > 0;) {
        if (ii % kGEnt == 0) continue;
        const fe zi = fe_mul(inv, pref[ii]);
        inv = fe_mul(inv, jt[ii].z);
        const fe zi2 = fe_sqr(zi);
        g_tab[ii].x = fe_mul(jt[ii].x, zi2);
        g_tab[ii].y = fe_mul(jt[ii].y, fe_mul(zi2, zi));
    }
}

static const std::vector<aff>& g_table() {
    std::call_once(g_tab_once, build_g_table);
    return g_tab;
}

const void* p256_g_table_host() { return g_table().data(); }

UPOW_HD jac mul_g(const fe& k, const aff* tab) {
    jac acc = jac_inf();
    for (int j = 0; j < kGWin; ++j) {
        const uint32_t b = fe_byte(k, j);
        if (b) acc = jac_madd(acc, tab[j * kGEnt + b]);
    }
    return acc;
}

// ------------------------------------------------------------------------------------------------
// shared verify core
// ------------------------------------------------------------------------------------------------
struct VerifyItem {  // 160 bytes, wire byte order
    uint8_t qx[32];  // little-endian
    uint8_t qy[32];  // little-endian
    uint8_t r[32];   // little-endian
    uint8_t s[32];   // little-endian
    uint8_t e[32];   // SHA-256 digest, big-endian
};
static_assert(sizeof(VerifyItem) == 160, "VerifyItem layout");

UPOW_HD uint8_t verify_prologue(const VerifyItem& it, aff& q, fe& r, fe& u1, fe& u2) {
    q.x = fe_from_le(it.qx);
    q.y = fe_from_le(it.qy);
    if (!aff_on_curve(q)) return 2;
    r = fe_from_le(it.r);
    const fe s = fe_from_le(it.s);
    const fe n = fe_const_n();
    // fastecdsa: raise if r > n or r < 1 (same for s)
    if (fe_is_zero(r) || (fe_geq(r, n) && !fe_eq(r, n))) return 3;
    if (fe_is_zero(s) || (fe_geq(s, n) && !fe_eq(s, n))) return 3;
    if (fe_eq(s, n)) return 0;  // s has no inverse mod n
    const fe e = sc_reduce(fe_from_be(it.e));
    const fe w_m = sc_inv_mont(sc_to_mont(s));  // s^-1 * R
    u1 = sc_mont_mul(e, w_m);                   // e * s^-1
    u2 = sc_mont_mul(sc_reduce(r), w_m);        // r * s^-1
    return 255;                                 // continue
}

UPOW_HD uint8_t verify_epilogue(const jac& R, const fe& r) {
    if (jac_is_inf(R)) return 0;
    const fe z2 = fe_sqr(R.z);
    if (fe_eq(fe_mul(r, z2), R.x)) return 1;
    // r + n < p ?  (x(R) in [n, p) maps to x mod n = x - n)
    fe rn;
    const uint32_t c = raw_add(rn, r, fe_const_n());
    if (!c && !fe_geq(rn, fe_const_p())) {
        if (fe_eq(fe_mul(rn, z2), R.x)) return 1;
    }
    return 0;
}

static uint8_t verify_one_host(const VerifyItem& it, const aff* gtab) {
    aff q;
    fe r, u1, u2;
    const uint8_t pro = verify_prologue(it, q, r, u1, u2);
    if (pro != 255) return pro;
    jac tbl[16];
    tbl[0] = jac_inf();
    tbl[1] = jac_from_aff(q);
    for (int k = 2; k < 16; ++k) tbl[k] = jac_madd(tbl[k - 1], q);
    jac acc = jac_inf();
    for (int w = 63; w >= 0; --w) {
        if (!jac_is_inf(acc)) { acc = jac_dbl(acc); acc = jac_dbl(acc); acc = jac_dbl(acc); acc = jac_dbl(acc); }
        const uint32_t nib = fe_nibble(u2, w);
        if (nib) acc = jac_add(acc, tbl[nib]);
    }
    const jac R = jac_add(mul_g(u1, gtab), acc);
    return verify_epilogue(R, r);
}

// ------------------------------------------------------------------------------------------------
// device kernels
// ------------------------------------------------------------------------------------------------
// Per-lane window table {1..15}Q lives in global scratch. SOA = false: [lane][k] Jacobian entries
// (each lane's 16 x 96 B contiguous; a table load gathers 64 scattered lines per dword). SOA = true:
// dword-major [k][dword][lane], so the lanes of a wave that picked the same window digit read one
// contiguous run per dword (at most 16 distinct runs per load instead of 64 lines).
template <bool SOA>
__device__ __forceinline__ void tab_store(jac* scratch, int64_t n, int64_t i, int k, const jac& p) {
    if (SOA) {
        uint32_t* s = reinterpret_cast<uint32_t*>(scratch);
        const uint32_t* src = reinterpret_cast<const uint32_t*>(&p);
#pragma unroll
        for (int d = 0; d < 24; ++d) s[(int64_t(k) * 24 + d) * n + i] = src[d];
    } else {
        scratch[i * 16 + k] = p;
    }
}

template <bool SOA>
__device__ __forceinline__ jac tab_load(const jac* scratch, int64_t n, int64_t i, int k) {
    if (SOA) {
        jac p;
        const uint32_t* s = reinterpret_cast<const uint32_t*>(scratch);
        uint32_t* dst = reinterpret_cast<uint32_t*>(&p);
#pragma unroll
        for (int d = 0; d < 24; ++d) dst[d] = s[(int64_t(k) * 24 + d) * n + i];
        return p;
    }
    return scratch[i * 16 + k];
}

template <int MIN_WAVES, bool SOA>
__global__ __launch_bounds__(64, MIN_WAVES) void p256_verify_kernel(const VerifyItem* __restrict__ items, int64_t n,
                                                          const aff* __restrict__ gtab, jac* __restrict__ scratch,
                                                          uint8_t* __restrict__ status) {
    const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const VerifyItem it = items[i];
    aff q;
    fe r, u1, u2;
    const uint8_t pro = verify_prologue(it, q, r, u1, u2);
    if (pro != 255) { status[i] = pro; return; }
    jac t = jac_from_aff(q);
    tab_store<SOA>(scratch, n, i, 1, t);
    for (int k = 2; k < 16; ++k) {
        t = jac_madd(t, q);
        tab_store<SOA>(scratch, n, i, k, t);
    }
    jac acc = jac_inf();
    for (int w = 63; w >= 0; --w) {
        acc = jac_dbl(acc); acc = jac_dbl(acc); acc = jac_dbl(acc); acc = jac_dbl(acc);
        const uint32_t nib = fe_nibble(u2, w);
        if (nib) acc = jac_add(acc, tab_load<SOA>(scratch, n, i, int(nib)));
    }
    const jac R = jac_add(mul_g(u1, gtab), acc);
    status[i] = verify_epilogue(R, r);
}

// item: 33-byte compressed address [spec | x LE]; out: x LE | y LE (64 B) and ok flag
__global__ __launch_bounds__(256) void p256_decompress_kernel(const uint8_t* __restrict__ in, int64_t n,
                                                               uint8_t* __restrict__ out, uint8_t* __restrict__ ok) {
    const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint8_t* a = in + 33 * i;
    const fe x = fe_from_le(a + 1);
    const bool odd = a[0] == 43;
    bool good = !fe_geq(x, fe_const_p());
    const fe x3 = fe_mul(fe_sqr(x), x);
    const fe rhs = fe_add(fe_sub(x3, fe_add(fe_add(x, x), x)), fe_const_b());
    fe y = fe_sqrt_candidate(rhs);
    good = good && fe_eq(fe_sqr(y), rhs);
    if ((y.v[0] & 1u) != uint32_t(odd)) y = fe_neg(y);
    fe_to_le(x, out + 64 * i);
    fe_to_le(y, out + 64 * i + 32);
    ok[i] = good ? 1 : 0;
}

static void hck(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

struct DeviceGTable {
    int device = -1;
    aff* d_tab = nullptr;
};
static std::mutex g_dev_mu;
static DeviceGTable g_dev_tabs[16];

static const aff* device_g_table() {
    int dev = 0;
    hck(hipGetDevice(&dev), "hipGetDevice");
    if (dev < 0 || dev >= 16) throw std::runtime_error("device index out of range");
    std::lock_guard<std::mutex> lk(g_dev_mu);
    DeviceGTable& t = g_dev_tabs[dev];
    if (!t.d_tab) {
        const auto& h = g_table();
        hck(hipMalloc(&t.d_tab, sizeof(aff) * h.size()), "hipMalloc gtab");
        node_h2d(t.d_tab, h.data(), sizeof(aff) * h.size(), "h2d gtab");
        node_sync("gtab upload");
        t.device = dev;
    }
    return t.d_tab;
}

// ------------------------------------------------------------------------------------------------
// host API
// ------------------------------------------------------------------------------------------------
std::vector<uint8_t> p256_verify_host(const uint8_t* items, int64_t n, int threads) {
    std::vector<uint8_t> st(static_cast<size_t>(n));
    const aff* tab = g_table().data();
    const VerifyItem* it = reinterpret_cast<const VerifyItem*>(items);
    static const bool legacy = [] {
        const char* v = std::getenv("UPOW_P256_HOST32");
        return v && v[0] == '1';
    }();
    threads = int(std::max<int64_t>(1, std::min<int64_t>(threads, n)));
    auto work = [&](int t) {
        if (legacy)  // UPOW_P256_HOST32=1: the 32-bit-limb field code the GPU kernel uses
            for (int64_t i = t; i < n; i += threads) st[i] = verify_one_host(it[i], tab);
        else
            for (int64_t i = t; i < n; i += threads)
                st[i] = p256_verify_one_host64(reinterpret_cast<const uint8_t*>(&it[i]));
    };
    if (threads <= 1) {
        work(0);
    } else {
        std::vector<std::thread> pool;
        for (int t = 0; t < threads; ++t) pool.emplace_back(work, t);
        for (auto& th : pool) th.join();
    }
    return st;
}

std::vector<uint8_t> p256_verify_gpu(const uint8_t* items, int64_t n) {
    std::vector<uint8_t> st(static_cast<size_t>(n));
    if (n == 0) return st;
    const aff* d_tab = device_g_table();
    PooledBuf<VerifyItem> b_items{size_t(n)};
    PooledBuf<jac> b_scratch(size_t(16) * size_t(n));
    PooledBuf<uint8_t> b_st{size_t(n)};
    VerifyItem* d_items = b_items.p;
    jac* d_scratch = b_scratch.p;
    uint8_t* d_st = b_st.p;
    node_h2d(d_items, items, sizeof(VerifyItem) * n, "h2d items");
    const int block = 64;
    const int grid = int((n + block - 1) / block);
    // Default (variant 1): __launch_bounds__(64, 4) -> 4 waves/SIMD at 128 VGPRs (a few spills), 7-9 %
    // faster than the compiler's 142-VGPR / 3-wave choice (variant 0) in the A/B runs of
    // scripts/p256_throughput.py (profiles/p256_variants_ab.txt). Variant 2: dword-major (SoA)
    // window tables, slower (the gathers were not the bottleneck).
    const char* var = std::getenv("UPOW_P256_VARIANT");
    const char v = var ? var[0] : '1';
    if (v == '0')
        hipLaunchKernelGGL((p256_verify_kernel<1, false>), dim3(grid), dim3(block), 0, node_stream(), d_items, n, d_tab, d_scratch,
                           d_st);
    else if (v == '2')
        hipLaunchKernelGGL((p256_verify_kernel<1, true>), dim3(grid), dim3(block), 0, node_stream(), d_items, n, d_tab, d_scratch,
                           d_st);
    else
        hipLaunchKernelGGL((p256_verify_kernel<4, false>), dim3(grid), dim3(block), 0, node_stream(), d_items, n, d_tab, d_scratch,
                           d_st);
    hck(hipGetLastError(), "p256_verify_kernel launch");
    node_d2h(st.data(), d_st, size_t(n), "d2h status");
    return st;
}

void p256_decompress_host(const uint8_t* in, int64_t n, uint8_t* out, uint8_t* ok) {
    for (int64_t i = 0; i < n; ++i) {
        const uint8_t* a = in + 33 * i;
        const fe x = fe_from_le(a + 1);
        const bool odd = a[0] == 43;
        bool good = !fe_geq(x, fe_const_p());
        const fe rhs = fe_add(fe_sub(fe_mul(fe_sqr(x), x), fe_add(fe_add(x, x), x)), fe_const_b());
        fe y = fe_sqrt_candidate(rhs);
        good = good && fe_eq(fe_sqr(y), rhs);
        if ((y.v[0] & 1u) != uint32_t(odd)) y = fe_neg(y);
        fe_to_le(x, out + 64 * i);
        fe_to_le(y, out + 64 * i + 32);
        ok[i] = good ? 1 : 0;
    }
}

void p256_decompress_gpu(const uint8_t* in, int64_t n, uint8_t* out, uint8_t* ok) {
    if (n == 0) return;
    PooledBuf<uint8_t> b_in{33 * size_t(n)}, b_out{64 * size_t(n)}, b_ok{size_t(n)};
    uint8_t *d_in = b_in.p, *d_out = b_out.p, *d_ok = b_ok.p;
    node_h2d(d_in, in, 33 * size_t(n), "h2d in");
    const int block = 256;
    hipLaunchKernelGGL(p256_decompress_kernel, dim3(int((n + block - 1) / block)), dim3(block), 0, node_stream(), d_in, n,
                       d_out, d_ok);
    hck(hipGetLastError(), "p256_decompress_kernel launch");
    node_d2h(out, d_out, 64 * size_t(n), "d2h out");
    node_d2h(ok, d_ok, size_t(n), "d2h ok");
}

bool p256_pubkey(const uint8_t d_be[32], uint8_t out_le[64]) {
    const fe d = fe_from_be(d_be);
    if (fe_is_zero(d) || fe_geq(d, fe_const_n())) return false;
    aff a;
    if (!jac_to_aff(mul_g(d, g_table().data()), a)) return false;
    fe_to_le(a.x, out_le);
    fe_to_le(a.y, out_le + 32);
    return true;
}

// HMAC-SHA256
static void hmac_sha256(const uint8_t* key, size_t klen, const uint8_t* msg, size_t mlen, uint8_t out[32]) {
    uint8_t k0[64] = {0};
    if (klen > 64) host_sha256(key, klen, k0); else std::memcpy(k0, key, klen);
    uint8_t ipad[64], opad[64];
    for (int i = 0; i < 64; ++i) { ipad[i] = k0[i] ^ 0x36; opad[i] = k0[i] ^ 0x5c; }
    HostSha256 h1;
    h1.update(ipad, 64);
    h1.update(msg, mlen);
    uint8_t inner[32];
    h1.final(inner);
    HostSha256 h2;
    h2.update(opad, 64);
    h2.update(inner, 32);
    h2.final(out);
}

// RFC 6979 (HMAC-SHA256, qlen = 256) + ECDSA sign over a SHA-256 digest. Returns r,s little-endian.
bool p256_sign(const uint8_t d_be[32], const uint8_t digest[32], uint8_t r_le[32], uint8_t s_le[32]) {
    const fe d = fe_from_be(d_be);
    const fe n = fe_const_n();
    if (fe_is_zero(d) || fe_geq(d, n)) return false;
    const fe e = sc_reduce(fe_from_be(digest));
    uint8_t h1[32];
    fe_to_be(e, h1);  // bits2octets(h1) = int2octets(bits2int(h1) mod q)
    uint8_t V[32], K[32];
    std::memset(V, 0x01, 32);
    std::memset(K, 0x00, 32);
    uint8_t buf[32 + 1 + 32 + 32];
    auto step = [&](uint8_t sep) {
        std::memcpy(buf, V, 32);
        buf[32] = sep;
        std::memcpy(buf + 33, d_be, 32);
        std::memcpy(buf + 65, h1, 32);
        hmac_sha256(K, 32, buf, sizeof(buf), K);
        hmac_sha256(K, 32, V, 32, V);
    };
    step(0x00);
    step(0x01);
    const aff* tab = g_table().data();
    for (int attempt = 0; attempt < 64; ++attempt) {
        hmac_sha256(K, 32, V, 32, V);
        const fe k = fe_from_be(V);
        if (!fe_is_zero(k) && !fe_geq(k, n)) {
            aff R;
            if (jac_to_aff(mul_g(k, tab), R)) {
                const fe r = sc_reduce(R.x);
                if (!fe_is_zero(r)) {
                    // s = k^-1 (e + r d) mod n
                    const fe k_m = sc_to_mont(k);
                    const fe kinv_m = sc_inv_mont(k_m);                  // k^-1 R
                    const fe rd = sc_mont_mul(sc_to_mont(r), d);         // r d
                    fe sum;
                    const uint32_t c = raw_add(sum, e, rd);
                    fe red;
                    const uint32_t br = raw_sub(red, sum, n);
                    sum = fe_select(c || br == 0, red, sum);
                    const fe s = sc_mont_mul(sum, kinv_m);               // (e + rd) k^-1
                    if (!fe_is_zero(s)) {
                        fe_to_le(r, r_le);
                        fe_to_le(s, s_le);
                        return true;
                    }
                }
            }
        }
        uint8_t b2[33];
        std::memcpy(b2, V, 32);
        b2[32] = 0x00;
        hmac_sha256(K, 32, b2, 33, K);
        hmac_sha256(K, 32, V, 32, V);
    }
    return false;
}

}  // namespace upow
