// K5/K6/K15: P-256 ECDSA batch verify, point decompression, keygen and RFC 6979 signing.
//
// reference: fastecdsa ecdsa.verify / ecdsa.sign / keys.get_public_key / util.mod_sqrt, called one
// signature at a time from upow/upow_transactions/transaction_input.py:84-120,
// upow/upow_transactions/transaction.py:148-180,484-497 and upow/helpers.py:58-62,135-144.
//
// GPU design (gfx950): batches up to 32k signatures (a block) take four lanes per signature (the quad
// kernel, see "four lanes per signature" below); larger batches one signature per lane:
//  * u1*G uses a fixed-base byte-window table T[j][b] = b*256^j*G (32 x 255 affine points, 522 KB,
//    L2/Infinity-Cache resident) -> 32 mixed additions and no doublings;
//  * u2*Q uses signed 5-bit windows (BoothW5) over a per-signature table {1..16}Q kept in global
//    scratch (1.5-2 KB per signature does not fit LDS at useful occupancy) -> 255 doublings + 52
//    additions (unsigned 4-bit windows: 252 + 64);
//  * no field inversion: x(R) == r is tested as X == r*Z^2 (and (r+n)*Z^2 when r+n < p);
//  * s^-1 mod n by Bernstein-Yang divsteps (p256_field.h sc_inv_safegcd_mont: 20 rounds of 30, no
//    divergence; the binary extended Euclid it replaced, sc_inv_bgcd_mont, stays for the A/B build);
//  * status per item: 1 valid, 0 invalid, 2 public key not on curve, 3 r/s out of [1, n]
//    (fastecdsa raises for 2/3; the Python layer turns them into EcdsaError).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <optional>
#include <stdexcept>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "dev_pool.h"
#include "native.h"
#include "thread_pool.h"
#include "streams.h"
#include "p256_field.h"
#include "p256_verify.h"
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

// field operations on one host thread (the same UPOW_HD code the kernels run), for differential tests:
// out = a*b, a^2, a+b, a-b (mod p) for canonical a, b; and an arbitrary 512-bit value reduced mod p
void p256_fe_ops_host(const uint32_t a[8], const uint32_t b[8], uint32_t out[32]) {
    fe x, y;
    std::memcpy(x.v, a, 32);
    std::memcpy(y.v, b, 32);
    const fe r[4] = {fe_mul(x, y), fe_sqr(x), fe_add(x, y), fe_sub(x, y)};
    for (int k = 0; k < 4; ++k) std::memcpy(out + 8 * k, r[k].v, 32);
}
void p256_fe_reduce_host(const uint32_t c[16], uint32_t out[8]) {
    const fe r = fe_reduce(c);
    std::memcpy(out, r.v, 32);
}

void p256_scalar_inv_mont_host(uint64_t out[4], const uint64_t s[4]) {
    fe a;
    std::memcpy(a.v, s, 32);
    const fe r = sc_inv_safegcd_mont(a);
    std::memcpy(out, r.v, 32);
}

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

static uint8_t verify_one_host(const VerifyItem& it, const aff* gtab) {
    aff q;
    fe r, u1, u2;
    const uint8_t pro = verify_prologue(it, q, r, u1, u2);
    if (pro != 255) return pro;
    jac tbl[17];  // k*Q, k = 1..16 (signed 5-bit windows)
    tbl[0] = jac_inf();
    tbl[1] = jac_from_aff(q);
    for (int k = 2; k <= 16; ++k) tbl[k] = jac_madd(tbl[k - 1], q);
    jac acc = jac_inf();
    BoothW5 bw(u2);
    for (int w = kBoothWindows - 1; w >= 0; --w) {
        if (!jac_is_inf(acc))
            for (int k = 0; k < 5; ++k) acc = jac_dbl(acc);
        const int d = bw.next();
        if (d) {
            jac e = tbl[d < 0 ? -d : d];
            if (d < 0) e.y = fe_neg(e.y);
            acc = jac_add(acc, e);
        }
    }
    const jac R = jac_add(mul_g(u1, gtab), acc);
    return verify_epilogue(R, r);
}

// ------------------------------------------------------------------------------------------------
// four lanes per signature (latency path for one block)
// ------------------------------------------------------------------------------------------------
// One 2 MB block is ~8,300 signatures = 130 waves at one signature per lane: 130 of the chip's 1,024
// SIMDs are busy and the launch takes as long as one wave's serial chain (~3 ms). A wave64 VALU op
// costs its four passes whatever the exec mask (profiles/p256_latency_ab.txt: 16 signatures per wave
// run no faster than 64), so the only way to cut that latency is to split each signature's chain over
// more lanes. Here a lane quad (4k .. 4k+3) owns one signature: all four lanes keep the whole point
// state (redundantly) and the field products of the point formulas are scheduled in "steps" of up to
// four independent products, one per lane; DPP quad_perm broadcasts hand every lane the others'
// results (8 v_mov_dpp per product). Adds/subs stay redundant: they are cheap next to a 256x256-bit
// product. Points are in XYZZ coordinates (x = X/ZZ, y = Y/ZZZ), whose formulas are shallow:
//   doubling (a = -3, dbl-2008-s-1)            9 products, depth 3  -> 3 steps (the first all squares)
//   addition (add-2008-s)                      14 products, depth 4 -> 4 steps
// (Jacobian doubling is 8 products but depth 4: 4 steps however many lanes.) A 4-bit window (4
// doublings + 1 addition) is 16 steps instead of 48 serial products; with signed 5-bit windows
// (Booth recoding: 52 windows of 5 doublings + 1 addition) u2*Q is 51 x 15 + 52 x 4 = 973 steps. The
// window table k*Q (k = 1..16) is built the same way (3 + 14 x 4 steps). u1*G (32 fixed-base byte windows) splits by quarters:
// each lane accumulates 8 windows on its own (Jacobian mixed adds), converts to XYZZ, and the four
// partial points are broadcast and added. s^-1 runs redundantly on all four lanes (binary Euclid).
// Waves go four to a workgroup so they land on four different SIMDs of a CU (single-wave workgroups
// double up on one SIMD once there are more waves than CUs: profiles/p256_latency_ab.txt).
//
// The schedule is written once over a policy type: QuadDev broadcasts through DPP on the GPU;
// QuadHost (one host thread) computes every product of a step itself, which lets the CPU tests check
// the formulas and the step schedule bit for bit against the reference verifier.
struct xz { fe x, y, zz, zzz; };  // XYZZ point; zz == 0 <=> infinity
static_assert(sizeof(xz) == 128, "xz layout");

struct QuadHost {
    UPOW_HD void sqr4(const fe& a0, const fe& a1, const fe& a2, const fe& a3, fe& r0, fe& r1, fe& r2, fe& r3) const {
        const fe m0 = fe_sqr(a0), m1 = fe_sqr(a1), m2 = fe_sqr(a2), m3 = fe_sqr(a3);
        r0 = m0;
        r1 = m1;
        r2 = m2;
        r3 = m3;
    }
    UPOW_HD void mul4(const fe& a0, const fe& b0, const fe& a1, const fe& b1, const fe& a2, const fe& b2,
                      const fe& a3, const fe& b3, fe& r0, fe& r1, fe& r2, fe& r3) const {
        const fe m0 = fe_mul(a0, b0), m1 = fe_mul(a1, b1), m2 = fe_mul(a2, b2), m3 = fe_mul(a3, b3);
        r0 = m0;
        r1 = m1;
        r2 = m2;
        r3 = m3;
    }
};

// the eight-lane kernel's pair-split product (OctDev below) on one host thread: both lanes' halves
UPOW_HD fe mul_pair_host(const fe& a, const fe& b);

struct OctHost {
    UPOW_HD void sqr4(const fe& a0, const fe& a1, const fe& a2, const fe& a3, fe& r0, fe& r1, fe& r2, fe& r3) const {
        const fe m0 = mul_pair_host(a0, a0), m1 = mul_pair_host(a1, a1), m2 = mul_pair_host(a2, a2),
                 m3 = mul_pair_host(a3, a3);
        r0 = m0;
        r1 = m1;
        r2 = m2;
        r3 = m3;
    }
    UPOW_HD void mul4(const fe& a0, const fe& b0, const fe& a1, const fe& b1, const fe& a2, const fe& b2,
                      const fe& a3, const fe& b3, fe& r0, fe& r1, fe& r2, fe& r3) const {
        const fe m0 = mul_pair_host(a0, b0), m1 = mul_pair_host(a1, b1), m2 = mul_pair_host(a2, b2),
                 m3 = mul_pair_host(a3, b3);
        r0 = m0;
        r1 = m1;
        r2 = m2;
        r3 = m3;
    }
};

template <int K>
__device__ __forceinline__ fe fe_quad_bcast(const fe& a) {  // every lane of the quad gets lane K's value
    fe r;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.v[i] = uint32_t(__builtin_amdgcn_mov_dpp(int(a.v[i]), K * 0x55, 0xF, 0xF, true));
    return r;
}
struct QuadDev {
    bool odd, hi;  // this lane's role in its quad (lane & 3): bit 0 and bit 1
    // a_role as a two-level select tree on the role's bits: the compiler folds a select of two identical
    // operands, so the schedule's repeated operands cost less than three selects per word — (a, b, c, c)
    // and (v, v, m, z) take two, (x, y, x, y) one (the linear chain on role == 1/2/3 folded less)
    __device__ __forceinline__ fe pick(const fe& a0, const fe& a1, const fe& a2, const fe& a3) const {
        fe r;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint32_t lo = odd ? a1.v[i] : a0.v[i];
            const uint32_t up = odd ? a3.v[i] : a2.v[i];
            r.v[i] = hi ? up : lo;
        }
        return r;
    }
    // a step whose four products are all squares: the squaring row code (36 partial products, not 64)
    __device__ __forceinline__ void sqr4(const fe& a0, const fe& a1, const fe& a2, const fe& a3, fe& r0, fe& r1, fe& r2,
                                         fe& r3) const {
        const fe m = fe_sqr(pick(a0, a1, a2, a3));
        r0 = fe_quad_bcast<0>(m);
        r1 = fe_quad_bcast<1>(m);
        r2 = fe_quad_bcast<2>(m);
        r3 = fe_quad_bcast<3>(m);
    }
    __device__ __forceinline__ void mul4(const fe& a0, const fe& b0, const fe& a1, const fe& b1, const fe& a2,
                                         const fe& b2, const fe& a3, const fe& b3, fe& r0, fe& r1, fe& r2,
                                         fe& r3) const {
        const fe m = fe_mul(pick(a0, a1, a2, a3), pick(b0, b1, b2, b3));
        r0 = fe_quad_bcast<0>(m);
        r1 = fe_quad_bcast<1>(m);
        r2 = fe_quad_bcast<2>(m);
        r3 = fe_quad_bcast<3>(m);
    }
};

// Eight lanes per signature (two quads, `hi` = the upper one): every product of a step is split over a lane
// PAIR (k, k + 4). Each lane runs four of the eight schoolbook rows (32 v_mad_u64_u32 instead of 64: the
// quarter-rate 64-bit multiply-adds are half of a step's time), the upper lane's 12-word partial sum
// crosses to its partner with DPP row_shl:4, the lower lane adds it and reduces, and row_shr:4 hands the
// reduced product back to the upper lane; quad_perm broadcasts then give all four products to every lane
// of both quads. 8,300 signatures fill 1,038 waves, one per SIMD of the chip, where the quad kernel left
// half of the SIMDs idle. `split_rows` / `combine_rows` are the arithmetic; the host test runs them on one
// thread (both halves) against fe_mul.
UPOW_HD void split_rows(uint32_t p[12], const fe& a, const fe& b, bool upper) {
    uint32_t ar[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) ar[i] = upper ? a.v[4 + i] : a.v[i];
#pragma unroll
    for (int i = 0; i < 12; ++i) p[i] = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        unsigned cy = 0;
        uint32_t prev = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const uint64_t t = uint64_t(ar[i]) * b.v[j] + p[i + j];
            p[i + j] = __builtin_addc(uint32_t(t), prev, cy, &cy);
            prev = uint32_t(t >> 32);
        }
        p[i + 8] = prev + cy;
    }
}
// lo: columns 0..11 of the lower rows; hi: columns 4..15 of the upper rows (hi[w] is column w + 4)
UPOW_HD fe combine_rows(const uint32_t lo[12], const uint32_t hi[12]) {
    uint32_t c[16];
#pragma unroll
    for (int w = 0; w < 4; ++w) c[w] = lo[w];
    unsigned cy = 0;
#pragma unroll
    for (int w = 4; w < 12; ++w) c[w] = __builtin_addc(lo[w], hi[w - 4], cy, &cy);
#pragma unroll
    for (int w = 12; w < 16; ++w) c[w] = __builtin_addc(0u, hi[w - 4], cy, &cy);
    return fe_reduce(c);
}

UPOW_HD fe mul_pair_host(const fe& a, const fe& b) {
    uint32_t lo[12], hi[12];
    split_rows(lo, a, b, false);
    split_rows(hi, a, b, true);
    return combine_rows(lo, hi);
}

struct OctDev {
    bool is1, is2, is3, hi;  // lane & 3, and whether the lane is in the octet's upper quad
    __device__ __forceinline__ fe pick(const fe& a0, const fe& a1, const fe& a2, const fe& a3) const {
        fe r;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            uint32_t t = a0.v[i];
            t = is1 ? a1.v[i] : t;
            t = is2 ? a2.v[i] : t;
            r.v[i] = is3 ? a3.v[i] : t;
        }
        return r;
    }
    __device__ __forceinline__ fe mul_pair(const fe& a, const fe& b) const {
        uint32_t p[12], q[12];
        split_rows(p, a, b, hi);
#pragma unroll
        for (int w = 0; w < 12; ++w) q[w] = uint32_t(__builtin_amdgcn_mov_dpp(int(p[w]), 0x104, 0xF, 0xF, true));  // row_shl:4
        const fe m = combine_rows(p, q);  // meaningful on the lower quad
        fe r;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint32_t from_lo = uint32_t(__builtin_amdgcn_mov_dpp(int(m.v[i]), 0x114, 0xF, 0xF, true));  // row_shr:4
            r.v[i] = hi ? from_lo : m.v[i];
        }
        return r;
    }
    __device__ __forceinline__ void sqr4(const fe& a0, const fe& a1, const fe& a2, const fe& a3, fe& r0, fe& r1, fe& r2,
                                         fe& r3) const {
        const fe a = pick(a0, a1, a2, a3);
        const fe m = mul_pair(a, a);
        r0 = fe_quad_bcast<0>(m);
        r1 = fe_quad_bcast<1>(m);
        r2 = fe_quad_bcast<2>(m);
        r3 = fe_quad_bcast<3>(m);
    }
    __device__ __forceinline__ void mul4(const fe& a0, const fe& b0, const fe& a1, const fe& b1, const fe& a2,
                                         const fe& b2, const fe& a3, const fe& b3, fe& r0, fe& r1, fe& r2,
                                         fe& r3) const {
        const fe m = mul_pair(pick(a0, a1, a2, a3), pick(b0, b1, b2, b3));
        r0 = fe_quad_bcast<0>(m);
        r1 = fe_quad_bcast<1>(m);
        r2 = fe_quad_bcast<2>(m);
        r3 = fe_quad_bcast<3>(m);
    }
};

// fewer products per step: the spare lanes repeat the last product (its broadcast is dead code)
template <class P>
UPOW_HD void mul3(const P& pp, const fe& a0, const fe& b0, const fe& a1, const fe& b1, const fe& a2, const fe& b2,
                  fe& r0, fe& r1, fe& r2) {
    fe d;
    pp.mul4(a0, b0, a1, b1, a2, b2, a2, b2, r0, r1, r2, d);
}
template <class P>
UPOW_HD void mul2(const P& pp, const fe& a0, const fe& b0, const fe& a1, const fe& b1, fe& r0, fe& r1) {
    fe d0, d1;
    pp.mul4(a0, b0, a1, b1, a1, b1, a1, b1, r0, r1, d0, d1);
}
template <class P>
UPOW_HD void mul1(const P& pp, const fe& a0, const fe& b0, fe& r0) {
    fe d0, d1, d2;
    pp.mul4(a0, b0, a0, b0, a0, b0, a0, b0, r0, d0, d1, d2);
}

UPOW_HD fe fe_x3(const fe& a) { return fe_add(fe_add(a, a), a); }

// dbl-2008-s-1 with a = -3: M = 3 X^2 - 3 ZZ^2. The first step is three squarings (U^2, X^2, ZZ^2),
// issued with the squaring code. Infinity (ZZ = 0) stays infinity.
template <class P>
UPOW_HD void dbl4(const P& pp, xz& p) {
    const fe u = fe_add(p.y, p.y);
    fe v, xx, zz2, unused;
    pp.sqr4(u, p.x, p.zz, p.zz, v, xx, zz2, unused);
    const fe m = fe_x3(fe_sub(xx, zz2));
    fe w, s, mm, zz3;
    pp.mul4(u, v, p.x, v, m, m, v, p.zz, w, s, mm, zz3);
    const fe x3 = fe_sub(mm, fe_add(s, s));
    fe ya, wy, zzz3;
    mul3(pp, m, fe_sub(s, x3), w, p.y, w, p.zzz, ya, wy, zzz3);
    p.x = x3;
    p.y = fe_sub(ya, wy);
    p.zz = zz3;
    p.zzz = zzz3;
}

// add-2008-s with the reference verifier's special cases (infinity, P == Q, P == -Q)
template <class P>
UPOW_HD void add4(const P& pp, xz& p, const xz& q) {
    if (fe_is_zero(q.zz)) return;
    if (fe_is_zero(p.zz)) { p = q; return; }
    fe u1, u2, s1, s2;
    pp.mul4(p.x, q.zz, q.x, p.zz, p.y, q.zzz, q.y, p.zzz, u1, u2, s1, s2);
    const fe ph = fe_sub(u2, u1), r = fe_sub(s2, s1);
    if (fe_is_zero(ph)) {
        if (fe_is_zero(r)) dbl4(pp, p);
        else p.zz = p.zzz = fe_zero();
        return;
    }
    fe pp2, rr, zz12, zzz12;
    pp.mul4(ph, ph, r, r, p.zz, q.zz, p.zzz, q.zzz, pp2, rr, zz12, zzz12);
    fe ppp, qq, zz3;
    mul3(pp, ph, pp2, u1, pp2, zz12, pp2, ppp, qq, zz3);
    const fe x3 = fe_sub(fe_sub(rr, ppp), fe_add(qq, qq));
    fe ya, s1p, zzz3;
    mul3(pp, r, fe_sub(qq, x3), s1, ppp, zzz12, ppp, ya, s1p, zzz3);
    p.x = x3;
    p.y = fe_sub(ya, s1p);
    p.zz = zz3;
    p.zzz = zzz3;
}

// u1*G over the byte windows [8*quarter, 8*quarter + 8) (one lane's share), Jacobian mixed adds
UPOW_HD jac mul_g_quarter(const fe& k, const aff* tab, int quarter) {
    jac acc = jac_inf();
    uint32_t lo = k.v[0], hi = k.v[1];  // this quarter's 64 bits, consumed a byte at a time
#pragma unroll
    for (int l = 1; l < 4; ++l) {
        lo = quarter == l ? k.v[2 * l] : lo;
        hi = quarter == l ? k.v[2 * l + 1] : hi;
    }
    const aff* t = tab + quarter * 8 * kGEnt;
    for (int j = 0; j < 8; ++j) {
        const uint32_t b = lo & 0xffu;
        lo = (lo >> 8) | (hi << 24);
        hi >>= 8;
        if (b) acc = jac_madd(acc, t[j * kGEnt + b]);
    }
    return acc;
}


UPOW_HD jac mul_g16_quarter(const fe& k, const aff* tab16, int quarter) {
    uint32_t lo = k.v[0], hi = k.v[1];  // this quarter's 64 bits, consumed 16 at a time
#pragma unroll
    for (int l = 1; l < 4; ++l) {
        lo = quarter == l ? k.v[2 * l] : lo;
        hi = quarter == l ? k.v[2 * l + 1] : hi;
    }
    const aff* t = tab16 + size_t(quarter) * 4 * kG16Ent;
    jac acc = jac_inf();
    for (int j = 0; j < 4; ++j) {
        const uint32_t b = lo & 0xffffu;
        lo = (lo >> 16) | (hi << 16);
        hi >>= 16;
        if (b) acc = jac_madd(acc, t[size_t(j) * kG16Ent + b]);
    }
    return acc;
}

// Jacobian (X, Y, Z) -> XYZZ (X, Y, Z^2, Z^3): the same affine point, one lane on its own
UPOW_HD xz jac_to_xz(const jac& p) {
    const fe zz = fe_sqr(p.z);
    return xz{p.x, p.y, zz, fe_mul(zz, p.z)};
}

// Shared verify body. `tab` holds this signature's 16 window entries 1Q..16Q (global scratch on the GPU, a
// local array on the host); `gpart(K)` yields quarter K of u1*G in XYZZ form (on the GPU: lane K's own
// quarter, broadcast). On the GPU every lane of the quad stores the (identical)
// entries, so each later table read is of the lane's own store.
template <class P, class GPart>
UPOW_HD uint8_t verify_quad_core(const P& pp, const aff& q, const fe& r, const fe& u2, xz* tab, GPart gpart) {
    const fe one = fe_one();
    const xz t1{q.x, q.y, one, one};
    xz t = t1;
    tab[0] = t;  // tab[k - 1] = k*Q, k = 1..16
    dbl4(pp, t);
    tab[1] = t;
    for (int k = 3; k <= 16; ++k) {
        add4(pp, t, t1);
        tab[k - 1] = t;
    }
    // u2*Q: 52 signed 5-bit windows (BoothW5) from the top, so 52 additions instead of the 64 of
    // unsigned 4-bit windows; a negative digit adds the entry with -Y
    xz acc{one, one, fe_zero(), fe_zero()};
    BoothW5 bw(u2);
    for (int w = kBoothWindows - 1; w >= 0; --w) {
        const int d = bw.next();
        xz e;
        if (d) {
            e = tab[(d < 0 ? -d : d) - 1];
            if (d < 0) e.y = fe_neg(e.y);
        }
        if (w != kBoothWindows - 1) {
            dbl4(pp, acc);
            dbl4(pp, acc);
            dbl4(pp, acc);
            dbl4(pp, acc);
            dbl4(pp, acc);
        }
        if (d) add4(pp, acc, e);
    }
    // + u1*G, added a quarter at a time
    add4(pp, acc, gpart(std::integral_constant<int, 0>{}));
    add4(pp, acc, gpart(std::integral_constant<int, 1>{}));
    add4(pp, acc, gpart(std::integral_constant<int, 2>{}));
    add4(pp, acc, gpart(std::integral_constant<int, 3>{}));
    // x(R) == r  <=>  X == r ZZ (and (r + n) ZZ when r + n < p)
    if (fe_is_zero(acc.zz)) return 0;
    if (fe_eq(fe_mul(r, acc.zz), acc.x)) return 1;
    fe rn;
    const uint32_t c = raw_add(rn, r, fe_const_n());
    if (!c && !fe_geq(rn, fe_const_p()) && fe_eq(fe_mul(rn, acc.zz), acc.x)) return 1;
    return 0;
}

template <class P>
static uint8_t verify_one_host_steps(const VerifyItem& it, const aff* gtab) {
    aff q;
    fe r, u1, u2;
    const uint8_t pro = verify_prologue(it, q, r, u1, u2);
    if (pro != 255) return pro;
    xz tab[16];
    return verify_quad_core(P{}, q, r, u2, tab, [&](auto K) { return jac_to_xz(mul_g_quarter(u1, gtab, K)); });
}
static uint8_t verify_one_host_quad(const VerifyItem& it, const aff* gtab) { return verify_one_host_steps<QuadHost>(it, gtab); }

// ------------------------------------------------------------------------------------------------
// device kernels
// ------------------------------------------------------------------------------------------------

// Four lanes per signature, four waves per workgroup (16 signatures per wave). Exits are quad-uniform.
static constexpr int64_t kQuadMaxBatch = 32 * 1024;  // 2,048 waves of 16 signatures: two per SIMD
static constexpr int64_t kBatchSlice = 4 * 1024 * 1024;  // one-lane batch launches: signatures per launch
__global__ __launch_bounds__(256, 1) void p256_verify_quad_kernel(const VerifyItem* __restrict__ items, int64_t n,
                                                                   const aff* __restrict__ gtab16,
                                                                   xz* __restrict__ scratch,
                                                                   uint8_t* __restrict__ status) {
    const int lane = int(threadIdx.x) & 63;
    const int64_t i = (int64_t(blockIdx.x) * 4 + (threadIdx.x >> 6)) * 16 + (lane >> 2);
    if (i >= n) return;
    const int role = lane & 3;
    const QuadDev pp{(role & 1) != 0, (role & 2) != 0};
    const VerifyItem it = items[i];
    aff q;
    fe r, u1, u2;
    const uint8_t pro = verify_prologue(it, q, r, u1, u2);
    if (pro != 255) {
        if (role == 0) status[i] = pro;
        return;
    }
    const xz mine = jac_to_xz(mul_g16_quarter(u1, gtab16, role));  // this lane's quarter of u1*G
    const uint8_t st = verify_quad_core(pp, q, r, u2, scratch + i * 16, [&](auto K) {
        constexpr int k = decltype(K)::value;
        return xz{fe_quad_bcast<k>(mine.x), fe_quad_bcast<k>(mine.y), fe_quad_bcast<k>(mine.zz), fe_quad_bcast<k>(mine.zzz)};
    });
    if (role == 0) status[i] = st;
}

// Eight lanes per signature (OctDev), four waves per workgroup (8 signatures per wave). Exits are
// octet-uniform. Both quads of an octet hold the same point state; the u1*G quarters are computed by each
// quad (lane & 3) and broadcast within it.
__global__ __launch_bounds__(256, 1) void p256_verify_oct_kernel(const VerifyItem* __restrict__ items, int64_t n,
                                                                  const aff* __restrict__ gtab16,
                                                                  xz* __restrict__ scratch,
                                                                  uint8_t* __restrict__ status) {
    const int lane = int(threadIdx.x) & 63;
    const int64_t i = (int64_t(blockIdx.x) * 4 + (threadIdx.x >> 6)) * 8 + (lane >> 3);
    if (i >= n) return;
    const int role = lane & 3;
    const bool upper = (lane & 4) != 0;
    const OctDev pp{role == 1, role == 2, role == 3, upper};
    const VerifyItem it = items[i];
    aff q;
    fe r, u1, u2;
    const uint8_t pro = verify_prologue(it, q, r, u1, u2);
    if (pro != 255) {
        if (role == 0 && !upper) status[i] = pro;
        return;
    }
    const xz mine = jac_to_xz(mul_g16_quarter(u1, gtab16, role));  // this lane's quarter of u1*G
    const uint8_t st = verify_quad_core(pp, q, r, u2, scratch + i * 16, [&](auto K) {
        constexpr int k = decltype(K)::value;
        return xz{fe_quad_bcast<k>(mine.x), fe_quad_bcast<k>(mine.y), fe_quad_bcast<k>(mine.zz), fe_quad_bcast<k>(mine.zzz)};
    });
    if (role == 0 && !upper) status[i] = st;
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

// The key kernel of p256_verify_fused_gpu. Thread t < n_jobs: signer key jobkeys[t] decompressed into verify
// item t, whose r | s | digest come from sigdig[t]; a key off the curve (or x >= p) gets x = y = 0, which the
// verify prologue reports as a bad key (status 2), as the separate decompression's failure did. Threads
// past n_jobs: output address t - n_jobs, curve check only (transaction_output.py: string_to_point).
__global__ __launch_bounds__(256) void p256_keyrec_kernel(const uint8_t* __restrict__ jobkeys,
                                                           const uint8_t* __restrict__ sigdig, int64_t n_jobs,
                                                           const uint8_t* __restrict__ outkeys, int64_t n_out,
                                                           VerifyItem* __restrict__ items, uint8_t* __restrict__ out_ok) {
    const int64_t t = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (t >= n_jobs + n_out) return;
    const bool job = t < n_jobs;
    const uint8_t* a = job ? jobkeys + 33 * t : outkeys + 33 * (t - n_jobs);
    const fe x = fe_from_le(a + 1);
    const bool odd = a[0] == 43;
    bool good = !fe_geq(x, fe_const_p());
    const fe x3 = fe_mul(fe_sqr(x), x);
    const fe rhs = fe_add(fe_sub(x3, fe_add(fe_add(x, x), x)), fe_const_b());
    fe y = fe_sqrt_candidate(rhs);
    good = good && fe_eq(fe_sqr(y), rhs);
    if (!job) {
        out_ok[t - n_jobs] = good ? 1 : 0;
        return;
    }
    if ((y.v[0] & 1u) != uint32_t(odd)) y = fe_neg(y);
    VerifyItem* it = items + t;
    fe_to_le(good ? x : fe_zero(), it->qx);
    fe_to_le(good ? y : fe_zero(), it->qy);
    const uint8_t* sd = sigdig + 96 * t;
    uint8_t* rse = reinterpret_cast<uint8_t*>(it) + 64;  // r | s | e: the item's last 96 bytes
#pragma unroll 8
    for (int k = 0; k < 96; ++k) rse[k] = sd[k];
}

// item: 64-byte full address x LE | y LE (transaction_output.py:25-26, is_point_on_curve per output)
UPOW_HD uint8_t on_curve_64(const uint8_t* a) {
    const aff q{fe_from_le(a), fe_from_le(a + 32)};
    return !fe_geq(q.x, fe_const_p()) && !fe_geq(q.y, fe_const_p()) && aff_on_curve(q) ? 1 : 0;
}

__global__ __launch_bounds__(256) void p256_on_curve_kernel(const uint8_t* __restrict__ in, int64_t n,
                                                             uint8_t* __restrict__ ok) {
    const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    ok[i] = on_curve_64(in + 64 * i);
}

static void hck(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

struct DeviceGTable {
    int device = -1;
    aff* d_tab = nullptr;
    aff* d_tab16 = nullptr;
};

// T16[j][b] = b * 2^(16 j) * G from the byte-window table: b = lo + 256 hi -> T[2j][lo] + T[2j+1][hi] (one
// mixed addition; the two are never equal or opposite, lo * 256^(2j) < 256^(2j+1) <= hi * 256^(2j+1)), then
// to affine with the thread's own inversion. One thread per entry; entry 0 of each window stays zero.
__global__ __launch_bounds__(256) void build_g16_kernel(const aff* __restrict__ tab8, aff* __restrict__ tab16) {
    const int64_t e = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (e >= int64_t(kG16Win) * kG16Ent) return;
    const int j = int(e / kG16Ent);
    const uint32_t b = uint32_t(e % kG16Ent), lo = b & 0xffu, hi = b >> 8;
    aff out{fe_zero(), fe_zero()};
    if (b) {
        jac acc = jac_inf();
        if (lo) acc = jac_madd(acc, tab8[(2 * j) * kGEnt + lo]);
        if (hi) acc = jac_madd(acc, tab8[(2 * j + 1) * kGEnt + hi]);
        (void)jac_to_aff(acc, out);
    }
    tab16[e] = out;
}
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

static const aff* device_g16_table() {
    const aff* tab8 = device_g_table();
    int dev = 0;
    hck(hipGetDevice(&dev), "hipGetDevice");
    std::lock_guard<std::mutex> lk(g_dev_mu);
    DeviceGTable& t = g_dev_tabs[dev];
    if (!t.d_tab16) {
        const int64_t n = int64_t(kG16Win) * kG16Ent;
        aff* d = nullptr;
        hck(hipMalloc(&d, sizeof(aff) * size_t(n)), "hipMalloc gtab16");
        hipLaunchKernelGGL(build_g16_kernel, dim3(unsigned((n + 255) / 256)), dim3(256), 0, node_stream(), tab8, d);
        hck(hipGetLastError(), "build_g16_kernel launch");
        node_sync("gtab16 build");
        t.d_tab16 = d;
    }
    return t.d_tab16;
}

// entries [first, first + count) of the device's 16-bit-window table, for its differential test
std::vector<uint8_t> p256_g16_entries(int64_t first, int64_t count) {
    const int64_t n = int64_t(kG16Win) * kG16Ent;
    if (first < 0 || count < 0 || first + count > n) throw std::invalid_argument("g16 entry range");
    node_device_enter();
    const aff* d = device_g16_table();
    std::vector<uint8_t> out(size_t(count) * sizeof(aff));
    node_d2h(out.data(), d + first, out.size(), "d2h gtab16");
    return out;
}

// ------------------------------------------------------------------------------------------------
// host API
// ------------------------------------------------------------------------------------------------
std::vector<uint8_t> p256_verify_host(const uint8_t* items, int64_t n, int threads) {
    std::vector<uint8_t> st(static_cast<size_t>(n));
    const aff* tab = g_table().data();
    const VerifyItem* it = reinterpret_cast<const VerifyItem*>(items);
    // UPOW_P256_HOST32 (read per call): '1' = the 32-bit-limb single-lane code the one-lane GPU kernels
    // run; 'quad' = the four-lane step schedule of the quad kernel played by one host thread (CPU tests
    // of both GPU code paths); 'oct' = the same schedule with the eight-lane kernel's pair-split products;
    // unset = the 64-bit-limb host verifier.
    const char* h32 = std::getenv("UPOW_P256_HOST32");
    const int mode = !h32 ? 0 : (std::strcmp(h32, "quad") == 0 ? 2 : std::strcmp(h32, "oct") == 0 ? 3 : (h32[0] == '1' ? 1 : 0));
    threads = int(std::max<int64_t>(1, std::min<int64_t>(threads, n)));
    auto work = [&](int t) {
        if (mode == 1)
            for (int64_t i = t; i < n; i += threads) st[i] = verify_one_host(it[i], tab);
        else if (mode == 2)
            for (int64_t i = t; i < n; i += threads) st[i] = verify_one_host_quad(it[i], tab);
        else if (mode == 3)  // the eight-lane kernel's pair-split products
            for (int64_t i = t; i < n; i += threads) st[i] = verify_one_host_steps<OctHost>(it[i], tab);
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

// Scratch of one verify launch: kept by the caller until its stream sync.
struct VerifyScratch {
    std::optional<PooledBuf<xz>> quad;
    std::optional<PooledBuf<jac>> one;
};

// Launches the verify of n device items into d_st on the node stream.
// Variant (UPOW_P256_VARIANT, read per call): unset/'a' = auto, '4' = four lanes per signature,
// '8' = eight, '0'..'3' = one lane per signature (below). Auto takes the quad kernel up to 32k signatures
// (2,048 waves, two per SIMD): there it cuts the latency of block-sized batches; past that the chip is
// full either way and one lane per signature does half the total work.
static void verify_launch(const VerifyItem* d_items, int64_t n, const aff* d_tab, uint8_t* d_st, VerifyScratch& sc) {
    const char* var = std::getenv("UPOW_P256_VARIANT");
    char v = var && var[0] ? var[0] : 'a';
    const bool autov = v == 'a';
    if (v == 'a') v = n <= kQuadMaxBatch ? '4' : '1';
    if (v == '8') {
        sc.quad.emplace(size_t(16) * size_t(n));
        const int64_t waves = (n + 7) / 8;
        hipLaunchKernelGGL(p256_verify_oct_kernel, dim3(unsigned((waves + 3) / 4)), dim3(256), 0, node_stream(), d_items, n,
                           d_tab, sc.quad->p, d_st);
        hck(hipGetLastError(), "p256_verify_oct_kernel launch");
        return;
    }
    if (v == '4') {
        sc.quad.emplace(size_t(16) * size_t(n));
        const int64_t waves = (n + 15) / 16;
        hipLaunchKernelGGL(p256_verify_quad_kernel, dim3(unsigned((waves + 3) / 4)), dim3(256), 0, node_stream(), d_items, n,
                           d_tab, sc.quad->p, d_st);
        hck(hipGetLastError(), "p256_verify_quad_kernel launch");
        return;
    }
    const char* spw_env = std::getenv("UPOW_P256_SPW");
    int spw = spw_env ? std::atoi(spw_env) : 64;
    if (spw < 1 || spw > 64) spw = 64;
    // one lane per signature (csrc/p256_batch.hip), one launch per kBatchSlice signatures (UPOW_P256_SLICE
    // for the A/B): slicing a 531,200-signature batch into 128 k or 256 k launches measured 12 % / 9 % slower
    // than one launch (each launch ends in a tail of half-idle SIMDs; profiles/r5/p256batch), so the default
    // slice only bounds the window-table scratch (16 x 96 B per signature)
    const char* sl_env = std::getenv("UPOW_P256_SLICE");
    const int64_t slice = std::max<int64_t>(1024, sl_env ? std::atoll(sl_env) : kBatchSlice);
    // Every one-lane wave runs the same fixed-window chain, so the kernel takes whole "rounds" of one wave
    // lifetime: 4 waves per SIMD x 1,024 SIMDs x 64 lanes = 262,144 signatures per round on MI355X. A batch
    // a little past a multiple of that (531,200 = 2 rounds + 6,912) paid a third round for 3 % of its work.
    // Auto mode runs the whole rounds on the one-lane kernel and a remainder of at most kQuadMaxBatch on the
    // four-lanes-per-signature kernel, which finishes it in a quarter of a wave lifetime.
    int64_t n_one = n, n_quad = 0;
    if (autov && v == '1' && spw == 64 && !sl_env && std::getenv("UPOW_P256_TAIL") == nullptr) {
        int dev = 0, cus = 0;
        hck(hipGetDevice(&dev), "hipGetDevice");
        hck(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev), "CU count");
        const int64_t round = int64_t(cus) * 4 /* SIMDs */ * 4 /* waves per SIMD */ * 64;
        const int64_t full = round > 0 ? (n / round) * round : 0, rem = n - full;
        if (full > 0 && rem > 0 && rem <= kQuadMaxBatch) {
            n_one = full;
            n_quad = rem;
        }
    }
    sc.one.emplace(size_t(16) * size_t(std::min(n_one, slice)));
    for (int64_t off = 0; off < n_one; off += slice)
        p256_batch_launch(v, d_items + off, std::min(slice, n_one - off), d_tab, sc.one->p, d_st + off, spw, node_stream());
    if (n_quad) {
        sc.quad.emplace(size_t(16) * size_t(n_quad));
        const int64_t waves = (n_quad + 15) / 16;
        hipLaunchKernelGGL(p256_verify_quad_kernel, dim3(unsigned((waves + 3) / 4)), dim3(256), 0, node_stream(),
                           d_items + n_one, n_quad, d_tab, sc.quad->p, d_st + n_one);
        hck(hipGetLastError(), "p256_verify_quad_kernel launch (remainder)");
    }
}

std::vector<uint8_t> p256_verify_gpu(const uint8_t* items, int64_t n) {
    std::vector<uint8_t> st(static_cast<size_t>(n));
    if (n == 0) return st;
    node_device_enter();
    const aff* d_tab = device_g16_table();
    PooledBuf<VerifyItem> b_items{size_t(n)};
    PooledBuf<uint8_t> b_st{size_t(n)};
    StagedIO io(sizeof(VerifyItem) * size_t(n) + size_t(n));
    io.h2d(b_items.p, items, sizeof(VerifyItem) * size_t(n));
    VerifyScratch sc;
    verify_launch(b_items.p, n, d_tab, b_st.p, sc);
    io.d2h(st.data(), b_st.p, size_t(n));
    io.finish("verify status");
    return st;
}

// One block's signatures from compressed keys (csrc/txcodec.cpp block_verify_fused): `fill` packs the
// inputs straight into pinned staging -- n_jobs 33-byte signer keys, n_jobs x 96 B (r | s | digest), n_out
// 33-byte output addresses -- then ONE stream order runs the key kernel (decompression into the verify items
// on the device, the outputs' curve check) and the verify, with one sync for the statuses and the output
// flags. `items_out` receives the device's verify items only when some status is INVALID (0): the caller's
// ASCII-hex retry rebuilds those records with another digest.
void p256_verify_fused_gpu(int64_t n_jobs, int64_t n_out, const std::function<void(uint8_t*, uint8_t*, uint8_t*)>& fill,
                           uint8_t* st, uint8_t* out_ok, std::vector<uint8_t>* items_out) {
    if (n_jobs + n_out == 0) return;
    node_device_enter();
    const aff* d_tab = device_g16_table();
    const size_t in_bytes = 129 * size_t(n_jobs) + 33 * size_t(n_out);
    PooledBuf<uint8_t> b_in{in_bytes}, b_st{size_t(n_jobs + n_out)};
    PooledBuf<VerifyItem> b_items{size_t(n_jobs)};
    StagedIO io(in_bytes + size_t(n_jobs + n_out));
    uint8_t* at = io.h2d_take(in_bytes);
    fill(at, at + 33 * size_t(n_jobs), at + 129 * size_t(n_jobs));
    io.h2d_issue(b_in.p, at, in_bytes);
    const int64_t nt = n_jobs + n_out;
    hipLaunchKernelGGL(p256_keyrec_kernel, dim3(unsigned((nt + 255) / 256)), dim3(256), 0, node_stream(), b_in.p,
                       b_in.p + 33 * n_jobs, n_jobs, b_in.p + 129 * n_jobs, n_out, b_items.p, b_st.p + n_jobs);
    hck(hipGetLastError(), "p256_keyrec_kernel launch");
    VerifyScratch sc;
    if (n_jobs) verify_launch(b_items.p, n_jobs, d_tab, b_st.p, sc);
    // statuses and output flags are adjacent on the device: one D2H for both
    const uint8_t* hst = io.d2h_arena(b_st.p, size_t(n_jobs + n_out));
    io.finish("fused verify");
    std::memcpy(st, hst, size_t(n_jobs));
    std::memcpy(out_ok, hst + n_jobs, size_t(n_out));
    if (items_out && std::find(st, st + n_jobs, uint8_t(0)) != st + n_jobs) {
        items_out->resize(sizeof(VerifyItem) * size_t(n_jobs));
        node_d2h(items_out->data(), b_items.p, items_out->size(), "d2h verify items");
    }
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

void p256_on_curve_host(const uint8_t* in, int64_t n, uint8_t* ok, int threads) {
    HostPool::get().parallel_for(n, threads, [&](int64_t i) { ok[i] = on_curve_64(in + 64 * i); });
}

void p256_on_curve_gpu(const uint8_t* in, int64_t n, uint8_t* ok) {
    if (n == 0) return;
    node_device_enter();
    PooledBuf<uint8_t> b_in{64 * size_t(n)}, b_ok{size_t(n)};
    StagedIO io(65 * size_t(n));
    io.h2d(b_in.p, in, 64 * size_t(n));
    const int block = 256;
    hipLaunchKernelGGL(p256_on_curve_kernel, dim3(int((n + block - 1) / block)), dim3(block), 0, node_stream(), b_in.p, n,
                       b_ok.p);
    hck(hipGetLastError(), "p256_on_curve_kernel launch");
    io.d2h(ok, b_ok.p, size_t(n));
    io.finish("on-curve");
}

void set_node_device_native(int dev) { set_node_device(dev); }

void p256_decompress_gpu(const uint8_t* in, int64_t n, uint8_t* out, uint8_t* ok) {
    if (n == 0) return;
    node_device_enter();
    PooledBuf<uint8_t> b_in{33 * size_t(n)}, b_out{64 * size_t(n)}, b_ok{size_t(n)};
    uint8_t *d_in = b_in.p, *d_out = b_out.p, *d_ok = b_ok.p;
    StagedIO io(98 * size_t(n));
    io.h2d(d_in, in, 33 * size_t(n));
    const int block = 256;
    hipLaunchKernelGGL(p256_decompress_kernel, dim3(int((n + block - 1) / block)), dim3(block), 0, node_stream(), d_in, n,
                       d_out, d_ok);
    hck(hipGetLastError(), "p256_decompress_kernel launch");
    io.d2h(out, d_out, 64 * size_t(n));
    io.d2h(ok, d_ok, size_t(n));
    io.finish("decompress");
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
