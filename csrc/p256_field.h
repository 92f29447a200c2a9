// NIST P-256 arithmetic shared by the host library and the gfx950 kernels (HIP __host__ __device__).
//
// Representation: 8 x 32-bit little-endian limbs. 32-bit limbs map the 32x32->64 partial products
// onto v_mad_u64_u32 on CDNA4 (64-bit limbs would need 4 of them per product anyway).
//  * field mod p: schoolbook 8x8 product + NIST/Solinas fast reduction (FIPS 186-4 D.2.3), using
//    p = 2^256 - 2^224 + 2^192 + 2^96 - 1 (no Montgomery form needed on the coordinate side);
//  * scalars mod n: Montgomery (CIOS) multiplication, used for s^-1, u1 = e*s^-1, u2 = r*s^-1;
//  * points: Jacobian coordinates with a = -3 doubling (dbl-2001-b), full add (add-2007-bl) and
//    mixed Jacobian+affine add (madd-2007-bl), all with explicit infinity/equal/opposite handling.
//
// reference semantics being reproduced: fastecdsa's ecdsa.verify/sign and util.mod_sqrt as used by
// upow/upow_transactions/transaction_input.py:84-120 and upow/helpers.py:58-62.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#define UPOW_HD __host__ __device__ __forceinline__

namespace upow {
namespace p256 {

struct fe { uint32_t v[8]; };

struct jac { fe x, y, z; };  // z == 0 <=> infinity
struct aff { fe x, y; };

// ------------------------------------------------------------------------------------------------
// constants (little-endian 32-bit limbs)
// ------------------------------------------------------------------------------------------------
#define P256_P {0xffffffffu, 0xffffffffu, 0xffffffffu, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000001u, 0xffffffffu}
#define P256_N {0xfc632551u, 0xf3b9cac2u, 0xa7179e84u, 0xbce6faadu, 0xffffffffu, 0xffffffffu, 0x00000000u, 0xffffffffu}
#define P256_B {0x27d2604bu, 0x3bce3c3eu, 0xcc53b0f6u, 0x651d06b0u, 0x769886bcu, 0xb3ebbd55u, 0xaa3a93e7u, 0x5ac635d8u}
#define P256_GX {0xd898c296u, 0xf4a13945u, 0x2deb33a0u, 0x77037d81u, 0x63a440f2u, 0xf8bce6e5u, 0xe12c4247u, 0x6b17d1f2u}
#define P256_GY {0x37bf51f5u, 0xcbb64068u, 0x6b315eceu, 0x2bce3357u, 0x7c0f9e16u, 0x8ee7eb4au, 0xfe1a7f9bu, 0x4fe342e2u}
#define P256_RN {0x039cdaafu, 0x0c46353du, 0x58e8617bu, 0x43190552u, 0x00000000u, 0x00000000u, 0xffffffffu, 0x00000000u}
#define P256_R2N {0xbe79eea2u, 0x83244c95u, 0x49bd6fa6u, 0x4699799cu, 0x2b6bec59u, 0x2845b239u, 0xf3d95620u, 0x66e12d94u}
static constexpr uint32_t P256_N0INV = 0xee00bc4fu;  // -n^-1 mod 2^32

UPOW_HD fe fe_const_p() { return fe{P256_P}; }
UPOW_HD fe fe_const_n() { return fe{P256_N}; }
UPOW_HD fe fe_const_b() { return fe{P256_B}; }
UPOW_HD fe fe_zero() { return fe{{0, 0, 0, 0, 0, 0, 0, 0}}; }
UPOW_HD fe fe_one() { return fe{{1, 0, 0, 0, 0, 0, 0, 0}}; }

UPOW_HD bool fe_is_zero(const fe& a) {
    uint32_t t = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) t |= a.v[i];
    return t == 0;
}
UPOW_HD bool fe_eq(const fe& a, const fe& b) {
    uint32_t t = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) t |= a.v[i] ^ b.v[i];
    return t == 0;
}
// a >= b (unsigned 256-bit): no final borrow of a - b
UPOW_HD bool fe_geq(const fe& a, const fe& b) {
    unsigned c = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) (void)__builtin_subc(a.v[i], b.v[i], c, &c);
    return c == 0;
}
// r = a + b, returns carry. Carry builtins map onto v_add_co_u32 / v_addc_co_u32 chains on gfx950
// (the uint64 formulation compiles to 64-bit shift-adds plus register moves: ~4x the instructions).
UPOW_HD uint32_t raw_add(fe& r, const fe& a, const fe& b) {
    unsigned c = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.v[i] = __builtin_addc(a.v[i], b.v[i], c, &c);
    return c;
}
// r = a - b, returns borrow
UPOW_HD uint32_t raw_sub(fe& r, const fe& a, const fe& b) {
    unsigned c = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.v[i] = __builtin_subc(a.v[i], b.v[i], c, &c);
    return c;
}
// r = cond ? a : b  (branch-free select)
UPOW_HD fe fe_select(bool cond, const fe& a, const fe& b) {
    fe r;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.v[i] = cond ? a.v[i] : b.v[i];
    return r;
}

// ------------------------------------------------------------------------------------------------
// field mod p
// ------------------------------------------------------------------------------------------------
UPOW_HD fe fe_add(const fe& a, const fe& b) {
    fe r, t;
    const uint32_t c = raw_add(r, a, b);
    const uint32_t br = raw_sub(t, r, fe_const_p());
    // use t when (carry) or (no borrow)
    return fe_select(c | (br ^ 1u), t, r);
}
// a - b, plus p when it borrows: p masked by the borrow (p's words are all-ones, zero or one), one chain
// of adds instead of computing r + p in full and selecting (17 instructions instead of 24)
UPOW_HD fe fe_sub(const fe& a, const fe& b) {
    fe r;
    const uint32_t br = raw_sub(r, a, b);
    const uint32_t m = 0u - br;
    unsigned c = 0;
    r.v[0] = __builtin_addc(r.v[0], m, c, &c);
    r.v[1] = __builtin_addc(r.v[1], m, c, &c);
    r.v[2] = __builtin_addc(r.v[2], m, c, &c);
    r.v[3] = __builtin_addc(r.v[3], 0u, c, &c);
    r.v[4] = __builtin_addc(r.v[4], 0u, c, &c);
    r.v[5] = __builtin_addc(r.v[5], 0u, c, &c);
    r.v[6] = __builtin_addc(r.v[6], br, c, &c);
    r.v[7] = __builtin_addc(r.v[7], m, c, &c);
    return r;
}
UPOW_HD fe fe_neg(const fe& a) { return fe_sub(fe_zero(), a); }

// 512-bit schoolbook product, one row per limb of a: t = a_i*b_j + c[i+j] is one v_mad_u64_u32
// with a zero-extended 32-bit addend (never overflows 64 bits); the row's high words are chained in
// with a single add-with-carry per product. (Writing the step as a 64-bit sum of three terms makes
// the compiler emit 64-bit shift-adds and ~2 register moves per product instead.)
UPOW_HD void mul_512(uint32_t c[16], const fe& a, const fe& b) {
#pragma unroll
    for (int i = 0; i < 16; ++i) c[i] = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        unsigned cy = 0;
        uint32_t prev = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const uint64_t t = uint64_t(a.v[i]) * b.v[j] + c[i + j];
            c[i + j] = __builtin_addc(uint32_t(t), prev, cy, &cy);
            prev = uint32_t(t >> 32);
        }
        c[i + 8] = prev + cy;  // cannot overflow: the row sum is < 2^(32(i+9))
    }
}

// squaring: off-diagonal rows once (28 products), double with funnel shifts, add the 8 squares.
UPOW_HD void sqr_512(uint32_t c[16], const fe& a) {
#pragma unroll
    for (int i = 0; i < 16; ++i) c[i] = 0;
#pragma unroll
    for (int i = 0; i < 7; ++i) {
        unsigned cy = 0;
        uint32_t prev = 0;
#pragma unroll
        for (int j = i + 1; j < 8; ++j) {
            const uint64_t t = uint64_t(a.v[i]) * a.v[j] + c[i + j];
            c[i + j] = __builtin_addc(uint32_t(t), prev, cy, &cy);
            prev = uint32_t(t >> 32);
        }
        c[i + 8] = prev + cy;
    }
    c[15] = c[14] >> 31;
#pragma unroll
    for (int k = 14; k > 0; --k) c[k] = (c[k] << 1) | (c[k - 1] >> 31);
    c[0] = c[0] << 1;
    unsigned cy = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint64_t sq = uint64_t(a.v[i]) * a.v[i];
        c[2 * i] = __builtin_addc(c[2 * i], uint32_t(sq), cy, &cy);
        c[2 * i + 1] = __builtin_addc(c[2 * i + 1], uint32_t(sq >> 32), cy, &cy);
    }
}

// NIST fast reduction of a 512-bit value mod p (FIPS 186-4 D.2.3):
//   c mod p = s1 + 2 s2 + 2 s3 + s4 + s5 - s6 - s7 - s8 - s9 (mod p)
// evaluated with 32-bit add/sub-with-carry chains (v_add_co/v_addc on gfx950; int64 limbs cost
// 64-bit shift-adds plus sign-extension moves), then the signed overflow T in [-4, 6] is folded with
// 2^256 == K = 2^224 - 2^192 - 2^96 + 1 (mod p) and the result brought into [0, p) branch-free.
#define UPOW_ACC(OP, S)                                                     \
    {                                                                       \
        unsigned cy_ = 0;                                                   \
        _Pragma("unroll") for (int i_ = 0; i_ < 8; ++i_) r[i_] = OP(r[i_], S[i_], cy_, &cy_); \
        top = (OP(top, 0u, cy_, &cy_));                                     \
    }
UPOW_HD fe fe_reduce(const uint32_t c[16]) {
    const uint32_t z = 0;
    const uint32_t s1[8] = {c[0], c[1], c[2], c[3], c[4], c[5], c[6], c[7]};
    const uint32_t s2[8] = {z, z, z, c[11], c[12], c[13], c[14], c[15]};
    const uint32_t s3[8] = {z, z, z, c[12], c[13], c[14], c[15], z};
    const uint32_t s4[8] = {c[8], c[9], c[10], z, z, z, c[14], c[15]};
    const uint32_t s5[8] = {c[9], c[10], c[11], c[13], c[14], c[15], c[13], c[8]};
    const uint32_t s6[8] = {c[11], c[12], c[13], z, z, z, c[8], c[10]};
    const uint32_t s7[8] = {c[12], c[13], c[14], c[15], z, z, c[9], c[11]};
    const uint32_t s8[8] = {c[13], c[14], c[15], c[8], c[9], c[10], z, c[12]};
    const uint32_t s9[8] = {c[14], c[15], z, c[9], c[10], c[11], z, c[13]};
    uint32_t r[8];
    uint32_t top = 0;  // signed 9th limb (two's complement)
    {
        unsigned cy = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) r[i] = __builtin_addc(s2[i], s3[i], cy, &cy);
        top = cy;
        cy = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) r[i] = __builtin_addc(r[i], r[i], cy, &cy);
        top = 2 * top + cy;
    }
    UPOW_ACC(__builtin_addc, s1)
    UPOW_ACC(__builtin_addc, s4)
    UPOW_ACC(__builtin_addc, s5)
    UPOW_ACC(__builtin_subc, s6)
    UPOW_ACC(__builtin_subc, s7)
    UPOW_ACC(__builtin_subc, s8)
    UPOW_ACC(__builtin_subc, s9)
    // W = r + T*K with T = (int32)top: add T at limb 0, subtract at limbs 3 and 6, add at limb 7;
    // every addend is sign-extended to the 9th limb h
    const uint32_t t = top;
    const uint32_t sx = uint32_t(int32_t(t) >> 31);
    uint32_t h = 0;
    {
        unsigned cy = 0;
        r[0] = __builtin_addc(r[0], t, cy, &cy);
#pragma unroll
        for (int i = 1; i < 8; ++i) r[i] = __builtin_addc(r[i], sx, cy, &cy);
        h = __builtin_addc(h, sx, cy, &cy);
        cy = 0;
        r[3] = __builtin_subc(r[3], t, cy, &cy);
#pragma unroll
        for (int i = 4; i < 8; ++i) r[i] = __builtin_subc(r[i], sx, cy, &cy);
        h = __builtin_subc(h, sx, cy, &cy);
        cy = 0;
        r[6] = __builtin_subc(r[6], t, cy, &cy);
        r[7] = __builtin_subc(r[7], sx, cy, &cy);
        h = __builtin_subc(h, sx, cy, &cy);
        cy = 0;
        r[7] = __builtin_addc(r[7], t, cy, &cy);
        h = __builtin_addc(h, sx, cy, &cy);
    }
    // W = r + h*2^256 with h in {-1, 0, 1}:
    //   h = 1  -> r + K            (< p, no carry)
    //   h = -1 -> r - K = r + p - 2^256
    //   h = 0  -> r - p = r + K - 2^256 when r >= p (i.e. when r + K carries), else r
    // one add chain of the selected constant, K or p masked word by word (their words are all-ones, zero,
    // one or all-but-one), after a carry-only chain for r >= p
    const uint32_t K[8] = {1u, 0u, 0u, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xfffffffeu, 0u};
    unsigned ck = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) (void)__builtin_addc(r[i], K[i], ck, &ck);
    const uint32_t mk = 0u - uint32_t(h == 1u || (h == 0u && ck));
    const uint32_t mp = 0u - uint32_t(h == 0xffffffffu);
    const uint32_t ad[8] = {(mk & 1u) | mp, mp, mp, mk, mk, mk, (mk & 0xfffffffeu) | (mp & 1u), mp};
    fe o;
    unsigned co = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) o.v[i] = __builtin_addc(r[i], ad[i], co, &co);
    return o;
}
#undef UPOW_ACC

UPOW_HD fe fe_mul(const fe& a, const fe& b) {
    uint32_t c[16];
    mul_512(c, a, b);
    return fe_reduce(c);
}
UPOW_HD fe fe_sqr(const fe& a) {
    uint32_t c[16];
    sqr_512(c, a);
    return fe_reduce(c);
}
UPOW_HD fe fe_sqr_n(fe a, int n) {
    for (int i = 0; i < n; ++i) a = fe_sqr(a);
    return a;
}
UPOW_HD fe fe_mul_small(const fe& a, uint32_t k) {
    fe r = fe_zero();
    for (uint32_t i = 0; i < k; ++i) r = fe_add(r, a);
    return r;
}

// a^(p-2) via an addition chain over runs of ones: p-2 = ffffffff 00000001 00000000 00000000
// 00000000 ffffffff ffffffff fffffffd (big-endian words).
UPOW_HD fe fe_inv(const fe& a) {
    const fe x2 = fe_mul(fe_sqr(a), a);             // 2^2-1
    const fe x3 = fe_mul(fe_sqr(x2), a);            // 2^3-1
    const fe x6 = fe_mul(fe_sqr_n(x3, 3), x3);      // 2^6-1
    const fe x12 = fe_mul(fe_sqr_n(x6, 6), x6);     // 2^12-1
    const fe x15 = fe_mul(fe_sqr_n(x12, 3), x3);    // 2^15-1
    const fe x30 = fe_mul(fe_sqr_n(x15, 15), x15);  // 2^30-1
    const fe x32 = fe_mul(fe_sqr_n(x30, 2), x2);    // 2^32-1
    fe t = fe_mul(fe_sqr_n(x32, 32), a);            // ffffffff 00000001
    t = fe_sqr_n(t, 96);                            // 00000000 00000000 00000000
    t = fe_mul(fe_sqr_n(t, 32), x32);               // ffffffff
    t = fe_mul(fe_sqr_n(t, 32), x32);               // ffffffff
    t = fe_mul(fe_sqr_n(t, 30), x30);               // fffffffd = 30 ones ...
    t = fe_mul(fe_sqr_n(t, 2), a);                  //            ... then "01"
    return t;
}

// a^((p+1)/4): (p+1)/4 = 3fffffffc0000000400000000000000000000000400000000000000000000000
UPOW_HD fe fe_sqrt_candidate(const fe& a) {
    const fe x2 = fe_mul(fe_sqr(a), a);
    const fe x4 = fe_mul(fe_sqr_n(x2, 2), x2);
    const fe x8 = fe_mul(fe_sqr_n(x4, 4), x4);
    const fe x16 = fe_mul(fe_sqr_n(x8, 8), x8);
    const fe x32 = fe_mul(fe_sqr_n(x16, 16), x16);
    // exponent bits (from the top): 30 ones ... we build (2^32-1) << ... then adjust:
    // (p+1)/4 = 2^254 - 2^222 + 2^190 + 2^94 ; compute a^(2^32-1) then shift patterns:
    fe t = fe_sqr_n(x32, 32);        // a^((2^32-1)*2^32)
    t = fe_mul(t, a);                // a^((2^32-1)*2^32 + 1)
    t = fe_sqr_n(t, 96);             // * 2^96
    t = fe_mul(t, a);                // + 1
    t = fe_sqr_n(t, 94);             // * 2^94
    // exponent = ((2^32-1)*2^32 + 1)*2^190 + 2^94 = 2^254 - 2^222 + 2^190 + 2^94 == (p+1)/4
    return t;
}

// ------------------------------------------------------------------------------------------------
// scalars mod n (Montgomery, R = 2^256)
// ------------------------------------------------------------------------------------------------
UPOW_HD fe sc_mont_mul(const fe& a, const fe& b) {
    const fe n = fe_const_n();
    uint32_t t[10];
#pragma unroll
    for (int i = 0; i < 10; ++i) t[i] = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        uint64_t C = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const uint64_t s = uint64_t(a.v[j]) * b.v[i] + t[j] + C;
            t[j] = uint32_t(s);
            C = s >> 32;
        }
        uint64_t s = uint64_t(t[8]) + C;
        t[8] = uint32_t(s);
        t[9] = uint32_t(s >> 32);
        const uint32_t m = t[0] * P256_N0INV;
        s = uint64_t(m) * n.v[0] + t[0];
        C = s >> 32;
#pragma unroll
        for (int j = 1; j < 8; ++j) {
            s = uint64_t(m) * n.v[j] + t[j] + C;
            t[j - 1] = uint32_t(s);
            C = s >> 32;
        }
        s = uint64_t(t[8]) + C;
        t[7] = uint32_t(s);
        t[8] = t[9] + uint32_t(s >> 32);
    }
    fe r, d;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.v[i] = t[i];
    const uint32_t br = raw_sub(d, r, n);
    return fe_select(t[8] != 0 || br == 0, d, r);
}
UPOW_HD fe sc_to_mont(const fe& a) { return sc_mont_mul(a, fe{P256_R2N}); }
UPOW_HD fe sc_from_mont(const fe& a) { return sc_mont_mul(a, fe_one()); }
// reduce a < 2^256 mod n (a < 2n always holds)
UPOW_HD fe sc_reduce(const fe& a) {
    fe d;
    const uint32_t br = raw_sub(d, a, fe_const_n());
    return fe_select(br == 0, d, a);
}
// a^(n-2) in the Montgomery domain (a_m = a*R): returns a^-1 * R.
// n-2 = ffffffff 00000000 ffffffff ffffffff | bce6faad a7179e84 f3b9cac2 fc63254f. The high half is
// runs of ones (addition chain through a^(2^32-1)); the low half is scanned bit by bit with the bit
// taken from a constant word, so the branch is wave-uniform and nothing is indexed dynamically
// (a windowed table in a local array would live in scratch memory on the GPU).
UPOW_HD fe sc_sqr_n_mont(fe a, int n) {
    for (int i = 0; i < n; ++i) a = sc_mont_mul(a, a);
    return a;
}
UPOW_HD fe sc_inv_mont(const fe& a_m) {
    const fe x2 = sc_mont_mul(sc_mont_mul(a_m, a_m), a_m);     // 2^2-1
    const fe x4 = sc_mont_mul(sc_sqr_n_mont(x2, 2), x2);       // 2^4-1
    const fe x8 = sc_mont_mul(sc_sqr_n_mont(x4, 4), x4);       // 2^8-1
    const fe x16 = sc_mont_mul(sc_sqr_n_mont(x8, 8), x8);      // 2^16-1
    const fe x32 = sc_mont_mul(sc_sqr_n_mont(x16, 16), x16);   // 2^32-1
    fe t = sc_mont_mul(sc_sqr_n_mont(x32, 64), x32);           // ffffffff 00000000 ffffffff
    t = sc_mont_mul(sc_sqr_n_mont(t, 32), x32);                // ... ffffffff
    for (int k = 0; k < 128; ++k) {
        const uint32_t word = k < 32 ? 0xbce6faadu : k < 64 ? 0xa7179e84u : k < 96 ? 0xf3b9cac2u : 0xfc63254fu;
        t = sc_mont_mul(t, t);
        if ((word >> (31 - (k & 31))) & 1u) t = sc_mont_mul(t, a_m);
    }
    return t;
}

// a^-1 * R mod n (the Montgomery form of the inverse, ready for sc_mont_mul) for a in [1, n), by the
// binary extended Euclid: u = x*a, v = y*a (mod n) hold throughout; every pass makes u even (subtracting
// the smaller of u, v from the larger when u is odd) and halves u and x, so log2(u*v) drops by at least
// one bit per pass and u reaches 0 after at most 512 passes (~360 for random a), leaving v = gcd = 1 and
// y = a^-1 (times R, which x starts at). Variable time, which is fine for verification (public data);
// the GPU wave runs until its slowest lane is done (~385 passes). Each pass is ~170 full-rate VALU ops
// with no multiplies: about a third of the VALU issue slots of the Fermat chain a^(n-2) (sc_inv_mont,
// ~300 Montgomery products of 128 quarter-rate v_mad_u64_u32 each), which sign() still uses.
UPOW_HD fe sc_inv_bgcd_mont(const fe& a) {
    const fe n = fe_const_n();
    fe u = a, v = n, x{P256_RN}, y = fe_zero();
    while (!fe_is_zero(u)) {
        const bool odd = u.v[0] & 1u;
        fe d1, d2, dx, t;
        const bool lt = raw_sub(d1, u, v) != 0;  // u < v
        raw_sub(d2, v, u);
        const uint32_t bx = raw_sub(dx, x, y);   // x - y mod n
        raw_add(t, dx, n);
        dx = fe_select(bx != 0, t, dx);
        fe ndx;                                   // y - x mod n = n - (x - y) unless zero
        raw_sub(ndx, n, dx);
        ndx = fe_select(fe_is_zero(dx), dx, ndx);
        const bool sw = odd && lt;
        const fe nu = fe_select(odd, fe_select(lt, d2, d1), u);
        const fe nx = fe_select(odd, fe_select(lt, ndx, dx), x);
        v = fe_select(sw, u, v);
        y = fe_select(sw, x, y);
        // u = nu / 2 (nu is even); x = nx / 2 mod n
#pragma unroll
        for (int i = 0; i < 7; ++i) u.v[i] = (nu.v[i] >> 1) | (nu.v[i + 1] << 31);
        u.v[7] = nu.v[7] >> 1;
        const uint32_t mask = 0u - (nx.v[0] & 1u);
        fe nm, xs;
#pragma unroll
        for (int i = 0; i < 8; ++i) nm.v[i] = n.v[i] & mask;
        const uint32_t c = raw_add(xs, nx, nm);
#pragma unroll
        for (int i = 0; i < 7; ++i) x.v[i] = (xs.v[i] >> 1) | (xs.v[i + 1] << 31);
        x.v[7] = (xs.v[7] >> 1) | (c << 31);
    }
    return y;
}

// a^-1 * R mod n by Bernstein-Yang divsteps (the "safegcd" recurrence, delta starting at 1/2). Values are
// in signed 30-bit limbs (nine int32, limb 8 signed). 20 rounds of 30 divsteps cover the 590 that any
// 256-bit input needs; each round runs its 30 divsteps on the low 32 bits of f and g alone (they decide
// every branch), collecting them into a 2x2 matrix scaled by 2^30, then applies the matrix to the full
// (f, g) and to (d, e), which track f = d*a*R^-1 and g = e*a*R^-1 (mod n): e starts at R, so d ends at
// +-a^-1*R, the Montgomery form verify_prologue wants. At most 20 rounds; a round's divsteps have no
// data-dependent branches, and the loop stops once g is zero (for random scalars after ~18 rounds). Cost per round: 30 divsteps of ~20 full-rate 32-bit ops, and 36 + 54 signed
// 32x32->64 multiply-adds for the matrix products; about a third of the binary Euclid above.
struct s30 { int32_t v[9]; };
static constexpr uint32_t kM30 = 0x3fffffffu;
static constexpr uint32_t kN30Inv = 0x11ff43b1u;  // n^-1 mod 2^30

UPOW_HD s30 s30_from_fe(const fe& a) {
    s30 r;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        const int bit = 30 * i, w = bit >> 5, sh = bit & 31;
        uint32_t x = a.v[w] >> sh;
        if (sh > 2 && w + 1 < 8) x |= a.v[w + 1] << (32 - sh);
        r.v[i] = int32_t(x & kM30);
    }
    return r;
}
// limbs 0..7 in [0, 2^30), limb 8 in [0, 2^16) (a canonical value below 2^256)
UPOW_HD fe fe_from_s30(const s30& a) {
    fe r;
#pragma unroll
    for (int w = 0; w < 8; ++w) {
        const int bit = 32 * w, i = bit / 30, sh = bit % 30;
        uint32_t x = uint32_t(a.v[i]) >> sh;
        if (i + 1 < 9) x |= uint32_t(a.v[i + 1]) << (30 - sh);
        if (sh > 28 && i + 2 < 9) x |= uint32_t(a.v[i + 2]) << (60 - sh);
        r.v[w] = x;
    }
    return r;
}

struct DivMatrix { int32_t u, v, q, r; };
// 30 divsteps on the low words: returns the new zeta = -(delta + 1/2)
UPOW_HD int32_t divsteps_30(int32_t zeta, uint32_t f, uint32_t g, DivMatrix& t) {
    uint32_t u = 1, v = 0, q = 0, r = 1;
#pragma unroll
    for (int i = 0; i < 30; ++i) {
        uint32_t c1 = uint32_t(zeta >> 31);  // all ones when delta > 0
        const uint32_t c2 = 0u - (g & 1u);   // all ones when g is odd
        // g odd: g += (delta > 0 ? -f : f), and the same on the matrix rows
        g += ((f ^ c1) - c1) & c2;
        q += ((u ^ c1) - c1) & c2;
        r += ((v ^ c1) - c1) & c2;
        c1 &= c2;  // delta > 0 and g odd: (f, g) <- (g, g - f), delta <- 1 - delta
        zeta = int32_t((uint32_t(zeta) ^ c1) - 1u);
        f += g & c1;
        u += q & c1;
        v += r & c1;
        g >>= 1;
        u <<= 1;
        v <<= 1;
    }
    t = DivMatrix{int32_t(u), int32_t(v), int32_t(q), int32_t(r)};
    return zeta;
}

// (f, g) <- (u f + v g, q f + r g) / 2^30 (exact)
UPOW_HD void s30_update_fg(s30& f, s30& g, const DivMatrix& t) {
    int64_t cf = int64_t(t.u) * f.v[0] + int64_t(t.v) * g.v[0];
    int64_t cg = int64_t(t.q) * f.v[0] + int64_t(t.r) * g.v[0];
    cf >>= 30;
    cg >>= 30;
#pragma unroll
    for (int i = 1; i < 9; ++i) {
        cf += int64_t(t.u) * f.v[i] + int64_t(t.v) * g.v[i];
        cg += int64_t(t.q) * f.v[i] + int64_t(t.r) * g.v[i];
        f.v[i - 1] = int32_t(uint32_t(cf) & kM30);
        g.v[i - 1] = int32_t(uint32_t(cg) & kM30);
        cf >>= 30;
        cg >>= 30;
    }
    f.v[8] = int32_t(cf);
    g.v[8] = int32_t(cg);
}

// (d, e) <- (u d + v e, q d + r e) / 2^30 mod n, keeping both in (-2n, n): a multiple of n is added to
// each numerator to clear its low 30 bits (plus n times the matrix row when d or e is negative)
UPOW_HD void s30_update_de(s30& d, s30& e, const DivMatrix& t, const s30& n) {
    const int32_t sd = d.v[8] >> 31, se = e.v[8] >> 31;
    int32_t md = (t.u & sd) + (t.v & se);
    int32_t me = (t.q & sd) + (t.r & se);
    int64_t cd = int64_t(t.u) * d.v[0] + int64_t(t.v) * e.v[0];
    int64_t ce = int64_t(t.q) * d.v[0] + int64_t(t.r) * e.v[0];
    md -= int32_t((kN30Inv * uint32_t(cd) + uint32_t(md)) & kM30);
    me -= int32_t((kN30Inv * uint32_t(ce) + uint32_t(me)) & kM30);
    cd += int64_t(n.v[0]) * md;
    ce += int64_t(n.v[0]) * me;
    cd >>= 30;
    ce >>= 30;
#pragma unroll
    for (int i = 1; i < 9; ++i) {
        cd += int64_t(t.u) * d.v[i] + int64_t(t.v) * e.v[i] + int64_t(n.v[i]) * md;
        ce += int64_t(t.q) * d.v[i] + int64_t(t.r) * e.v[i] + int64_t(n.v[i]) * me;
        d.v[i - 1] = int32_t(uint32_t(cd) & kM30);
        e.v[i - 1] = int32_t(uint32_t(ce) & kM30);
        cd >>= 30;
        ce >>= 30;
    }
    d.v[8] = int32_t(cd);
    e.v[8] = int32_t(ce);
}

// carry-normalise: limbs 0..7 into [0, 2^30), the sign in limb 8
UPOW_HD void s30_carry(s30& a) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        a.v[i + 1] += a.v[i] >> 30;
        a.v[i] = int32_t(uint32_t(a.v[i]) & kM30);
    }
}
// a += n & mask (limb-wise), then carry
UPOW_HD void s30_add_masked(s30& a, const s30& n, int32_t mask) {
#pragma unroll
    for (int i = 0; i < 9; ++i) a.v[i] += n.v[i] & mask;
    s30_carry(a);
}

UPOW_HD fe sc_inv_safegcd_mont(const fe& a) {
    const s30 n = s30_from_fe(fe_const_n());
    s30 f = n, g = s30_from_fe(a), d{{0, 0, 0, 0, 0, 0, 0, 0, 0}}, e = s30_from_fe(fe{P256_RN});
    int32_t zeta = -1;
    for (int round = 0; round < 20; ++round) {
        // g = 0: f = +-1 and the remaining rounds would only keep d, e in range (their matrix is
        // diag(2^30, 1)); random inputs finish in ~517 divsteps (18 rounds), 590 bounds every input.
        // Public data, so the exit may depend on it; a wave runs until its last lane is done.
        uint32_t gz = 0;
#pragma unroll
        for (int i = 0; i < 9; ++i) gz |= uint32_t(g.v[i]);
        if (gz == 0) break;
        DivMatrix t;
        zeta = divsteps_30(zeta, uint32_t(f.v[0]) | (uint32_t(f.v[1]) << 30), uint32_t(g.v[0]) | (uint32_t(g.v[1]) << 30), t);
        s30_update_de(d, e, t, n);
        s30_update_fg(f, g, t);
    }
    // g = 0 and f = +-1 (f's sign is its top limb's): d = +-a^-1*R in (-2n, n)
    const int32_t sf = f.v[8] >> 31;
#pragma unroll
    for (int i = 0; i < 9; ++i) d.v[i] = (d.v[i] ^ sf) - sf;
    s30_carry(d);                        // (-2n, 2n): d was in (-2n, n) and may have been negated
    s30_add_masked(d, n, d.v[8] >> 31);  // (-n, 2n)
    s30_add_masked(d, n, d.v[8] >> 31);  // [0, 2n)
    s30 t = d;                           // d - n, kept when non-negative
#pragma unroll
    for (int i = 0; i < 9; ++i) t.v[i] -= n.v[i];
    s30_carry(t);
    const bool ge = t.v[8] >= 0;
#pragma unroll
    for (int i = 0; i < 9; ++i) d.v[i] = ge ? t.v[i] : d.v[i];
    return fe_from_s30(d);
}

// ------------------------------------------------------------------------------------------------
// points
// ------------------------------------------------------------------------------------------------
UPOW_HD bool jac_is_inf(const jac& p) { return fe_is_zero(p.z); }
UPOW_HD jac jac_inf() { return jac{fe_one(), fe_one(), fe_zero()}; }
UPOW_HD jac jac_from_aff(const aff& a) { return jac{a.x, a.y, fe_one()}; }

UPOW_HD bool aff_on_curve(const aff& a) {
    const fe p = fe_const_p();
    if (fe_geq(a.x, p) || fe_geq(a.y, p)) return false;
    // y^2 == x^3 - 3x + b
    const fe y2 = fe_sqr(a.y);
    fe rhs = fe_mul(fe_sqr(a.x), a.x);
    const fe x3 = fe_add(fe_add(a.x, a.x), a.x);
    rhs = fe_add(fe_sub(rhs, x3), fe_const_b());
    return fe_eq(y2, rhs);
}

// dbl-2001-b (a = -3): 3M + 5S
UPOW_HD jac jac_dbl(const jac& p) {
    if (fe_is_zero(p.z) || fe_is_zero(p.y)) return jac_inf();
    const fe delta = fe_sqr(p.z);
    const fe gamma = fe_sqr(p.y);
    const fe beta = fe_mul(p.x, gamma);
    const fe t0 = fe_sub(p.x, delta);
    const fe t1 = fe_add(p.x, delta);
    fe alpha = fe_mul(t0, t1);
    alpha = fe_add(fe_add(alpha, alpha), alpha);
    const fe beta4 = fe_add(fe_add(beta, beta), fe_add(beta, beta));
    const fe beta8 = fe_add(beta4, beta4);
    jac r;
    r.x = fe_sub(fe_sqr(alpha), beta8);
    const fe yz = fe_add(p.y, p.z);
    r.z = fe_sub(fe_sub(fe_sqr(yz), gamma), delta);
    fe g2 = fe_sqr(gamma);
    g2 = fe_add(g2, g2);
    g2 = fe_add(g2, g2);
    g2 = fe_add(g2, g2);  // 8 gamma^2
    r.y = fe_sub(fe_mul(alpha, fe_sub(beta4, r.x)), g2);
    return r;
}

// add-2007-bl: 11M + 5S
UPOW_HD jac jac_add(const jac& p, const jac& q) {
    if (fe_is_zero(p.z)) return q;
    if (fe_is_zero(q.z)) return p;
    const fe z1z1 = fe_sqr(p.z);
    const fe z2z2 = fe_sqr(q.z);
    const fe u1 = fe_mul(p.x, z2z2);
    const fe u2 = fe_mul(q.x, z1z1);
    const fe s1 = fe_mul(fe_mul(p.y, q.z), z2z2);
    const fe s2 = fe_mul(fe_mul(q.y, p.z), z1z1);
    const fe h = fe_sub(u2, u1);
    const fe rr0 = fe_sub(s2, s1);
    if (fe_is_zero(h)) {
        if (fe_is_zero(rr0)) return jac_dbl(p);
        return jac_inf();
    }
    const fe h2 = fe_add(h, h);
    const fe i = fe_sqr(h2);
    const fe j = fe_mul(h, i);
    const fe rr = fe_add(rr0, rr0);
    const fe v = fe_mul(u1, i);
    jac r;
    r.x = fe_sub(fe_sub(fe_sqr(rr), j), fe_add(v, v));
    const fe s1j = fe_mul(s1, j);
    r.y = fe_sub(fe_mul(rr, fe_sub(v, r.x)), fe_add(s1j, s1j));
    const fe zz = fe_add(p.z, q.z);
    r.z = fe_mul(fe_sub(fe_sub(fe_sqr(zz), z1z1), z2z2), h);
    return r;
}

// madd-2007-bl (q affine, z2 = 1): 7M + 4S
UPOW_HD jac jac_madd(const jac& p, const aff& q) {
    if (fe_is_zero(p.z)) return jac_from_aff(q);
    const fe z1z1 = fe_sqr(p.z);
    const fe u2 = fe_mul(q.x, z1z1);
    const fe s2 = fe_mul(fe_mul(q.y, p.z), z1z1);
    const fe h = fe_sub(u2, p.x);
    const fe rr0 = fe_sub(s2, p.y);
    if (fe_is_zero(h)) {
        if (fe_is_zero(rr0)) return jac_dbl(p);
        return jac_inf();
    }
    const fe hh = fe_sqr(h);
    fe i = fe_add(hh, hh);
    i = fe_add(i, i);
    const fe j = fe_mul(h, i);
    const fe rr = fe_add(rr0, rr0);
    const fe v = fe_mul(p.x, i);
    jac r;
    r.x = fe_sub(fe_sub(fe_sqr(rr), j), fe_add(v, v));
    const fe y1j = fe_mul(p.y, j);
    r.y = fe_sub(fe_mul(rr, fe_sub(v, r.x)), fe_add(y1j, y1j));
    const fe zh = fe_add(p.z, h);
    r.z = fe_sub(fe_sub(fe_sqr(zh), z1z1), hh);
    return r;
}

UPOW_HD bool jac_to_aff(const jac& p, aff& out) {
    if (fe_is_zero(p.z)) return false;
    const fe zi = fe_inv(p.z);
    const fe zi2 = fe_sqr(zi);
    out.x = fe_mul(p.x, zi2);
    out.y = fe_mul(p.y, fe_mul(zi2, zi));
    return true;
}

// Byte helpers: 32-byte big-endian <-> limbs
UPOW_HD fe fe_from_be(const uint8_t* b) {
    fe r;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint8_t* q = b + 28 - 4 * i;
        r.v[i] = (uint32_t(q[0]) << 24) | (uint32_t(q[1]) << 16) | (uint32_t(q[2]) << 8) | uint32_t(q[3]);
    }
    return r;
}
UPOW_HD void fe_to_be(const fe& a, uint8_t* b) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        uint8_t* q = b + 28 - 4 * i;
        q[0] = uint8_t(a.v[i] >> 24); q[1] = uint8_t(a.v[i] >> 16); q[2] = uint8_t(a.v[i] >> 8); q[3] = uint8_t(a.v[i]);
    }
}
// 32-byte little-endian (the upow wire order for x/y/r/s)
UPOW_HD fe fe_from_le(const uint8_t* b) {
    fe r;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint8_t* q = b + 4 * i;
        r.v[i] = uint32_t(q[0]) | (uint32_t(q[1]) << 8) | (uint32_t(q[2]) << 16) | (uint32_t(q[3]) << 24);
    }
    return r;
}
UPOW_HD void fe_to_le(const fe& a, uint8_t* b) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        uint8_t* q = b + 4 * i;
        q[0] = uint8_t(a.v[i]); q[1] = uint8_t(a.v[i] >> 8); q[2] = uint8_t(a.v[i] >> 16); q[3] = uint8_t(a.v[i] >> 24);
    }
}
UPOW_HD uint32_t fe_nibble(const fe& a, int w) { return (a.v[w >> 3] >> ((w & 7) * 4)) & 0xfu; }
UPOW_HD uint32_t fe_byte(const fe& a, int k) { return (a.v[k >> 2] >> ((k & 3) * 8)) & 0xffu; }

}  // namespace p256
}  // namespace upow
