// The P-256 verify pieces shared by the block-latency kernels (csrc/p256.hip: four and eight lanes per
// signature, compiled with the ILP-first scheduler) and the one-lane batch kernel (csrc/p256_batch.hip,
// compiled with the default occupancy-first scheduler so it keeps four waves per SIMD without spilling):
// the 160-byte work item, the scalar prologue (range checks, s^-1, u1, u2), the x-coordinate epilogue, the
// signed 5-bit windows of u2 and the 16-bit fixed-base windows of u1*G.
//
// reference: fastecdsa ecdsa.verify as called from upow/upow_transactions/transaction_input.py:84-120.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "p256_field.h"

namespace upow {
using namespace p256;

struct VerifyItem {  // 160 bytes, wire byte order
    uint8_t qx[32];  // little-endian
    uint8_t qy[32];  // little-endian
    uint8_t r[32];   // little-endian
    uint8_t s[32];   // little-endian
    uint8_t e[32];   // SHA-256 digest, big-endian
};
static_assert(sizeof(VerifyItem) == 160, "VerifyItem layout");

// 1 builds the previous inverse (binary Euclid) for the A/B (_build.py variant 'p256bgcd')
#ifndef UPOW_P256_INV_BGCD
#define UPOW_P256_INV_BGCD 0
#endif

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
    const fe w_m = UPOW_P256_INV_BGCD ? sc_inv_bgcd_mont(s) : sc_inv_safegcd_mont(s);  // s^-1 * R
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

// Signed 5-bit windows of a scalar k < 2^256 (Booth recoding): 52 digits in [-16, 16], top first, with
// k = sum d_i 32^i. Digit i comes from bits [5i+4 .. 5i-1] of k (bit -1 = 0): d = b0 + b1 + 2 b2 + 4 b3
// + 8 b4 - 16 b5 of those six bits. They are read from the top of a 288-bit shift register s = k << 28
// and shifted out five at a time (no dynamic register indexing on the GPU).
struct BoothW5 {
    uint32_t s9[9];
    UPOW_HD explicit BoothW5(const fe& k) {
        s9[0] = k.v[0] << 28;
#pragma unroll
        for (int l = 1; l < 8; ++l) s9[l] = (k.v[l] << 28) | (k.v[l - 1] >> 4);
        s9[8] = k.v[7] >> 4;
    }
    UPOW_HD int next() {
        const uint32_t v = s9[8] >> 26;
#pragma unroll
        for (int l = 8; l > 0; --l) s9[l] = (s9[l] << 5) | (s9[l - 1] >> 27);
        s9[0] <<= 5;
        return int((v >> 1) & 15u) + int(v & 1u) - 16 * int(v >> 5);
    }
};
static constexpr int kBoothWindows = 52;

// The GPU kernels' u1*G: 16 windows of 16 bits over T16[j][b] = b * 2^(16 j) * G (16 x 65,536 affine
// points, 64 MiB in HBM, built on the device from the byte-window table: build_g16_kernel). Half the mixed
// additions of the byte windows (a lane's quarter is 4 windows: 3 additions instead of 7); the table
// reads are 4 random 64-byte lines per lane, served from the 256 MB Infinity Cache once warm.
static constexpr int kG16Win = 16;
static constexpr int kG16Ent = 65536;  // entry 0 unused (zero)
UPOW_HD jac mul_g16(const fe& k, const aff* tab16) {
    jac acc = jac_inf();
    for (int j = 0; j < kG16Win; ++j) {
        const uint32_t b = (k.v[j >> 1] >> (16 * (j & 1))) & 0xffffu;
        if (b) acc = jac_madd(acc, tab16[size_t(j) * kG16Ent + b]);
    }
    return acc;
}
}  // namespace upow
