// Host-side P-256 ECDSA verify on 64-bit limbs: the one-signature-at-a-time path (a /push_tx
// admission, a CPU-only node), where a GPU round trip would cost more than the verify itself.
//
// reference: fastecdsa ecdsa.verify called from upow/upow_transactions/transaction_input.py:100-120.
//
// Same status codes and the same acceptance rules as the GPU kernel (csrc/p256.hip verify_prologue /
// verify_epilogue); only the arithmetic differs. The GPU field code uses 32-bit limbs because that is
// the native width of the CDNA4 VALU; on the host the same code costs 4x the multiplies of a 64 x 64
// -> 128-bit schoolbook, so this file has its own:
//  * Montgomery multiplication (CIOS, R = 2^256) for both the field prime p and the group order n, with
//    the constants (R mod m, R^2 mod m, -m^-1 mod 2^64) derived at start-up, not typed in;
//  * u1*G from the fixed-base byte-window table of p256.hip (32 mixed additions), converted once into
//    the Montgomery domain;
//  * u2*Q with a 4-bit fixed window (252 doublings + <= 64 additions), a = -3 doubling formula;
//  * no inversion in the field: x(R) == r is checked as X == r*Z^2 (and (r+n)*Z^2 when r+n < p).
#include <cstdint>
#include <cstring>
#include <mutex>
#include <vector>

#include "native.h"

namespace upow {
namespace {

typedef unsigned __int128 u128;

struct Mod {
    uint64_t m[4];
    uint64_t n0;     // -m^-1 mod 2^64
    uint64_t rr[4];  // R^2 mod m
    uint64_t one[4]; // R mod m
};

inline bool geq(const uint64_t a[4], const uint64_t b[4]) {
    for (int i = 3; i >= 0; --i) {
        if (a[i] != b[i]) return a[i] > b[i];
    }
    return true;
}

inline uint64_t sub4(uint64_t r[4], const uint64_t a[4], const uint64_t b[4]) {
    uint64_t borrow = 0;
    for (int i = 0; i < 4; ++i) {
        const u128 d = u128(a[i]) - b[i] - borrow;
        r[i] = uint64_t(d);
        borrow = uint64_t(d >> 64) & 1;
    }
    return borrow;
}

inline uint64_t add4(uint64_t r[4], const uint64_t a[4], const uint64_t b[4]) {
    u128 c = 0;
    for (int i = 0; i < 4; ++i) {
        c += u128(a[i]) + b[i];
        r[i] = uint64_t(c);
        c >>= 64;
    }
    return uint64_t(c);
}

inline void mod_add(uint64_t r[4], const uint64_t a[4], const uint64_t b[4], const uint64_t m[4]) {
    uint64_t t[4], s[4];
    const uint64_t c = add4(t, a, b);
    const uint64_t borrow = sub4(s, t, m);
    if (c || !borrow) std::memcpy(r, s, 32);
    else std::memcpy(r, t, 32);
}

inline void mod_sub(uint64_t r[4], const uint64_t a[4], const uint64_t b[4], const uint64_t m[4]) {
    uint64_t t[4];
    if (sub4(t, a, b)) add4(t, t, m);
    std::memcpy(r, t, 32);
}

// r = a * b * R^-1 mod m (a, b < m)
inline void mont_mul(uint64_t r[4], const uint64_t a[4], const uint64_t b[4], const Mod& M) {
    uint64_t t[6] = {0, 0, 0, 0, 0, 0};
    for (int i = 0; i < 4; ++i) {
        u128 c = 0;
        for (int j = 0; j < 4; ++j) {
            c += u128(a[j]) * b[i] + t[j];
            t[j] = uint64_t(c);
            c >>= 64;
        }
        c += t[4];
        t[4] = uint64_t(c);
        t[5] = uint64_t(c >> 64);
        const uint64_t q = t[0] * M.n0;
        c = u128(q) * M.m[0] + t[0];
        c >>= 64;
        for (int j = 1; j < 4; ++j) {
            c += u128(q) * M.m[j] + t[j];
            t[j - 1] = uint64_t(c);
            c >>= 64;
        }
        c += t[4];
        t[3] = uint64_t(c);
        t[4] = t[5] + uint64_t(c >> 64);
    }
    uint64_t s[4];
    const uint64_t borrow = sub4(s, t, M.m);
    if (t[4] || !borrow) std::memcpy(r, s, 32);
    else std::memcpy(r, t, 32);
}

Mod make_mod(const uint64_t m[4]) {
    Mod M;
    std::memcpy(M.m, m, 32);
    uint64_t inv = 1;  // Newton: inv = m0^-1 mod 2^64
    for (int i = 0; i < 6; ++i) inv *= 2 - m[0] * inv;
    M.n0 = 0 - inv;
    uint64_t x[4] = {1, 0, 0, 0};
    for (int i = 0; i < 512; ++i) {  // x = 2^i mod m; R at i = 256, R^2 at i = 512
        mod_add(x, x, x, m);
        if (i == 255) std::memcpy(M.one, x, 32);
    }
    std::memcpy(M.rr, x, 32);
    return M;
}

const uint64_t kP[4] = {0xFFFFFFFFFFFFFFFFull, 0x00000000FFFFFFFFull, 0x0000000000000000ull, 0xFFFFFFFF00000001ull};
const uint64_t kN[4] = {0xF3B9CAC2FC632551ull, 0xBCE6FAADA7179E84ull, 0xFFFFFFFFFFFFFFFFull, 0xFFFFFFFF00000000ull};
const uint64_t kB[4] = {0x3BCE3C3E27D2604Bull, 0x651D06B0CC53B0F6ull, 0xB3EBBD55769886BCull, 0x5AC635D8AA3A93E7ull};

struct Fe { uint64_t v[4]; };
struct Jac { Fe x, y, z; bool inf; };
struct Aff { Fe x, y; };

struct Ctx {
    Mod p, n;
    Fe b_m, three_m;
    std::vector<Aff> g;  // [32][256] Montgomery-form copy of p256.hip's fixed-base table
};

inline void to_mont(Fe& r, const uint64_t a[4], const Mod& M) { mont_mul(r.v, a, M.rr, M); }

const Ctx& ctx() {
    static Ctx c;
    static std::once_flag once;
    std::call_once(once, [] {
        c.p = make_mod(kP);
        c.n = make_mod(kN);
        to_mont(c.b_m, kB, c.p);
        const uint64_t three[4] = {3, 0, 0, 0};
        to_mont(c.three_m, three, c.p);
        const uint32_t* tab = static_cast<const uint32_t*>(p256_g_table_host());  // 8192 x (x[8], y[8]) u32 LE
        c.g.resize(32 * 256);
        for (size_t i = 0; i < c.g.size(); ++i) {
            uint64_t x[4], y[4];
            std::memcpy(x, tab + i * 16, 32);
            std::memcpy(y, tab + i * 16 + 8, 32);
            to_mont(c.g[i].x, x, c.p);
            to_mont(c.g[i].y, y, c.p);
        }
    });
    return c;
}

// ---- field helpers (Montgomery domain mod p)
struct FOps {
    const Mod& P;
    explicit FOps(const Mod& p) : P(p) {}
    Fe mul(const Fe& a, const Fe& b) const { Fe r; mont_mul(r.v, a.v, b.v, P); return r; }
    Fe sqr(const Fe& a) const { return mul(a, a); }
    Fe add(const Fe& a, const Fe& b) const { Fe r; mod_add(r.v, a.v, b.v, P.m); return r; }
    Fe sub(const Fe& a, const Fe& b) const { Fe r; mod_sub(r.v, a.v, b.v, P.m); return r; }
    Fe dbl(const Fe& a) const { return add(a, a); }
    static bool eq(const Fe& a, const Fe& b) { return std::memcmp(a.v, b.v, 32) == 0; }
    static bool zero(const Fe& a) { return (a.v[0] | a.v[1] | a.v[2] | a.v[3]) == 0; }
};

// dbl-2001-b (a = -3)
Jac jdbl(const Jac& p, const FOps& F) {
    if (p.inf || FOps::zero(p.y)) return Jac{{}, {}, {}, true};
    const Fe delta = F.sqr(p.z);
    const Fe gamma = F.sqr(p.y);
    const Fe beta = F.mul(p.x, gamma);
    const Fe t = F.mul(F.sub(p.x, delta), F.add(p.x, delta));
    const Fe alpha = F.add(F.dbl(t), t);
    const Fe beta4 = F.dbl(F.dbl(beta));
    Jac r;
    r.inf = false;
    r.x = F.sub(F.sqr(alpha), F.dbl(beta4));
    r.z = F.sub(F.sub(F.sqr(F.add(p.y, p.z)), gamma), delta);
    const Fe g2 = F.sqr(gamma);
    const Fe g8 = F.dbl(F.dbl(F.dbl(g2)));
    r.y = F.sub(F.mul(alpha, F.sub(beta4, r.x)), g8);
    return r;
}

// add-2007-bl (general Jacobian)
Jac jadd(const Jac& p, const Jac& q, const FOps& F) {
    if (p.inf) return q;
    if (q.inf) return p;
    const Fe z1z1 = F.sqr(p.z), z2z2 = F.sqr(q.z);
    const Fe u1 = F.mul(p.x, z2z2), u2 = F.mul(q.x, z1z1);
    const Fe s1 = F.mul(F.mul(p.y, q.z), z2z2), s2 = F.mul(F.mul(q.y, p.z), z1z1);
    const Fe h = F.sub(u2, u1);
    const Fe rr = F.sub(s2, s1);
    if (FOps::zero(h)) {
        if (FOps::zero(rr)) return jdbl(p, F);
        return Jac{{}, {}, {}, true};
    }
    const Fe i = F.sqr(F.dbl(h));
    const Fe j = F.mul(h, i);
    const Fe r2 = F.dbl(rr);
    const Fe v = F.mul(u1, i);
    Jac o;
    o.inf = false;
    o.x = F.sub(F.sub(F.sqr(r2), j), F.dbl(v));
    o.y = F.sub(F.mul(r2, F.sub(v, o.x)), F.dbl(F.mul(s1, j)));
    o.z = F.mul(F.sub(F.sub(F.sqr(F.add(p.z, q.z)), z1z1), z2z2), h);
    return o;
}

// madd-2007-bl (q affine)
Jac jmadd(const Jac& p, const Aff& q, const Mod& Pm, const FOps& F) {
    if (p.inf) return Jac{q.x, q.y, Fe{{Pm.one[0], Pm.one[1], Pm.one[2], Pm.one[3]}}, false};
    const Fe z1z1 = F.sqr(p.z);
    const Fe u2 = F.mul(q.x, z1z1);
    const Fe s2 = F.mul(F.mul(q.y, p.z), z1z1);
    const Fe h = F.sub(u2, p.x);
    const Fe rr = F.sub(s2, p.y);
    if (FOps::zero(h)) {
        if (FOps::zero(rr)) return jdbl(p, F);
        return Jac{{}, {}, {}, true};
    }
    const Fe hh = F.sqr(h);
    const Fe i = F.dbl(F.dbl(hh));
    const Fe j = F.mul(h, i);
    const Fe r2 = F.dbl(rr);
    const Fe v = F.mul(p.x, i);
    Jac o;
    o.inf = false;
    o.x = F.sub(F.sub(F.sqr(r2), j), F.dbl(v));
    o.y = F.sub(F.mul(r2, F.sub(v, o.x)), F.dbl(F.mul(p.y, j)));
    o.z = F.sub(F.sub(F.sqr(F.add(p.z, h)), z1z1), hh);
    return o;
}

void load_le(uint64_t r[4], const uint8_t* b) { std::memcpy(r, b, 32); }

void load_be(uint64_t r[4], const uint8_t* b) {
    for (int i = 0; i < 4; ++i) {
        uint64_t w = 0;
        for (int k = 0; k < 8; ++k) w = (w << 8) | b[(3 - i) * 8 + k];
        r[i] = w;
    }
}

bool is_zero4(const uint64_t a[4]) { return (a[0] | a[1] | a[2] | a[3]) == 0; }

}  // namespace

uint8_t p256_verify_one_host64(const uint8_t* item) {
    const Ctx& C = ctx();
    const FOps F(C.p);
    const Mod& N = C.n;
    uint64_t qx[4], qy[4], r[4], s[4], e[4];
    load_le(qx, item);
    load_le(qy, item + 32);
    load_le(r, item + 64);
    load_le(s, item + 96);
    load_be(e, item + 128);
    // public key on the curve: y^2 == x^3 - 3x + b, coordinates in [0, p)
    if (geq(qx, kP) || geq(qy, kP)) return 2;
    Aff q;
    to_mont(q.x, qx, C.p);
    to_mont(q.y, qy, C.p);
    {
        const Fe x2 = F.sqr(q.x);
        const Fe rhs = F.add(F.sub(F.mul(x2, q.x), F.mul(C.three_m, q.x)), C.b_m);
        if (!FOps::eq(F.sqr(q.y), rhs)) return 2;
    }
    // fastecdsa: r, s must lie in [1, n]; s == n has no inverse
    const bool r_big = geq(r, kN) && std::memcmp(r, kN, 32) != 0;
    const bool s_big = geq(s, kN) && std::memcmp(s, kN, 32) != 0;
    if (is_zero4(r) || r_big) return 3;
    if (is_zero4(s) || s_big) return 3;
    if (std::memcmp(s, kN, 32) == 0) return 0;
    if (geq(e, kN)) sub4(e, e, kN);
    uint64_t r_red[4];
    std::memcpy(r_red, r, 32);
    if (geq(r_red, kN)) sub4(r_red, r_red, kN);
    uint64_t wm[4], u1[4], u2[4];
    p256_scalar_inv_mont_host(wm, s);  // s^-1 * R (divsteps, p256_field.h)
    mont_mul(u1, e, wm, N);     // e * s^-1
    mont_mul(u2, r_red, wm, N); // r * s^-1
    // u2 * Q: 4-bit fixed window
    Jac tbl[16];
    tbl[0] = Jac{{}, {}, {}, true};
    tbl[1] = jmadd(tbl[0], q, C.p, F);
    for (int k = 2; k < 16; ++k) tbl[k] = jmadd(tbl[k - 1], q, C.p, F);
    Jac acc{{}, {}, {}, true};
    for (int w = 63; w >= 0; --w) {
        if (!acc.inf) {
            acc = jdbl(acc, F);
            acc = jdbl(acc, F);
            acc = jdbl(acc, F);
            acc = jdbl(acc, F);
        }
        const uint32_t nib = uint32_t(u2[w / 16] >> ((w % 16) * 4)) & 15u;
        if (nib) acc = jadd(acc, tbl[nib], F);
    }
    // u1 * G: byte windows over the fixed-base table, mixed additions
    Jac g{{}, {}, {}, true};
    for (int j = 0; j < 32; ++j) {
        const uint32_t b = uint32_t(u1[j / 8] >> ((j % 8) * 8)) & 0xFFu;
        if (b) g = jmadd(g, C.g[size_t(j) * 256 + b], C.p, F);
    }
    const Jac R = jadd(g, acc, F);
    if (R.inf) return 0;
    const Fe z2 = F.sqr(R.z);
    Fe rm;
    to_mont(rm, r, C.p);
    if (FOps::eq(F.mul(rm, z2), R.x)) return 1;
    uint64_t rn[4];
    if (!add4(rn, r, kN) && !geq(rn, kP)) {
        to_mont(rm, rn, C.p);
        if (FOps::eq(F.mul(rm, z2), R.x)) return 1;
    }
    return 0;
}

}  // namespace upow
