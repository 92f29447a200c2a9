"""Pure-Python NIST P-256 oracle: point arithmetic, RFC 6979 signing, ECDSA verify, decompression.

This is the *correctness oracle* for the native C++ host library and the HIP batch kernels
(csrc/p256.h, csrc/p256_verify.hip). It reproduces the behaviour the reference obtains from
``fastecdsa`` (upow/upow_transactions/transaction_input.py:84-120, upow/helpers.py:58-62):

* ``verify`` raises :class:`EcdsaError` when the public key is off-curve or when r/s are outside
  ``[1, n]`` (fastecdsa checks ``r > q or r < 1``; ``r == n`` passes the check and then fails
  the comparison), otherwise returns the boolean result of ``x(u1*G + u2*Q) mod n == r``.
* the message digest is SHA-256 of the message bytes; a ``str`` message is UTF-8 encoded first
  (that is how the reference's "ASCII hex" fallback verify works).
* ``sign`` uses the RFC 6979 deterministic nonce with HMAC-SHA-256, no low-s normalisation.
"""
from __future__ import annotations

import hashlib
import hmac
import secrets
from typing import Optional, Tuple, Union

P = 0xffffffff00000001000000000000000000000000ffffffffffffffffffffffff
A = P - 3
B = 0x5ac635d8aa3a93e7b3ebbd55769886bc651d06b0cc53b0f63bce3c3e27d2604b
N = 0xffffffff00000000ffffffffffffffffbce6faada7179e84f3b9cac2fc632551
GX = 0x6b17d1f2e12c4247f8bce6e563a440f277037d812deb33a0f4a13945d898c296
GY = 0x4fe342e2fe1a7f9b8ee7eb4a7c0f9e162bce33576b315ececbb6406837bf51f5


class EcdsaError(Exception):
    pass


class Point:
    """Affine point on P-256 (``None`` coordinates == point at infinity)."""
    __slots__ = ('x', 'y')

    def __init__(self, x: int, y: int, check: bool = True):
        if check and not is_on_curve(x, y):
            raise ValueError(f'coordinates are not on curve P256\n\tx={x:x}\n\ty={y:x}')
        self.x = x
        self.y = y

    def __eq__(self, other):
        return isinstance(other, Point) and self.x == other.x and self.y == other.y

    def __hash__(self):
        return hash((self.x, self.y))

    def __repr__(self):
        return f'Point(x=0x{self.x:064x}, y=0x{self.y:064x})'


def is_on_curve(x: int, y: int) -> bool:
    if not (0 <= x < P and 0 <= y < P):
        return False
    return (y * y - (x * x * x + A * x + B)) % P == 0


def mod_sqrt(a: int) -> Tuple[int, int]:
    """Square root modulo P (P = 3 mod 4). Returns (root, P - root) like fastecdsa.util.mod_sqrt.

    When ``a`` is not a quadratic residue the returned value is not a root (the caller's
    on-curve check then fails, which is how the reference rejects such x).
    """
    r = pow(a % P, (P + 1) // 4, P)
    return r, (P - r) % P


def x_to_y(x: int, is_odd: bool = False) -> int:
    """reference: upow/helpers.py:58-62."""
    y2 = (x * x * x + A * x + B) % P
    y_res, y_mod = mod_sqrt(y2)
    return y_res if y_res % 2 == is_odd else y_mod


# ----------------------------------------------------------------------------------------------
# Jacobian arithmetic (a = -3)
# ----------------------------------------------------------------------------------------------
_INF = (0, 1, 0)


def _jdouble(X1, Y1, Z1):
    if Z1 == 0 or Y1 == 0:
        return _INF
    delta = Z1 * Z1 % P
    gamma = Y1 * Y1 % P
    beta = X1 * gamma % P
    alpha = 3 * (X1 - delta) * (X1 + delta) % P
    X3 = (alpha * alpha - 8 * beta) % P
    Z3 = ((Y1 + Z1) ** 2 - gamma - delta) % P
    Y3 = (alpha * (4 * beta - X3) - 8 * gamma * gamma) % P
    return X3, Y3, Z3


def _jadd(p1, p2):
    X1, Y1, Z1 = p1
    X2, Y2, Z2 = p2
    if Z1 == 0:
        return p2
    if Z2 == 0:
        return p1
    Z1Z1 = Z1 * Z1 % P
    Z2Z2 = Z2 * Z2 % P
    U1 = X1 * Z2Z2 % P
    U2 = X2 * Z1Z1 % P
    S1 = Y1 * Z2 * Z2Z2 % P
    S2 = Y2 * Z1 * Z1Z1 % P
    if U1 == U2:
        if S1 != S2:
            return _INF
        return _jdouble(X1, Y1, Z1)
    H = (U2 - U1) % P
    I = (2 * H) ** 2 % P
    J = H * I % P
    r = 2 * (S2 - S1) % P
    V = U1 * I % P
    X3 = (r * r - J - 2 * V) % P
    Y3 = (r * (V - X3) - 2 * S1 * J) % P
    Z3 = ((Z1 + Z2) ** 2 - Z1Z1 - Z2Z2) * H % P
    return X3, Y3, Z3


def _to_affine(pt) -> Optional[Tuple[int, int]]:
    X, Y, Z = pt
    if Z == 0:
        return None
    zi = pow(Z, P - 2, P)
    zi2 = zi * zi % P
    return X * zi2 % P, Y * zi2 * zi % P


def _jmul(k: int, pt) -> tuple:
    acc = _INF
    for bit in bin(k)[2:] if k > 0 else '':
        acc = _jdouble(*acc)
        if bit == '1':
            acc = _jadd(acc, pt)
    return acc


def scalar_mult(k: int, x: int, y: int) -> Optional[Tuple[int, int]]:
    return _to_affine(_jmul(k % N, (x, y, 1)))


def shamir(u1: int, u2: int, qx: int, qy: int) -> Optional[Tuple[int, int]]:
    """u1*G + u2*Q (Straus/Shamir's trick)."""
    g = (GX, GY, 1)
    q = (qx, qy, 1)
    gq = _jadd(g, q)
    acc = _INF
    nb = max(u1.bit_length(), u2.bit_length())
    for i in range(nb - 1, -1, -1):
        acc = _jdouble(*acc)
        b1 = (u1 >> i) & 1
        b2 = (u2 >> i) & 1
        if b1 and b2:
            acc = _jadd(acc, gq)
        elif b1:
            acc = _jadd(acc, g)
        elif b2:
            acc = _jadd(acc, q)
    return _to_affine(acc)


def get_public_key(d: int) -> Point:
    x, y = scalar_mult(d, GX, GY)
    return Point(x, y, check=False)


def gen_private_key() -> int:
    while True:
        d = secrets.randbits(256)
        if 1 <= d < N:
            return d


def _msg_bytes(msg: Union[str, bytes, bytearray]) -> bytes:
    if isinstance(msg, str):
        return msg.encode()
    return bytes(msg)


def hash_to_int(msg: Union[str, bytes]) -> int:
    return int.from_bytes(hashlib.sha256(_msg_bytes(msg)).digest(), 'big')


def _bits2int(b: bytes) -> int:
    v = int.from_bytes(b, 'big')
    blen = len(b) * 8
    if blen > 256:
        v >>= blen - 256
    return v


def rfc6979_nonce(d: int, h1: bytes) -> int:
    """RFC 6979 §3.2 with HMAC-SHA-256, qlen = hlen = 256."""
    x = d.to_bytes(32, 'big')
    h1i = _bits2int(h1) % N
    h1o = h1i.to_bytes(32, 'big')
    V = b'\x01' * 32
    K = b'\x00' * 32
    K = hmac.new(K, V + b'\x00' + x + h1o, hashlib.sha256).digest()
    V = hmac.new(K, V, hashlib.sha256).digest()
    K = hmac.new(K, V + b'\x01' + x + h1o, hashlib.sha256).digest()
    V = hmac.new(K, V, hashlib.sha256).digest()
    while True:
        V = hmac.new(K, V, hashlib.sha256).digest()
        k = _bits2int(V)
        if 1 <= k < N:
            return k
        K = hmac.new(K, V + b'\x00', hashlib.sha256).digest()
        V = hmac.new(K, V, hashlib.sha256).digest()


def sign(msg: Union[str, bytes], d: int) -> Tuple[int, int]:
    """Deterministic ECDSA-P256/SHA-256 signature (r, s) (fastecdsa.ecdsa.sign contract)."""
    h = hashlib.sha256(_msg_bytes(msg)).digest()
    e = int.from_bytes(h, 'big')
    k = rfc6979_nonce(d, h)
    while True:
        x, _ = scalar_mult(k, GX, GY)
        r = x % N
        s = pow(k, -1, N) * (e + r * d) % N
        if r != 0 and s != 0:
            return r, s
        k = (k + 1) % N  # unreachable in practice


def verify_digest(r: int, s: int, e: int, qx: int, qy: int) -> bool:
    """Core verify on an already-hashed message. Raises EcdsaError on invalid key or r/s range."""
    if not is_on_curve(qx, qy):
        raise EcdsaError('Invalid public key, point is not on curve P256')
    if r > N or r < 1:
        raise EcdsaError('Invalid Signature: r is not a positive integer smaller than the curve order')
    if s > N or s < 1:
        raise EcdsaError('Invalid Signature: s is not a positive integer smaller than the curve order')
    if s == N:
        return False
    w = pow(s, -1, N)
    u1 = e * w % N
    u2 = r * w % N
    pt = shamir(u1, u2, qx, qy)
    if pt is None:
        return False
    return pt[0] % N == r


def verify(sig: Tuple[int, int], msg: Union[str, bytes], q: Point) -> bool:
    r, s = sig
    return verify_digest(r, s, hash_to_int(msg), q.x, q.y)


G = Point(GX, GY)
