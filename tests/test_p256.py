"""P-256: Python oracle, host C++ core and gfx950 batch kernels against each other."""
import hashlib
import random

import numpy as np
import pytest

from upow_amd.ops import p256 as op
from upow_amd.utils import p256 as o

RFC6979_D = 0xC9AFA9D845BA75166B5C215767B1D6934E50C3DB36E89B127B8A622B120F6721


def test_rfc6979_sample_vector():
    # RFC 6979 A.2.5, P-256 + SHA-256, message "sample"
    r, s = o.sign(b'sample', RFC6979_D)
    assert r == 0xEFD48B2AACB6A8FD1140DD9CD45E81D69D2C877B56AAF991C34D0EA84EAF3716
    assert s == 0xF7CB1C942D657C41D436C7A1B6E29F65F3E900DBB9AFF4064DC4AB2F843ACDA8
    q = o.get_public_key(RFC6979_D)
    assert q.x == 0x60FED4BA255A9D31C961EB74C6356D68C049B8923B61FA6CE669622E60F29FB6
    assert q.y == 0x7903FE1008B8BC99A41AE9E95628BC64F2F1B20C2D7E9F5177A3C294D4462299


def test_native_sign_pubkey_match_oracle(native):
    rng = random.Random(2)
    for _ in range(20):
        d = rng.randrange(1, o.N)
        msg = rng.randbytes(rng.randrange(0, 300))
        assert op.public_key(d) == o.get_public_key(d)
        assert op.sign(msg, d) == o.sign(msg, d)
    assert op.sign(b'sample', RFC6979_D) == o.sign(b'sample', RFC6979_D)


def test_scalar_inverse_divsteps_matches_pow(native):
    """s^-1 * 2^256 mod n by the verifier's divsteps inverse (p256_field.h sc_inv_safegcd_mont) against
    Python's pow, on random scalars and on the shapes that stress a gcd: small values, powers of two, n - k,
    values just below 2^256 reduced, and runs of ones."""
    from upow_amd.ops.native import lib
    inv = lib().p256_scalar_inv_mont
    n = o.N
    R = (1 << 256) % n
    rng = random.Random(11)
    cases = [1, 2, 3, n - 1, n - 2, (n - 1) // 2, (1 << 255) % n, (1 << 256) - 1 - n, (1 << 128) - 1]
    cases += [1 << k for k in range(256)] + [n - (1 << k) for k in range(255)]
    cases += [((1 << k) - 1) % n for k in range(1, 257)] + [rng.randrange(1, n) for _ in range(3000)]
    for s in cases:
        s %= n
        if s == 0:
            continue
        got = int.from_bytes(inv(s.to_bytes(32, 'little')), 'little')
        assert got == pow(s, -1, n) * R % n, hex(s)


def test_field_arithmetic_matches_python(native):
    """The kernels' field code (p256_field.h, run on the host): products, squares, sums and differences
    mod p against Python integers, and the Solinas reduction of arbitrary 512-bit values — including the
    words patterns that drive its signed overflow to both ends of [-4, 6] (the h = -1 and h = 1 folds)."""
    from upow_amd.ops.native import lib
    L = lib()
    p = o.P
    rng = random.Random(13)
    edge = [0, 1, 2, p - 1, p - 2, (p - 1) // 2, 1 << 255, (1 << 224) - 1, (1 << 96) + 5, p - (1 << 96),
            (1 << 256) - 1 - (1 << 224) - p // 3]
    vals = [v % p for v in edge] + [rng.randrange(p) for _ in range(1500)]
    vals += [sum(rng.choice((0, 0xffffffff, 1)) << (32 * k) for k in range(8)) % p for _ in range(500)]
    for k in range(len(vals)):
        a, b = vals[k], vals[rng.randrange(len(vals))]
        out = L.p256_fe_ops(a.to_bytes(32, 'little'), b.to_bytes(32, 'little'))
        got = [int.from_bytes(out[32 * i:32 * i + 32], 'little') for i in range(4)]
        assert got == [a * b % p, a * a % p, (a + b) % p, (a - b) % p], (hex(a), hex(b))
    words = (0, 1, 0xffffffff, 0x80000000, 0xfffffffe)
    for _ in range(4000):
        c = sum(rng.choice(words) << (32 * k) for k in range(16)) if rng.random() < 0.7 else rng.getrandbits(512)
        assert int.from_bytes(L.p256_fe_reduce(c.to_bytes(64, 'little')), 'little') == c % p, hex(c)


def test_verify_semantics(native):
    d = 12345
    q = o.get_public_key(d)
    msg = b'\x01\x02hello'
    sig = o.sign(msg, d)
    assert op.verify(sig, msg, q) and o.verify(sig, msg, q)
    assert not op.verify((sig[0], sig[1] ^ 1), msg, q)
    # the reference's second try hashes the ASCII-hex string (str is utf-8 encoded)
    sig2 = o.sign(msg.hex(), d)
    assert op.verify(sig2, msg.hex(), q) and not op.verify(sig2, msg, q)
    # fastecdsa contract: out-of-range r/s and off-curve keys raise
    for bad in [(0, sig[1]), (sig[0], 0), (o.N + 1, sig[1]), (sig[0], o.N + 1)]:
        with pytest.raises(o.EcdsaError):
            op.verify(bad, msg, q)
        with pytest.raises(o.EcdsaError):
            o.verify(bad, msg, q)
    # r == n and s == n pass the range check and fail verification
    assert op.verify((o.N, sig[1]), msg, q) is False
    assert op.verify((sig[0], o.N), msg, q) is False
    off = o.Point(q.x, (q.y + 1) % o.P, check=False)
    with pytest.raises(o.EcdsaError):
        op.verify(sig, msg, off)


def _batch(n, seed):
    rng = random.Random(seed)
    recs, exp = [], []
    keys = [rng.randrange(1, o.N) for _ in range(8)]
    pubs = [o.get_public_key(k) for k in keys]
    for i in range(n):
        k = i % 8
        msg = rng.randbytes(40)
        r, s = op.sign(msg, keys[k])
        q = pubs[k]
        kind = i % 7
        if kind == 1:
            s = (s * 3) % o.N or 1
        elif kind == 2:
            msg += b'!'
        elif kind == 3:
            q = pubs[(k + 1) % 8]
        elif kind == 4:
            r = o.N  # passes range check, never verifies
        elif kind == 5:
            r = 0    # range error
        e = hashlib.sha256(msg).digest()
        recs.append(op.record(q, (r, s), e))
        if kind == 5:
            exp.append(3)
        else:
            try:
                exp.append(1 if o.verify_digest(r, s, int.from_bytes(e, 'big'), q.x, q.y) else 0)
            except o.EcdsaError:
                exp.append(3)
    return b''.join(recs), np.array(exp, dtype=np.uint8)


def test_host_batch_matches_oracle(native):
    recs, exp = _batch(70, 3)
    st = op.verify_records(recs, device='cpu', threads=4)
    assert (st == exp).all()
    assert exp.tolist().count(1) > 10


def test_decompress_host(native):
    rng = random.Random(4)
    addrs, want = [], []
    for _ in range(30):
        q = o.get_public_key(rng.randrange(1, o.N))
        addrs.append(bytes([42 if q.y % 2 == 0 else 43]) + q.x.to_bytes(32, 'little'))
        want.append((q.x, q.y))
    addrs.append(bytes([42]) + (5).to_bytes(32, 'little'))  # x=5: check against the oracle
    try:
        want.append((5, o.x_to_y(5, False)) if o.is_on_curve(5, o.x_to_y(5, False)) else None)
    except Exception:
        want.append(None)
    assert op.decompress(addrs, device='cpu') == want


def _chosen_s_batch():
    """Valid signatures for chosen s (edge values of the binary-Euclid s^-1): pick k, R = kG, e, s and
    solve for the key d = (s k - e) / r, so each record verifies; every one is followed by a copy with
    s + 1 (or s - 1 at the top), which must not."""
    rng = random.Random(41)
    svals = [1, 2, 3, 5, o.N - 1, o.N - 2, (o.N + 1) // 2, 1 << 255, (1 << 128) + 1, 0xffffffff]
    svals += [rng.randrange(1, o.N) for _ in range(6)]
    recs, exp = [], []
    for s in svals:
        k = rng.randrange(1, o.N)
        r = o.get_public_key(k).x % o.N
        e = rng.randbytes(32)
        d = (s * k - int.from_bytes(e, 'big')) * pow(r, -1, o.N) % o.N
        q = o.get_public_key(d)
        assert o.verify_digest(r, s, int.from_bytes(e, 'big'), q.x, q.y)
        s2 = s + 1 if s + 1 < o.N else s - 1
        recs += [op.record(q, (r, s), e), op.record(q, (r, s2), e)]
        exp += [1, 0]
    return b''.join(recs), np.array(exp, dtype=np.uint8)


@pytest.mark.parametrize('mode', ['1', 'quad', 'oct'])  # one-lane 32-bit code; four-lane steps; pair-split products
def test_host_gpu_code_paths(native, mode, monkeypatch):
    """The GPU kernels' field/point code run on the host: the one-lane 32-bit path and the quad
    kernel's four-product step schedule in XYZZ coordinates (QuadHost), both with the binary-Euclid
    s^-1."""
    monkeypatch.setenv('UPOW_P256_HOST32', mode)
    for recs, exp in (_batch(140, 5), _high_x_batch(4, 33), _chosen_s_batch()):
        assert (op.verify_records(recs, device='cpu', threads=4) == exp).all()


@pytest.mark.gpu
@pytest.mark.parametrize('variant', ['0', '1', '2', '4', '8', 'a'])  # 3 / 4 waves/SIMD, SoA tables, quad, oct, auto
def test_gpu_batch_verify_matches_host(gpu, variant, monkeypatch):
    monkeypatch.setenv('UPOW_P256_VARIANT', variant)
    recs, exp = _batch(700, 5)
    st_gpu = op.verify_records(recs, device='gpu')
    assert (st_gpu == exp).all()
    recs, exp = _chosen_s_batch()
    assert (op.verify_records(recs, device='gpu') == exp).all()


@pytest.mark.gpu
def test_gpu_decompress(gpu):
    rng = random.Random(6)
    addrs = []
    for _ in range(600):
        q = o.get_public_key(rng.randrange(1, o.N))
        addrs.append(bytes([42 if q.y % 2 == 0 else 43]) + q.x.to_bytes(32, 'little'))
    addrs.append(bytes([43]) + (o.P - 1).to_bytes(32, 'little'))
    assert op.decompress(addrs, device='gpu') == op.decompress(addrs, device='cpu')


def _high_x_batch(count: int, seed: int):
    """Signatures whose R = u1*G + u2*Q has x(R) in [n, p), so r = x(R) - n: the kernels' inversion-free
    x-check must also compare (r + n)*Z^2 against X. Such R are ~2^-130 rare for honest signers, so the
    key is solved for instead: pick R, e, s; Q = u2^-1 * (R - u1*G). Each valid record is followed by
    the same signature with r = x(R) (>= n: a range error) and with r + 1 (a plain mismatch)."""
    rng = random.Random(seed)
    recs, exp = [], []
    x = o.N
    while len(exp) < 3 * count:
        x += rng.randrange(1, 1 << 20)
        try:
            y = o.x_to_y(x, rng.random() < 0.5)
        except Exception:
            continue
        if not o.is_on_curve(x, y):
            continue
        r = x - o.N
        s = rng.randrange(1, o.N)
        e = rng.randbytes(32)
        w = pow(s, -1, o.N)
        u1 = int.from_bytes(e, 'big') * w % o.N
        u2 = r * w % o.N
        t = o._to_affine(o._jadd((x, y, 1), o._jmul(o.N - u1, (o.GX, o.GY, 1))))
        q = o.Point(*o.scalar_mult(pow(u2, -1, o.N), *t))
        assert o.verify_digest(r, s, int.from_bytes(e, 'big'), q.x, q.y)
        recs += [op.record(q, (r, s), e), op.record(q, (x, s), e), op.record(q, (r + 1, s), e)]
        exp += [1, 3, 0]
    return b''.join(recs), np.array(exp, dtype=np.uint8)


def test_high_x_r_plus_n_host(native):
    recs, exp = _high_x_batch(8, 31)
    assert (op.verify_records(recs, device='cpu', threads=2) == exp).all()


@pytest.mark.gpu
@pytest.mark.parametrize('variant', ['0', '1', '2', '4', '8'])
def test_high_x_r_plus_n_gpu(gpu, variant, monkeypatch):
    monkeypatch.setenv('UPOW_P256_VARIANT', variant)
    recs, exp = _high_x_batch(40, 32)
    assert (op.verify_records(recs, device='gpu') == exp).all()


@pytest.mark.gpu
def test_node_device_pin_from_worker_thread(gpu):
    """set_node_device pins node-side GPU calls made from other threads (a cluster rank's ledger worker
    and executor threads start on device 0) to the rank's device."""
    import threading
    from upow_amd.ops.native import lib
    lib().set_node_device(0)
    try:
        recs, exp = _batch(100, 9)
        out = {}
        t = threading.Thread(target=lambda: out.update(st=op.verify_records(recs, device='gpu')))
        t.start()
        t.join()
        assert (out['st'] == exp).all()
    finally:
        lib().set_node_device(-1)


def test_on_curve_batch_matches_oracle(native):
    """Native batch on-curve check of 64-byte addresses (csrc/p256.hip p256_on_curve, host pool) against the
    pure-int oracle: valid points, y flipped to the other root, x or y >= p, off-curve noise."""
    import random
    from upow_amd.utils import p256 as o
    rng = random.Random(17)
    rows, want = [], []
    for k in range(300):
        pt = o.get_public_key(rng.randrange(1, o.N))
        x, y = pt.x, pt.y
        kind = k % 5
        if kind == 1:
            y = o.P - y
        elif kind == 2:
            y = (y + 1) % o.P
        elif kind == 3:
            x = x + o.P if x + o.P < 1 << 256 else x
        elif kind == 4:
            x, y = rng.randrange(1 << 256), rng.randrange(1 << 256)
        rows.append(x.to_bytes(32, 'little') + y.to_bytes(32, 'little'))
        want.append(1 if (x < o.P and y < o.P and o.is_on_curve(x, y)) else 0)
    got = native.p256_on_curve(b''.join(rows), False, 4)
    assert list(got) == want and sum(want) > 100


@pytest.mark.gpu
def test_on_curve_batch_gpu_matches_host(gpu):
    import random
    from upow_amd.utils import p256 as o
    rng = random.Random(23)
    pubs = gpu.p256_pubkey_batch(b''.join(rng.randrange(1, o.N).to_bytes(32, 'big') for _ in range(5000)), 8)
    rows = []
    for k in range(5000):
        x, y = int.from_bytes(pubs[64 * k:64 * k + 32], 'little'), int.from_bytes(pubs[64 * k + 32:64 * k + 64], 'little')
        if k % 3 == 0:
            x, y = rng.randrange(1 << 256), rng.randrange(1 << 256)
        elif k % 2 == 0:
            y = o.P - y
        rows.append(x.to_bytes(32, 'little') + y.to_bytes(32, 'little'))
    buf = b''.join(rows)
    assert gpu.p256_on_curve(buf, True) == gpu.p256_on_curve(buf, False, 8)


@pytest.mark.gpu
def test_g16_window_table_matches_python(gpu):
    """The GPU kernels' fixed-base table T16[j][b] = b * 2^(16 j) * G (built on the device from the byte
    windows): sampled entries of every window, both byte halves zero / non-zero, against Python."""
    from upow_amd.ops.native import lib
    L = lib()
    rng = random.Random(17)
    for j in range(16):
        for b in [0, 1, 2, 255, 256, 257, 0xff00, 0xffff] + [rng.randrange(1, 1 << 16) for _ in range(6)]:
            raw = L.p256_g16_entries(j * 65536 + b, 1)
            x, y = int.from_bytes(raw[:32], 'little'), int.from_bytes(raw[32:], 'little')
            if b == 0:
                assert x == y == 0
                continue
            q = o.get_public_key((b << (16 * j)) % o.N)
            assert (x, y) == (q.x, q.y), (j, b)


def _addr33(q) -> bytes:
    return bytes([42 if q.y % 2 == 0 else 43]) + q.x.to_bytes(32, 'little')


def _off_curve_x(rng) -> int:
    """An x with no curve point (x^3 - 3x + b a non-residue mod p)."""
    while True:
        x = rng.randrange(1, o.P)
        rhs = (x ** 3 - 3 * x + o.B) % o.P
        if pow(rhs, (o.P - 1) // 2, o.P) != 1:
            return x


def _fused_block(seed, bad_out=False, bad_signer=False):
    """Block-path columns (csrc/txcodec.cpp block_signer_records / block_verify_fused) for 48 jobs over 60
    inputs and 70 outputs, with bad signatures, a wrong key, r = n and r = 0 among them."""
    rng = random.Random(seed)
    keys = [rng.randrange(1, o.N) for _ in range(6)]
    pubs = [o.get_public_key(k) for k in keys]
    n_jobs, n_in, n_out = 48, 60, 70
    pay = np.zeros((n_in, 64), np.uint8)
    owner = [j % 6 for j in range(n_in)]
    for i in range(n_in):
        pay[i, :33] = np.frombuffer(_addr33(pubs[owner[i]]), np.uint8)
    if bad_signer:
        pay[5, :33] = np.frombuffer(bytes([42]) + _off_curve_x(rng).to_bytes(32, 'little'), np.uint8)
    out = np.zeros((n_out, 64), np.uint8)
    for i in range(n_out):
        out[i, :33] = np.frombuffer(_addr33(o.get_public_key(rng.randrange(1, o.N))), np.uint8)
    if bad_out:
        out[7, :33] = np.frombuffer(bytes([43]) + _off_curve_x(rng).to_bytes(32, 'little'), np.uint8)
    job_input = np.array(rng.sample(range(n_in), n_jobs), np.int64)
    digest = np.frombuffer(b''.join(rng.randbytes(32) for _ in range(n_jobs)), np.uint8).reshape(-1, 32)
    job_tx = np.arange(n_jobs, dtype=np.int64)[::-1].copy()
    sigs = np.zeros((n_jobs, 64), np.uint8)
    for j in range(n_jobs):
        k = owner[int(job_input[j])]
        msg_e = digest[job_tx[j]].tobytes()
        z = int.from_bytes(msg_e, 'big')
        kk = rng.randrange(1, o.N)
        r = o.get_public_key(kk).x % o.N
        s = pow(kk, -1, o.N) * (z + r * keys[k]) % o.N
        kind = j % 6
        if kind == 1:
            s = (s * 3) % o.N or 1
        elif kind == 2:
            r = o.N
        elif kind == 3:
            r = 0
        sigs[j] = np.frombuffer(r.to_bytes(32, 'little') + s.to_bytes(32, 'little'), np.uint8)
    return (pay, np.full(n_in, 33, np.uint8), out, np.full(n_out, 33, np.uint8), job_input, sigs,
            np.arange(n_jobs, dtype=np.int64), digest, job_tx)


def _fused_reference(native, cols):
    pay, pay_len, out, out_len, job_input, sigs, sig_ids, digest, job_tx = cols
    kst, recs = native.block_signer_records(pay, pay_len, out, out_len, job_input, sigs, sig_ids, digest, job_tx,
                                            1 << 62)
    return kst, recs


@pytest.mark.parametrize('case', ['plain', 'bad_out', 'bad_signer'])
def test_fused_block_verify_host_matches_separate_stages(native, case):
    """block_verify_fused (keys decompressed into the verify items, every address curve-checked, signatures
    verified) gives the verdicts of block_signer_records + p256_verify; its items, returned when a signature
    fails, are the separate path's records."""
    cols = _fused_block(7, bad_out=case == 'bad_out', bad_signer=case == 'bad_signer')
    code, st, ok, items = native.block_verify_fused(*cols, threads=3, gpu=False)
    kst, recs = _fused_reference(native, cols)
    assert code == 1
    if case == 'plain':
        assert kst == 1 and ok
        exp = op.verify_records(recs, device='cpu', threads=2)
        assert np.frombuffer(st, np.uint8).tolist() == exp.tolist()
        assert set(exp.tolist()) == {0, 1, 3} and items == recs
    elif case == 'bad_out':
        assert kst == 0 and not ok
    else:  # every spent output's owner is curve-checked too; the signer's own job also says bad key
        assert kst == 0 and not ok
        assert all(st[j] == 2 for j in range(len(cols[4])) if cols[4][j] == 5)
    # a 64-byte address hands the block to the general path, as block_signer_records does
    pay_len = cols[1].copy()
    pay_len[0] = 64
    assert native.block_verify_fused(cols[0], pay_len, *cols[2:], gpu=False)[0] == -1


@pytest.mark.gpu
@pytest.mark.parametrize('case', ['plain', 'bad_out', 'bad_signer'])
def test_fused_block_verify_gpu_matches_host(gpu, case):
    from upow_amd.ops.native import lib
    cols = _fused_block(9, bad_out=case == 'bad_out', bad_signer=case == 'bad_signer')
    assert lib().block_verify_fused(*cols, threads=3, gpu=True) == lib().block_verify_fused(*cols, threads=3, gpu=False)
