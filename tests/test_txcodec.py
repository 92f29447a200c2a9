"""Native block codec (csrc/txcodec.cpp) against the Python Transaction model, byte for byte."""
import hashlib
import json
import random
from decimal import Decimal

import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings, strategies as st

from upow_amd.ledger.database import arena_list

from upow_amd.models.block import get_transactions_merkle_tree
from upow_amd.models.transaction import Transaction, TransactionInput, TransactionOutput
from upow_amd.utils.codec import OutputType, point_to_string
from upow_amd.utils.p256 import GX, GY, Point


@pytest.fixture(scope='module')
def L(native):
    return native


def _addr(rng, compressed=True):
    from upow_amd.ops import p256 as op
    pt = op.public_key(rng.randrange(1, 1 << 200))
    return point_to_string(pt) if compressed else (pt.x.to_bytes(32, 'little') + pt.y.to_bytes(32, 'little')).hex()


def _tx(rng, version=None, n_in=None, n_out=None, msg=None, one_sig=None):
    n_in = n_in or rng.randint(1, 4)
    n_out = n_out or rng.randint(1, 3)
    v1 = version == 1
    ins = [TransactionInput(rng.randbytes(32).hex(), rng.randrange(256)) for _ in range(n_in)]
    outs = [TransactionOutput(_addr(rng, not v1), Decimal(rng.randrange(1, 10 ** 12)) / 10 ** 8) for _ in range(n_out)]
    tx = Transaction(ins, outs, msg, version)
    one = one_sig if one_sig is not None else rng.random() < 0.5
    if one:
        s = (rng.randrange(1, 1 << 256), rng.randrange(1, 1 << 256))
        for i in ins:
            i.signed = s
    else:
        for i in ins:
            i.signed = (rng.randrange(1, 1 << 256), rng.randrange(1, 1 << 256))
    return tx


def _check_fast(d, hexes):
    assert d['all_fast'], list(d['flags'])
    i32 = lambda k: np.frombuffer(d[k], dtype=np.int32)
    in_start, out_start = i32('in_start'), i32('out_start')
    in_keys = np.frombuffer(d['in_keys'], dtype=np.uint8).reshape(-1, 40)
    out_amount = np.frombuffer(d['out_amount'], dtype=np.uint64)
    out_addr_json, out_amount_json = arena_list(d['out_addr_json']), arena_list(d['out_amount_json'])
    out_addr_str = arena_list(d['out_addr_str'])
    grouped = np.frombuffer(d['grouped'], dtype=np.uint8)
    parsed = []
    for k, h in enumerate(hexes):
        tx, pending = Transaction.parse(h)
        parsed.append(tx)
        assert bool(grouped[k]) == (pending is not None)
        if pending is not None:
            # 1 < k < n signatures: the owner groups come from the UTXO set (transaction.py:578-590, resolved
            # later by fastpath._resolve_groups). Any grouping whose groups first appear in signature order
            # serialises to the same bytes: one input per signature, the remaining inputs on the last one
            for j, i in enumerate(tx.inputs):
                i.signed = pending[min(j, len(pending) - 1)]
        assert d['hex'][k] == tx.hex()
        assert d['txid'][32 * k:32 * k + 32].hex() == tx.hash()
        assert d['digest'][32 * k:32 * k + 32] == hashlib.sha256(bytes.fromhex(tx.hex(False))).digest()
        assert i32('signed_len')[k] * 2 == len(tx.hex(False))
        assert out_addr_json[k] == json.dumps([o.address for o in tx.outputs], separators=(',', ':'))
        assert out_amount_json[k] == json.dumps([int(o.amount * 10 ** 8) for o in tx.outputs], separators=(',', ':'))
        assert out_addr_str[out_start[k]:out_start[k + 1]] == [o.address for o in tx.outputs]
        assert [int(a) for a in out_amount[out_start[k]:out_start[k + 1]]] == [int(o.amount * 10 ** 8) for o in tx.outputs]
        for j, i in enumerate(tx.inputs):
            rec = in_keys[in_start[k] + j]
            assert bytes(rec[:32]).hex() == i.tx_hash and int(rec[32]) == i.index
            if pending is not None:
                assert i32('in_sig')[in_start[k] + j] == -1  # assigned once the owners are known
                continue
            sig = d['sigs'][64 * i32('in_sig')[in_start[k] + j]:][:64]
            assert (int.from_bytes(sig[:32], 'little'), int.from_bytes(sig[32:], 'little')) == i.signed
    assert d['merkle_job'].result() == get_transactions_merkle_tree(parsed)


def test_decode_matches_python_model(L):
    rng = random.Random(5)
    txs = [_tx(rng) for _ in range(60)]
    txs += [_tx(rng, version=1) for _ in range(5)]
    txs += [_tx(rng, msg=b'hello world') for _ in range(5)]
    txs += [_tx(rng, version=2, msg=b'x' * 200) for _ in range(3)]
    txs += [_tx(rng, msg=b'') for _ in range(2)]
    hexes = [t.hex() for t in txs]
    _check_fast(L.decode_block_txs(hexes, 4), hexes)


def test_non_canonical_encodings_are_canonicalised(L):
    rng = random.Random(9)
    tx = _tx(rng, n_in=2, n_out=1, one_sig=True)
    h = tx.hex()
    b = bytearray(bytes.fromhex(h))
    # widen the amount to 8 bytes (non-minimal) and use prefix 0x07 instead of 42 for the address
    pos = 2 + 2 * 34 + 1
    addr, alen = b[pos:pos + 33], b[pos + 33]
    amount = int.from_bytes(b[pos + 34:pos + 34 + alen], 'little')
    wide = bytes(addr[:1] if addr[0] == 43 else b'\x07') + bytes(addr[1:]) + bytes([8]) + amount.to_bytes(8, 'little')
    b2 = b[:pos] + wide + b[pos + 34 + alen:]
    for variant in (bytes(b2).hex(), bytes(b2).hex().upper()):
        d = L.decode_block_txs([variant], 1)
        _check_fast(d, [variant])
        assert d['hex'][0] == Transaction.parse(variant)[0].hex() != variant


def test_general_and_malformed_flags(L):
    rng = random.Random(2)
    coinbase_like = _tx(rng, n_in=1).hex()[:-128 - 2] + '24'
    gov = Transaction([TransactionInput(rng.randbytes(32).hex(), 0)],
                      [TransactionOutput(_addr(rng), Decimal(1), OutputType.STAKE)])
    gov.inputs[0].signed = (1, 2)
    four = _tx(rng, n_in=3, one_sig=False)
    gh = four.hex() + four.hex()[-128:]  # 4 signatures for 3 inputs: the parser's IndexError
    cases = {'coinbase': coinbase_like, 'more sigs than inputs': gh,
             'odd hex': 'abc', 'bad char': 'zz' + _tx(rng).hex()[2:], 'version 4': '04' + _tx(rng).hex()[2:],
             'truncated': _tx(rng).hex()[:100]}
    d = L.decode_block_txs(list(cases.values()), 2)
    assert not d['all_fast']
    assert all(f != 0 for f in d['flags']), dict(zip(cases, d['flags']))
    # 2 signatures for 3 inputs decode natively, grouped (assignment by owner key in the block path)
    grouped = _tx(rng, n_in=3, one_sig=False).hex()[:-128]
    d = L.decode_block_txs([grouped], 1)
    assert d['all_fast'] and list(d['grouped']) == [1] and list(np.frombuffer(d['sig_first_in'], np.int32)) == [-1, -1]
    # governance outputs decode natively: the output-type column carries them
    d = L.decode_block_txs([gov.hex()], 1)
    assert d['all_fast'] and list(d['out_type']) == [int(OutputType.STAKE)] and list(d['tx_type']) == [0]


_MESSAGES = [b'5', b'05', b'0005', b'4', b'9', b'10', b'3', b'0', b'', b' 5', b'5 ', b'+5', b'-5', b'5_0', b'1_0',
             '\u0665'.encode(), '\uff15'.encode(), b'\xff5', b'\x80\x05', b'abc', b'hello 7', b'7\n', b'\t6',
             b'99999999999999999999', b'00000000000000000007', b'\xc3\xa9', b'\xe2\x80', b'8']


@settings(max_examples=200, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(st.one_of(st.sampled_from(_MESSAGES), st.binary(min_size=0, max_size=6),
                 st.text(alphabet='0123456789 +-_\u0665\u0e55a', max_size=5).map(lambda t: t.encode())))
def test_message_tx_type_matches_python(native, msg):
    """The codec's tx type (helpers.py:97-112 get_transaction_type_from_message) equals Python's whenever it
    decides (255 = left to Python's int())."""
    from upow_amd.utils.codec import get_transaction_type_from_message
    rng = random.Random(len(msg))
    tx = _tx(rng, n_in=1, n_out=1, one_sig=True)
    tx.message = msg
    tx.transaction_type = get_transaction_type_from_message(msg)
    h = tx.hex()
    d = native.decode_block_txs([h], 1)
    assert d['all_fast']
    t = d['tx_type'][0]
    if t != 255:
        assert t == int(get_transaction_type_from_message(msg)), (msg, t)


@settings(max_examples=150, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(st.binary(min_size=1, max_size=400), st.integers(0, 10 ** 6))
def test_fuzz_fast_implies_python_agrees(native, data, seed):
    """Random byte strings and mutated valid txs: whenever the native codec claims the fast path,
    the Python parser must accept the same bytes and serialise/hash them identically."""
    rng = random.Random(seed)
    base = bytearray(bytes.fromhex(_tx(rng, n_in=1, n_out=1, one_sig=True).hex()))
    for _ in range(rng.randint(0, 3)):
        base[rng.randrange(len(base))] = rng.randrange(256)
    for cand in (bytes(data).hex(), bytes(base).hex()):
        d = native.decode_block_txs([cand], 1)
        if d['all_fast']:
            _check_fast(d, [cand])


def test_input_address_strings(L):
    from upow_amd.ops import p256 as op
    rng = random.Random(3)
    pts = [op.public_key(rng.randrange(1, 1 << 200)) for _ in range(6)]
    addrs, lens = bytearray(), bytearray()
    for k, p in enumerate(pts):
        if k % 2:
            raw = p.x.to_bytes(32, 'little') + p.y.to_bytes(32, 'little')
        else:
            raw = bytes([42 if p.y % 2 == 0 else 43]) + p.x.to_bytes(32, 'little')
        addrs += raw + bytes(64 - len(raw))
        lens.append(len(raw))
    starts = np.array([0, 2, 6], dtype=np.int32).tobytes()
    js = arena_list(L.input_address_strings(bytes(addrs), bytes(lens), starts, 2))
    strs = [point_to_string(p) for p in pts]
    assert js == [json.dumps(strs[:2], separators=(',', ':')), json.dumps(strs[2:], separators=(',', ':'))]


def test_fee_strings_match_python(L):
    from decimal import Decimal
    from upow_amd.ledger.database import numeric
    rng = random.Random(4)
    fees = [0, 1, 49, 50, 51, 149, 150, 10 ** 8, 123456789012345] + [rng.randrange(1 << 50) for _ in range(300)]
    got = arena_list(L.fee_strings(np.array(fees, dtype=np.int64).tobytes()))
    assert got == [numeric(Decimal(f) / 10 ** 8, 6) for f in fees]
    # the other row columns of the bulk writes are bound natively from the codec's buffers: see
    # tests/test_ledger_sql.py (hex32 / arena / gather columns) and tests/test_fastpath.py


def test_address_pairs_distinct_per_tx(L):
    # each tx's distinct addresses, inputs first then outputs, in first-seen order (the address index rows)
    rng = random.Random(11)
    pool = [''.join(rng.choice('abcdefgh') for _ in range(rng.randrange(1, 50))) for _ in range(12)]
    txs = [([rng.choice(pool) for _ in range(rng.randrange(0, 5))], [rng.choice(pool) for _ in range(rng.randrange(0, 90))])
           for _ in range(300)]

    def arena(strs):
        off = np.cumsum([0] + [len(x) for x in strs]).astype(np.int64)
        return ''.join(strs).encode(), off.tobytes()

    ins = [a for t in txs for a in t[0]]
    outs = [a for t in txs for a in t[1]]
    ist = np.cumsum([0] + [len(t[0]) for t in txs]).astype(np.int32).tobytes()
    ost = np.cumsum([0] + [len(t[1]) for t in txs]).astype(np.int32).tobytes()
    blob, off, tx = L.address_pairs(*arena(ins), ist, *arena(outs), ost, 3)
    got = list(zip(np.frombuffer(tx, np.int64).tolist(), arena_list((blob, off))))
    want = [(k, a) for k, t in enumerate(txs) for a in dict.fromkeys(t[0] + t[1])]
    assert got == want


def _mutate(rng, raw: bytes, other: bytes) -> bytes:
    """One structural mutation of a serialised tx: flip/overwrite a byte, insert or delete a run, truncate,
    duplicate a range, bump a count byte, splice in a piece of another tx, or upper-case / odd-length hex."""
    b = bytearray(raw)
    op = rng.randrange(8)
    if not b:
        return bytes(other[:rng.randrange(len(other) + 1)])
    i = rng.randrange(len(b))
    if op == 0:
        b[i] ^= 1 << rng.randrange(8)
    elif op == 1:
        b[i] = rng.choice([0, 1, 2, 3, 4, 10, 33, 36, 42, 43, 64, 127, 128, 254, 255])
    elif op == 2:
        b[i:i] = rng.randbytes(rng.randint(1, 70))
    elif op == 3:
        del b[i:i + rng.randint(1, 70)]
    elif op == 4:
        del b[i:]
    elif op == 5:
        j = rng.randrange(len(b))
        b[i:i] = b[min(i, j):max(i, j)][:200]
    elif op == 6:
        for k in (1, 2 + 34 * raw[1] if len(raw) > 1 else 1):  # the input / output count bytes
            if k < len(b):
                b[k] = (b[k] + rng.choice([-1, 1, 2, 255])) % 256
    else:
        j = rng.randrange(len(other) + 1)
        b[i:] = other[j:j + rng.randint(1, 200)]
    return bytes(b)


@settings(max_examples=400, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(st.integers(0, 10 ** 9), st.integers(1, 4))
def test_mutated_txs_rejected_or_agree_with_python_parser(native, seed, n_mut):
    """Structured mutations of valid txs of every shape (multi-input, one or n signatures, messages, v1
    64-byte addresses): for every mutant the native codec either does not claim the fast path, or the
    Python parser (reference transaction.py:520-592) accepts the same bytes and serialises, hashes and
    splits them identically. A block holding a mutant among valid txs is all-fast only if the mutant is."""
    rng = random.Random(seed)
    shapes = [dict(), dict(version=1), dict(msg=b'hello'), dict(n_in=3, one_sig=False), dict(n_in=2, one_sig=True)]
    a, b = (_tx(rng, **rng.choice(shapes)).hex() for _ in range(2))
    raw = bytes.fromhex(a)
    for _ in range(n_mut):
        raw = _mutate(rng, raw, bytes.fromhex(b))
    cands = [raw.hex()]
    if rng.random() < 0.3:
        cands.append(raw.hex().upper())
    for cand in cands:
        d = native.decode_block_txs([cand], 1)
        if d['all_fast']:
            _check_fast(d, [cand])
        blk = native.decode_block_txs([b, cand, a], 2)
        assert bool(blk['all_fast']) == bool(d['all_fast'])
        if blk['all_fast']:
            _check_fast(blk, [b, cand, a])


def test_sha256_hex_prefixes_matches_hashlib(L):
    # the ASCII-hex retry's batch hash: SHA-256 of the first n characters of the selected hex strings
    import hashlib
    import random
    rng = random.Random(7)
    hexes = [rng.randbytes(rng.randrange(1, 300)).hex() for _ in range(200)]
    idx = np.array([rng.randrange(len(hexes)) for _ in range(500)], np.int64)
    nch = np.array([rng.randrange(len(hexes[i]) + 1) for i in idx], np.int64)
    got = L.sha256_hex_prefixes(hexes, idx, nch, 4)
    want = b''.join(hashlib.sha256(hexes[i][:c].encode()).digest() for i, c in zip(idx, nch))
    assert got == want
    assert L.sha256_hex_prefixes(hexes, np.zeros(0, np.int64), np.zeros(0, np.int64), 4) == b''
    with pytest.raises(IndexError):
        L.sha256_hex_prefixes(hexes, np.array([len(hexes)], np.int64), np.array([0], np.int64), 1)
    with pytest.raises(ValueError):
        L.sha256_hex_prefixes(hexes, np.array([0], np.int64), np.array([len(hexes[0]) + 1], np.int64), 1)
