"""UTXO index: host dict backend vs the HBM hash-table kernels (probe / insert / erase / grow)."""
import random

import numpy as np
import pytest

from upow_amd.ledger.utxo import MISSING, UtxoIndex, make_payload, pack_records


def _keys(n, seed):
    rng = random.Random(seed)
    return [(rng.randbytes(32).hex(), rng.randrange(0, 256)) for _ in range(n)]


def _exercise(backend):
    idx = UtxoIndex(backend=backend)
    keys = _keys(5000, 1)
    tags = [k % 7 for k in range(5000)]
    idx.reset(keys[:1000], tags[:1000])
    idx.insert(keys[1000:3000], 0)
    idx.insert(keys[3000:], tags[3000:])
    got = idx.probe(keys)
    want = np.array(tags[:1000] + [0] * 2000 + tags[3000:], dtype=np.uint8)
    assert (got == want).all()
    assert (idx.probe(_keys(100, 2)) == MISSING).all()
    # erase with tag filter + duplicate keys in one batch: each outpoint erased once
    er = idx.erase(keys[:10] + keys[:10], tag=None)
    assert ((er[:10] + er[10:]) == 1).all()  # exactly one copy wins (on the GPU either lane may)
    assert (idx.probe(keys[:10]) == MISSING).all()
    # tag-filtered erase leaves other tables alone
    k7 = [k for k, t in zip(keys[3000:3100], tags[3000:3100]) if t == 3]
    kn = [k for k, t in zip(keys[3000:3100], tags[3000:3100]) if t != 3]
    assert idx.erase(k7 + kn, tag=3)[:len(k7)].all()
    assert (idx.probe(kn) != MISSING).all()
    # filter() keeps first-seen order and uniqueness
    f = idx.filter([keys[2000], keys[2000], keys[1500], keys[0]], 0)
    assert f == [keys[2000], keys[1500]]
    # re-insert after tombstones
    idx.insert(keys[:10], 5)
    assert (idx.probe(keys[:10]) == 5).all()
    # payloads: (amount, address bytes) come back with the tag; absent -> len 0
    rng = random.Random(4)
    pk = _keys(300, 3)
    amounts = [rng.randrange(1 << 63) for _ in pk]
    addrs = [bytes([42]) + rng.randbytes(32) if k % 3 else rng.randbytes(64) for k in range(300)]
    idx.insert(pk, 0, make_payload(amounts, addrs))
    tags, pay = idx.lookup(pk + _keys(5, 77))
    assert (tags[:300] == 0).all() and (tags[300:] == MISSING).all()
    assert [int(a) for a in pay['amount'][:300]] == amounts and (pay['len'][300:] == 0).all()
    assert all(bytes(pay['addr'][k][:pay['len'][k]]) == addrs[k] for k in range(300))
    t2, p2 = idx.lookup_records(pack_records(pk[:50]))
    assert (t2 == 0).all() and [int(a) for a in p2['amount']] == amounts[:50]
    recs, allpay = idx.records_payload()
    assert len(recs) == len(idx) and len(allpay) == len(idx)
    return idx


def test_host_backend():
    idx = _exercise('host')
    assert len(idx) == 5000 + 300 - len([1 for t in range(3000, 3100) if t % 7 == 3])


@pytest.mark.gpu
def test_gpu_backend_matches_host(gpu):
    _exercise('gpu')
    # growth past 50% load triggers a rehash on device
    idx = UtxoIndex(backend='gpu')
    keys = _keys(1 << 19 | 12345, 9)
    amounts = list(range(len(keys)))
    idx.insert(keys, 1, make_payload(amounts, [bytes([43]) + bytes(32)] * len(keys)))
    assert len(idx) == len(keys)
    assert (idx.probe(keys[::97]) == 1).all()
    t, p = idx.lookup(keys[::97])  # payloads survive the device rehash
    assert (t == 1).all() and [int(a) for a in p['amount']] == amounts[::97]
