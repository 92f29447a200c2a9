"""UTXO index: host dict backend vs the HBM hash-table kernels (probe / insert / erase / grow)."""
import random

import numpy as np
import pytest

from upow_amd.ledger.utxo import MISSING, UtxoIndex


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
    return idx


def test_host_backend():
    idx = _exercise('host')
    assert len(idx) == 5000 - len([1 for t in range(3000, 3100) if t % 7 == 3])


@pytest.mark.gpu
def test_gpu_backend_matches_host(gpu):
    _exercise('gpu')
    # growth past 50% load triggers a rehash on device
    idx = UtxoIndex(backend='gpu')
    keys = _keys(1 << 19 | 12345, 9)
    idx.insert(keys, 1)
    assert len(idx) == len(keys)
    assert (idx.probe(keys[::97]) == 1).all()
