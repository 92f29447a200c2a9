"""K3/K4 batched SHA-256 (txids, merkle leaves): host C++ core and the gfx950 lane-per-message kernel
against hashlib, over every padding boundary (lengths 0..200 cover 55/56/63/64/119/120 bytes), real tx
sizes and maximum-size messages (a 65 535-byte message field plus the tx framing)."""
import hashlib
import random

import pytest

from upow_amd.ops import sha256 as sh


def _messages(seed):
    rng = random.Random(seed)
    msgs = [rng.randbytes(n) for n in range(201)]                 # every padding boundary
    msgs += [rng.randbytes(rng.randrange(182, 319)) for _ in range(3000)]  # 1-5 input regular txs
    msgs += [rng.randbytes(n) for n in (65_535, 65_535 + 255 * 107, 4096 * 1024 // 2)]
    rng.shuffle(msgs)
    return msgs


def _merkle_oracle(txs):
    """upow/manager.py:365-378: SHA-256 over the concatenated SHA-256 digests of the raw-byte-sorted txs."""
    return hashlib.sha256(b''.join(hashlib.sha256(t).digest() for t in sorted(txs))).hexdigest()


def test_host_batch_matches_hashlib(native):
    msgs = _messages(1)
    assert sh.batch(msgs, device='cpu') == [hashlib.sha256(m).digest() for m in msgs]
    assert sh.batch([], device='cpu') == []
    txs = msgs[:500]
    assert sh.merkle_root(txs, device='cpu') == _merkle_oracle(txs)


@pytest.mark.gpu
def test_gpu_batch_matches_hashlib(gpu):
    msgs = _messages(2)
    assert sh.batch(msgs, device='gpu') == [hashlib.sha256(m).digest() for m in msgs]
    # one partial tail word at the very end of the packed buffer (length % 4 != 0 on the last message)
    tail = [b'\x01' * 5, b'\x02' * 7]
    assert sh.batch(tail, device='gpu') == [hashlib.sha256(m).digest() for m in tail]
    txs = msgs[:5000]
    assert sh.merkle_root(txs, device='gpu') == _merkle_oracle(txs)
