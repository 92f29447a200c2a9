"""bench_verify's distinct-key block builder (BASELINE: random-keypair data): the bulk-signed synthetic txs
are byte-identical to what the Transaction model serialises and signs (RFC 6979 is deterministic), and the
native batch key/sign bindings agree with the single-key ones."""
import random
from decimal import Decimal

from upow_amd.bench_verify import batch_keys, signed_spend_txs
from upow_amd.models.transaction import Transaction, TransactionInput, TransactionOutput
from upow_amd.ops import p256 as op
from upow_amd.ops.native import lib
from upow_amd.utils.codec import bytes_to_string


def test_bulk_signed_txs_match_transaction_model():
    rng = random.Random(5)
    keys, pubs, a33 = batch_keys(24, rng)
    _, _, r33 = batch_keys(24, rng)
    spends = [((rng.randbytes(32).hex(), rng.randrange(3)), (rng.randbytes(32).hex(), 7)) for _ in range(24)]
    fast = signed_spend_txs(spends, keys, a33, r33)
    assert len(set(a33)) == 24 and len(set(fast)) == 24
    for j in range(24):
        q = op.public_key(keys[j])
        assert pubs[64 * j:64 * j + 64] == q.x.to_bytes(32, 'little') + q.y.to_bytes(32, 'little')
        ins = [TransactionInput(h, i, amount=Decimal(10)) for h, i in spends[j]]
        for i in ins:
            i.public_key = q
        tx = Transaction(ins, [TransactionOutput(bytes_to_string(r33[j]), Decimal('12.5')),
                               TransactionOutput(bytes_to_string(a33[j]), Decimal('7.49'))])
        tx.sign([keys[j]])
        assert tx.hex() == fast[j]


def test_sign_batch_matches_single_and_zero_key_is_left_empty():
    rng = random.Random(9)
    keys = [rng.randrange(1, op.oracle.N) for _ in range(70)] + [0]
    digests = [rng.randbytes(32) for _ in keys]
    out = lib().p256_sign_batch(b''.join(k.to_bytes(32, 'big') for k in keys), b''.join(digests), 4)
    for j, (k, d) in enumerate(zip(keys[:-1], digests)):
        r, s = lib().p256_sign(k.to_bytes(32, 'big'), d)
        assert out[64 * j:64 * j + 64] == r + s
    assert out[-64:] == bytes(64)
