"""The native emission cascade (csrc/gov_index.cpp GovStore, via ledger/governance.py) against the
reference's sequential recomputation (database.py:1127-1136, 1189-1205, 1390-1418): after random stake /
ballot additions and removals with fractional and near-28-digit amounts, every delegate stake, validator
stake and inode power equals the left-to-right Decimal sum in value AND representation (str), which is
what lands in emission_details and the coinbase split. A sum the store cannot keep exactly must come back
as "unknown" (recomputed sequentially), never as a different number."""
import random
from decimal import Decimal

from upow_amd.ledger.governance import STAKE, GovernanceIndex, _forms, point_key_of
from upow_amd.ops import p256 as op
from upow_amd.utils.codec import point_to_string


class _NoDb:
    _mempool_ver = 0


class _Off:
    """The store with its cascade answers withheld: the facade then recomputes the reference's way."""

    def __init__(self, store):
        self._s = store

    def __getattr__(self, name):
        if name in ('stake', 'validator_stake', 'inode_power'):
            return lambda pt: None
        return getattr(self._s, name)


def _sequential(g, fn):
    saved = g.store
    g.store = _Off(saved)
    g.version += 1  # no memoised aggregate from the native answers
    try:
        return fn()
    finally:
        g.store = saved
        g.version += 1


def _index():
    g = GovernanceIndex(_NoDb())
    g._pending = (0, set(), {}, 0)
    return g


def test_cascade_matches_sequential_sums():
    rng = random.Random(7)
    g = _index()
    addrs = [point_to_string(op.public_key(rng.randrange(1, 1 << 200))) for _ in range(24)]
    delegates, validators, inodes = addrs[:14], addrs[14:20], addrs[20:]
    live = {STAKE: [], 'validators_ballot': [], 'inodes_ballot': []}
    n = 0
    for step in range(1500):
        table = rng.choice(list(live))
        if live[table] and rng.random() < 0.35:
            key = live[table].pop(rng.randrange(len(live[table])))
            assert g.tables[table].remove(key)
        else:
            n += 1
            key = (f'{n:064x}', rng.randrange(3))
            amount = rng.choice([10 * 10 ** 8, rng.randrange(1, 10 ** 10), 123456789, 5 * 10 ** 7,
                                 10 ** 18 - rng.randrange(1, 1000)])
            if table == STAKE:
                a = rng.choice(delegates + validators)
                g.tables[table].add(key, a, amount, a, 1)
            elif table == 'validators_ballot':
                g.tables[table].add(key, rng.choice(validators), rng.randrange(1, 11) * 10 ** 7, rng.choice(delegates), 1)
            else:
                g.tables[table].add(key, rng.choice(inodes), rng.randrange(1, 11) * 10 ** 8 // 3, rng.choice(validators), 1)
            live[table].append(key)
        if step % 7 == 6 or rng.random() < 0.05:
            for v in validators:
                fast = g.validators_stake(_forms(v), False)
                slow = _sequential(g, lambda: g.validators_stake(_forms(v), False))
                assert fast == slow and str(fast) == str(slow), (v, fast, slow)
            for i in inodes:
                fast = g.inode_power(_forms(i), False)
                slow = _sequential(g, lambda: g.inode_power(_forms(i), False))
                assert fast == slow and str(fast) == str(slow), (i, fast, slow)
            for d in delegates:
                fast = g.address_stake(_forms(d), False)
                slow = _sequential(g, lambda: g.address_stake(_forms(d), False))
                assert fast == slow and str(fast) == str(slow)
    # a rebuild of the cascade from the rows gives the same answers
    before = [str(g.inode_power(_forms(i), False)) for i in inodes]
    g.store.build()
    g.version += 1
    assert [str(g.inode_power(_forms(i), False)) for i in inodes] == before


def test_store_rows_indexes_and_exponents():
    g = _index()
    rng = random.Random(3)
    a, b = (point_to_string(op.public_key(rng.randrange(1, 1 << 200))) for _ in range(2))
    t = g.tables[STAKE]
    t.add(('aa' * 32, 0), a, 150000000, a, 5)
    t.add(('bb' * 32, 1), a, 50000000, a, 6)
    t.add(('cc' * 32, 0), b, 300000000, b, 7)
    assert len(t) == 3
    assert list(t.rows) == [('aa' * 32, 0), ('bb' * 32, 1), ('cc' * 32, 0)]  # rowid order
    assert str(g.address_stake(_forms(a), False)) == '2.0'  # Decimal('1.5') + Decimal('0.5')
    assert str(g.address_stake(_forms(b), False)) == '3'
    assert g.amount_rows(STAKE, _forms(a), False) == [('aa' * 32, 0, 150000000), ('bb' * 32, 1, 50000000)]
    # both string forms of an address denote the same point
    assert all(g.has_point(STAKE, point_key_of(f), False)
               for f in _forms(a))
    assert t.remove(('aa' * 32, 0)) and not t.remove(('aa' * 32, 0))
    assert str(g.address_stake(_forms(a), False)) == '0.5'
    g.tables['validators_ballot'].add(('dd' * 32, 0), b, 5 * 10 ** 7, a, 8)
    assert str(g.validators_stake(_forms(b), False)) == '0.025'  # 0.5 * 0.5 / 10
    assert g.ballot_rows('validators_ballot', _forms(b), False)[0][2:4] == (Decimal('0.5'), a)
