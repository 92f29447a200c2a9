"""The incremental emission cascade (ledger/governance.py _Cascade) against the reference's sequential
recomputation (database.py:1127-1136, 1189-1205, 1390-1418): after random stake / ballot additions and
removals with fractional amounts, every validator stake and inode power equals the left-to-right Decimal
sum in value AND representation (str), which is what lands in emission_details and the coinbase split."""
import random
from decimal import Decimal

from upow_amd.ledger.governance import STAKE, GovernanceIndex, _Cascade, _forms
from upow_amd.ops import p256 as op
from upow_amd.utils.codec import point_to_string


class _NoDb:
    _mempool_ver = 0


def _sequential(g, forms_fn):
    """validators_stake / inode_power recomputed the reference's way (no cascade)."""
    saved = g.cascade
    g.cascade = type('Off', (), {'stake': lambda s, pt: None, 'validator_stake': lambda s, pt: None,
                                 'inode_power': lambda s, pt: None})()
    try:
        return forms_fn()
    finally:
        g.cascade = saved


def test_cascade_matches_sequential_sums():
    rng = random.Random(7)
    g = GovernanceIndex.__new__(GovernanceIndex)
    import threading
    g.db, g.lock, g.version = _NoDb(), threading.RLock(), 0
    from upow_amd.ledger.governance import GOV_TABLES, _Table
    g.tables = {t: _Table(t, None) for t in (*GOV_TABLES, STAKE)}
    g._memo, g._memo_version, g._pending, g._parsed = {}, -1, (0, set(), {}, 0), {}
    g.cascade = _Cascade(g)
    for t in g.tables.values():
        t.changed = g._changed
    addrs = [point_to_string(op.public_key(rng.randrange(1, 1 << 200))) for _ in range(24)]
    delegates, validators, inodes = addrs[:14], addrs[14:20], addrs[20:]
    live = {STAKE: [], 'validators_ballot': [], 'inodes_ballot': []}
    n = 0
    for step in range(1500):
        table = rng.choice(list(live))
        if live[table] and rng.random() < 0.35:
            key = live[table].pop(rng.randrange(len(live[table])))
            g.tables[table].remove(key)
        else:
            n += 1
            key = (f'{n:064x}', rng.randrange(3))
            amount = rng.choice([10 * 10 ** 8, rng.randrange(1, 10 ** 10), 123456789, 5 * 10 ** 7])
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
    g.cascade.build()
    assert [str(g.inode_power(_forms(i), False)) for i in inodes] == before
