"""Governance transactions on the native block path (ledger/fastpath.py + ledger/govcheck.py) against the
object path (reference transaction.py:240-479, manager.py:470-529, database.py:589-621): a full lifecycle —
stakes, inode and validator registrations, votes, revokes, unstake, de-registration — goes through both,
accepted blocks natively, and every rejected block (MAX_INODES, vote range, double registration, the 48 h
revoke rule, a forged voter signature) is handed to the object path with the same verdict and error. After
each block every table, the UTXO index with payloads and the UTXO-set hash are identical (Pair.push), and
the native side's governance index equals one rebuilt from SQL."""
import asyncio
import time
from decimal import Decimal

import pytest

from test_fastpath import GENESIS, Pair, _dump  # noqa: F401
from upow_amd.ledger import fastpath, govcheck, manager
from upow_amd.ledger.database import Database
from upow_amd.models import transaction as txmod
from upow_amd.models.transaction import Transaction, TransactionInput, TransactionOutput
from upow_amd.utils.codec import OutputType, TransactionType
from upow_amd.wallet import builders as B

I1, I2, I3, V1, V2, D1, D2 = (0x7100 + k for k in range(7))


@pytest.fixture(autouse=True)
def _small_world(monkeypatch):
    monkeypatch.setattr(manager, 'START_DIFFICULTY', Decimal('1.0'))
    monkeypatch.setattr(txmod, 'MAX_INODES', 2)
    monkeypatch.setattr(govcheck, 'MAX_INODES', 2)
    manager.cache.clear()


async def _chain(n_blocks: int):
    a = await Database.create(utxo_backend='host')
    b = await Database.create(utxo_backend='host')
    p = Pair(a, b)
    base = 1_700_000_000
    for k in range(n_blocks):  # empty blocks, both paths, no per-block dump (funding only)
        p.use(a)
        c = await p.mine(ts=base + 60 * k)
        for db in (a, b):
            p.use(db)
            assert await fastpath.create_block_from_hex(c, []) if db is b else await manager.create_block(c, [])
    return p, base + 60 * n_blocks


def _gov_rows(db):
    return {t: dict(tab.rows) for t, tab in db.gov.tables.items()}


async def _push(p, txs, ts, expect, path):
    hexes = [t.hex() for t in txs]
    p.use(p.a)
    c = await p.mine(hexes, ts=ts)
    ok, err = await p.push(c, hexes, expect=expect)
    assert fastpath.last_path == path, (fastpath.last_path, err)
    rows = _gov_rows(p.b)
    p.b.gov.rebuild()
    assert _gov_rows(p.b) == rows  # the native side's incremental governance index == a rebuild from SQL
    return err


def _raw(inputs, outputs, tx_type=None, keys=()):
    msg = B.type_message(tx_type) if tx_type is not None else None
    return Transaction(inputs, outputs, msg).sign(list(keys))


def test_governance_lifecycle_native_matches_object():
    async def go():
        p, ts = await _chain(700)
        A = {k: B.address_of(k) for k in (I1, I2, I3, V1, V2, D1, D2)}
        fund = []
        for k, amount in zip((I1, I2, I3, V1, V2, D1, D2), ('1100', '1100', '1100', '150', '150', '50', '50')):
            p.use(p.a)
            tx = await B.create_transaction(GENESIS, A[k], amount)  # <= 255 coinbase inputs each
            for db in (p.a, p.b):  # both mempools: the next selection skips pending inputs
                p.use(db)
                assert await db.add_pending_transaction(tx)
            fund.append(tx)
        await _push(p, fund, ts, True, 'native')
        # stakes (REGULAR txs with STAKE + DELEGATE_VOTING_POWER outputs)
        p.use(p.a)
        stakes = [await B.create_stake_transaction(k, '10') for k in (I1, I2, I3, V1, V2, D1, D2)]
        await _push(p, stakes, ts + 60, True, 'native')
        # registrations: two inodes (MAX_INODES = 2 here), two validators
        p.use(p.a)
        regs = [await B.create_inode_registration_transaction(I1), await B.create_inode_registration_transaction(I2),
                await B.create_validator_registration_transaction(V1),
                await B.create_validator_registration_transaction(V2)]
        await _push(p, regs, ts + 120, True, 'native')
        # votes: validators -> inodes, delegates -> validators
        p.use(p.a)
        votes = [await B.create_voting_transaction(V1, 5, A[I1]), await B.create_voting_transaction(V2, 3, A[I2]),
                 await B.create_voting_transaction(D1, 7, A[V1]), await B.create_voting_transaction(D2, 4, A[V2])]
        await _push(p, votes, ts + 180, True, 'native')
        # rejections, each handed to the object path with the same verdict
        p.use(p.a)
        outs = await p.a.get_spendable_outputs(A[I3])
        third = _raw(outs, [TransactionOutput(A[I3], Decimal(1000), OutputType.INODE_REGISTRATION),
                            TransactionOutput(A[I3], sum(o.amount for o in outs) - 1000)], keys=[I3])
        err = await _push(p, [third], ts + 240, False, 'object')  # 2 active inodes already (MAX_INODES)
        assert err
        dvp = await p.a.get_delegates_voting_power(A[D2])
        over = _raw(dvp, [TransactionOutput(A[V2], Decimal(11), OutputType.VOTE_AS_DELEGATE)],
                    TransactionType.VOTE_AS_DELEGATE, [D2])
        await _push(p, [over], ts + 240, False, 'object')  # vote range > 10
        outs = await p.a.get_spendable_outputs(A[V1])
        again = _raw(outs, [TransactionOutput(A[V1], Decimal(100), OutputType.VALIDATOR_REGISTRATION),
                            TransactionOutput(A[V1], Decimal(10), OutputType.VALIDATOR_VOTING_POWER)],
                     TransactionType.VALIDATOR_REGISTRATION, [V1])
        await _push(p, [again], ts + 240, False, 'object')  # validator already registered
        # revokes (the votes are far older than 48 h), signed by the voters
        p.use(p.a)
        rv = [await B.create_revoke_transaction(D1, A[V1]), await B.create_revoke_transaction(V2, A[I2])]
        forged, _ = Transaction.parse(rv[0].hex())
        forged.inputs[0].signed = Transaction.parse((await B.create_revoke_transaction(D2, A[V2])).hex())[0].inputs[0].signed
        await _push(p, [forged], ts + 240, False, 'native')  # signature of another voter: same error, native
        await _push(p, rv, ts + 300, True, 'native')
        # unstake (D1 released its vote) and inode de-registration (I2 lost its votes, registered long ago)
        p.use(p.a)
        un = await B.create_unstake_transaction(D1)
        dereg = await B.create_inode_de_registration_transaction(I2)
        await _push(p, [un, dereg], ts + 360, True, 'native')
        assert await p.b.get_address_stake(A[D1]) == 0
        # the 48 h revoke rule: a vote cast now cannot be revoked yet
        now = int(time.time())
        p.use(p.a)
        fresh = await B.create_voting_transaction(V1, 2, A[I1])
        await _push(p, [fresh], now - 100, True, 'native')
        p.use(p.a)
        early = await B.create_revoke_transaction(V1, A[I1])
        assert len(early.inputs) == 2  # the old ballot (revocable) and the fresh one
        fresh_only = _raw([TransactionInput(i.tx_hash, i.index, public_key=i.public_key)
                           for i in early.inputs if i.tx_hash == fresh.hash()],
                          [TransactionOutput(A[V1], Decimal(2), OutputType.VALIDATOR_VOTING_POWER)],
                          TransactionType.REVOKE_AS_VALIDATOR, [V1])
        await _push(p, [fresh_only], now - 50, False, 'object')
        await _push(p, [early], now - 40, True, 'native')  # any() over the inputs: the old ballot qualifies
        # regular traffic still native next to governance txs
        p.use(p.a)
        mix = [await B.create_transaction(GENESIS, A[D2], "1"), await B.create_stake_transaction(D1, "5")]
        await _push(p, mix, now - 30, True, 'native')
        # inode rewards reach the coinbase identically on both paths after all of this
        assert _dump(p.a)['transactions'] == _dump(p.b)['transactions']
    asyncio.run(go())


def test_native_block_prep_matches_numpy():
    """gov_block_mask / gov_block_inputs (csrc/gov_index.cpp) against the numpy forms of BlockGovernance."""
    import numpy as np
    from upow_amd.ledger.govcheck import BlockGovernance, SPEND_TABLE, _seg
    from upow_amd.ledger.utxo import PAYLOAD_DTYPE, TAG_BY_TABLE
    from upow_amd.utils.codec import OutputType as O
    rng = np.random.default_rng(11)
    for trial in range(20):
        n = int(rng.integers(1, 300))
        n_out_per = rng.integers(1, 4, n)
        n_in_per = rng.integers(1, 4, n)
        out_start = np.concatenate([[0], np.cumsum(n_out_per)]).astype(np.int32)
        in_start = np.concatenate([[0], np.cumsum(n_in_per)]).astype(np.int32)
        n_out, n_in = int(out_start[-1]), int(in_start[-1])
        tx_type = np.where(rng.random(n) < 0.2, rng.choice([4, 5, 6, 7, 8, 9], n), 0).astype(np.uint8)
        out_type = np.where(rng.random(n_out) < 0.1, rng.integers(0, 10, n_out), 0).astype(np.uint8)
        out_tx = np.repeat(np.arange(n, dtype=np.int32), n_out_per)
        in_tx = np.repeat(np.arange(n, dtype=np.int32), n_in_per)
        out_amount = rng.integers(0, 1 << 40, n_out).astype(np.uint64)
        fee = rng.integers(-(1 << 30), 1 << 30, n).astype(np.int64)
        bg = BlockGovernance(tx_type, out_type, out_tx, out_start, in_tx)
        has = np.zeros(n, bool)
        has[np.unique(out_tx[out_type != 0])] = True
        assert np.array_equal(bg.gov, (tx_type != 0) | has) and bg.any == bool(((tx_type != 0) | has).any())
        want_tag = bg.spend_tags(TAG_BY_TABLE)
        tags = want_tag.copy()
        pay = np.zeros(n_in, PAYLOAD_DTYPE)
        pay['len'] = 33
        flip = trial % 3
        if flip == 1:
            tags[int(rng.integers(n_in))] ^= 1
        elif flip == 2:
            pay['len'][int(rng.integers(n_in))] = 0
        in_tag, bad, f = bg.inputs(TAG_BY_TABLE, tags, pay, fee, out_amount)
        assert np.array_equal(in_tag, want_tag)
        assert bad == bool(((tags != want_tag) | (pay['len'] == 0)).any()) == (flip != 0)
        assert np.array_equal(f, bg.fee_adjust(fee, out_amount))
