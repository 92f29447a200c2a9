"""Governance flow on a devnet: staking, validator/inode registration, votes, emission, inode
rewards in the coinbase, revokes, unstake rules (reference transaction.py:240-479, database.py:939-1436)."""
import asyncio
from decimal import Decimal

import pytest

from upow_amd import devnet
from upow_amd.ledger import manager
from upow_amd.ledger.database import Database
from upow_amd.models.transaction import Transaction
from upow_amd.utils.codec import TransactionType
from upow_amd.wallet import builders as B

KA, KV, KI, KD = 0xA1, 0xB2, 0xC3, 0xD4


@pytest.fixture
def db(monkeypatch):
    monkeypatch.setattr(manager, 'START_DIFFICULTY', Decimal('1.0'))
    manager.Manager.difficulty = None
    manager.cache.clear()
    d = asyncio.run(Database.create(utxo_backend='host'))
    yield d
    d.close()


def test_governance_lifecycle(db):
    async def go():
        A, V, I, D = (B.address_of(k) for k in (KA, KV, KI, KD))
        ts = [1_700_000_000]

        async def block(txs=()):
            ts[0] += 1
            return await devnet.mine_block(A, list(txs), ts=ts[0])

        async def push_and_mine(*txs):
            for t in txs:
                assert await db.add_pending_transaction(t), t.transaction_type
            await block(await db.get_pending_transactions_limit())

        for _ in range(240):
            await block()
        await push_and_mine(await B.create_transaction_to_send_multiple_wallet(KA, [I, V, D], ['1100', '200', '50']))
        assert await db.get_address_balance(I) == 1100
        # delegates: stake 10 each (first stake mints 10 delegate voting power)
        await push_and_mine(await B.create_stake_transaction(KI, '10'), await B.create_stake_transaction(KV, '10'),
                            await B.create_stake_transaction(KD, '10'))
        for k in (I, V, D):
            assert await db.get_address_stake(k) == 10
            assert len(await db.get_delegates_voting_power(k)) == 1
        with pytest.raises(Exception, match='Already staked'):
            await B.create_stake_transaction(KD, '1')
        # registrations
        await push_and_mine(await B.create_inode_registration_transaction(KI),
                            await B.create_validator_registration_transaction(KV))
        assert await db.is_inode_registered(I) and await db.is_validator_registered(V)
        assert not await db.is_validator_registered(I)
        # votes: validator -> inode (5), delegate -> validator (7)
        vtx = await B.create_voting_transaction(KV, 5, I)
        dtx = await B.create_voting_transaction(KD, 7, V)
        assert vtx.transaction_type == TransactionType.VOTE_AS_VALIDATOR
        assert dtx.transaction_type == TransactionType.VOTE_AS_DELEGATE
        await push_and_mine(vtx, dtx)
        ballots = await db.get_inode_ballot(0, 100)
        assert [(b[1], b[2], b[3]) for b in ballots] == [(I, Decimal(5), V)]
        assert await db.get_validators_stake(V) == Decimal(7)  # 7 * stake(D)=10 / 10
        active = await db.get_active_inodes()
        assert [a['wallet'] for a in active] == [I] and active[0]['power'] == Decimal('3.5')
        assert active[0]['emission'] == 100
        # the next block pays the inode half of the reward through the coinbase
        h = await block()
        cb = [t for t in await db.get_block_transactions(h) if not isinstance(t, Transaction)][0]
        assert [(o.address, o.amount) for o in cb.outputs] == [(A, Decimal(3)), (I, Decimal(3))]
        # an active inode cannot de-register; a delegate with cast votes cannot unstake
        with pytest.raises(Exception, match='active inode'):
            await B.create_inode_de_registration_transaction(KI)
        with pytest.raises(Exception, match='release the votes'):
            await B.create_unstake_transaction(KD)
        # revokes (blocks are > 48 h old): voting power comes back
        rv = await B.create_revoke_transaction(KV, I)
        rd = await B.create_revoke_transaction(KD, V)
        assert rv.transaction_type == TransactionType.REVOKE_AS_VALIDATOR
        await push_and_mine(rv, rd)
        assert await db.get_inode_ballot(0, 100) == []
        assert sum(i.amount for i in await db.get_validators_voting_power(V)) == 10
        assert await db.get_active_inodes() == []
        # now D may unstake
        await push_and_mine(await B.create_unstake_transaction(KD))
        assert await db.get_address_stake(D) == 0
        # the UTXO-set hash still matches a full replay
        import hashlib
        outs = await db.get_unspent_outputs_from_all_transactions()
        regular = set(await db.get_unspent_outputs(outs))
        assert regular  # governance outputs live in their own tables
    asyncio.run(go())


GOV_QUERIES = ('get_active_inodes', 'get_inode_count', 'get_all_registered_inode', 'get_inode_ballot',
               'get_validator_ballot')


async def _gov_answers(db, people, check_pending):
    """Every indexed governance query, for every address (reference: database.py:939-1436)."""
    out = {}
    cp = check_pending
    out['active'] = await db.get_active_inodes(cp)
    out['count'] = await db.get_inode_count(cp)
    out['registered'] = await db.get_all_registered_inode(cp)
    out['inode_ballot'] = await db.get_inode_ballot(0, 1000, cp)
    out['validator_ballot'] = await db.get_validator_ballot(0, 1000, cp)
    out['page'] = await db.get_validator_ballot(1, 2, cp)
    out['multi'] = await db.get_multiple_address_stakes(set(people), cp)
    for a in people:
        row = out.setdefault(a, {})
        row['stake'] = await db.get_address_stake(a, cp)
        row['vstake'] = await db.get_validators_stake(a, cp)
        row['ratio'] = await db.get_inode_vote_ratio_by_address(a, cp)
        row['iballot'] = await db.get_inode_ballot_by_address(0, 1000, a, cp)
        row['vballot'] = await db.get_validator_ballot_by_address(0, 1000, a, cp)
        for fn in ('get_stake_outputs', 'get_inode_registration_outputs', 'get_validator_registration_outputs',
                   'get_validators_voting_power', 'get_delegates_voting_power', 'get_validators_spent_votes',
                   'get_delegates_spent_votes', 'get_delegates_all_power'):
            row[fn] = [(i.tx_hash, i.index, i.amount) for i in await getattr(db, fn)(a, cp)]
        for other in people:
            row[('iin', other)] = [(i.tx_hash, i.index, i.amount)
                                   for i in await db.get_inode_ballot_input_by_address(a, other, cp)]
            row[('vin', other)] = [(i.tx_hash, i.index, i.amount)
                                   for i in await db.get_validator_ballot_input_by_address(a, other, cp)]
    return out


async def _compare_index_with_sql(db, people):
    for cp in (False, True):
        fast = await _gov_answers(db, people, cp)
        gov, db.gov = db.gov, None
        try:
            ref = await _gov_answers(db, people, cp)
        finally:
            db.gov = gov
        for k in ref:
            assert fast[k] == ref[k], (cp, k)
    return fast


def test_governance_index_matches_sql(db):
    """The in-memory governance index (ledger/governance.py) answers every governance query exactly
    like the SQL implementation, with and without the mempool overlay, through registrations, votes,
    pending governance txs, revokes and a rollback."""
    async def go():
        A = B.address_of(KA)
        inodes = [0x1100 + k for k in range(2)]
        validators = [0x2200 + k for k in range(3)]
        delegates = [0x3300 + k for k in range(5)]
        people_keys = inodes + validators + delegates
        people = [B.address_of(k) for k in people_keys]
        ts = [1_700_000_000]

        async def block(txs=()):
            ts[0] += 60  # one block per target interval: the difficulty stays at the start value
            return await devnet.mine_block(A, list(txs), ts=ts[0])

        async def push_and_mine(*txs):
            for t in txs:
                assert await db.add_pending_transaction(t), t.transaction_type
            await block(await db.get_pending_transactions_limit())

        for _ in range(500):
            await block()
        # funding in three txs (at most 255 inputs each), each admitted before the next is built
        for p in people[:len(inodes)]:
            assert await db.add_pending_transaction(await B.create_transaction(KA, p, '1100'))
        assert await db.add_pending_transaction(await B.create_transaction_to_send_multiple_wallet(
            KA, people[len(inodes):], ['150'] * len(validators) + ['40'] * len(delegates)))
        await block(await db.get_pending_transactions_limit())
        await push_and_mine(*[await B.create_stake_transaction(k, '10' if k in delegates else '12')
                              for k in people_keys])
        await push_and_mine(*[await B.create_inode_registration_transaction(k) for k in inodes],
                            *[await B.create_validator_registration_transaction(k) for k in validators])
        votes = []
        for j, k in enumerate(validators):
            votes.append(await B.create_voting_transaction(k, 3 + j, B.address_of(inodes[j % 2])))
        for j, k in enumerate(delegates):
            votes.append(await B.create_voting_transaction(k, 2 + j % 4, B.address_of(validators[j % 3])))
        await push_and_mine(*votes)
        await _compare_index_with_sql(db, people)
        active = await db.get_active_inodes()
        assert sorted(a['wallet'] for a in active) == sorted(B.address_of(k) for k in inodes)
        # pending governance state: a revoke and a second-round stake wait in the mempool
        assert await db.add_pending_transaction(await B.create_revoke_transaction(delegates[0],
                                                                                  B.address_of(validators[0])))
        tip = (await db.get_last_block())['id']
        await _compare_index_with_sql(db, people)
        # revokes confirmed, then rolled back
        await block(await db.get_pending_transactions_limit())
        await _compare_index_with_sql(db, people)
        await db.remove_blocks(tip + 1)
        manager.Manager.difficulty = None
        await _compare_index_with_sql(db, people)
        # the index equals one rebuilt from the tables
        rows = {t: dict(tab.rows) for t, tab in db.gov.tables.items()}
        db.gov.rebuild()
        assert rows == {t: dict(tab.rows) for t, tab in db.gov.tables.items()}
    asyncio.run(go())
