"""Rollback from undo data (reference upow/database.py:146-169 remove_blocks, upow/node/main.py:167-185
500-block fork window): the UTXO index and the governance index are rolled back from the undo log —
no rebuild — and must equal a fresh rebuild from the SQL tables record for record, including after
rolling back governance spends (votes, revokes, unstakes) and across journal rotations."""
import asyncio
from decimal import Decimal

import pytest

from upow_amd import devnet
from upow_amd.ledger import manager
from upow_amd.ledger.database import Database
from upow_amd.wallet import builders as B

KA = 0xA7
KV, KI, KD = 0xB7, 0xC7, 0xD7


@pytest.fixture
def fast_chain(monkeypatch):
    monkeypatch.setattr(manager, 'START_DIFFICULTY', Decimal('1.0'))
    manager.Manager.difficulty = None
    manager.cache.clear()


def _index_state(db):
    recs, pay = db.utxo.records_payload()
    return recs.tobytes(), pay.tobytes()


def _assert_equals_rebuild(db):
    before = _index_state(db)
    gov = {t: dict(tab.rows) for t, tab in db.gov.tables.items()}
    k12 = db.utxo.set_hash(0)
    db._rebuild_utxo_index()  # also rebuilds the governance index from SQL
    assert _index_state(db) == before
    assert {t: dict(tab.rows) for t, tab in db.gov.tables.items()} == gov
    assert k12 == db.sql_unspent_outputs_hash() == db.utxo.set_hash(0)


def test_rollback_of_governance_spends_matches_rebuild(fast_chain):
    async def go():
        db = await Database.create(utxo_backend='host')
        try:
            A, V, I, D = (B.address_of(k) for k in (KA, KV, KI, KD))
            ts = [1_700_000_000]

            async def block(txs=()):
                ts[0] += 60
                return await devnet.mine_block(A, list(txs), ts=ts[0])

            async def push_and_mine(*txs):
                for t in txs:
                    assert await db.add_pending_transaction(t), t.transaction_type
                await block(await db.get_pending_transactions_limit())

            for _ in range(240):
                await block()
            await push_and_mine(await B.create_transaction_to_send_multiple_wallet(KA, [I, V, D], ['1100', '150', '50']))
            await push_and_mine(await B.create_stake_transaction(KI, '10'), await B.create_stake_transaction(KV, '10'),
                                await B.create_stake_transaction(KD, '10'))
            await push_and_mine(await B.create_inode_registration_transaction(KI),
                                await B.create_validator_registration_transaction(KV))
            first_gov = (await db.get_last_block())['id'] + 1
            await push_and_mine(await B.create_voting_transaction(KV, 5, I), await B.create_voting_transaction(KD, 7, V))
            await push_and_mine(await B.create_revoke_transaction(KV, I), await B.create_revoke_transaction(KD, V))
            await push_and_mine(await B.create_unstake_transaction(KD))
            assert await db.get_address_stake(D) == 0
            # roll back the vote, revoke and unstake blocks: their spent governance/stake outputs come back
            # as plain unstaked UTXOs in SQL (the reference's add_unspent_outputs), and in the index too
            await db.remove_blocks(first_gov)
            manager.Manager.difficulty = None
            assert db.last_rollback_undo is True
            _assert_equals_rebuild(db)
            # the chain continues cleanly on top
            await block()
            _assert_equals_rebuild(db)
        finally:
            db.close()
    asyncio.run(go())


@pytest.mark.slow
def test_rollback_300_blocks_across_journal_rotation(fast_chain, monkeypatch, tmp_path):
    monkeypatch.setenv('UPOW_JOURNAL_MAX_MB', '1')
    monkeypatch.setenv('UPOW_SNAPSHOT', '0')

    async def go():
        db = await Database.create(str(tmp_path / 'ledger.sqlite3'), utxo_backend='host')
        try:
            A, Bd = B.address_of(KA), B.address_of(KV)
            ts = [1_700_000_000]

            async def block(txs=()):
                ts[0] += 60
                return await devnet.mine_block(A, list(txs), ts=ts[0])

            for _ in range(20):
                await block()
            snapshot_at = None
            for k in range(330):
                if k == 30:
                    db.flush()
                    snapshot_at = ((await db.get_last_block())['id'], _index_state(db), db.utxo.set_hash(0))
                # one transfer per block (spends an older output, so every undo record has both halves)
                tx = await B.create_transaction(KA, Bd, '0.5')
                assert await db.add_pending_transaction(tx)
                await block(await db.get_pending_transactions_limit())
                db.flush()
            st = db.writer.stats()
            assert st['rotations'] >= 1, st['journal_bytes']
            tip = (await db.get_last_block())['id']
            height, state, k12 = snapshot_at
            assert tip - height == 300
            await db.remove_blocks(height + 1)
            manager.Manager.difficulty = None
            assert db.last_rollback_undo is True
            assert (await db.get_last_block())['id'] == height
            assert _index_state(db) == state and db.utxo.set_hash(0) == k12
            _assert_equals_rebuild(db)
        finally:
            db.close()
    asyncio.run(go())


def test_recent_block_rows_match_sql_and_follow_a_rollback(fast_chain):
    """The recent-rows cache that serves the retarget's block lookup (Database._recent_rows) returns the row
    SQL holds, and a rollback drops the rows it removed."""
    async def go():
        db = await Database.create(utxo_backend='host')
        try:
            A = B.address_of(KA)
            for k in range(40):
                await devnet.mine_block(A, [], ts=1_700_000_000 + 60 * (k + 1))
            assert 1 in db._recent_rows and 40 in db._recent_rows
            cached = {i: await db.get_block_by_id(i) for i in (1, 20, 39, 40)}
            db._recent_rows.clear()
            for i, row in cached.items():
                assert row == await db.get_block_by_id(i), i
            for k in range(40, 45):
                await devnet.mine_block(A, [], ts=1_700_000_000 + 60 * (k + 1))
            await db.remove_blocks(43)
            assert all(i < 43 for i in db._recent_rows)
            assert await db.get_block_by_id(43) is None
            assert (await db.get_block_by_id(42))['id'] == 42
        finally:
            db.close()
    asyncio.run(go())
