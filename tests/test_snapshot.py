"""UTXO-index checkpoint/resume (ledger/snapshot.py), index-side K12 hash, and the ledger lock."""
import asyncio
from decimal import Decimal

import pytest

from upow_amd import devnet
from upow_amd.ledger import manager, snapshot
from upow_amd.ledger.database import Database
from upow_amd.wallet.builders import address_of, create_stake_transaction, create_transaction

KEY = 0x5A5A


@pytest.fixture(autouse=True)
def _low_difficulty(monkeypatch):
    monkeypatch.setattr(manager, 'START_DIFFICULTY', Decimal('1.0'))


async def _chain(path, blocks=4):
    db = await Database.create(path=str(path), utxo_backend='host')
    manager.Manager.difficulty = None
    addr = address_of(KEY)
    for b in range(blocks):
        await devnet.mine_block(addr, ts=1_700_000_000 + 60 * b, device='cpu')
    tx = await create_transaction(KEY, address_of(0x77), '2.5')
    await db.add_pending_transaction(tx)
    st = await create_stake_transaction(KEY, '1')
    await db.add_pending_transaction(st)
    await devnet.mine_block(addr, [tx, st], ts=1_700_000_000 + 60 * blocks, device='cpu')
    return db


def test_snapshot_roundtrip_and_stale_fallback(tmp_path):
    async def go():
        path = tmp_path / 'ledger.sqlite3'
        db = await _chain(path)
        sql_hash = await db.get_unspent_outputs_hash()
        assert db.utxo.set_hash() == sql_hash  # index-side K12 == SQL K12
        hdr = snapshot.save(db)
        assert hdr['height'] == 5 and hdr['utxo_hash'] == sql_hash and hdr['count'] == len(db.utxo)
        db.close()
        db2 = await Database.create(path=str(path), utxo_backend='host')
        assert db2.utxo_source == 'snapshot'
        assert db2.utxo.set_hash() == sql_hash and snapshot.verify(db2)['ok']
        # a block after the snapshot makes it stale -> rebuild from SQL
        await devnet.mine_block(address_of(KEY), ts=1_700_000_000 + 60 * 9, device='cpu')
        db2.close()
        db3 = await Database.create(path=str(path), utxo_backend='host')
        assert db3.utxo_source == 'sql' and snapshot.verify(db3)['ok']
        snapshot.save(db3)
        db3.close()
        # corrupt payload -> rejected
        raw = bytearray(open(snapshot.default_path(db3), 'rb').read())
        raw[-3] ^= 0xFF
        open(snapshot.default_path(db3), 'wb').write(bytes(raw))
        db4 = await Database.create(path=str(path), utxo_backend='host')
        assert db4.utxo_source == 'sql' and snapshot.verify(db4)['ok']
        db4.close()
    asyncio.run(go())


def test_periodic_snapshot_is_written_off_the_block_path(tmp_path, monkeypatch):
    """The block path's periodic snapshot (manager._maybe_snapshot) only dumps the index; the sort, K12 and file
    write run on the snapshot thread. The file it leaves equals a synchronous save's, byte for byte, and the
    ledger restarts from it."""
    monkeypatch.setattr(manager, 'SNAPSHOT_EVERY', 5)
    monkeypatch.setattr(manager, 'SNAPSHOT_ASYNC', True)

    async def go():
        path = tmp_path / 'ledger.sqlite3'
        db = await _chain(path)  # block 5 takes the periodic snapshot
        hdr = snapshot.wait_pending(60, snapshot.default_path(db))
        assert hdr is not None and hdr['height'] == 5 and hdr['utxo_hash'] == await db.get_unspent_outputs_hash()
        bg = open(snapshot.default_path(db), 'rb').read()
        sync_hdr = snapshot.save(db)
        assert sync_hdr == hdr and open(snapshot.default_path(db), 'rb').read() == bg
        db.close()
        db2 = await Database.create(path=str(path), utxo_backend='host')
        assert db2.utxo_source == 'snapshot' and snapshot.verify(db2)['ok']
        db2.close()
    asyncio.run(go())


def test_verify_detects_index_drift(tmp_path):
    async def go():
        db = await _chain(tmp_path / 'l.sqlite3', blocks=2)
        assert snapshot.verify(db)['ok']
        db.utxo.erase_records(db.utxo.records()[:1])  # the index drops an outpoint SQL still has
        rep = snapshot.verify(db)
        assert not rep['ok'] and rep['mismatched_tables']
        db.close()
    asyncio.run(go())


def test_concurrent_blocks_at_same_height_serialised(tmp_path):
    async def go():
        db = await _chain(tmp_path / 'c.sqlite3', blocks=2)
        addr = address_of(KEY)
        a = await devnet.mine_header(addr, [], ts=1_700_000_000 + 600, device='cpu')
        b = await devnet.mine_header(addr, [], ts=1_700_000_000 + 601, device='cpu')
        res = await asyncio.gather(manager.create_block(a, []), manager.create_block(b, []))
        assert sorted(res) == [False, True]
        assert await db.get_next_block_id() == 5
        db.close()
    asyncio.run(go())


def test_lazy_address_index_follows_rollback(tmp_path):
    async def go():
        db = await _chain(tmp_path / 'a.sqlite3', blocks=3)
        dest = address_of(0x77)
        assert len(await db.get_address_transactions(dest)) == 1  # catch-up happens on query
        assert db._address_index_height() == 4
        tx = await create_transaction(KEY, dest, '0.5')
        await devnet.mine_block(address_of(KEY), [tx], ts=1_700_000_000 + 60 * 8, device='cpu')
        # a caught-up index follows the chain inside each block's journal batch (materialiser thread)
        assert db._address_index_height() == 5
        assert len(await db.get_address_transactions(dest)) == 2 and db._address_index_height() == 5
        await db.remove_blocks(5)
        assert db._address_index_height() == 4
        assert len(await db.get_address_transactions(dest)) == 1
        n = db._q1('SELECT COUNT(*) FROM address_transactions')[0]
        assert db.index_addresses() == 0 and db._q1('SELECT COUNT(*) FROM address_transactions')[0] == n
        db.close()
    asyncio.run(go())
