"""Ledger file layout (ledger/database.py): ``transactions`` and ``unspent_outputs`` split over files of their
own by the first tx-hash byte, each materialised by its own writer thread; the layout recorded at creation;
ledgers in the layout from before the transactions split (table in the main file, two UTXO files) keep
working; the reference's ON DELETE CASCADE applied by hand across files on rollback."""
import asyncio
import os
import sqlite3
from decimal import Decimal

import pytest

from upow_amd import devnet
from upow_amd.ledger import manager
from upow_amd.ledger.database import Database, file_of, ledger_files
from upow_amd.wallet import builders

KEY_A = 0x3333333333333333333333333333333333333333333333333333333333333333
KEY_B = 0x4444444444444444444444444444444444444444444444444444444444444444


@pytest.fixture(autouse=True)
def _easy(monkeypatch):
    monkeypatch.setattr(manager, 'START_DIFFICULTY', Decimal('1.5'))
    monkeypatch.setenv('UPOW_SNAPSHOT', '0')
    manager.Manager.difficulty = None
    manager.cache.clear()


async def _grow(db, n_tx: int = 3):
    a, b = builders.address_of(KEY_A), builders.address_of(KEY_B)
    base = 1_700_000_000
    for k in range(3):
        await devnet.mine_block(a, ts=base + k + 1)
    txs = []
    for k in range(n_tx):
        tx = await builders.create_transaction(KEY_A, b, '0.25')
        assert await db.add_pending_transaction(tx)
        txs.append(tx)
    block_txs = await db.get_pending_transactions_limit()
    await devnet.mine_block(a, block_txs, ts=base + 10)
    return a, b, block_txs


@pytest.mark.parametrize('n_utxo,n_tx,mixed', [(4, 4, False), (5, 5, False), (6, 4, False), (2, 3, False),
                                                (2, 0, False), (10, 10, True), (3, 3, True)])
def test_layouts_apply_read_and_roll_back(tmp_path, monkeypatch, n_utxo, n_tx, mixed):
    """Separate layouts (each split table in files of its own) and mixed ones (UPOW_LEDGER_MIXED: every split
    file holds both tables for one hash range)."""
    monkeypatch.setenv('UPOW_LEDGER_MIXED', '1' if mixed else '0')
    if mixed:
        monkeypatch.setenv('UPOW_LEDGER_FILES', str(n_utxo))
    monkeypatch.setenv('UPOW_UTXO_FILES', str(n_utxo if not mixed else 5))
    monkeypatch.setenv('UPOW_TX_FILES', str(n_tx if not mixed else 5))
    path = str(tmp_path / 'ledger.sqlite3')

    async def go():
        db = await Database.create(path=path, utxo_backend='host')
        a, b, txs = await _grow(db)
        assert (len(db.utxo_schemas), len(db.tx_schemas)) == (n_utxo, n_tx)
        db.flush()
        # every row sits in the file its hash routes to; the view reads them all
        for k, sch in enumerate(db.tx_schemas):
            for (h,) in db._conn.execute(f'SELECT tx_hash FROM {sch}.transactions'):
                assert file_of(h, n_tx) == k
        for k, sch in enumerate(db.utxo_schemas):
            for (h,) in db._conn.execute(f'SELECT tx_hash FROM {sch}.unspent_outputs'):
                assert file_of(h, n_utxo) == k
        tip = await db.get_last_block()
        block = await db.get_block_transactions_hashes(tip['hash'])
        assert block[1:] == [t.hash() for t in txs]  # coinbase row first, then the block's order
        assert await db.get_address_balance(b) == Decimal('0.25') * len(txs)
        hist = await db.get_address_transactions(b)
        assert sorted(t.hash() for t in hist) == sorted(t.hash() for t in txs)
        nice = await db.get_nice_transaction(txs[0].hash())
        assert nice['block_hash'] == tip['hash']
        k12 = await db.get_unspent_outputs_hash()
        assert k12 == db.sql_unspent_outputs_hash()
        # rollback: the tx rows, their address rows and outputs go; the spent outputs come back
        await db.remove_blocks(tip['id'])
        db.flush()
        assert db._q1('SELECT COUNT(*) FROM transactions WHERE block_hash = ?', (tip['hash'],))[0] == 0
        gone = [t.hash() for t in txs]
        ph = ','.join('?' * len(gone))
        assert db._q1(f'SELECT COUNT(*) FROM address_transactions WHERE tx_hash IN ({ph})', gone)[0] == 0
        assert await db.get_address_balance(b) == 0
        assert await db.get_address_balance(a) == Decimal(18)
        assert db.utxo.set_hash(0) == db.sql_unspent_outputs_hash()
        db.close()
        assert db.mixed == mixed and len(db.writer.stats()['shards']) == 1 + n_utxo + (0 if mixed else n_tx)
        db.close()
        # reopened: the recorded layout wins over the environment
        monkeypatch.setenv('UPOW_TX_FILES', '1')
        monkeypatch.setenv('UPOW_LEDGER_MIXED', '0' if mixed else '1')
        db = await Database.create(path=path, utxo_backend='host')
        assert (len(db.utxo_schemas), len(db.tx_schemas), db.mixed) == (n_utxo, n_tx, mixed)
        assert await db.get_address_balance(a) == Decimal(18)
        db.close()
    asyncio.run(go())
    names = [os.path.basename(f) for f in ledger_files(path)]
    assert sum(n.startswith('ledger.sqlite3-tx') for n in names) == (0 if mixed else n_tx)
    assert sum(n.startswith('ledger.sqlite3-utxo') for n in names) == n_utxo
    if n_tx == 0:  # the pre-split layout: transactions in the main file
        c = sqlite3.connect(path)
        assert c.execute("SELECT COUNT(*) FROM sqlite_master WHERE name = 'transactions'").fetchone()[0] == 1
        c.close()


def test_layout_beyond_sqlite_attach_limit_is_refused(tmp_path, monkeypatch):
    # one ATTACH per split file; SQLite allows 10, so 8 + 8 must fail loudly at creation, not on ATTACH
    monkeypatch.setenv('UPOW_LEDGER_MIXED', '0')
    monkeypatch.setenv('UPOW_UTXO_FILES', '8')
    monkeypatch.setenv('UPOW_TX_FILES', '8')
    with pytest.raises(ValueError, match='at most 10'):
        asyncio.run(Database.create(path=str(tmp_path / 'ledger.sqlite3'), utxo_backend='host'))
    monkeypatch.setenv('UPOW_LEDGER_MIXED', '1')
    monkeypatch.setenv('UPOW_LEDGER_FILES', '11')
    with pytest.raises(ValueError, match='at most 10'):
        asyncio.run(Database.create(path=str(tmp_path / 'ledger2.sqlite3'), utxo_backend='host'))
