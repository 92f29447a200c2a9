"""Native bulk ledger writer (csrc/ledger_sql.cpp) — column binding, error mapping, transaction
membership, and equality with the ``sqlite3.executemany`` fallback through the native block path."""
import os
import sqlite3

import numpy as np
import pytest

from upow_amd.ledger.database import Database
from upow_amd.ops.native import lib


def test_probe_enabled_for_memory_and_file(tmp_path):
    mem = Database(':memory:', utxo_backend='host')
    assert mem.native_sql
    f = Database(str(tmp_path / 'ledger.sqlite3'), utxo_backend='host')
    assert f.native_sql
    fn, _, autocommit = lib().sql_probe(f.conn)
    assert os.path.realpath(fn) == os.path.realpath(str(tmp_path / 'ledger.sqlite3')) and autocommit == 1
    mem.close()
    f.close()


def test_probe_respects_env(monkeypatch):
    monkeypatch.setenv('UPOW_NATIVE_SQL', '0')
    assert not Database(':memory:', utxo_backend='host').native_sql


def test_column_kinds_and_order():
    L = lib()
    c = sqlite3.connect(':memory:', isolation_level=None)
    c.execute('CREATE TABLE t (h TEXT UNIQUE, i INTEGER, g TEXT, k TEXT, z INTEGER, nul TEXT)')
    raw = np.frombuffer(bytes(range(256)) * 2, dtype=np.uint8)[:40 * 4].copy()
    words = ['w0', None, 'w2']
    n = L.sql_executemany(c, 'INSERT INTO t VALUES (?, ?, ?, ?, ?, ?)',
                          [('hex32', raw, 40, 0), np.array([7, 8, 9, 10], np.int64),
                           ('gather', words, np.array([2, 0, 1, 2], np.int32)), 'const', 5, None], 4)
    assert n == 4 and c.total_changes == 4
    rows = c.execute('SELECT * FROM t ORDER BY rowid').fetchall()
    assert rows[0] == (bytes(raw[:32]).hex(), 7, 'w2', 'const', 5, None)
    assert rows[1][2] == 'w0' and rows[2][2] is None and rows[3][0] == bytes(raw[120:152]).hex()
    # text arena (the codec's form): blob + int64 offsets, as bytes or as an array
    c.execute('CREATE TABLE a (s TEXT)')
    blob, off = b'alphabetagamma', np.array([0, 5, 9, 14], np.int64)
    for offs in (off, off.tobytes()):
        assert L.sql_executemany(c, 'INSERT INTO a VALUES (?)', [('arena', blob, offs)], 3) == 3
    assert [r[0] for r in c.execute('SELECT s FROM a')] == ['alpha', 'beta', 'gamma'] * 2
    from upow_amd.ledger.database import _expand_col, arena_list
    assert arena_list((blob, off.tobytes())) == ['alpha', 'beta', 'gamma']
    assert _expand_col(('hex32', raw, 40, 0), 2) == [bytes(raw[:32]).hex(), bytes(raw[40:72]).hex()]
    with pytest.raises(IndexError):
        L.sql_executemany(c, 'INSERT INTO a VALUES (?)', [('arena', blob, np.array([0, 5, 99], np.int64))], 2)
    # explicit row order: the last row first
    c.execute('CREATE TABLE o (x INTEGER)')
    L.sql_executemany(c, 'INSERT INTO o VALUES (?)', [np.array([10, 20, 30], np.int64)], 3,
                      np.array([2, 0, 1], np.int64))
    assert [r[0] for r in c.execute('SELECT x FROM o ORDER BY rowid')] == [30, 10, 20]
    # deletes report their row changes; a missing key changes nothing
    d = L.sql_executemany(c, 'DELETE FROM o WHERE x = ?', [np.array([10, 99, 30], np.int64)], 3)
    assert d == 2
    # UNIQUE violations surface as sqlite3.IntegrityError (callers map it to UniqueViolationError)
    with pytest.raises(sqlite3.IntegrityError):
        L.sql_executemany(c, 'INSERT INTO t (h) VALUES (?)', [('hex32', raw, 40, 0)], 1)
    with pytest.raises(sqlite3.OperationalError):
        L.sql_executemany(c, 'INSERT INTO missing VALUES (?)', [1], 1)
    with pytest.raises(ValueError):
        L.sql_executemany(c, 'INSERT INTO o VALUES (?)', [np.array([1], np.int64)], 2)
    with pytest.raises(IndexError):
        L.sql_executemany(c, 'INSERT INTO t (g) VALUES (?)', [('gather', words, np.array([3], np.int32))], 1)
    with pytest.raises(TypeError):  # never reinterprets anything but a sqlite3.Connection
        L.sql_executemany(object(), 'INSERT INTO o VALUES (?)', [1], 1)


def test_native_writes_join_the_open_transaction():
    db = Database(':memory:', utxo_backend='host')
    assert db.native_sql
    db.conn.execute('CREATE TABLE x (v INTEGER)')
    with pytest.raises(RuntimeError):
        with db.transaction():
            db.bulk('INSERT INTO x VALUES (?)', [np.arange(5, dtype=np.int64)], 5)
            assert db._q1('SELECT COUNT(*) FROM x')[0] == 5
            raise RuntimeError('roll back')
    assert db._q1('SELECT COUNT(*) FROM x')[0] == 0  # rolled back with the Python-side BEGIN
    with db.transaction():
        db.bulk('INSERT INTO x VALUES (?)', [np.arange(3, dtype=np.int64)], 3)
    assert db._q1('SELECT COUNT(*) FROM x')[0] == 3


def test_small_outpoint_lookups_via_sql_match_index():
    """GPU-backend nodes answer a single tx's outpoint lookups from SQLite (no device round trip);
    the answer must equal the UTXO index's for every table, including absent and repeated keys."""
    import asyncio
    import random
    from decimal import Decimal

    from upow_amd import devnet
    from upow_amd.ledger import manager
    from upow_amd.ledger.database import OUTPUT_TABLES
    from upow_amd.ledger.utxo import TAG_BY_TABLE
    from upow_amd.wallet.builders import address_of

    async def go():
        db = await Database.create(utxo_backend='host')
        manager.Manager.difficulty = None
        manager.START_DIFFICULTY, saved = Decimal('1.0'), manager.START_DIFFICULTY
        try:
            for b in range(4):
                await devnet.mine_block(address_of(0xABC), ts=1_700_000_000 + 60 * b, device='cpu')
        finally:
            manager.START_DIFFICULTY = saved
        live = [(r[0], r[1]) for r in db._q('SELECT tx_hash, "index" FROM unspent_outputs')]
        rng = random.Random(3)
        for _ in range(40):
            req = rng.sample(live, min(len(live), rng.randint(0, 3))) + [('ef' * 32, rng.randint(0, 3))]
            req += req[:1]  # a repeated key
            rng.shuffle(req)
            for table in OUTPUT_TABLES:
                want = db.utxo.filter(req, TAG_BY_TABLE[table])
                db.utxo.backend_name = 'gpu'  # take the SQL branch
                try:
                    got = db._filter_outputs(table, req)
                finally:
                    db.utxo.backend_name = 'host'
                assert got == want, (table, req)
    asyncio.run(go())


def test_block_trace_file(tmp_path, monkeypatch):
    """UPOW_TRACE_FILE: one JSON line per validated block with the stage timings."""
    import asyncio
    import json
    from decimal import Decimal

    from upow_amd import devnet
    from upow_amd.ledger import manager
    from upow_amd.wallet.builders import address_of
    trace = tmp_path / 'blocks.jsonl'
    monkeypatch.setattr(manager, '_TRACE_PATH', str(trace))
    monkeypatch.setattr(manager, 'START_DIFFICULTY', Decimal('1.0'))

    async def go():
        await Database.create(utxo_backend='host')
        manager.Manager.difficulty = None
        for b in range(3):
            await devnet.mine_block(address_of(0x5EED), ts=1_700_000_000 + 60 * b, device='cpu')
    asyncio.run(go())
    recs = [json.loads(ln) for ln in trace.read_text().splitlines()]
    assert len(recs) == 3 and all(r['ok'] for r in recs)
    assert [r['height'] for r in recs] == [1, 2, 3] and all('ms' in r and 'stages_ms' in r for r in recs)
