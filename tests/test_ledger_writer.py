"""Native ledger writer (csrc/ledger_writer.cpp): undo log retention across restarts and journal rotation,
rollback tombstones, fatal row-count mismatches, SQLITE_BUSY retry, queue backpressure, and the
durability watermark (a journal cut at the last synced offset reopens to a consistent ledger)."""
import asyncio
import os
import shutil
import sqlite3
import threading
import time
from decimal import Decimal

import numpy as np
import pytest

from upow_amd import devnet
from upow_amd.ops.native import lib
from upow_amd.ledger import manager
from upow_amd.ledger.database import UTXO_SUFFIXES, Database, ledger_files
from upow_amd.wallet import builders

KEY_A, KEY_B = 0x5151, 0x6262


def _writer(tmp_path, name='w', **kw):
    from upow_amd.ops.native import lib
    dbs = [str(tmp_path / f'{name}.db'), str(tmp_path / f'{name}.u1.db')]
    return lib().LedgerWriter(dbs, str(tmp_path / f'{name}.journal'), kw.pop('sync_mode', 1), 16, 8,
                              kw.pop('journal_max_bytes', 1 << 30), kw.pop('undo_keep', 600),
                              kw.pop('max_queue_bytes', 512 << 20), kw.pop('throttle_timeout_s', 300.0),
                              kw.pop('busy_timeout_ms', 5000)), dbs


def _meta(i: int) -> bytes:
    return i.to_bytes(8, 'little') * 16


def test_undo_log_retention_restart_and_tombstone(tmp_path):
    w, _ = _writer(tmp_path, undo_keep=50)
    for i in range(1, 301):
        w.submit([], _meta(i), i)
    st = w.stats()
    assert st['undo_blocks'] >= 50 and st['undo_pruned_segments'] >= 2
    assert st['undo_first_block'] <= 300 - 50 and st['undo_first_block'] > 1
    assert w.journal_meta(300) == _meta(300) and w.journal_meta(251) == _meta(251)
    assert w.journal_meta(1) is None
    w.forget_blocks_from(280)
    assert w.journal_meta(280) is None and w.journal_meta(279) == _meta(279)
    w.submit([], b'replaced', 280)
    w.close()
    w, _ = _writer(tmp_path, undo_keep=50)  # restart: tombstone honoured, newest record per block wins
    assert w.journal_meta(281) is None and w.journal_meta(280) == b'replaced' and w.journal_meta(279) == _meta(279)
    w.close()


def test_undo_survives_journal_rotation(tmp_path):
    w, dbs = _writer(tmp_path, journal_max_bytes=4096)
    blob = b'x' * 2048
    w.submit([lib().ledger_encode_stmt('CREATE TABLE IF NOT EXISTS t (x TEXT)', [], 1)], b'', -1)
    stmt = lib().ledger_encode_stmt('INSERT INTO t (x) VALUES (?)', [['y' * 2048]], 1)
    for i in range(1, 40):
        w.submit([stmt], _meta(i) + blob, i)
        w.wait(w.stats()['submitted'], -1, 30.0)
    st = w.stats()
    assert st['rotations'] >= 1
    assert all(w.journal_meta(i) == _meta(i) + blob for i in range(1, 40))
    w.close()


def test_row_count_mismatch_stops_writer(tmp_path):
    async def go():
        db = await Database.create(str(tmp_path / 'l.sqlite3'), utxo_backend='host')
        try:
            stmt = db.encode('DELETE FROM unspent_outputs WHERE tx_hash = ? AND "index" = ?',
                             [['00' * 32], np.array([0], np.int64)], 1, None, None, 1)
            db.submit_batch([stmt], {'unspent_outputs'})
            with pytest.raises(RuntimeError, match='1 rows changed|0 of 1 rows'):
                db.flush()
            st = db.writer.stats()
            assert st['failed'] and st['change_mismatches'] == 1
            with pytest.raises(RuntimeError, match='stopped after an error'):
                db.submit_batch([stmt], {'unspent_outputs'})
            from upow_amd.utils import metrics
            db.publish_writer_metrics()
            text = metrics.prometheus_text()
            assert 'upow_ledger_writer_failed 1' in text and 'upow_ledger_row_mismatches 1' in text
        finally:
            db.writer.close()
    asyncio.run(go())


def test_busy_file_is_retried_and_block_submit_is_throttled(tmp_path):
    w, dbs = _writer(tmp_path, max_queue_bytes=4096, throttle_timeout_s=0.4, busy_timeout_ms=20)
    stmt = lib().ledger_encode_stmt('CREATE TABLE IF NOT EXISTS t (x TEXT)', [], 1)
    w.submit([stmt], b'', -1)
    w.wait(w.stats()['submitted'], -1, 30.0)
    blocker = sqlite3.connect(dbs[0], isolation_level=None, timeout=1)
    blocker.execute('BEGIN IMMEDIATE')  # holds the write lock: the materialiser of file 0 gets SQLITE_BUSY
    ins = lib().ledger_encode_stmt('INSERT INTO t (x) VALUES (?)', [['y' * 3000]], 1)
    w.submit([ins], b'', -1)
    w.submit([ins], b'', -1)
    t0 = time.time()
    w.submit([ins], b'', 1)  # a block: file 0 lags by > 4 KB queued -> waits (bounded by the timeout)
    waited = time.time() - t0
    st = w.stats()
    assert st['throttle_waits'] >= 1 and waited >= 0.3
    assert st['queued_bytes'] > 0 and not st['failed']
    blocker.execute('COMMIT')
    blocker.close()
    w.wait(w.stats()['submitted'], -1, 60.0)  # the busy group was retried, not fatal
    st = w.stats()
    assert not st['failed'] and st['busy_retries'] >= 1
    assert sqlite3.connect(dbs[0]).execute('SELECT COUNT(*) FROM t').fetchone()[0] == 3
    w.close()


def test_journal_cut_at_synced_offset_reopens_consistent(tmp_path, monkeypatch):
    """Power loss model: only the fdatasync'd journal prefix survives. With the default 'block' mode every
    applied block is inside it; a later, unsynced mempool admission may be lost. Reopening the surviving
    files replays the journal into SQL and reaches the same tip and UTXO-set hash (K12) as before."""
    monkeypatch.setattr(manager, 'START_DIFFICULTY', Decimal('1.5'))
    monkeypatch.setenv('UPOW_SNAPSHOT', '0')
    monkeypatch.delenv('UPOW_JOURNAL_SYNC', raising=False)
    manager.Manager.difficulty = None
    manager.cache.clear()
    src = tmp_path / 'src'
    dst = tmp_path / 'dst'
    src.mkdir()
    dst.mkdir()

    async def build():
        db = await Database.create(str(src / 'ledger.sqlite3'), utxo_backend='host')
        a, b = builders.address_of(KEY_A), builders.address_of(KEY_B)
        base = 1_700_000_000
        for k in range(3):
            await devnet.mine_block(a, ts=base + k)
        tx = await builders.create_transaction(KEY_A, b, '2.5')
        assert await db.add_pending_transaction(tx)
        late = await builders.create_transaction(KEY_A, b, '1')  # another input (the first one is pending)
        db.flush()
        db.writer.set_paused(True)  # SQL stops at block 3; blocks 4-5 live only in the journal
        await devnet.mine_block(a, [tx], ts=base + 10)
        await devnet.mine_block(a, ts=base + 11)
        tip = await db.get_last_block()
        k12 = db.utxo.set_hash(0)
        assert await db.add_pending_transaction(late)  # journaled after the last block, not synced
        st = db.writer.stats()
        assert st['sync_mode'] == 3 and st['synced_bytes'] < st['journal_bytes']
        # the crash: copy the files as they are on disk now, cutting the journal at the synced offset
        s0, d0 = str(src / 'ledger.sqlite3'), str(dst / 'ledger.sqlite3')
        for s_ in ledger_files(s0):
            d_ = d0 + s_[len(s0):]
            for sfx in ('', '-wal'):
                if os.path.exists(s_ + sfx):
                    shutil.copy(s_ + sfx, d_ + sfx)
        with open(str(dst / 'ledger.sqlite3') + '.journal', 'r+b') as f:
            f.truncate(st['synced_bytes'])
        db.writer.set_paused(False)
        db.close()
        return tip, k12, late.hash()

    tip, k12, late_hash = asyncio.run(build())

    async def reopen():
        db = await Database.create(str(dst / 'ledger.sqlite3'), utxo_backend='host')
        try:
            assert db.writer.stats()['replayed'] >= 2
            assert (await db.get_last_block())['hash'] == tip['hash']
            assert db.utxo.set_hash(0) == k12 == db.sql_unspent_outputs_hash()
            assert await db.get_pending_transaction(late_hash) is None
        finally:
            db.close()
    asyncio.run(reopen())


def _crc32c_ref(data: bytes, crc: int = 0) -> int:
    table = []
    for i in range(256):
        c = i
        for _ in range(8):
            c = (c >> 1) ^ (0x82F63B78 if c & 1 else 0)
        table.append(c)
    crc ^= 0xFFFFFFFF
    for b in data:
        crc = (crc >> 8) ^ table[(crc ^ b) & 0xFF]
    return crc ^ 0xFFFFFFFF


def test_crc32c_three_stream_path_matches_reference():
    # the record checksum switches to three interleaved crc32 streams at 3 x 8 KiB: sizes around every
    # boundary of that path (and a multi-step buffer with a ragged tail) against the bitwise definition
    rng = np.random.default_rng(7)
    assert lib().crc32c(b'123456789') == 0xE3069283  # the CRC-32C check value
    for n in (0, 1, 7, 8, 24575, 24576, 24577, 49152 + 13, 3 * 24576 + 4095):
        data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert lib().crc32c(data) == _crc32c_ref(data), n


def test_deferred_block_record_is_durable_and_replayed(tmp_path):
    # a block record handed to the journal I/O thread (sync=False): durable() returns once it is written,
    # published, fdatasync'd and its undo data stored; a later inline record keeps the sequence order
    w, dbs = _writer(tmp_path, sync_mode=3)
    w.submit([lib().ledger_encode_stmt('CREATE TABLE IF NOT EXISTS t (x TEXT)', [], 1)], b'', -1)
    ins = lib().ledger_encode_stmt('INSERT INTO t (x) VALUES (?)', [['b' * 100_000]], 1)
    seq = w.submit([ins, ins], _meta(7), 7, False)
    seq2 = w.submit([lib().ledger_encode_stmt('INSERT INTO t (x) VALUES (?)', [['after']], 1)], b'', -1)
    assert seq2 == seq + 1
    w.durable(seq)
    st = w.stats()
    assert st['synced'] >= seq and w.journal_meta(7) == _meta(7)
    w.wait(seq2)
    w.close()
    rows = [r[0] for r in sqlite3.connect(dbs[0]).execute('SELECT x FROM t ORDER BY rowid')]
    assert rows == ['b' * 100_000, 'b' * 100_000, 'after']


def test_hexarena_column_binds_lowercase_hex(tmp_path):
    # ('hexarena', blob, offsets[, sel]): raw bytes in the journal, lowercase hex text in SQL
    w, dbs = _writer(tmp_path)
    w.submit([lib().ledger_encode_stmt('CREATE TABLE IF NOT EXISTS t (i INTEGER, h TEXT)', [], 1)], b'', -1)
    rows = [b'', b'\x00\xff', bytes(range(200))]
    blob = b''.join(rows)
    off = np.cumsum([0] + [len(r) for r in rows]).astype(np.int64)
    ins = 'INSERT INTO t (i, h) VALUES (?, ?)'
    seq = w.submit([lib().ledger_encode_stmt(ins, [np.arange(3, dtype=np.int64), ('hexarena', blob, off.tobytes())], 3),
                    lib().ledger_encode_stmt(ins, [np.array([7, 8], dtype=np.int64),
                                                   ('hexarena', blob, off.tobytes(), np.array([2, 1], np.int64))], 2)],
                   b'', -1)
    w.wait(seq)
    w.close()
    got = sqlite3.connect(dbs[0]).execute('SELECT i, h FROM t ORDER BY rowid').fetchall()
    assert got == [(0, ''), (1, '00ff'), (2, bytes(range(200)).hex()), (7, bytes(range(200)).hex()), (8, '00ff')]


@pytest.mark.parametrize('early', ['1', '0'])
def test_block_sized_record_is_written_in_slices_and_replays(tmp_path, monkeypatch, early):
    """A record of at least 1 MB (a block's) is written body first, in 1 MB slices whose writeback starts at
    once, with its checksum computed alongside, and its header last. Replayed from the journal alone (fresh
    database files) it gives the same rows; cut anywhere inside it (a crash before the header or mid-body),
    recovery drops it and keeps the records before it."""
    monkeypatch.setenv('UPOW_JOURNAL_EARLY_WRITEBACK', early)
    w, dbs = _writer(tmp_path, sync_mode=3)
    w.submit([lib().ledger_encode_stmt('CREATE TABLE IF NOT EXISTS t (x TEXT)', [], 1)], b'', -1)
    rng = np.random.default_rng(5)
    vals = [rng.integers(97, 123, n, dtype=np.uint8).tobytes().decode() for n in (700_000, 1_300_001, 5, 999_999)]
    parts = [lib().ledger_encode_stmt('INSERT INTO t (x) VALUES (?)', [[v]], 1) for v in vals]
    first = w.submit([parts[2]], b'', -1)
    w.durable(first)
    before = w.stats()['journal_bytes']
    seq = w.submit(parts, _meta(9), 9, False)  # the I/O thread's split write (3 MB over four parts)
    w.durable(seq)
    seq2 = w.submit(parts[::-1], _meta(10), 10)  # the inline path, split too
    w.durable(seq2)
    w.wait(seq2)
    st = w.stats()
    w.close()
    journal = str(tmp_path / 'w.journal')
    want = [vals[2]] + vals + vals[::-1]
    assert [r[0] for r in sqlite3.connect(dbs[0]).execute('SELECT x FROM t ORDER BY rowid')] == want
    assert st['io_records'] >= 1 and st['io_write_s'] > 0
    size = os.path.getsize(journal)

    def replay(cut_at=None, zero_header_at=None):
        d = tmp_path / f'replay{cut_at}{zero_header_at}'
        d.mkdir()
        shutil.copy(journal, d / 'w.journal')
        if cut_at is not None:
            with open(d / 'w.journal', 'r+b') as f:
                f.truncate(cut_at)
        if zero_header_at is not None:  # the body is on disk, its header is not yet
            with open(d / 'w.journal', 'r+b') as f:
                f.seek(zero_header_at)
                f.write(bytes(48))
        w2, dbs2 = _writer(d, sync_mode=3)
        w2.wait(w2.stats()['submitted'], -1, 60.0)
        rows = [r[0] for r in sqlite3.connect(dbs2[0]).execute('SELECT x FROM t ORDER BY rowid')]
        jb = w2.stats()['journal_bytes']
        w2.close()
        return rows, jb

    assert replay() == (want, size)
    rows, jb = replay(cut_at=before + 1_500_000)  # mid-body of the deferred record
    assert rows == [vals[2]] and jb == before
    rows, jb = replay(zero_header_at=before)
    assert rows == [vals[2]] and jb == before
