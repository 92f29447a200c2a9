"""Crash consistency of a file-backed ledger: a node process applying full blocks (native block path,
WAL + background checkpoints, periodic UTXO snapshots) is SIGKILLed at an arbitrary point. Reopening
the ledger must give a chain of whole blocks only, an UTXO index equal to the SQL UTXO set (K12 hash
on both sides) and a snapshot that is either valid for the tip or refused."""
import os
import random
import signal
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TXS = 60
BLOCKS = 14

WRITER = r'''
import asyncio, hashlib, sys
sys.path.insert(0, sys.argv[2])
from upow_amd import bench_verify, devnet
from upow_amd.constants import START_DIFFICULTY
from upow_amd.ledger import fastpath
from upow_amd.models.block import get_transactions_merkle_tree

async def main(path, n_blocks, n_txs, pause):
    db, addr, blocks, base_ts = await bench_verify._setup(n_blocks, n_txs, 99, 'host', 'cpu', ledger_path=path)
    prev = (await db.get_last_block())['hash']
    print('ready', (await db.get_last_block())['id'], flush=True)
    if pause:  # committed to the journal, never materialised: the kill lands before SQL catch-up
        db.flush()
        db.writer.set_paused(True)
    for b, txs in enumerate(blocks):
        content = devnet.mine_header_raw(prev, addr, get_transactions_merkle_tree(txs), base_ts + 10 + b,
                                         START_DIFFICULTY, device='cpu')
        assert await fastpath.create_block_from_hex(content, txs)
        assert fastpath.last_path == 'native'
        prev = hashlib.sha256(bytes.fromhex(content)).hexdigest()
        print('applied', b, flush=True)
    print('done', flush=True)

asyncio.run(main(sys.argv[1], int(sys.argv[3]), int(sys.argv[4]), sys.argv[5] == 'pause'))
'''


def _run_and_kill(tmp_path, kill_after: int, delay: float, pause: bool = False) -> str:
    path = str(tmp_path / 'ledger.sqlite3')
    env = dict(os.environ, UPOW_START_DIFFICULTY='1.5', UPOW_SNAPSHOT_EVERY='3', UPOW_DISABLE_GPU='1',
               UPOW_WAL_CHECKPOINT_PERIOD='0.05')
    p = subprocess.Popen([sys.executable, '-c', WRITER, path, ROOT, str(BLOCKS), str(TXS),
                          'pause' if pause else 'run'], env=env,
                         stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True)
    try:
        applied = -1
        deadline = time.time() + 240
        while applied < kill_after and time.time() < deadline:
            line = p.stdout.readline()
            if not line:
                break
            if line.startswith('applied'):
                applied = int(line.split()[1])
        assert applied >= kill_after, f'writer stopped early at block {applied}'
        time.sleep(delay)  # land somewhere inside the next block's validation / writes / commit
        p.send_signal(signal.SIGKILL)
        p.wait(timeout=30)
    finally:
        if p.poll() is None:
            p.kill()
    return path


@pytest.mark.parametrize('kill_after,delay', [(2, 0.0), (4, 0.03), (6, 0.11)])
def test_sigkill_mid_chain_recovers_whole_blocks(tmp_path, kill_after, delay):
    random.seed(kill_after)
    path = _run_and_kill(tmp_path, kill_after, delay)
    import asyncio

    from upow_amd.ledger import snapshot
    from upow_amd.ledger.database import Database

    async def check():
        db = Database(path, utxo_backend='host')
        try:
            tip = db._tip_id()
            # genesis + funding + at least the blocks reported as applied
            assert tip >= 2 + kill_after + 1
            # whole blocks only: every spending block has its coinbase + all of its txs
            counts = db._q('SELECT b.id, COUNT(t.tx_hash) FROM blocks b LEFT JOIN transactions t '
                           'ON t.block_hash = b.hash WHERE b.id > 2 GROUP BY b.id')
            assert counts and all(c == TXS + 1 for _, c in counts), counts
            assert len(counts) == tip - 2
            # referential integrity of the output tables
            orphans = db._q1('SELECT COUNT(*) FROM unspent_outputs u LEFT JOIN transactions t '
                             'ON t.tx_hash = u.tx_hash WHERE t.tx_hash IS NULL')[0]
            assert orphans == 0
            # the UTXO index (snapshot-restored or rebuilt) equals the SQL UTXO set
            assert db.utxo.set_hash() == db.sql_unspent_outputs_hash()
            assert snapshot.verify(db)['ok']
            # each spending block spent exactly its 2 * TXS funding outputs and created 2 * TXS + 1
            n_unspent = db._q1('SELECT COUNT(*) FROM unspent_outputs')[0]
            n_blocks = tip - 2
            funding_outputs = BLOCKS * TXS * 2
            assert n_unspent == 2 + funding_outputs + n_blocks * 1  # genesis/funding coinbases + block coinbases
            return tip
        finally:
            db.close()

    asyncio.run(check())


def test_sigkill_between_journal_append_and_sql_catch_up(tmp_path):
    """The materialiser is held back, so every block after the setup is only in the journal (and the
    HBM/host index) when the process dies. Reopening must re-apply the journal to the tables: the tip
    includes every block reported as applied, and the rebuilt index hashes like the SQL UTXO set."""
    kill_after = 3
    path = _run_and_kill(tmp_path, kill_after, 0.0, pause=True)
    import asyncio

    from upow_amd.ledger.database import Database

    async def check():
        db = Database(path, utxo_backend='host')
        try:
            assert db.writer.stats()['replayed'] >= kill_after + 1
            tip = db._tip_id()
            assert tip >= 2 + kill_after + 1
            counts = db._q('SELECT b.id, COUNT(t.tx_hash) FROM blocks b LEFT JOIN transactions t '
                           'ON t.block_hash = b.hash WHERE b.id > 2 GROUP BY b.id')
            assert len(counts) == tip - 2 and all(c == TXS + 1 for _, c in counts), counts
            assert db.utxo.set_hash() == db.sql_unspent_outputs_hash()
            n_unspent = db._q1('SELECT COUNT(*) FROM unspent_outputs')[0]
            assert n_unspent == 2 + BLOCKS * TXS * 2 + (tip - 2)
        finally:
            db.close()
        # a second open finds nothing left to replay
        db2 = Database(path, utxo_backend='host')
        try:
            assert db2.writer.stats()['replayed'] == 0 and db2._tip_id() == tip
        finally:
            db2.close()

    asyncio.run(check())


def test_single_utxo_file_ledger_is_split_on_open(tmp_path, monkeypatch):
    """A ledger written with one UTXO file (before the 00-7f / 80-ff split) opens with the rows of the
    high half moved to the second file (row ids kept), the same UTXO set and K12 hash, and keeps
    applying blocks. (Built in the layout of that era: transactions in the main file, two UTXO files.)"""
    monkeypatch.setenv('UPOW_LEDGER_MIXED', '0')
    monkeypatch.setenv('UPOW_UTXO_FILES', '2')
    monkeypatch.setenv('UPOW_TX_FILES', '0')
    import asyncio
    import sqlite3
    sys.path.insert(0, ROOT)
    from upow_amd import bench_verify
    from upow_amd.ledger.database import Database

    path = str(tmp_path / 'ledger.sqlite3')

    async def build():
        db, *_ = await bench_verify._setup(2, 40, 7, 'host', 'cpu', ledger_path=path)
        rows = sorted(tuple(r) for r in db._q('SELECT rowid, tx_hash, "index", address, is_stake FROM unspent_outputs'))
        h = db.sql_unspent_outputs_hash()
        db.close()
        return rows, h
    rows, h = asyncio.run(build())
    assert any(r[1] >= '8' for r in rows) and any(r[1] < '8' for r in rows)
    # fold the second file back into the first: the layout of a ledger from before the split
    c = sqlite3.connect(path + '-utxo', isolation_level=None)
    c.execute('ATTACH DATABASE ? AS hi', (path + '-utxo2',))
    c.execute('INSERT INTO unspent_outputs (rowid, tx_hash, "index", address, is_stake) '
              'SELECT rowid, tx_hash, "index", address, is_stake FROM hi.unspent_outputs')
    c.execute('DETACH DATABASE hi')
    c.close()
    for sfx in ('', '-wal', '-shm'):
        if os.path.exists(path + '-utxo2' + sfx):
            os.remove(path + '-utxo2' + sfx)

    async def reopen():
        db = await Database.create(path=path, utxo_backend='host')
        got = sorted(tuple(r) for r in db._q('SELECT rowid, tx_hash, "index", address, is_stake FROM unspent_outputs'))
        hi = db._q1("SELECT COUNT(*) FROM utxo.unspent_outputs WHERE tx_hash >= '8'")[0]
        lo2 = db._q1("SELECT COUNT(*) FROM utxo2.unspent_outputs WHERE tx_hash < '8'")[0]
        ok = (got == rows, hi, lo2, db.sql_unspent_outputs_hash() == h, h == db.utxo.set_hash())
        nxt = db._utxo_next_rowid
        db.close()
        return ok, nxt, len(got)
    ok, nxt, n_got = asyncio.run(reopen())
    assert ok == (True, 0, 0, True, True), (ok, n_got, len(rows))
    assert nxt == max(r[0] for r in rows) + 1


SYNCER = r'''
import asyncio, hashlib, json, sys
sys.path.insert(0, sys.argv[3])
from upow_amd import bench_verify, devnet
from upow_amd.constants import START_DIFFICULTY
from upow_amd.ledger import fastpath, manager, pagesync
from upow_amd.models.block import get_transactions_merkle_tree

async def main(src_path, dst_path, n_blocks, n_txs, out):
    base_ts = 1_700_000_000
    src, addr, blocks, _ = await bench_verify._setup(n_blocks, n_txs, 99, 'host', 'cpu', ledger_path=src_path,
                                                     base_ts=base_ts)
    prev = (await src.get_last_block())['hash']
    for b, txs in enumerate(blocks):
        manager.Manager.difficulty = None
        content = devnet.mine_header_raw(prev, addr, get_transactions_merkle_tree(txs), base_ts + 60 * (b + 2),
                                         START_DIFFICULTY, device='cpu')
        assert await fastpath.create_block_from_hex(content, txs)
        prev = hashlib.sha256(bytes.fromhex(content)).hexdigest()
    page = await src.get_blocks(3, n_blocks)
    with open(out, 'w') as f:
        json.dump({'page': page, 'utxo': src.sql_unspent_outputs_hash(), 'tip': prev}, f, default=str)
    src.close()
    dst, *_ = await bench_verify._setup(n_blocks, n_txs, 99, 'host', 'cpu', ledger_path=dst_path, base_ts=base_ts,
                                        make_blocks=False)
    orig = fastpath.create_block_from_hex

    async def traced(*a, **kw):
        ok = await orig(*a, **kw)
        print('applied', dst._tip_id(), flush=True)
        return ok
    fastpath.create_block_from_hex = traced
    print('syncing', flush=True)
    assert await pagesync.create_blocks(page)
    print('done', flush=True)

asyncio.run(main(sys.argv[1], sys.argv[2], int(sys.argv[4]), int(sys.argv[5]), sys.argv[6]))
'''


@pytest.mark.parametrize('kill_at', [5, 9])
def test_sigkill_mid_sync_page_resumes_at_the_last_durable_block(tmp_path, kill_at, monkeypatch):
    """A page-batched sync (ledger/pagesync.py: one fdatasync for the whole page, deferred index writes) is
    SIGKILLed in the middle of its page. Reopening gives whole blocks only (up to the last record the journal
    writer had written; any of the page's blocks, since none is promised durable before the page ends) and an
    index equal to the SQL UTXO set; syncing the rest of the page from the reopened tip (what the node does:
    fetch from its next block id) ends in the source chain's exact state."""
    import asyncio
    import json
    n_blocks = 14
    src, dst, out = str(tmp_path / 'src.sqlite3'), str(tmp_path / 'dst.sqlite3'), str(tmp_path / 'page.json')
    env = dict(os.environ, UPOW_START_DIFFICULTY='1.5', UPOW_DISABLE_GPU='1', UPOW_SYNC_CHUNK='4',
               UPOW_WAL_CHECKPOINT_PERIOD='0.05', UPOW_SNAPSHOT_EVERY='3')
    p = subprocess.Popen([sys.executable, '-c', SYNCER, src, dst, ROOT, str(n_blocks), str(TXS), out], env=env,
                         stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True)
    try:
        tip = 0
        deadline = time.time() + 240
        while tip < kill_at and time.time() < deadline:
            line = p.stdout.readline()
            if not line:
                break
            if line.startswith('applied'):
                tip = int(line.split()[1])
        assert tip >= kill_at, f'syncer stopped early at block {tip}'
        p.send_signal(signal.SIGKILL)
        p.wait(timeout=30)
    finally:
        if p.poll() is None:
            p.kill()
    ref = json.load(open(out))
    sys.path.insert(0, ROOT)
    from decimal import Decimal
    from upow_amd.ledger import manager, pagesync
    from upow_amd.ledger.database import Database
    monkeypatch.setattr(manager, 'START_DIFFICULTY', Decimal('1.5'))  # the syncer's chain

    async def resume():
        db = await Database.create(path=dst, utxo_backend='host')
        manager.Manager.difficulty = None
        try:
            t = db._tip_id()
            # inside a page nothing is promised durable before the page's one fdatasync, and the writer's I/O
            # thread writes the block records behind the apply: the reopened tip is any whole block of the page
            assert 2 <= t <= 2 + n_blocks
            counts = db._q('SELECT b.id, COUNT(t.tx_hash) FROM blocks b LEFT JOIN transactions t '
                           'ON t.block_hash = b.hash WHERE b.id > 2 GROUP BY b.id')
            assert len(counts) == t - 2 and all(c == TXS + 1 for _, c in counts), counts
            assert db.utxo.set_hash() == db.sql_unspent_outputs_hash()
            rest = [b for b in ref['page'] if int(b['block']['id']) > t]
            if rest:
                assert await pagesync.create_blocks(rest)
            db.flush()
            return db._tip_id(), (await db.get_last_block())['hash'], db.sql_unspent_outputs_hash(), db.utxo.set_hash()
        finally:
            db.close()
    tip, h, sql_hash, idx_hash = asyncio.run(resume())
    assert (tip, h) == (2 + n_blocks, ref['tip'])
    assert sql_hash == idx_hash == ref['utxo']
