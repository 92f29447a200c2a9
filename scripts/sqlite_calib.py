"""Materialiser calibration: the SQL side of one 2 MB block (8,300 tx rows, 16,600 unspent-output inserts,
16,600 deletes of the previous block's outputs) pushed through the native ledger writer
(csrc/ledger_writer.cpp) on the ledger's real schema, without validation in front of it.

    python scripts/sqlite_calib.py [--blocks 12] [--txs 8300] [--dir /tmp/calib]

Prints the writer's per-statement times and the sustained block rate of the materialiser. Run in the
same gpurun call as the verify bench so box-to-box host variance can be told apart from code changes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import upow_amd  # noqa: E402,F401  (before sqlite3: see upow_amd._sqlite_no_memstatus)
import argparse  # noqa: E402
import json  # noqa: E402
import random  # noqa: E402
import shutil  # noqa: E402
import sqlite3  # noqa: E402
import tempfile  # noqa: E402
import time  # noqa: E402

import numpy as np  # noqa: E402

from upow_amd.ledger.database import SCHEMA, tx_schema, utxo_schema  # noqa: E402
from upow_amd.ops.native import lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--blocks', type=int, default=12)
    ap.add_argument('--txs', type=int, default=8300)
    ap.add_argument('--dir', default=None)
    ap.add_argument('--group', type=int, default=8)
    ap.add_argument('--single-file', action='store_true',
                    help='materialise every table on one connection (the layout before the UTXO file split)')
    ap.add_argument('--sorted-inserts', action='store_true', help='UTXO INSERTs in tx-hash order (index locality)')
    ap.add_argument('--without-rowid', action='store_true',
                    help='UTXO table clustered on (tx_hash, index): one B-tree per row instead of table + index')
    ap.add_argument('--utxo-shards', type=int, default=1,
                    help='UTXO rows split over this many files by the first txid byte (A/B for a wider split)')
    a = ap.parse_args()
    L = lib()
    utxo_ddl = utxo_schema('utxo')
    if a.without_rowid:
        utxo_ddl = ('CREATE TABLE IF NOT EXISTS utxo.unspent_outputs (tx_hash TEXT, "index" INTEGER NOT NULL, '
                    'address TEXT NULL, is_stake INTEGER, PRIMARY KEY (tx_hash, "index")) WITHOUT ROWID;')
    d = tempfile.mkdtemp(prefix='calib_', dir=a.dir)
    path = os.path.join(d, 'ledger.sqlite3')
    c = sqlite3.connect(path, isolation_level=None)
    c.execute('PRAGMA journal_mode = WAL')
    c.executescript(SCHEMA + tx_schema('main', legacy=True))
    c.execute('ATTACH DATABASE ? AS utxo', (path + '-utxo',))
    c.execute('PRAGMA utxo.journal_mode = WAL')
    c.executescript(utxo_ddl)
    extra = [path + f'-utxo{k + 1}' for k in range(1, a.utxo_shards)] if not a.single_file else []
    for f in extra:
        c.execute('ATTACH DATABASE ? AS ux', (f,))
        c.execute('PRAGMA ux.journal_mode = WAL')
        c.executescript(utxo_ddl.replace('utxo.', 'ux.'))
        c.execute('DETACH DATABASE ux')
    c.close()
    files = [path] if a.single_file else [path, path + '-utxo', *extra]
    nsh = 1 if a.single_file else a.utxo_shards
    if a.single_file:  # the UTXO table next to the others
        c = sqlite3.connect(path, isolation_level=None)
        c.executescript(utxo_ddl.replace('utxo.', ''))
        c.close()
    w = L.LedgerWriter(files, path + '.journal', 1, 1024, a.group, 1 << 40)
    def shard_rows(keys):  # (shard, row indices) by the first txid byte
        if nsh == 1:
            return [(0 if a.single_file else 1, np.arange(len(keys)))]
        b0 = keys[:, 0].astype(np.int64) * nsh // 256
        return [(1 + k, np.nonzero(b0 == k)[0]) for k in range(nsh)]
    rng = random.Random(1)
    addrs = [rng.randbytes(30).hex()[:45] for _ in range(256)]
    n = a.txs
    prev = None
    enc = L.ledger_encode_stmt
    batches = []
    for b in range(a.blocks + 1):  # encoded up front: only the materialiser runs in the timed region
        bh = rng.randbytes(32).hex()
        txid = np.frombuffer(rng.randbytes(32 * n), np.uint8).reshape(n, 32)
        tx_hex = [rng.randbytes(216).hex() for _ in range(n)]
        js = [json.dumps([rng.choice(addrs), rng.choice(addrs)]) for _ in range(n)]
        out_txid = np.repeat(txid, 2, axis=0)
        out_idx = np.tile(np.arange(2, dtype=np.int64), n)
        stmts = [enc('INSERT INTO blocks (id, hash, content, address, random, difficulty, reward, timestamp) '
                     'VALUES (?, ?, ?, ?, ?, ?, ?, ?)', [b + 1, bh, 'c' * 216, addrs[0], 0, '6.0', '6.0', 1000 + b], 1),
                 enc('INSERT INTO transactions (block_hash, tx_hash, tx_hex, inputs_addresses, outputs_addresses, '
                     'outputs_amounts, fees) VALUES (?, ?, ?, ?, ?, ?, ?)',
                     [bh, ('hex32', txid, 32, 0), tx_hex, js, js, '[1250000000,749000000]', '0.010000'], n)]
        out_addr = [rng.choice(addrs) for _ in range(2 * n)]
        for sh, rows in shard_rows(out_txid):
            ot = np.ascontiguousarray(out_txid[rows])
            iord = np.argsort(ot[:, :8].copy().view('>u8').ravel(), kind='stable').astype(np.int64) \
                if a.sorted_inserts else None
            stmts.append(enc('INSERT INTO unspent_outputs (tx_hash, "index", address, is_stake) VALUES (?, ?, ?, ?)',
                             [('hex32', ot, 32, 0), np.ascontiguousarray(out_idx[rows]),
                              [out_addr[r] for r in rows.tolist()], 0], len(rows), iord, shard=sh))
        if prev is not None:
            keys = np.zeros((2 * n, 40), np.uint8)
            keys[:, :32] = prev
            keys[:, 32:36] = np.tile(np.array([[0, 0, 0, 0], [1, 0, 0, 0]], np.uint8), (n, 1))
            idx = np.tile(np.arange(2, dtype=np.int64), n)
            for sh, rows in shard_rows(keys):
                kk = np.ascontiguousarray(keys[rows])
                order = np.argsort(kk[:, :8].copy().view('>u8').ravel(), kind='stable').astype(np.int64)
                stmts.append(enc('DELETE FROM unspent_outputs WHERE tx_hash = ? AND "index" = ?',
                                 [('hex32', kk, 40, 0), np.ascontiguousarray(idx[rows])], len(rows), order,
                                 None, len(rows), sh))
        batches.append(stmts)
        prev = out_txid
    w.submit(batches[0], b'', 1)
    w.wait(1)
    t0 = time.perf_counter()
    t_submit = 0.0
    for b, stmts in enumerate(batches[1:], start=2):
        ts = time.perf_counter()
        w.submit(stmts, b'', b)
        t_submit += time.perf_counter() - ts
    w.wait(a.blocks + 1)
    dt = time.perf_counter() - t0
    st = w.stats()
    w.close()
    shutil.rmtree(d, ignore_errors=True)
    per = {k[:32]: {'ms_per_block': round(v[0] * 1e3 / (a.blocks + 1), 2), 'us_per_row': round(v[0] * 1e6 / max(1, v[1]), 3)}
           for k, v in st['statements'].items()}
    print(json.dumps({'files': len(files), 'utxo_shards': nsh, 'sorted_inserts': a.sorted_inserts,
                      'without_rowid': a.without_rowid, 'memstatus_rc': upow_amd.SQLITE_MEMSTATUS_RC, 'blocks': a.blocks, 'txs': n, 'materialiser_ms_per_block': round(dt * 1e3 / a.blocks, 2),
                      'materialiser_tx_per_s': round(a.blocks * n / dt, 1),
                      'submit_ms_per_block': round(t_submit * 1e3 / a.blocks, 2),
                      'commit_ms_per_block': round(st['commit_s'] * 1e3 / (a.blocks + 1), 2),
                      'groups': st['groups'], 'shards': st['shards'], 'statements': per}))


if __name__ == '__main__':
    main()
