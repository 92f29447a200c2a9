"""Host calibration for the ledger-write numbers: raw SQLite cost of one 2 MB block's UTXO writes
(16,600 inserts + deletes with the unspent_outputs indexes) through the native writer. Run in the same
gpurun call as the verify bench so box-to-box host variance can be told apart from code changes."""
import json
import os
import random
import sqlite3
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from upow_amd.ops.native import lib  # noqa: E402

L = lib()
rng = random.Random(1)
addrs = [rng.randbytes(30).hex()[:45] for _ in range(256)]
c = sqlite3.connect(':memory:', isolation_level=None)
c.execute('CREATE TABLE u (tx_hash TEXT, "index" INTEGER NOT NULL, address TEXT NULL, is_stake INTEGER)')
c.execute('CREATE INDEX a ON u (tx_hash, "index")')
c.execute('CREATE INDEX b ON u (address)')
n0 = 200_000
raw = np.frombuffer(rng.randbytes(32 * n0), np.uint8)
c.execute('BEGIN')
L.sql_executemany(c, 'INSERT INTO u VALUES (?,?,?,?)',
                  [('hex32', raw, 32, 0), np.zeros(n0, np.int64), [rng.choice(addrs) for _ in range(n0)], 0], n0)
c.execute('COMMIT')
ins, dels = [], []
for rep in range(5):
    n = 16_600
    raw = np.frombuffer(rng.randbytes(32 * n), np.uint8)
    ad = [rng.choice(addrs) for _ in range(n)]
    c.execute('BEGIN')
    t = time.perf_counter()
    L.sql_executemany(c, 'INSERT INTO u VALUES (?,?,?,?)', [('hex32', raw, 32, 0), np.zeros(n, np.int64), ad, 0], n)
    ins.append(time.perf_counter() - t)
    c.execute('COMMIT')
    c.execute('BEGIN')
    t = time.perf_counter()
    L.sql_executemany(c, 'DELETE FROM u WHERE tx_hash = ? AND "index" = ?', [('hex32', raw, 32, 0), np.zeros(n, np.int64)], n)
    dels.append(time.perf_counter() - t)
    c.execute('COMMIT')
print(json.dumps({'sqlite_insert_ms': round(1e3 * float(np.median(ins)), 2),
                  'sqlite_delete_ms': round(1e3 * float(np.median(dels)), 2), 'rows': 16_600}))
