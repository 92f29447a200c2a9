"""SQLite page size vs ledger size: per-block insert of 8,300 transaction rows (the reference's
`transactions` layout: UNIQUE tx_hash, block_hash index, ~540-char tx hex) into a table that already
holds N rows, WAL mode, 1 GiB page cache, one checkpoint per block. Prints (median ms per block,
median WAL bytes per block in MB) for each page size.

    python scripts/sqlite_page_scale.py [N_PRE [PAGE,PAGE,...]]

A fresh ledger (the verify bench's) favours large pages; once the unique index is much larger than
one block's inserts, every insert dirties its own leaf and large pages write proportionally more."""
import os, sqlite3, time, random, sys, tempfile
def run(page, n_pre, blocks=6, per=8300):
    d = tempfile.mkdtemp(dir='/tmp'); f = d + '/t.db'
    c = sqlite3.connect(f, isolation_level=None)
    c.execute(f'PRAGMA page_size={page}'); c.execute('PRAGMA journal_mode=WAL'); c.execute('PRAGMA synchronous=OFF')
    c.execute('PRAGMA cache_size=-1048576'); c.execute('PRAGMA wal_autocheckpoint=0')
    c.execute('CREATE TABLE t (block_hash TEXT, tx_hash TEXT UNIQUE, tx_hex TEXT, a TEXT, b TEXT, c TEXT, fees TEXT)')
    c.execute('CREATE INDEX bh ON t(block_hash)')
    rng = random.Random(1)
    hexpad = 'ab' * 270
    def batch(n, bh):
        return [(bh, '%064x' % rng.getrandbits(256), hexpad, '["x"]', '["y","z"]', '[1,2]', '0.000001') for _ in range(n)]
    c.execute('BEGIN')
    for k in range(0, n_pre, 50000):
        c.executemany('INSERT INTO t VALUES (?,?,?,?,?,?,?)', batch(min(50000, n_pre - k), 'pre%d' % k))
    c.execute('COMMIT'); c.execute('PRAGMA wal_checkpoint(TRUNCATE)')
    ts = []; wal = []
    for b in range(blocks):
        rows = batch(per, 'b%d' % b)
        t = time.perf_counter()
        c.execute('BEGIN'); c.executemany('INSERT INTO t VALUES (?,?,?,?,?,?,?)', rows); c.execute('COMMIT')
        ts.append(time.perf_counter() - t)
        wal.append(os.path.getsize(f + '-wal')); c.execute('PRAGMA wal_checkpoint(TRUNCATE)')
    c.close()
    import shutil; shutil.rmtree(d)
    return round(sorted(ts)[len(ts)//2]*1e3, 1), round(sorted(wal)[len(wal)//2]/1e6, 1)
for n_pre in ((100_000, 2_000_000) if len(sys.argv) < 2 else [int(sys.argv[1])]):
    for page in ((4096, 16384, 32768) if len(sys.argv) < 3 else [int(x) for x in sys.argv[2].split(",")]):
        print(n_pre, page, run(page, n_pre), flush=True)
