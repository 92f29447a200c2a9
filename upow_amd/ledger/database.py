"""Embedded ledger store with the reference's query API (reference: upow/database.py:26-1654).

The reference keeps everything in PostgreSQL through asyncpg. This build keeps the exact
``schema.sql`` table/column layout (reference: schema.sql:1-84) in an embedded SQLite database
(TEXT[]/BIGINT[] columns stored as JSON, NUMERIC stored as canonical decimal text with PostgreSQL's
NUMERIC(p,s) rounding), so a restart resumes from the last block with no server, and keeps the UTXO
set additionally in an in-memory / HBM hash index (:mod:`upow_amd.ledger.utxo`) that the batched
block validator probes instead of issuing SQL per input.

Method names, arguments, return shapes and ordering follow the reference one-for-one (each method
cites its reference line range) so the consensus and node layers read the same.
"""
from __future__ import annotations

import asyncio
import json
import os
import re
import sqlite3
import struct
import threading
import weakref
from collections import OrderedDict, defaultdict
from datetime import datetime, timedelta, timezone
from decimal import ROUND_HALF_UP, Decimal
from statistics import mean
from time import perf_counter
from typing import Any, Dict, Iterable, List, Optional, Set, Tuple, Union

import numpy as np

from ..constants import MAX_BLOCK_SIZE_HEX, SMALLEST
from ..models.transaction import CoinbaseTransaction, Transaction, TransactionInput
from ..utils import codec, roctx
from ..utils.codec import (AddressFormat, OutputType, TransactionType, normalize_block, point_to_bytes,
                           point_to_string, round_up_decimal, sha256, string_to_bytes, string_to_point)
from ..utils import coalesce
from ..utils.logstore import LogStore
from ..utils.logger import get_logger
from .governance import STAKE, GovernanceIndex
from .governance import TID as GOV_TID
from .governance import _row_args as _gov_row
from .mempool import MempoolIndex
from .utxo import FLAG_STAKE, PAYLOAD_DTYPE, TAG_BY_TABLE, UtxoIndex, make_payload

logger = get_logger(__name__)

OUTPUT_TABLES = ('unspent_outputs', 'inode_registration_output', 'validator_registration_output',
                 'validators_voting_power', 'delegates_voting_power', 'validators_ballot', 'inodes_ballot')

SCHEMA = """
CREATE TABLE IF NOT EXISTS blocks (
    id INTEGER PRIMARY KEY,
    hash TEXT UNIQUE,
    content TEXT NOT NULL,
    address TEXT NOT NULL,
    random INTEGER NOT NULL,
    difficulty TEXT NOT NULL,
    reward TEXT NOT NULL,
    timestamp INTEGER
);
CREATE TABLE IF NOT EXISTS pending_transactions (
    tx_hash TEXT UNIQUE,
    tx_hex TEXT,
    inputs_addresses TEXT,
    fees TEXT NOT NULL,
    propagation_time INTEGER NOT NULL
);
CREATE TABLE IF NOT EXISTS pending_spent_outputs (
    tx_hash TEXT REFERENCES transactions(tx_hash) ON DELETE CASCADE,
    "index" INTEGER NOT NULL
);
CREATE TABLE IF NOT EXISTS address_transactions (
    address TEXT NOT NULL,
    tx_hash TEXT NOT NULL REFERENCES transactions(tx_hash) ON DELETE CASCADE
);
CREATE TABLE IF NOT EXISTS address_index_state (
    k TEXT PRIMARY KEY,
    height INTEGER NOT NULL
);
"""
for _t in OUTPUT_TABLES[1:]:
    SCHEMA += f"""
CREATE TABLE IF NOT EXISTS {_t} (
    tx_hash TEXT REFERENCES transactions(tx_hash) ON DELETE CASCADE,
    "index" INTEGER NOT NULL,
    address TEXT NULL
);"""
SCHEMA += """
CREATE INDEX IF NOT EXISTS pending_spent_idx ON pending_spent_outputs (tx_hash, "index");
CREATE INDEX IF NOT EXISTS address_transactions_idx ON address_transactions (address);
CREATE INDEX IF NOT EXISTS address_transactions_tx_idx ON address_transactions (tx_hash);
"""
for _t in OUTPUT_TABLES[1:]:
    SCHEMA += f'CREATE INDEX IF NOT EXISTS {_t}_outpoint_idx ON {_t} (tx_hash, "index");\n'
    SCHEMA += f'CREATE INDEX IF NOT EXISTS {_t}_address_idx ON {_t} (address);\n'


# Row-heavy tables live in database files of their own, each table split over several files by the first
# byte of the tx hash (file k of n holds the hashes whose first byte b has b * n >> 8 == k). A 2 MB block
# inserts ~8.3k transaction rows and ~33k UTXO rows and deletes as many; once a ledger holds millions of
# rows every one of them is a random B-tree update, and each file has a native materialiser thread of its
# own (csrc/ledger_writer.cpp routes a statement's rows by that byte), so the files apply in parallel.
#
#   ``<ledger>-utxo``, ``-utxo2``, ...  ``unspent_outputs``, attached as ``utxo``, ``utxo2``, ...
#   ``<ledger>-tx``, ``-tx2``, ...      ``transactions``, attached as ``tx``, ``tx2``, ...
#
# * Row ids come from one ledger-wide counter per table (explicit ``rowid`` on every insert), so
#   ``rowid`` order over the files is insertion order, as in the single tables of schema.sql.
# * On the Python connection each split table is a TEMP view over its files for reads; Python-side
#   writes are routed by :meth:`Database._routed_exec` (a trigger body cannot name an attached table).
# * SQLite cannot declare a foreign key across files: the reference's ``ON DELETE CASCADE`` clauses that
#   point at a split table (or from it at ``blocks``) are applied by the block-deleting methods themselves.
# * The layout of a ledger is recorded in its main file (``upow_layout``) when it is created. Ledgers from
#   before the transactions split keep ``transactions`` in the main file (one "file", no view) and two
#   UTXO files.
_SQL_READERS = None  # Database._off_loop


def _commit_point():
    """On a cluster node, the block's agree-before-commit vote resolves here, right before its journal write
    (parallel/cluster.py ``commit_point``); raises when a replica is not ready."""
    from ..parallel.cluster import commit_point
    commit_point()
# 5 + 5 (eleven files with the main one; SQLite attaches at most ten): ~20 % faster materialisation of an
# aged ledger than 4 + 4 (profiles/r4/verify_aged_writer_ab_r4g.json, verify_aged60_s55_r4x.json), 11 %
# faster than 6 + 4 on the aged ledger (profiles/r5/verify_aged_split_*_r5i.json). 6 + 4 is 12 % faster on a
# fresh ledger (three interleaved pairs, profiles/r5/verify_split_*): the aged ledger is what a node runs.
UTXO_FILES_DEFAULT = 5
TX_FILES_DEFAULT = 5
# New ledgers take the mixed layout: LEDGER_FILES_DEFAULT files, each with both split tables of one hash
# range, so every materialiser carries the same share of UTXO and transaction rows whatever their cost ratio
# (fresh: the UTXO files of 5 + 5 were busy 9-10 ms per block against 6-7 for the tx files). Interleaved A/Bs
# against 5 + 5 (profiles/r5/ledger_mixed_ab/): fresh 10.02-10.58 vs 10.76-12.35 ms per block (five pairs,
# one noisy mixed run at 12.93), aged 60-block run 19.01 vs 20.85 ms per block.
LEDGER_MIXED_DEFAULT = '1'
LEDGER_FILES_DEFAULT = 10
ROUTED = ('unspent_outputs', 'transactions')


def _names(kind: str, n: int) -> Tuple[List[str], List[str]]:
    """(schema names, file suffixes) of the ``n`` files of ``kind`` ('utxo' | 'tx')."""
    schemas = [kind if k == 0 else f'{kind}{k + 1}' for k in range(n)]
    return schemas, ['-' + sch for sch in schemas]


# the two-file UTXO layout of earlier ledgers (still what ``_migrate_utxo_split`` produces)
UTXO_SCHEMAS, UTXO_SUFFIXES = _names('utxo', 2)


def file_of(tx_hash: str, n: int) -> int:
    """Which of ``n`` files holds ``tx_hash``: the writer's routing (first byte * n >> 8; non-hex -> 0)."""
    try:
        return (int(tx_hash[:2], 16) * n) >> 8 if n > 1 else 0
    except (ValueError, TypeError):
        return 0


TX_COLUMNS = 'block_hash, tx_hash, tx_hex, inputs_addresses, outputs_addresses, outputs_amounts, fees'
UTXO_COLUMNS = 'tx_hash, "index", address, is_stake'


def tx_schema(schema: str, legacy: bool = False) -> str:
    """``transactions`` (schema.sql) in one of its files; ``legacy``: the main-file table of a ledger from
    before the split, with the reference's cascade from ``blocks``."""
    parent = ' REFERENCES blocks(hash) ON DELETE CASCADE' if legacy else ''
    return f"""
CREATE TABLE IF NOT EXISTS {schema}.transactions (
    block_hash TEXT NOT NULL{parent},
    tx_hash TEXT UNIQUE,
    tx_hex TEXT,
    inputs_addresses TEXT,
    outputs_addresses TEXT,
    outputs_amounts TEXT,
    fees TEXT NOT NULL
);
CREATE INDEX IF NOT EXISTS {schema}.block_hash_idx ON transactions (block_hash);
"""


def utxo_schema(schema: str = 'utxo') -> str:
    return f"""
CREATE TABLE IF NOT EXISTS {schema}.unspent_outputs (
    tx_hash TEXT,
    "index" INTEGER NOT NULL,
    address TEXT NULL,
    is_stake INTEGER
);
CREATE INDEX IF NOT EXISTS {schema}.tx_hash_idx ON unspent_outputs (tx_hash, "index");
"""


def split_view(table: str, schemas: List[str]) -> str:
    """The TEMP view that reads a split table over its files (``rowid``: the ledger-wide row id)."""
    if table == 'unspent_outputs':
        arms = [f'SELECT rowid AS rowid, {UTXO_COLUMNS} FROM {sch}.unspent_outputs' for sch in schemas]
    else:
        arms = [f'SELECT {TX_COLUMNS}, rowid AS rowid FROM {sch}.transactions' for sch in schemas]
    return f'CREATE TEMP VIEW IF NOT EXISTS {table} AS\n    ' + '\n    UNION ALL\n    '.join(arms) + ';\n'


def utxo_file_of(tx_hash: str) -> int:
    """0 for ``utxo`` (hash 00-7f), 1 for ``utxo2`` (80-ff) in the two-file layout."""
    return file_of(tx_hash, 2)


def ledger_files(path: str) -> List[str]:
    """Every file of a (closed) file ledger: the main database, its table files and the journal."""
    import glob
    parts = sorted(glob.glob(glob.escape(path) + '-utxo*') + glob.glob(glob.escape(path) + '-tx*'))
    parts = [f for f in parts if not f.endswith(('-wal', '-shm', '-journal'))]
    return [path] + parts + [path + '.journal']


def copy_ledger(src: str, dst: str):
    """Copy a closed file ledger (all of its files) to ``dst``."""
    import shutil
    src, dst = str(src), str(dst)
    for f in ledger_files(src):
        if os.path.exists(f):
            shutil.copy(f, dst + f[len(src):])


def numeric(value, scale: int) -> str:
    """PostgreSQL NUMERIC(p, scale) storage: round half away from zero to ``scale`` digits."""
    q = Decimal(1).scaleb(-scale)
    return str(Decimal(value).quantize(q, rounding=ROUND_HALF_UP))


def _probe_batch(items: list) -> list:
    """Coalesced admission probes: items are (database, tag, outpoints); one index lookup per (database,
    tag) over the union, each item gets the set of its outpoints that are present."""
    groups: Dict[tuple, tuple] = {}
    for k, (db, tag, keys) in enumerate(items):
        groups.setdefault((id(db), tag), (db, tag, []))[2].append(k)
    res: list = [None] * len(items)
    for db, tag, idxs in groups.values():
        allkeys = list(dict.fromkeys(key for k in idxs for key in items[k][2]))
        found = set(db.utxo.filter(allkeys, tag))
        for k in idxs:
            res[k] = found
    return res


def _utcnow() -> datetime:
    return datetime.now(timezone.utc).replace(tzinfo=None)


def _dt(ts: int) -> datetime:
    return datetime.fromtimestamp(int(ts), timezone.utc).replace(tzinfo=None)


def _j(x) -> str:
    return json.dumps(x, separators=(',', ':'))


def _arr(s) -> list:
    return json.loads(s) if s else []


_CANON: dict = {}


async def _input_address(tx_input) -> str:
    """``point_to_string(await input.get_public_key())`` memoised by the owning address string
    (the canonical compressed base58 form of the spent output's address)."""
    if tx_input.public_key is not None:
        return point_to_string(tx_input.public_key)
    addr = await tx_input.get_address()
    hit = _CANON.get(addr)
    if hit is None:
        hit = point_to_string(string_to_point(addr))
        if len(_CANON) > (1 << 20):
            _CANON.clear()
        _CANON[addr] = hit
    return hit


def _addr_bytes(address: Optional[str]) -> Optional[bytes]:
    if not address:
        return None
    try:
        return string_to_bytes(address)
    except ValueError:
        return None


def _at(arr: list, index: int):
    """PostgreSQL 1-based array subscript semantics for ``arr[index + 1]`` (NULL when out of range)."""
    return arr[index] if 0 <= index < len(arr) else None


_ENCODE_POOL = None
_ENCODE_THREADS = int(os.environ.get('UPOW_ENCODE_THREADS', '4'))


def _expand_col(spec, n: int) -> list:
    """Python values of one bulk column spec (the ``sqlite3.executemany`` fallback of Database.bulk)."""
    if isinstance(spec, list):
        return spec
    if isinstance(spec, tuple):
        kind = spec[0]
        if kind == 'gather':
            return [spec[1][i] for i in np.asarray(spec[2]).tolist()]
        if kind == 'hex32':  # optional 5th element: the rows to take
            raw = np.frombuffer(spec[1], dtype=np.uint8)
            stride, off = spec[2], spec[3]
            rows = np.asarray(spec[4]).tolist() if len(spec) > 4 else range(n)
            return [bytes(raw[r * stride + off:r * stride + off + 32]).hex() for r in rows]
        if kind == 'arena':  # optional 4th element: the rows to take
            blob = bytes(spec[1]).decode()  # ASCII: byte offsets are character offsets
            off = np.frombuffer(spec[2], dtype=np.int64).tolist()
            rows = np.asarray(spec[3]).tolist() if len(spec) > 3 else range(n)
            return [blob[off[i]:off[i + 1]] for i in rows]
        if kind == 'hexarena':  # raw bytes per row, stored as their lowercase hex
            blob = bytes(spec[1])
            off = np.frombuffer(spec[2], dtype=np.int64).tolist()
            rows = np.asarray(spec[3]).tolist() if len(spec) > 3 else range(n)
            return [blob[off[i]:off[i + 1]].hex() for i in rows]
        raise ValueError(f'unknown column kind {kind}')
    if isinstance(spec, np.ndarray):
        return spec.tolist()
    return [spec] * n


def arena_list(arena) -> List[str]:
    """The strings of a (blob, int64 offsets) text arena from csrc/txcodec.cpp."""
    blob, off = arena
    return _expand_col(('arena', blob, off), len(off) // 8 - 1)


_TABLES = ('blocks', 'transactions', 'unspent_outputs', 'pending_transactions', 'pending_spent_outputs',
           'address_transactions', 'address_index_state', *OUTPUT_TABLES[1:])
_TABLE_RE = re.compile(r'\b(' + '|'.join(_TABLES) + r')\b')
# tables whose rows reference transactions(tx_hash) / blocks(hash): a write to them must see the parents
_FK_PARENTS = {t: ('transactions', 'blocks') for t in ('unspent_outputs', 'pending_spent_outputs',
                                                       'address_transactions', *OUTPUT_TABLES[1:])}
_FK_PARENTS['transactions'] = ('blocks',)
_SQL_TABLES: Dict[Tuple[str, bool], Optional[frozenset]] = {}


def _tables_of(sql: str, write: bool) -> Optional[frozenset]:
    """Ledger tables a statement reads (or writes, with their FK parents); None = all of them
    (a DELETE/UPDATE on blocks or transactions cascades through the output tables)."""
    key = (sql, write)
    hit = _SQL_TABLES.get(key, False)
    if hit is not False:
        return hit
    names = set(_TABLE_RE.findall(sql))
    res: Optional[frozenset]
    head = sql.lstrip()[:6].upper()
    if write and head in ('DELETE', 'UPDATE') and names & {'blocks', 'transactions'}:
        res = None
    else:
        if write:
            for t in list(names):
                names.update(_FK_PARENTS.get(t, ()))
        res = frozenset(names)
    if len(_SQL_TABLES) > 4096:
        _SQL_TABLES.clear()
    _SQL_TABLES[key] = res
    return res


def _ephemeral_dir() -> str:
    """A private directory on tmpfs for an in-memory ledger (``':memory:'``): the ledger's SQLite file
    must be openable by two connections (Python's and the native writer's), which a SQLite
    ``:memory:`` database is not."""
    import tempfile
    base = os.environ.get('UPOW_EPHEMERAL_DIR') or ('/dev/shm' if os.path.isdir('/dev/shm') and
                                                     os.access('/dev/shm', os.W_OK) else None)
    return tempfile.mkdtemp(prefix='upow_ledger_', dir=base)


def _cleanup_ephemeral(state: dict):
    w = state.get('writer')
    if w is not None:
        try:
            w.close()
        except Exception:
            pass
    c = state.get('conn')
    if c is not None:
        try:
            c.close()
        except Exception:
            pass
    d = state.get('dir')
    if d:
        import shutil
        shutil.rmtree(d, ignore_errors=True)


class Database:
    """SQLite-backed ledger. ``Database.instance`` is the process singleton (as in the reference).

    Block applications of the native path are written through :class:`LedgerWriter`
    (csrc/ledger_writer.cpp): a journal append is the commit point and a background thread on a
    connection of its own materialises the tables. Every read through this class first waits until
    the tables it names are materialised up to the last committed batch (:meth:`_settle`); writes
    through the Python connection wait for the tables they write and their FK parents."""
    instance: 'Database' = None
    credentials: dict = {}
    is_indexed = True

    def __init__(self, path: str = ':memory:', utxo_backend: Optional[str] = None):
        self.path = path
        self._eph = {}
        if path == ':memory:':
            self._eph['dir'] = _ephemeral_dir()
            self.file = os.path.join(self._eph['dir'], 'ledger.sqlite3')
            weakref.finalize(self, _cleanup_ephemeral, self._eph)
        else:
            self.file = path
        self._conn = sqlite3.connect(self.file, check_same_thread=False, isolation_level=None, timeout=120)
        self._eph['conn'] = self._conn if path == ':memory:' else None
        self._conn.row_factory = sqlite3.Row
        if os.environ.get('UPOW_SQL_TRACE'):  # every statement of the Python connection (query-plan audits)
            trace = open(os.environ['UPOW_SQL_TRACE'], 'a')
            self._conn.set_trace_callback(lambda q: trace.write(q.replace('\n', ' ') + '\n'))
        self.lock = threading.RLock()
        self.writer = None
        self._submitted = 0
        self._applied_seen: Dict[int, int] = {}  # shard (-1: all) -> applied sequence already observed
        self._table_seq: Dict[str, int] = {}
        self._tip_cache: Optional[dict] = None
        # the rows of the last RECENT_ROWS blocks applied on this process's block path, by id: the difficulty
        # retarget reads the block 99 below the tip every 100 blocks, which from SQL first waits for the
        # materialisers to write the blocks table (~3 ms per retarget in the page sync's profile)
        self._recent_rows: Dict[int, dict] = {}
        self._tip_gen = 0
        self._genesis_cache: Optional[str] = None
        self._pending_empty: Optional[bool] = None
        self._mempool_ver = 0
        # lean cluster follower (ledger/lean.py): blocks go to the HBM/governance/mempool indexes, the chain-tip
        # header rows below and the op log, not to SQL; _lean_tip is the tip row while lean
        self.lean = False
        self.lean_log = None
        self._lean_rows: Dict[int, dict] = {}
        self._lean_by_hash: Dict[str, int] = {}
        self._lean_tip: Optional[dict] = None
        self.on_admit = None  # cluster leader: row hook of every admission (parallel/cluster.py)
        self.on_confirm = None  # cluster leader: hook (index, hit txs, hit inputs) of a block's mempool confirm
        self._mp: Optional[MempoolIndex] = None  # ledger/mempool.py; None: (re)load from SQL on next use
        self.mempool_reloads = 0
        self._seq_lock = threading.Lock()  # journal submission + per-table sequence bookkeeping
        # parsed rows of confirmed txs by hash (immutable until a rollback, which clears it): a funding
        # tx with hundreds of outputs is spent by many pushed txs, each would re-read and re-parse it
        self._info_cache: 'OrderedDict[str, dict]' = OrderedDict()
        self.mempool_index = os.environ.get('UPOW_MEMPOOL_INDEX', '1') != '0'
        self._conn.execute('PRAGMA foreign_keys = ON')
        # B-tree page size of a NEW ledger file (fixed once the file exists in WAL mode). A block inserts
        # ~8.3k wide transaction rows and ~33k UTXO rows and deletes as many. Larger pages mean fewer
        # splits and levels (a fresh ledger materialises 1.5x faster on 32 KB pages than on 4 KB:
        # profiles/r2/sqlite_page_size_ab.txt), but once an index is far larger than one block's
        # inserts every insert dirties its own leaf, and large pages then write more WAL and lose
        # (profiles/r2/sqlite_page_scale_cpu.txt, 2 M rows). 8 KB beats 4 KB at both ends.
        page = int(os.environ.get('UPOW_SQLITE_PAGE_SIZE', '8192'))
        self._conn.execute(f'PRAGMA page_size = {page}')
        self._conn.execute('PRAGMA journal_mode = WAL')
        self._conn.execute('PRAGMA synchronous = ' + ('OFF' if path == ':memory:' else 'NORMAL'))
        # a 2 MB block rewrites ~10 MB of B-tree pages: keep the hot index levels in a large page
        # cache (MI355X hosts have RAM to spare), and take WAL checkpoints (page copy-back + fsync)
        # off the block-apply path: a background thread with its own connection runs PASSIVE
        # checkpoints; the commit-time auto-checkpoint only remains as a 400 MB safety net
        cache_mb = int(os.environ.get('UPOW_SQLITE_CACHE_MB', '1024' if path != ':memory:' else '256'))
        self._conn.execute(f'PRAGMA cache_size = -{cache_mb * 1024}')
        bg = os.environ.get('UPOW_WAL_CHECKPOINT_THREAD', '1') != '0'
        auto = int(os.environ.get('UPOW_WAL_AUTOCHECKPOINT', '100000' if bg else '10000'))
        self._conn.execute(f'PRAGMA wal_autocheckpoint = {auto}')
        n_utxo, n_tx, self.mixed = self._layout()
        self._conn.executescript(SCHEMA)
        self.utxo_schemas, sfx = _names('utxo', n_utxo)
        self.utxo_files = [self.file + x for x in sfx]
        self.utxo_file = self.utxo_files[0]
        if self.mixed:
            # every split file holds both split tables for one hash range (the UTXO rows and the txs of the
            # same tx hashes): each materialiser gets an equal share of both workloads, whatever their ratio
            self.tx_schemas, self.tx_files = list(self.utxo_schemas), list(self.utxo_files)
        else:
            # n_tx == 0: a ledger from before the transactions split keeps the table in its main file
            self.tx_schemas, sfx = _names('tx', n_tx)
            self.tx_files = [self.file + x for x in sfx]
        fresh2 = n_utxo == 2 and not self.mixed and not os.path.exists(self.utxo_files[1])
        for schema, f in self._split_files():
            self._conn.execute(f'ATTACH DATABASE ? AS {schema}', (f,))
            self._conn.execute(f'PRAGMA {schema}.page_size = {page}')
            self._conn.execute(f'PRAGMA {schema}.journal_mode = WAL')
            self._conn.execute(f'PRAGMA {schema}.synchronous = ' + ('OFF' if path == ':memory:' else 'NORMAL'))
            self._conn.execute(f'PRAGMA {schema}.cache_size = -{cache_mb * 1024}')
            if self.mixed:
                self._conn.executescript(utxo_schema(schema) + tx_schema(schema))
            else:
                self._conn.executescript(utxo_schema(schema) if schema.startswith('utxo') else tx_schema(schema))
        if not n_tx:
            self._conn.executescript(tx_schema('main', legacy=True))
        else:
            # the reference's cascades into and out of the split table are applied by the deleting methods
            self._conn.execute('PRAGMA foreign_keys = OFF')
        self._fk = not n_tx
        self._migrate_single_file_utxo()
        if fresh2:
            self._migrate_utxo_split()
        self._conn.executescript(split_view('unspent_outputs', self.utxo_schemas))
        if n_tx:
            self._conn.executescript(split_view('transactions', self.tx_schemas))
        # table -> writer files holding it (main file = 0); routed tables: (first file, number of files)
        self._routed = {'unspent_outputs': (1, n_utxo)}
        if n_tx:
            self._routed['transactions'] = (1, n_utxo) if self.mixed else (1 + n_utxo, n_tx)
        self._shard_of = {t: tuple(range(a, a + k)) for t, (a, k) in self._routed.items()}
        if bg:
            self._start_checkpointer(float(os.environ.get('UPOW_WAL_CHECKPOINT_PERIOD', '0.5')))
        if os.environ.get('UPOW_LEDGER_WRITER', '1') != '0':
            self._open_writer(cache_mb)
            if fresh2:
                # journal records written under the one-file layout were just replayed into the first UTXO
                # file only (they carry no routing): move their 80-ff rows across like the migration did
                self._resplit_utxo()
        # next row ids: one counter per split table over its files (row id order = insertion order)
        self._utxo_next_rowid = 1 + max(self._conn.execute(f'SELECT COALESCE(MAX(rowid), 0) FROM {s}.unspent_outputs')
                                        .fetchone()[0] for s in self.utxo_schemas)
        self._tx_next_rowid = 1 + max(self._conn.execute(f'SELECT COALESCE(MAX(rowid), 0) FROM {s}.transactions')
                                      .fetchone()[0] for s in (self.tx_schemas or ['main']))
        store_dir = os.path.dirname(path) if path != ':memory:' else None
        # per-block inode emission records (reference: pickledb emission_details.json): an append-only log
        self.emission_details = LogStore(os.path.join(store_dir, 'emission_details.jsonl') if store_dir else None,
                                         legacy_json=os.path.join(store_dir, 'emission_details.json') if store_dir else None)
        self.utxo = UtxoIndex(backend=utxo_backend)
        self.utxo_source = 'sql'
        if path != ':memory:' and os.environ.get('UPOW_SNAPSHOT', '1') != '0':
            from . import snapshot
            if snapshot.try_restore(self):
                self.utxo_source = 'snapshot'
        if self.utxo_source == 'sql':
            self._rebuild_utxo_index()
        # spendable-output / balance queries answered by the UTXO index (K14) instead of SQL
        self.address_queries_from_index = os.environ.get('UPOW_ADDRESS_SQL', '0') != '1'
        self.gov: Optional[GovernanceIndex] = None
        if os.environ.get('UPOW_GOV_INDEX', '1') != '0':
            self.gov = GovernanceIndex(self)
            self.gov.rebuild()
        # the address-index watermark row must exist before the first block: the per-block statements
        # of the journal batches only advance an existing watermark
        self._address_index_height()

    def _layout(self) -> Tuple[int, int, bool]:
        """(UTXO files, transaction files; 0 = in the main file, mixed) of this ledger, recorded at creation.
        A mixed layout (``UPOW_LEDGER_MIXED=1``) has ``UPOW_LEDGER_FILES`` files each holding both split
        tables for one tx-hash range, so its materialisers share the UTXO and the transaction workloads
        evenly; the separate layout gives each table files of its own."""
        c = self._conn
        c.execute('CREATE TABLE IF NOT EXISTS upow_layout (k TEXT PRIMARY KEY, v INTEGER NOT NULL)')
        got = {r[0]: int(r[1]) for r in c.execute('SELECT k, v FROM upow_layout')}
        if 'utxo_files' in got and 'tx_files' in got:
            return got['utxo_files'], got['tx_files'], bool(got.get('mixed', 0))
        legacy = c.execute("SELECT 1 FROM main.sqlite_master WHERE type = 'table' AND name = 'blocks'").fetchone()
        mixed = False
        if legacy:
            n_utxo, n_tx = 2, 0
        elif os.environ.get('UPOW_LEDGER_MIXED', LEDGER_MIXED_DEFAULT) == '1':
            mixed = True
            n_utxo = n_tx = int(os.environ.get('UPOW_LEDGER_FILES', str(LEDGER_FILES_DEFAULT)))
            if not 2 <= n_utxo <= 10:
                raise ValueError('UPOW_LEDGER_FILES must be in 2..10 (SQLite attaches at most 10 files to a connection)')
        else:
            n_utxo = int(os.environ.get('UPOW_UTXO_FILES', str(UTXO_FILES_DEFAULT)))
            n_tx = int(os.environ.get('UPOW_TX_FILES', str(TX_FILES_DEFAULT)))
            # every split file is one ATTACH of the Python connection: SQLite allows 10 by default
            if not (2 <= n_utxo <= 8 and 0 <= n_tx <= 8 and n_utxo + n_tx <= 10):
                raise ValueError('UPOW_UTXO_FILES must be in 2..8, UPOW_TX_FILES in 0..8, and their sum at most 10 '
                                 '(SQLite attaches at most 10 files to a connection)')
        c.executemany('INSERT OR REPLACE INTO upow_layout (k, v) VALUES (?, ?)',
                      [('utxo_files', n_utxo), ('tx_files', n_tx), ('mixed', int(mixed))])
        return n_utxo, n_tx, mixed

    def _split_files(self) -> List[Tuple[str, str]]:
        """(schema, file) of every attached split file, each once."""
        if self.mixed:
            return list(zip(self.utxo_schemas, self.utxo_files))
        return [*zip(self.utxo_schemas, self.utxo_files), *zip(self.tx_schemas, self.tx_files)]

    def _migrate_single_file_utxo(self):
        """Ledgers written before the UTXO table got its own file keep ``unspent_outputs`` in the main
        file: move the rows once (unqualified names would otherwise resolve to the main copy)."""
        c = self._conn
        if c.execute("SELECT 1 FROM main.sqlite_master WHERE type = 'table' AND name = 'unspent_outputs'").fetchone():
            c.execute('BEGIN')
            c.execute('INSERT INTO utxo.unspent_outputs (rowid, tx_hash, "index", address, is_stake) '
                      'SELECT rowid, tx_hash, "index", address, is_stake FROM main.unspent_outputs ORDER BY rowid')
            c.execute('DROP TABLE main.unspent_outputs')
            c.execute('COMMIT')
            logger.info('ledger: moved unspent_outputs into its own database file')

    def _resplit_utxo(self):
        c = self._conn
        if c.execute("SELECT 1 FROM utxo.unspent_outputs WHERE tx_hash >= '8' LIMIT 1").fetchone() is None:
            return
        c.execute('BEGIN')
        c.execute('INSERT INTO utxo2.unspent_outputs (rowid, tx_hash, "index", address, is_stake) '
                  "SELECT rowid, tx_hash, \"index\", address, is_stake FROM utxo.unspent_outputs "
                  "WHERE tx_hash >= '8' ORDER BY rowid")
        c.execute("DELETE FROM utxo.unspent_outputs WHERE tx_hash >= '8'")
        c.execute('COMMIT')
        logger.info('ledger: moved replayed one-file-layout UTXO rows into the second file')

    def _migrate_utxo_split(self):
        """Ledgers written with one UTXO file: move the rows of hashes 80-ff (with their row ids) into
        the second file, whose journal watermark starts where the first file's stands."""
        c = self._conn
        move = c.execute("SELECT 1 FROM utxo.unspent_outputs WHERE tx_hash >= '8' LIMIT 1").fetchone() is not None
        c.execute('BEGIN')
        if move:
            c.execute('INSERT INTO utxo2.unspent_outputs (rowid, tx_hash, "index", address, is_stake) '
                      "SELECT rowid, tx_hash, \"index\", address, is_stake FROM utxo.unspent_outputs "
                      "WHERE tx_hash >= '8' ORDER BY rowid")
            c.execute("DELETE FROM utxo.unspent_outputs WHERE tx_hash >= '8'")
        if c.execute("SELECT 1 FROM utxo.sqlite_master WHERE type = 'table' AND name = 'upow_journal_state'").fetchone():
            c.execute('CREATE TABLE IF NOT EXISTS utxo2.upow_journal_state (k INTEGER PRIMARY KEY CHECK (k = 0), '
                      'seq INTEGER NOT NULL)')
            c.execute('INSERT OR REPLACE INTO utxo2.upow_journal_state (k, seq) SELECT k, seq FROM utxo.upow_journal_state')
        c.execute('COMMIT')
        if move:
            logger.info('ledger: split unspent_outputs over two database files')

    def _open_writer(self, cache_mb: int):
        """The native writer owns its own connection to the same file. Opening it re-applies any
        journal records that were committed but not yet materialised when the process stopped."""
        from ..ops.native import lib
        # durability: 'block' (default) fdatasyncs every block record before push_block answers and gossips;
        # mempool admissions are synced by the materialisers' group sync (a lost admission is a lost mempool
        # entry, never a lost block). 'group' syncs only there; 'commit' syncs every record; 'off' never.
        mode = {'off': 0, 'group': 1, 'commit': 2, 'block': 3}[os.environ.get('UPOW_JOURNAL_SYNC', 'block')]
        if self.path == ':memory:':
            mode = 0
        self._journal_sync_mode = mode
        journal = os.environ.get('UPOW_JOURNAL_PATH') or os.path.join(os.path.dirname(os.path.abspath(self.file)),
                                                                       os.path.basename(self.file) + '.journal')
        self.writer = lib().LedgerWriter([self.file, *(f for _, f in self._split_files())], journal, mode, cache_mb,
                                         # records per materialiser transaction: a lagging materialiser takes
                                         # up to this many per commit (an aged 5 M-row ledger: 32 vs 8 halves the
                                         # commit time, profiles/r4/verify_aged_writer_ab_r4g.json)
                                         int(os.environ.get('UPOW_WRITER_GROUP', '32')),
                                         int(os.environ.get('UPOW_JOURNAL_MAX_MB', '1024')) << 20,
                                         # undo data of the last N blocks survives journal rotation: a
                                         # rollback over the reference's 500-block fork window never rebuilds
                                         int(os.environ.get('UPOW_UNDO_KEEP', '600')),
                                         # a block submit waits while a materialiser's backlog exceeds this (a
                                         # 2 MB block is one ~8 MB record in every materialiser's queue): the SQL
                                         # files trail the journal by at most ~3 blocks, a short drain instead of a
                                         # backlog that grows through a long sync (profiles/r4/verify_aged60_*)
                                         int(os.environ.get('UPOW_WRITER_MAX_QUEUE_MB', '24')) << 20,
                                         float(os.environ.get('UPOW_WRITER_THROTTLE_TIMEOUT', '300')),
                                         int(os.environ.get('UPOW_WRITER_BUSY_MS', '5000')))
        self._eph['writer'] = self.writer if self.path == ':memory:' else None
        self.journal_path = journal
        st = self.writer.stats()
        self._submitted = st['submitted']
        self._applied_seen = {-1: st['applied']}
        if st['replayed']:
            logger.info(f'ledger journal: re-applied {st["replayed"]} committed batch(es) to the SQL tables')

    # ------------------------------------------------------------------ lifecycle
    @staticmethod
    async def create(path: Optional[str] = None, ignore: bool = False, utxo_backend: Optional[str] = None,
                     **_ignored) -> 'Database':
        """reference: database.py:34-85 (asyncpg pool + migrations) -> embedded store + UTXO index."""
        path = path or os.environ.get('UPOW_DATABASE_PATH') or ':memory:'
        if path != ':memory:':
            os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        self = Database(path, utxo_backend=utxo_backend)
        Database.instance = self
        return self

    @staticmethod
    async def get() -> 'Database':
        if Database.instance is None:
            await Database.create(**Database.credentials)
        return Database.instance

    def _tip_id(self) -> int:
        tip = self._lean_tip if self._lean_tip is not None else self._tip_cache
        if tip is not None:
            return int(tip['id'])
        row = self._q1('SELECT MAX(id) FROM blocks')
        return int(row[0] or 0)

    _ckpt_stop: Optional[threading.Event] = None
    _ckpt_thread: Optional[threading.Thread] = None

    def _start_checkpointer(self, period: float):
        """WAL checkpoints on a daemon thread: ``PRAGMA wal_checkpoint(PASSIVE)`` copies committed frames
        back into the database file without blocking the writer (the fsync happens here, not at the
        block's COMMIT). sqlite3 releases the GIL while the checkpoint runs."""
        self._ckpt_stop = threading.Event()
        path = self.file
        files = self._split_files()

        # one file per period, round-robin: a checkpoint of every attached file at once (11 WALs copied back
        # and fsync'd in one statement) made readers of those files wait for ~200 ms at a time, among them
        # the HTTP loop's push_tx lookups (profiles/r4/node_soak_checkpoint_ab_r4w.json)
        schemas = ['main', *(sch for sch, _ in files)]

        def run(stop: threading.Event):
            conn = sqlite3.connect(path, check_same_thread=False, isolation_level=None)
            for schema, f in files:
                conn.execute(f'ATTACH DATABASE ? AS {schema}', (f,))
            k = 0
            try:
                while not stop.wait(period / len(schemas)):
                    schema = schemas[k % len(schemas)]
                    k += 1
                    try:
                        conn.execute(f'PRAGMA {schema}.wal_checkpoint(PASSIVE)').fetchall()
                    except sqlite3.Error as e:  # busy/locked: try again next round
                        logger.debug(f'WAL checkpoint of {schema} skipped: {e}')
            finally:
                conn.close()

        self._ckpt_thread = threading.Thread(target=run, args=(self._ckpt_stop,), name='upow-wal-checkpoint',
                                             daemon=True)
        self._ckpt_thread.start()

    def close(self):
        if self.lean_log is not None:
            self.lean_log.close()
        if self._ckpt_stop is not None:
            self._ckpt_stop.set()
            self._ckpt_thread.join(timeout=10)
            self._ckpt_stop = None
        if self.writer is not None:
            self.writer.close()  # drains the queue into SQL first
        self.emission_details.close()
        with self.lock:
            self._conn.close()
        if self.path == ':memory:':
            _cleanup_ephemeral(self._eph)

    # ------------------------------------------------------------------ materialisation barrier
    def _settle(self, tables: Optional[frozenset] = None):
        """Wait until the SQL tables in ``tables`` (None: all) hold every batch committed to the
        journal that writes them. No-op when the writer is idle or absent."""
        if self.writer is None:
            return
        if self._tx_depth and self._tx_owner == threading.get_ident():
            # inside this thread's open SQL transaction: a batch journaled since BEGIN cannot be
            # materialised before COMMIT (it needs the write lock), so waiting would deadlock
            return
        if tables is None:
            waits = {-1: self._submitted}
        else:
            ts = self._table_seq
            waits = {}
            for t in tables:
                seq = ts.get(t, 0)
                for sh in self._shard_of.get(t, (0,)):
                    if seq > waits.get(sh, 0):
                        waits[sh] = seq
        seen = self._applied_seen
        for sh, target in waits.items():
            if target <= seen.get(sh, 0) or target <= seen.get(-1, 0):
                continue
            applied = self.writer.applied(sh)
            if applied < target:
                self.writer.wait(target, sh, float(os.environ.get('UPOW_WRITER_WAIT_TIMEOUT', '600')))
                applied = target
            seen[sh] = max(seen.get(sh, 0), applied)

    def _fresh(self, table: str) -> bool:
        """Does ``table`` already hold every journaled batch that writes it? (never waits)"""
        if self.writer is None:
            return True
        seq = self._table_seq.get(table, 0)
        seen = self._applied_seen
        if seq <= seen.get(-1, 0):
            return True
        for sh in self._shard_of.get(table, (0,)):
            if seq <= seen.get(sh, 0):
                continue
            applied = self.writer.applied(sh)
            if applied < seq:
                return False
            seen[sh] = max(seen.get(sh, 0), applied)
        return True

    def lagging(self) -> bool:
        """Is any journaled batch not yet in SQL? (never waits)"""
        if self.writer is None:
            return False
        target = self._submitted
        return target > self._applied_seen.get(-1, 0) and self.writer.applied(-1) < target

    async def asettle(self, tables: Optional[frozenset] = None):
        """:meth:`_settle` for an event loop: the wait runs on an executor thread (the native wait
        releases the GIL), so one request waiting for the materialiser does not stall the others."""
        if self.lagging():
            import asyncio
            await asyncio.get_running_loop().run_in_executor(None, self._settle, tables)

    def publish_writer_metrics(self):
        """Journal/materialiser state as gauges for GET /metrics: a stopped writer (row-count mismatch = the
        HBM index and SQL diverged, or an I/O error) must be visible to monitoring, not only in the log."""
        if self.writer is None:
            return
        from ..utils import metrics
        st = self.writer.stats()
        g = metrics.set_gauge
        g('upow_ledger_writer_failed', int(bool(st['failed'])), help='1 when the ledger writer stopped after an error')
        g('upow_ledger_row_mismatches', st['change_mismatches'], help='statements whose row count differed from the block')
        g('upow_ledger_journal_lag', st['submitted'] - st['applied'], help='journal records not yet in SQL')
        g('upow_ledger_queued_bytes', st['queued_bytes'], help='bytes queued for the slowest materialiser')
        g('upow_ledger_throttle_seconds', st['throttle_s'], help='time block submits waited on a lagging materialiser')
        g('upow_ledger_busy_retries', st['busy_retries'], help='materialiser groups retried after SQLITE_BUSY')
        g('upow_ledger_journal_synced', st['synced'], help='last journal sequence made durable (fdatasync)')
        g('upow_ledger_undo_blocks', st['undo_blocks'], help='blocks with undo data retained for rollback')

    def flush(self):
        """Block until the SQL tables hold every committed block (tests, tools, shutdown)."""
        self._settle(None)

    @property
    def conn(self) -> sqlite3.Connection:
        """The Python connection, after the tables are fully materialised (direct callers may read or
        write anything). Hot paths use :meth:`_q`/:meth:`_x`, which only wait for what they touch."""
        self._settle(None)
        self._invalidate_for(None)
        return self._conn

    def _invalidate_for(self, tables: Optional[frozenset]):
        if tables is None or 'blocks' in tables or 'transactions' in tables:
            self._info_cache.clear()
        if tables is None or 'blocks' in tables:
            self._tip_cache = None
            self._recent_rows.clear()
            self._genesis_cache = None
            self._tip_gen += 1
        if tables is None or 'pending_transactions' in tables or 'pending_spent_outputs' in tables:
            self._pending_empty = None
            self._mempool_ver += 1
            self._mp = None

    _journal_sync_mode = 0

    def submit_batch(self, stmts: List[bytes], tables: Iterable[str], meta: bytes = b'', block_id: int = -1,
                     defer_sync: bool = False, write_behind: bool = False) -> int:
        """Commit a batch of encoded statements (``lib().ledger_encode_stmt``) through the journal.

        Does not take the connection lock: a block's batch is megabytes, and the /push_tx path must not
        queue behind its journal write. A batch journaled while another thread has a Python-side SQL
        transaction open is materialised after that transaction commits (the materialiser needs the
        write lock), which is the order the two would have had if the batch had waited; the
        transaction's own reads do not wait for it (see :meth:`_settle`).

        The native submit orders records itself (its journal mutex assigns the sequence numbers); the
        sequence lock here only guards the per-table bookkeeping, which takes maxima and so does not
        care in which order concurrent submitters get there. A /push_tx admission therefore waits at
        most for the journal write of a concurrent block, not for its payload assembly too."""
        if self._tx_depth and self._tx_owner == threading.get_ident():
            raise RuntimeError('ledger batch submitted inside an open SQL transaction')
        if defer_sync:
            # the writer's journal I/O thread checksums, writes and fdatasyncs the block record (and stores
            # its undo data) while the caller updates its indexes; the sequence number is fixed here. The
            # block is not answered or gossiped before wait_durable() (UPOW_JOURNAL_SYNC=block semantics).
            # Inside a group commit (a sync page, ledger/pagesync.py) the record is not synced on its own: the
            # page's closing wait_durable() makes every block of the page durable with one fdatasync.
            seq = self.writer.submit(stmts, meta, block_id, False, self.group_commit > 0)
            self._durable_seq = seq
        elif write_behind and self._journal_sync_mode != 2:
            # a mempool record (not synced on its own unless UPOW_JOURNAL_SYNC=commit): the sequence number
            # is reserved here and the writer's I/O thread writes it, so the HTTP loop never waits behind a
            # block record's multi-megabyte write on the same file
            seq = self.writer.submit(stmts, meta, block_id, False)
        else:
            seq = self.writer.submit(stmts, meta, block_id)
        with self._seq_lock:
            if seq > self._submitted:
                self._submitted = seq
            for t in tables:
                if seq > self._table_seq.get(t, 0):
                    self._table_seq[t] = seq
        return seq

    _durable_seq = 0
    utxo_defer = False  # True while a sync page applies plan-checked blocks (UtxoIndex.defer_block)
    group_commit = 0  # > 0 while a sync page applies its blocks (ledger/pagesync.py): one fdatasync per page

    def wait_durable(self, force: bool = False):
        """Block until the last block record submitted with ``defer_sync`` is written and on disk (raises when
        the writer failed on it: a journal write error after the commit point stops the ledger). During a group
        commit this is a no-op unless ``force``: the page's end makes the whole page durable at once."""
        if self.group_commit > 0 and not force:
            return
        seq, self._durable_seq = self._durable_seq, 0
        if seq and self.writer is not None:
            self.writer.durable(seq)

    # ------------------------------------------------------------------ SQL helpers
    def _q(self, sql: str, args: Iterable = ()) -> List[sqlite3.Row]:
        self._settle(_tables_of(sql, False))
        with self.lock:
            return self._conn.execute(sql, tuple(args)).fetchall()

    def _q1(self, sql: str, args: Iterable = ()):
        self._settle(_tables_of(sql, False))
        with self.lock:
            return self._conn.execute(sql, tuple(args)).fetchone()

    def _x(self, sql: str, args: Iterable = ()):
        t = _tables_of(sql, True)
        self._settle(t)
        with self.lock:
            self._invalidate_for(t)
            split = self._split_target(sql)
            if split is not None:
                return self._routed_exec(split, sql, [tuple(args)])
            return self._conn.execute(sql, tuple(args))

    def _xm(self, sql: str, rows: Iterable):
        t = _tables_of(sql, True)
        self._settle(t)
        with self.lock:
            self._invalidate_for(t)
            split = self._split_target(sql)
            if split is not None:
                return self._routed_exec(split, sql, list(rows))
            return self._conn.executemany(sql, rows)

    class _Changed:
        def __init__(self, n: int):
            self.rowcount = n

    _SPLIT_INSERT = re.compile(r'^\s*INSERT\s+(OR\s+\w+\s+)?INTO\s+(unspent_outputs|transactions)\s*\(([^)]*)\)\s*VALUES',
                               re.I)
    _SPLIT_TARGET = re.compile(r'^(\s*(?:DELETE\s+FROM|UPDATE))\s+(unspent_outputs|transactions)\b', re.I)

    def _split_target(self, sql: str) -> Optional[str]:
        """The split table a write statement targets (None: an ordinary table, or ``transactions`` of a
        ledger that keeps it in the main file). Memoised per statement text: the block path encodes the same
        handful of statements for every block."""
        cache = self.__dict__.setdefault('_split_cache', {})
        hit = cache.get(sql, cache)
        if hit is not cache:
            return hit
        m = self._SPLIT_INSERT.match(sql) or self._SPLIT_TARGET.match(sql)
        t = None if m is None else m.group(2).lower()
        t = t if t in self._routed else None
        if len(cache) < 4096:
            cache[sql] = t
        return t

    def _utxo_rowids(self, n: int) -> int:
        """First of ``n`` consecutive row ids from the ledger-wide UTXO counter."""
        with self._seq_lock:
            base = self._utxo_next_rowid
            self._utxo_next_rowid += n
        return base

    def _tx_rowids(self, n: int) -> int:
        """First of ``n`` consecutive row ids from the ledger-wide transactions counter."""
        with self._seq_lock:
            base = self._tx_next_rowid
            self._tx_next_rowid += n
        return base

    # the journaled tx-row insert: tx hash in column 0 (a split table's routing key), explicit row id
    _TX_INSERT = ('INSERT INTO transactions (tx_hash, block_hash, tx_hex, inputs_addresses, outputs_addresses, '
                  'outputs_amounts, fees, rowid) VALUES (?, ?, ?, ?, ?, ?, ?, ?)')

    def _routed_exec(self, table: str, sql: str, rows: list) -> '_Changed':
        """A Python-side write to a split table (caller holds the lock, tables settled), routed to the
        file(s) holding the rows: INSERTs by tx hash with row ids from the table's ledger-wide counter,
        ``DELETE ... WHERE tx_hash = ? ...`` by tx hash, anything else on every file."""
        c = self._conn
        schemas = self.utxo_schemas if table == 'unspent_outputs' else self.tx_schemas
        nf = len(schemas)
        m = self._SPLIT_INSERT.match(sql)
        if m:
            cols = [x.strip().strip('"') for x in m.group(3).split(',')]
            h = cols.index('tx_hash')
            values = sql[m.end():]
            if 'rowid' not in cols:
                base = (self._utxo_rowids if table == 'unspent_outputs' else self._tx_rowids)(len(rows))
                rows = [(*r, base + k) for k, r in enumerate(rows)]
                values = values.replace(')', ', ?)', 1)
                cols.append('rowid')
            names = ', '.join(chr(34) + x + chr(34) if x == 'index' else x for x in cols)
            head = f'INSERT {m.group(1) or ""}INTO %s.{table} ({names}) VALUES'
            n = 0
            for f, schema in enumerate(schemas):
                part = [r for r in rows if file_of(r[h], nf) == f]
                if part:
                    n += c.executemany(head % schema + values, part).rowcount
            return self._Changed(n)
        m = self._SPLIT_TARGET.match(sql)
        by_hash = re.search(r'\bWHERE\s+tx_hash\s*=\s*\?', sql, re.I) is not None
        n = 0
        for f, schema in enumerate(schemas):
            part = [r for r in rows if file_of(r[0], nf) == f] if by_hash else rows
            if part:
                q = m.group(1) + f' {schema}.{table}' + sql[m.end():]
                n += c.executemany(q, part).rowcount if part != [()] else c.execute(q).rowcount
        return self._Changed(n)

    def _utxo_cascade(self, tx_hashes: Iterable[str]):
        """``ON DELETE CASCADE`` from transactions to unspent_outputs (schema.sql) for deleted txs."""
        hs = [(h,) for h in tx_hashes]
        if hs:
            self._xm('DELETE FROM unspent_outputs WHERE tx_hash = ?', hs)

    # ------------------------------------------------------------------ native bulk writes
    def encode(self, sql: str, cols: list, n: int, order=None, guard: Optional[str] = None,
               expect: Optional[int] = None) -> bytes:
        """One column-major bulk statement for :meth:`submit_batch`. Column specs as in
        csrc/ledger_writer.cpp: text lists, int64 arrays, ('gather'|'hex32'|'arena', ...) views of the
        block codec's buffers, or one constant for every row. A statement on a split table is spread over
        its files by the tx hash in column 0."""
        from ..ops.native import lib
        split = self._split_target(sql)
        if split is not None:
            first, count = self._routed[split]
            return lib().ledger_encode_stmt(sql, cols, n, order, guard, expect, first, count)
        return lib().ledger_encode_stmt(sql, cols, n, order, guard, expect, 0)  # every other table: main file

    def encode_many(self, stmts: list) -> list:
        """:meth:`encode` of a block's statements, the large ones concurrently: each encode copies its
        columns with the GIL released, so a block's ~4 multi-MB statements (tx rows, UTXO rows, spends,
        address rows) are copied on pool threads side by side instead of one after another."""
        out = [None] * len(stmts)
        todo = list(range(len(stmts)))
        big = [k for k in todo if stmts[k][2] >= 1024]
        if len(big) < 2 or _ENCODE_THREADS < 2:
            for k in todo:
                out[k] = self.encode(*stmts[k])
            return out
        global _ENCODE_POOL
        if _ENCODE_POOL is None:
            from concurrent.futures import ThreadPoolExecutor
            _ENCODE_POOL = ThreadPoolExecutor(max_workers=_ENCODE_THREADS, thread_name_prefix='upow-encode')
        futs = {k: _ENCODE_POOL.submit(self.encode, *stmts[k]) for k in big[1:]}
        for k in todo:
            if k not in futs:
                out[k] = self.encode(*stmts[k])  # the first big one and the small ones on this thread meanwhile
        for k, f in futs.items():
            out[k] = f.result()
        return out

    def bulk(self, sql: str, cols: list, n: int, order=None) -> int:
        """Column-major executemany on the Python connection (synchronous); returns the row changes."""
        if n == 0:
            return 0
        rows = list(zip(*[_expand_col(c, n) for c in cols]))
        if isinstance(order, str):  # 'key': by the leading 8 bytes of the column-0 hashes
            order = np.argsort(np.array([bytes.fromhex(r[0][:16]) for r in rows], dtype='S8'), kind='stable')
        if order is not None:
            rows = [rows[i] for i in np.asarray(order).tolist()]
        return self._xm(sql, rows).rowcount

    class _Tx:
        """Re-entrant SQL transaction: only the outermost level issues BEGIN/COMMIT/ROLLBACK, so a
        whole block application (many helper calls) commits or rolls back as one unit. The outermost
        level first waits for the native writer to drain (it cannot take the write lock meanwhile)."""

        def __init__(self, db, foreign_keys: bool = True, invalidate: bool = True):
            self.db = db
            self.fk = foreign_keys
            self.inv = invalidate

        def __enter__(self):
            self.db.lock.acquire()
            if self.db._tx_depth == 0:
                try:  # no SQL transaction is open on this connection: safe to wait for the writer
                    self.db._settle(None)
                except BaseException:
                    self.db.lock.release()
                    raise
                c = self.db._conn
                if not self.fk:  # only settable outside a transaction
                    c.execute('PRAGMA foreign_keys = OFF')
                c.execute('BEGIN')
                self.db._tx_owner = threading.get_ident()
                self.db._fk_off = not self.fk
                self.db._tx_inv = self.inv
                if self.inv:
                    self.db._invalidate_for(None)
            self.db._tx_depth += 1
            return self.db

        def __exit__(self, et, ev, tb):
            try:
                self.db._tx_depth -= 1
                if self.db._tx_depth == 0:
                    self.db._conn.execute('COMMIT' if et is None else 'ROLLBACK')
                    if self.db._tx_inv:
                        self.db._invalidate_for(None)
                    if self.db._fk_off:
                        if self.db._fk:
                            self.db._conn.execute('PRAGMA foreign_keys = ON')
                        self.db._fk_off = False
                elif et is not None:
                    self.db._tx_failed = True
            finally:
                self.db.lock.release()
            return False

    _tx_depth = 0
    _tx_owner = None
    _tx_inv = True
    _tx_failed = False
    _fk_off = False

    def transaction(self, foreign_keys: bool = True, invalidate: bool = True):
        """``foreign_keys=False``: skip FK enforcement for this (outermost) transaction.
        ``invalidate=False``: the caller writes only through ``_x``/``_xm`` (which invalidate per table)
        or invalidates what it wrote itself; the host caches are not dropped wholesale."""
        return Database._Tx(self, foreign_keys, invalidate)

    # fault injection (tests): raise inside block application after the named stage
    fail_after_stage: Optional[str] = None

    def checkpoint(self, stage: str):
        if self.fail_after_stage == stage:
            raise RuntimeError(f'injected failure after {stage}')

    @staticmethod
    def _txq(col: str, key: str) -> str:
        """Column ``col`` of the tx whose hash is the SQL expression ``key``, as a correlated lookup. Where
        ``transactions`` is split over several files, SQLite materialises the whole view to join it, but a
        correlated lookup is pushed into each file's tx-hash index (rows without their tx come back NULL,
        which callers of an INNER JOIN form skip)."""
        return f'(SELECT t_.{col} FROM transactions t_ WHERE t_.tx_hash = {key})'

    def _tx_source_for_utxo(self, k: int) -> Optional[str]:
        """The one transactions table holding the txs of every row of UTXO file ``k`` (same hash routing), or
        None when its hash range spans several tx files."""
        if not self.tx_schemas:
            return 'main.transactions'
        nu, nt = len(self.utxo_schemas), len(self.tx_schemas)
        lo, hi = (k * 256 + nu - 1) // nu, ((k + 1) * 256 + nu - 1) // nu  # first bytes b with b * nu >> 8 == k
        files = {file_of(f'{b:02x}', nt) for b in range(lo, hi)}
        return f'{self.tx_schemas[files.pop()]}.transactions' if len(files) == 1 else None

    def _rebuild_utxo_index(self):
        """Rebuild the HBM/host UTXO set from the output tables; each entry's payload (amount,
        address bytes) comes from its creating tx's JSON columns, read with SQLite's json_extract."""
        keys, tags, amounts, addrs, stake = [], [], [], [], []
        am = 'json_extract(t.outputs_amounts, \'$[\' || u."index" || \']\')'
        ad = 'json_extract(t.outputs_addresses, \'$[\' || u."index" || \']\')'
        queries = []
        for table in OUTPUT_TABLES:
            if table != 'unspent_outputs':
                queries.append((table, f'SELECT u.tx_hash, u."index", '
                                       f'(SELECT {am} FROM transactions t WHERE t.tx_hash = u.tx_hash), '
                                       f'(SELECT {ad} FROM transactions t WHERE t.tx_hash = u.tx_hash), NULL '
                                       f'FROM {table} u'))
                continue
            for k, sch in enumerate(self.utxo_schemas):  # each UTXO file against the tx file of its hash range
                src = self._tx_source_for_utxo(k)
                if src is not None:
                    queries.append((table, f'SELECT u.tx_hash, u."index", {am}, {ad}, u.is_stake '
                                           f'FROM {sch}.unspent_outputs u LEFT JOIN {src} t ON t.tx_hash = u.tx_hash'))
                else:
                    queries.append((table, f'SELECT u.tx_hash, u."index", '
                                           f'(SELECT {am} FROM transactions t WHERE t.tx_hash = u.tx_hash), '
                                           f'(SELECT {ad} FROM transactions t WHERE t.tx_hash = u.tx_hash), u.is_stake '
                                           f'FROM {sch}.unspent_outputs u'))
        for table, sql in queries:
            tag = TAG_BY_TABLE[table]
            for r in self._q(sql):
                keys.append((r[0], r[1]))
                tags.append(tag)
                amounts.append(r[2])
                addrs.append(_addr_bytes(r[3]))
                stake.append(r[4] == 1)
        self.utxo.reset(keys, tags, make_payload(amounts, addrs, stake))
        if getattr(self, 'gov', None) is not None:
            self.gov.rebuild()

    async def _payload_from_ledger(self, outpoints: List[Tuple[str, int]], stake=None):
        infos = await self.get_transactions_info([h for h, _ in outpoints])
        amounts, addrs = [], []
        for h, i in outpoints:
            info = infos.get(h)
            amounts.append(_at(info['outputs_amounts'], i) if info else None)
            addrs.append(_addr_bytes(_at(info['outputs_addresses'], i)) if info else None)
        return make_payload(amounts, addrs, stake)

    def _select_outpoints(self, table: str, outputs: List[Tuple[str, int]]) -> List[Tuple[str, int]]:
        """``SELECT tx_hash, index FROM <table> WHERE (tx_hash, index) = ANY($1)`` (rows in table order)."""
        if not outputs:
            return []
        want = {(str(h), int(i)) for h, i in outputs}
        if len(want) <= 32:
            # a single tx's inputs (mempool admission): exact (tx_hash, index) probes on the outpoint
            # index, instead of pulling every row of each funding tx (often hundreds) into Python
            found = []
            self._settle(frozenset((table,)))
            with self.lock:
                for h, i in want:
                    for r in self._conn.execute(f'SELECT rowid FROM {table} WHERE tx_hash = ? AND "index" = ?', (h, i)):
                        found.append((r[0], (h, i)))
            found.sort()
            return [o for _, o in found]
        hashes = sorted({h for h, _ in want})
        out = []
        for k in range(0, len(hashes), 500):
            chunk = hashes[k:k + 500]
            ph = ','.join('?' * len(chunk))
            for r in self._q(f'SELECT rowid, tx_hash, "index" FROM {table} WHERE tx_hash IN ({ph})', chunk):
                if (r[1], r[2]) in want:
                    out.append((r[0], (r[1], r[2])))
        out.sort()
        return [o for _, o in out]

    def _delete_outpoints(self, table: str, inputs: List[Tuple[str, int]]) -> int:
        return self._xm(f'DELETE FROM {table} WHERE tx_hash = ? AND "index" = ?',
                        [(h, int(i)) for h, i in inputs]).rowcount

    _PENDING = frozenset(('pending_transactions', 'pending_spent_outputs'))

    def _mempool(self) -> Optional[MempoolIndex]:
        """The host mempool index (ledger/mempool.py), loaded from SQL when dropped; None without the
        journal writer (SQL is then always current) or with ``UPOW_MEMPOOL_INDEX=0``."""
        if self.writer is None or not self.mempool_index:
            return None
        mp = self._mp
        if mp is None:
            self._settle(self._PENDING)
            with self.lock:
                mp = MempoolIndex(self._conn.execute('SELECT tx_hash, propagation_time, tx_hex, fees '
                                                     'FROM pending_transactions'),
                                  self._conn.execute('SELECT tx_hash, "index" FROM pending_spent_outputs'))
                self._mp = mp
            self.mempool_reloads += 1
        return mp

    def _mempool_confirm(self, mempool_deleted: bool, txids=None, in_keys=None, hashes=None, inputs=None,
                         block_seq: int = 0):
        """A committed block's txs and inputs leave the mempool index. The block's own batch deletes them
        from the tables only if it carried the mempool DELETEs and the tx's INSERTs were journaled before
        it; a tx of the block whose admission batch came after the block's (admitted on the HTTP loop while
        the block was being applied) is deleted by a follow-up batch, journaled after those INSERTs."""
        mp = self._mp
        if mp is None:
            if self.on_confirm is not None:  # no index: the block's SQL deletes cover all its txs and inputs
                if txids is not None:
                    kk = np.asarray(in_keys, dtype=np.uint8)
                    self.on_confirm(None, [bytes(r) for r in np.asarray(txids, np.uint8).reshape(-1, 32)],
                                    [bytes(r[:36]) for r in kk.reshape(-1, kk.shape[-1] if kk.ndim == 2 else 40)])
                else:
                    from .mempool import outpoint_key
                    self.on_confirm(None, [bytes.fromhex(h) for h in hashes or []],
                                    [outpoint_key(h, i) for h, i in inputs or []])
            return
        if txids is not None:
            hit_tx, hit_in, late_tx, late_in = mp.confirm_raw(txids, in_keys, block_seq, self.on_confirm)
        else:
            hit_tx, hit_in, late_tx, late_in = mp.confirm(hashes or [], inputs or [], block_seq, self.on_confirm)
        if not (hit_tx or hit_in):
            return
        self._pending_empty = None
        self._mempool_ver += 1
        if not mempool_deleted:
            late_tx, late_in = hit_tx, hit_in
        if not (late_tx or late_in):
            return
        stmts = []
        if late_tx:
            stmts.append(self.encode('DELETE FROM pending_transactions WHERE tx_hash = ?',
                                     [[h.hex() for h in late_tx]], len(late_tx)))
        if late_in:
            stmts.append(self.encode('DELETE FROM pending_spent_outputs WHERE tx_hash = ? AND "index" = ?',
                                     [[k[:32].hex() for k in late_in],
                                      np.array([int.from_bytes(k[32:36], 'little') for k in late_in], np.int64)],
                                     len(late_in)))
        self.submit_batch(stmts, self._PENDING, write_behind=True)

    def _pending_spent_set(self) -> Set[Tuple[str, int]]:
        return {(r[0], r[1]) for r in self._q('SELECT tx_hash, "index" FROM pending_spent_outputs')}

    # ------------------------------------------------------------------ mempool (database.py:93-231)
    async def add_pending_transaction(self, transaction: Transaction, verify: bool = True) -> bool:
        logger.info('Adding in pending transaction')
        if isinstance(transaction, CoinbaseTransaction):
            logger.error('CoinbaseTransaction in add_pending_transaction')
            return False
        tx_hex = transaction.hex()
        if verify and not await transaction.verify_pending():
            logger.error('Error in adding transaction.')
            return False
        inputs_addresses = [await _input_address(i) for i in transaction.inputs]
        mp = self._mempool() if verify else None
        if mp is not None:
            return self._admit(mp, transaction, tx_hex, inputs_addresses)
        ptime = int(_utcnow().replace(tzinfo=timezone.utc).timestamp())
        try:
            self._x('INSERT INTO pending_transactions (tx_hash, tx_hex, inputs_addresses, fees, propagation_time) '
                    'VALUES (?, ?, ?, ?, ?)',
                    (sha256(tx_hex), tx_hex, _j(inputs_addresses), numeric(transaction.fees, 6), ptime))
        except sqlite3.IntegrityError as e:
            raise UniqueViolationError(str(e)) from e
        await self.add_transactions_pending_spent_outputs([transaction])
        if self.on_admit is not None:
            self.on_admit([tx_hex, _j(inputs_addresses), numeric(transaction.fees, 6), ptime,
                           [[i.tx_hash, int(i.index)] for i in transaction.inputs], sha256(tx_hex)])
        return True

    def _admit(self, mp: MempoolIndex, transaction: Transaction, tx_hex: str, inputs_addresses: list) -> bool:
        """Journaled admission of a verified tx: reserve it in the mempool index, then commit its
        pending_transactions and pending_spent_outputs rows as one batch (both under the index lock,
        so a block that later finds the tx in the index knows its rows are already journaled)."""
        tx_hash = sha256(tx_hex)
        ptime = int(_utcnow().replace(tzinfo=timezone.utc).timestamp())
        inputs = [(i.tx_hash, int(i.index)) for i in transaction.inputs]
        fees = numeric(transaction.fees, 6)
        with mp.lock:
            why = mp.try_add(tx_hash, ptime, inputs, tx_hex, fees)
            if why == 'duplicate':
                raise UniqueViolationError(f'UNIQUE constraint failed: pending_transactions.tx_hash ({tx_hash})')
            if why is not None:
                logger.error(f'Double spending in pending {tx_hash}')
                return False
            # OR IGNORE: a statement error would stop the materialiser; the index already refused duplicates
            stmts = [self.encode('INSERT OR IGNORE INTO pending_transactions (tx_hash, tx_hex, inputs_addresses, fees, '
                                 'propagation_time) VALUES (?, ?, ?, ?, ?)',
                                 [tx_hash, tx_hex, _j(inputs_addresses), fees, ptime], 1)]
            if inputs:
                stmts.append(self.encode('INSERT INTO pending_spent_outputs (tx_hash, "index") VALUES (?, ?)',
                                         [[h for h, _ in inputs], np.array([i for _, i in inputs], np.int64)],
                                         len(inputs)))
            seq = self.submit_batch(stmts, self._PENDING, write_behind=True)
            mp.set_seq(tx_hash, inputs, seq)
            if self.on_admit is not None:  # cluster leader: replicate the admitted row (under the index lock)
                self.on_admit([tx_hex, _j(inputs_addresses), fees, ptime, [[h, i] for h, i in inputs], tx_hash])
        self._pending_empty = False
        self._mempool_ver += 1
        return True

    def admit_replicated(self, rows: List[list]) -> int:
        """Insert mempool rows admitted (and verified) by the cluster leader: ``[tx_hex, inputs_addresses
        JSON, fees, propagation_time, [[txid, index], ...]]`` each (parallel/cluster.py). No re-verification:
        the rows reproduce the leader's tables and index exactly, as one index pass under the index lock and
        one journal batch. Returns how many rows were inserted."""
        if not rows:
            return 0
        mp = self._mempool()
        if mp is None:
            n = 0
            for tx_hex, ia, fees, ptime, inputs in rows:
                try:
                    self._x('INSERT INTO pending_transactions (tx_hash, tx_hex, inputs_addresses, fees, '
                            'propagation_time) VALUES (?, ?, ?, ?, ?)', (sha256(tx_hex), tx_hex, ia, fees, int(ptime)))
                except sqlite3.IntegrityError:
                    continue
                if inputs:
                    self._xm('INSERT INTO pending_spent_outputs (tx_hash, "index") VALUES (?, ?)',
                             [(h, int(i)) for h, i in inputs])
                n += 1
            return n
        acc = []
        with mp.lock:
            for tx_hex, ia, fees, ptime, inputs in rows:
                h = sha256(tx_hex)
                ins = [(a, int(b)) for a, b in inputs]
                why = mp.try_add(h, int(ptime), ins, tx_hex, fees)
                if why is not None:
                    logger.error(f'cluster replica: leader mempool row {h} refused ({why})')
                    continue
                acc.append((h, tx_hex, ia, fees, int(ptime), ins))
            if not acc:
                return 0
            stmts = [self.encode('INSERT OR IGNORE INTO pending_transactions (tx_hash, tx_hex, inputs_addresses, fees, '
                                 'propagation_time) VALUES (?, ?, ?, ?, ?)',
                                 [[a[0] for a in acc], [a[1] for a in acc], [a[2] for a in acc], [a[3] for a in acc],
                                  np.array([a[4] for a in acc], np.int64)], len(acc))]
            spent = [(h, i) for a in acc for h, i in a[5]]
            if spent:
                stmts.append(self.encode('INSERT INTO pending_spent_outputs (tx_hash, "index") VALUES (?, ?)',
                                         [[h for h, _ in spent], np.array([i for _, i in spent], np.int64)], len(spent)))
            seq = self.submit_batch(stmts, self._PENDING, write_behind=True)
            for a in acc:
                mp.set_seq(a[0], a[5], seq)
        self._pending_empty = False
        self._mempool_ver += 1
        return len(acc)

    def clear_mempool(self):
        """Empty both mempool tables (a cluster replica about to take the leader's mempool)."""
        self.flush()
        self._x('DELETE FROM pending_spent_outputs')
        self._x('DELETE FROM pending_transactions')
        self._pending_empty = None
        self._mempool_ver += 1

    async def remove_pending_transaction(self, tx_hash: str):
        self._x('DELETE FROM pending_transactions WHERE tx_hash = ?', (tx_hash,))

    def remove_pending_by_txids(self, txids: np.ndarray) -> int:
        """``remove_pending_transactions_by_hash`` for a block given as n x 32 raw txids. Empty mempool:
        nothing to do. A mempool much smaller than the block: delete only the hashes it holds. Otherwise
        (the usual case for a mined block, whose txs came from the mempool) one native bulk delete."""
        txids = np.ascontiguousarray(txids, dtype=np.uint8).reshape(-1, 32)
        n_pending = self._q1('SELECT COUNT(*) FROM pending_transactions')[0]
        if n_pending == 0 or not len(txids):
            return 0
        if 4 * n_pending < len(txids):
            pending = {r[0] for r in self._q('SELECT tx_hash FROM pending_transactions')}
            keep = [k for k, t in enumerate(txids) if bytes(t).hex() in pending]
            txids = txids[keep]
            if not len(txids):
                return 0
        return self.bulk('DELETE FROM pending_transactions WHERE tx_hash = ?', [('hex32', txids, 32, 0)],
                         len(txids), self._key_order(txids))

    async def remove_pending_transactions_by_hash(self, tx_hashes: List[str]):
        # only the hashes present in the (small) mempool: no index probe per confirmed tx
        pending = {r[0] for r in self._q('SELECT tx_hash FROM pending_transactions')}
        hit = [(h,) for h in tx_hashes if h in pending] if pending else []
        if hit:
            self._xm('DELETE FROM pending_transactions WHERE tx_hash = ?', hit)

    async def remove_pending_transactions(self):
        with self.transaction():
            deleted = [r[0] for r in self.conn.execute('SELECT tx_hash FROM pending_transactions').fetchall()]
            self.conn.execute('DELETE FROM pending_transactions')
            self.conn.execute('DELETE FROM pending_spent_outputs')
        if deleted:
            logger.info(f'remove_pending_transactions: removed {len(deleted)} transactions: {deleted}')
        else:
            logger.info('remove_pending_transactions: no transactions to remove')

    async def delete_blockchain(self):
        with self.transaction():
            # the cascade from blocks and transactions (every split-table row belongs to a tx)
            for schema in self.tx_schemas or ['main']:
                self._conn.execute(f'DELETE FROM {schema}.transactions')
            for schema in self.utxo_schemas:
                self._conn.execute(f'DELETE FROM {schema}.unspent_outputs')
            if self.tx_schemas:
                for child in self._TX_CHILDREN:
                    self._conn.execute(f'DELETE FROM {child}')
            self.conn.execute('DELETE FROM blocks')
            self.conn.execute("UPDATE address_index_state SET height = 0 WHERE k = 'height'")
        self._rebuild_utxo_index()

    def _block_tx_hashes(self, where: str, args: tuple) -> List[str]:
        """Hashes of the txs of the blocks matching ``where`` (a condition on ``blocks``)."""
        return self._txs_of_blocks([r[0] for r in self._q(f'SELECT hash FROM blocks WHERE {where}', args)], 'tx_hash')

    def _txs_of_blocks(self, block_hashes: List[str], cols: str) -> list:
        """``SELECT cols FROM transactions WHERE block_hash IN (...)`` with literal lists (pushed into each
        file's block_hash index; an IN (subquery) is not), in row id order per chunk of blocks."""
        out = []
        single = ',' not in cols
        for k in range(0, len(block_hashes), 200):
            chunk = block_hashes[k:k + 200]
            rows = self._q(f'SELECT {cols} FROM transactions WHERE block_hash IN ({",".join("?" * len(chunk))}) '
                           f'ORDER BY rowid', chunk)
            out.extend(r[0] for r in rows) if single else out.extend(rows)
        return out

    # tables whose rows belong to a tx (schema.sql: tx_hash REFERENCES transactions ON DELETE CASCADE)
    _TX_CHILDREN = ('pending_spent_outputs', 'address_transactions', *OUTPUT_TABLES[1:])

    def _delete_blocks(self, where: str, args: tuple) -> List[str]:
        """``DELETE FROM blocks WHERE <where>`` with the reference's cascade: blocks -> transactions -> every
        table keyed by their tx hash. A split layout has no foreign keys across its files, so the cascade
        is applied here (one temp table of the deleted hashes); unspent_outputs always is. Returns the
        deleted txs' hashes."""
        gone = self._block_tx_hashes(where, args)
        if self.tx_schemas and gone:
            with self.transaction():
                c = self._conn
                c.execute('CREATE TEMP TABLE IF NOT EXISTS upow_gone (h TEXT PRIMARY KEY)')
                c.execute('DELETE FROM temp.upow_gone')
                c.executemany('INSERT OR IGNORE INTO temp.upow_gone (h) VALUES (?)', [(h,) for h in gone])
                for child in self._TX_CHILDREN:
                    c.execute(f'DELETE FROM main.{child} WHERE tx_hash IN (SELECT h FROM temp.upow_gone)')
                for schema in self.tx_schemas:
                    c.execute(f'DELETE FROM {schema}.transactions WHERE tx_hash IN (SELECT h FROM temp.upow_gone)')
                c.execute('DELETE FROM temp.upow_gone')
        self._x(f'DELETE FROM blocks WHERE {where}', args)
        self._utxo_cascade(gone)
        return gone

    async def delete_block(self, id: int):
        self._delete_blocks('id = ?', (id,))
        self._address_index_rollback()
        self._rebuild_utxo_index()

    async def delete_blocks(self, offset: int):
        self._delete_blocks('id > ?', (offset,))
        self._address_index_rollback()
        self._rebuild_utxo_index()

    async def remove_blocks(self, block_no: int):
        """database.py:146-169: roll back blocks >= block_no and restore the outputs they spent. The UTXO
        index is rolled back from the journal's undo records when every removed block has one, else
        rebuilt from the tables."""
        tip = self._tip_id()
        blocks_to_remove = await self.get_blocks(block_no, 500)
        transactions_to_remove, transactions_hashes = [], []
        for b in blocks_to_remove:
            transactions_to_remove.extend([await Transaction.from_hex(tx, False) for tx in b['transactions']])
            transactions_hashes.extend([sha256(tx) for tx in b['transactions']])
        hashes = set(transactions_hashes)
        outputs_to_be_restored = []
        for tx in transactions_to_remove:
            if isinstance(tx, Transaction):
                outputs_to_be_restored.extend([(i.tx_hash, i.index) for i in tx.inputs if i.tx_hash not in hashes])
        created = self._undo_blocks_in_index(block_no, tip)
        undone = created is not None
        self._delete_blocks('id >= ?', (block_no,))
        self._address_index_rollback()
        await self.add_unspent_outputs(outputs_to_be_restored, index=not undone)
        if self.writer is not None:
            self.writer.forget_blocks_from(block_no)
        if not undone:
            self._rebuild_utxo_index()
        elif self.gov is not None:
            # governance rows of the removed blocks' txs go with them (FK cascade); restored outpoints
            # return as plain unstaked UTXOs, so no governance row comes back: removing is the whole undo
            with self.gov.lock:
                for t in self.gov.tables:
                    self.gov.removed(t, created)
                self.gov.version += 1
        self.utxo_rollbacks = getattr(self, 'utxo_rollbacks', 0) + 1
        self.last_rollback_undo = undone

    def _pending_rows_ordered(self):
        """``ORDER BY fees / LENGTH(tx_hex) DESC, LENGTH(tx_hex), tx_hex`` (database.py:173-174)."""
        rows = self._q('SELECT tx_hash, tx_hex, fees, propagation_time FROM pending_transactions')
        return sorted(rows, key=lambda r: (-(Decimal(r['fees']) / len(r['tx_hex'])), len(r['tx_hex']), r['tx_hex']))

    async def get_pending_transactions_limit(self, limit: int = MAX_BLOCK_SIZE_HEX, hex_only: bool = False,
                                             check_signatures: bool = True) -> List[Union[Transaction, str]]:
        mp = self._mempool()
        if mp is not None:
            return_txs = mp.ordered_hex(limit)
        else:
            return_txs, size = [], 0
            for r in self._pending_rows_ordered():
                tx = r['tx_hex']
                if size + len(tx) > limit:
                    break
                return_txs.append(tx)
                size += len(tx)
        if hex_only:
            return return_txs
        return [await Transaction.from_hex(t, check_signatures) for t in return_txs]

    def mining_template(self, limit: int = MAX_BLOCK_SIZE_HEX, head: int = 10) -> Tuple[List[str], List[str], bytes]:
        """The next block template as ``/get_mining_info`` publishes it (reference main.py:675-695: the
        selected pending txs sorted by hex): (first ``head`` hexes, all tx hashes, those hashes as one JSON
        array body without brackets). From the mempool index in one native call when there is one."""
        mp = self._mempool()
        if mp is not None:
            return mp.mining_template(limit, head)
        hexes, hashes = self.pending_template(limit)
        order = sorted(range(len(hexes)), key=hexes.__getitem__)
        ordered_hashes = [hashes[k] for k in order]
        return [hexes[k] for k in order[:head]], ordered_hashes, ','.join(f'"{h}"' for h in ordered_hashes).encode()

    def pending_template(self, limit: int = MAX_BLOCK_SIZE_HEX) -> Tuple[List[str], List[str]]:
        """(tx hex, tx hash) lists of ``get_pending_transactions_limit(hex_only=True)``; the hashes come
        from the mempool index when there is one instead of being recomputed per call."""
        mp = self._mempool()
        if mp is not None:
            rows = mp.ordered(limit)
            return [hx for hx, _ in rows], [h.hex() for _, h in rows]
        hexes = []
        size = 0
        for r in self._pending_rows_ordered():
            tx = r['tx_hex']
            if size + len(tx) > limit:
                break
            hexes.append(tx)
            size += len(tx)
        return hexes, [sha256(t) for t in hexes]

    async def get_need_propagate_transactions(self, last_propagation_delta: int = 600,
                                              limit: int = MAX_BLOCK_SIZE_HEX) -> List[str]:
        now = int(_utcnow().replace(tzinfo=timezone.utc).timestamp())
        # the node's middleware asks this on EVERY request: only stale txs can be returned, so when no
        # pending tx is older than the delta the answer is [] without ordering the whole mempool (from
        # the mempool index when there is one: no SQL at all)
        mp = self._mempool()
        if mp is not None and not mp.maybe_stale(now, last_propagation_delta):
            return []
        if self._q1('SELECT 1 FROM pending_transactions WHERE propagation_time < ? LIMIT 1',
                    (now - last_propagation_delta,)) is None:
            return []
        return_txs, size = [], 0
        for r in self._pending_rows_ordered():
            tx_hex = r['tx_hex']
            if size + len(tx_hex) > limit:
                break
            size += len(tx_hex)
            if now - r['propagation_time'] > last_propagation_delta:
                return_txs.append(tx_hex)
        return return_txs

    async def update_pending_transactions_propagation_time(self, txs_hash: List[str]):
        now = int(_utcnow().replace(tzinfo=timezone.utc).timestamp())
        self._xm('UPDATE pending_transactions SET propagation_time = ? WHERE tx_hash = ?', [(now, h) for h in txs_hash])

    async def get_next_block_average_fee(self):
        rows = sorted(self._q('SELECT LENGTH(tx_hex) AS size, fees FROM pending_transactions'),
                      key=lambda r: (-(Decimal(r['fees']) / r['size']), r['size']))
        fees, size = [], 0
        for r in rows:
            if size + r['size'] > MAX_BLOCK_SIZE_HEX:
                break
            fees.append(Decimal(r['fees']))
            size += r['size']
        return int(mean(fees) * SMALLEST) // Decimal(SMALLEST)

    async def get_pending_blocks_count(self):
        rows = self._q('SELECT LENGTH(tx_hex) AS size FROM pending_transactions')
        return int(sum(r['size'] for r in rows) / MAX_BLOCK_SIZE_HEX + 1)

    async def clear_duplicate_pending_transactions(self):
        self._x('DELETE FROM pending_transactions WHERE EXISTS '
                '(SELECT 1 FROM transactions t WHERE t.tx_hash = pending_transactions.tx_hash)')

    # ------------------------------------------------------------------ blocks / txs (database.py:233-437)
    async def add_transaction(self, transaction, block_hash: str):
        await self.add_transactions([transaction], block_hash)

    async def _tx_row(self, transaction, block_hash):
        if isinstance(transaction, Transaction):
            inputs_addresses = [await _input_address(i) for i in transaction.inputs]
        else:
            inputs_addresses = []
        return (block_hash, transaction.hash(), transaction.hex(), _j(inputs_addresses),
                _j([o.address for o in transaction.outputs]),
                _j([int(o.amount * SMALLEST) for o in transaction.outputs]),
                numeric(transaction.fees if isinstance(transaction, Transaction) else 0, 6))

    async def add_transactions(self, transactions, block_hash: str):
        rows = [await self._tx_row(t, block_hash) for t in transactions]
        self.insert_transaction_rows(rows)

    def insert_transaction_rows(self, rows: List[tuple]):
        """Confirmed tx rows. The per-address index (``address_transactions``) is maintained lazily by
        :meth:`index_addresses` — off the block-apply critical path."""
        try:
            with self.transaction():
                self._xm('INSERT INTO transactions (block_hash, tx_hash, tx_hex, inputs_addresses, '
                         'outputs_addresses, outputs_amounts, fees) VALUES (?, ?, ?, ?, ?, ?, ?)', rows)
        except sqlite3.IntegrityError as e:
            raise UniqueViolationError(str(e)) from e

    def insert_transaction_columns(self, n: int, block_hash: str, tx_hash, tx_hex, inputs_addresses,
                                   outputs_addresses, outputs_amounts, fees):
        """``insert_transaction_rows`` from bulk column specs (native block path, see :meth:`bulk`)."""
        try:
            with self.transaction():
                self.bulk('INSERT INTO transactions (block_hash, tx_hash, tx_hex, inputs_addresses, '
                          'outputs_addresses, outputs_amounts, fees) VALUES (?, ?, ?, ?, ?, ?, ?)',
                          [block_hash, tx_hash, tx_hex, inputs_addresses, outputs_addresses, outputs_amounts, fees], n)
        except sqlite3.IntegrityError as e:
            raise UniqueViolationError(str(e)) from e

    # ---------------------------------------------------------------- lazy address index
    def _address_index_height(self) -> int:
        row = self._q1("SELECT height FROM address_index_state WHERE k = 'height'")
        if row is not None:
            return int(row[0])
        # ledgers written before the watermark existed indexed every tx eagerly
        has_rows = self._q1('SELECT 1 FROM address_transactions LIMIT 1') is not None
        h = self._tip_id() if has_rows else 0
        self._x("INSERT OR REPLACE INTO address_index_state (k, height) VALUES ('height', ?)", (h,))
        return h

    def index_addresses(self) -> int:
        """Bring ``address_transactions`` up to the tip: one INSERT … SELECT over json_each of the
        inputs/outputs address columns of every tx in blocks above the watermark (all in SQLite's C
        code). Returns the number of blocks indexed."""
        if self._address_index_height() >= self._tip_id():
            return 0  # kept current by the block batches: no write transaction
        # the transaction only writes the two address tables: invalidate those, not every cache (a
        # blanket invalidation would drop the mempool and tip caches the /push_tx path runs on)
        with self.transaction(invalidate=False):
            wm = self._address_index_height()
            tip = self._tip_id()
            if tip <= wm:
                return 0
            hashes = [r[0] for r in self._conn.execute('SELECT hash FROM blocks WHERE id > ? AND id <= ?', (wm, tip))]
            for k in range(0, len(hashes), 200):  # literal lists: pushed into each tx file's block_hash index
                chunk = hashes[k:k + 200]
                ph = ','.join('?' * len(chunk))
                self._conn.execute(
                    'INSERT INTO address_transactions (address, tx_hash) '
                    f'SELECT j.value, t.tx_hash FROM transactions t, json_each(t.inputs_addresses) j '
                    f'WHERE t.block_hash IN ({ph}) '
                    'UNION '
                    f'SELECT j.value, t.tx_hash FROM transactions t, json_each(t.outputs_addresses) j '
                    f'WHERE t.block_hash IN ({ph})', (*chunk, *chunk))
            self._conn.execute("UPDATE address_index_state SET height = ? WHERE k = 'height'", (tip,))
        return tip - wm  # (address tables feed no host cache: nothing to invalidate)

    # the per-address index of one block, inside the block's own journal batch (materialiser thread):
    # only when the watermark stands at the previous block, so a lagging index is left to the catch-up
    # above (rows are a set: ``get_address_transactions`` orders by block and tx rowid)
    _ADDR_ROWS = 'INSERT INTO address_transactions (address, tx_hash) VALUES (?, ?)'
    _ADDR_BLOCK_WM = "UPDATE address_index_state SET height = ?2 + 1 WHERE k = 'height' AND height = ?2 AND ?1 IS NOT NULL"

    @staticmethod
    def address_rows(tx_rows) -> Tuple[List[str], List[str]]:
        """(addresses, tx hashes) of the address_transactions rows of tx rows (block_hash, tx_hash, tx_hex,
        inputs_addresses, outputs_addresses, ...): each distinct address among a tx's inputs and outputs
        (json_each(inputs_addresses) UNION json_each(outputs_addresses))."""
        addrs, hashes = [], []
        for r in tx_rows:
            seen = dict.fromkeys(a for col in (r[3], r[4]) for a in (json.loads(col) if col else [])
                                 if isinstance(a, str))
            addrs.extend(seen)
            hashes.extend([r[1]] * len(seen))
        return addrs, hashes

    def _address_index_stmts(self, block_hash: str, block_id: int, rows: list) -> list:
        """The block's address_transactions rows (``rows``: (address column spec, tx hash column spec, n)
        parts) and the watermark update, applied only while the index is caught up to the block before
        (otherwise :meth:`index_addresses` catches it up lazily). Rows are a set: ``get_address_transactions``
        orders by block and tx row id."""
        if os.environ.get('UPOW_ADDRESS_INDEX_INLINE', '1') == '0':
            return []
        guard = f"SELECT EXISTS(SELECT 1 FROM address_index_state WHERE k = 'height' AND height = {int(block_id) - 1})"
        out = [(self._ADDR_ROWS, [a, h], n, None, guard, None) for a, h, n in rows if n]
        out.append((self._ADDR_BLOCK_WM, [block_hash, block_id - 1], 1, None, None, None))
        return out

    def _address_index_rollback(self):
        """After blocks were deleted (their address rows cascade away), pull the watermark down."""
        tip = self._tip_id()
        self._x("UPDATE address_index_state SET height = MIN(height, ?) WHERE k = 'height'", (tip,))

    async def add_block(self, id: int, block_hash: str, block_content: str, address: str, random: int,
                        difficulty: Decimal, reward: Decimal, timestamp: Union[datetime, int]):
        if isinstance(timestamp, datetime):
            timestamp = int(timestamp.replace(tzinfo=timezone.utc).timestamp())
        try:
            self._x('INSERT INTO blocks (id, hash, content, address, random, difficulty, reward, timestamp) '
                    'VALUES (?, ?, ?, ?, ?, ?, ?, ?)',
                    (id, block_hash, block_content, address, int(random), numeric(difficulty, 1),
                     numeric(reward, 6), int(timestamp)))
        except sqlite3.IntegrityError as e:
            raise UniqueViolationError(str(e)) from e
        from .manager import Manager
        Manager.difficulty = None

    @staticmethod
    def _block_row(row) -> Optional[dict]:
        if row is None:
            return None
        d = dict(row)
        d['difficulty'] = Decimal(d['difficulty'])
        d['reward'] = Decimal(d['reward'])
        return normalize_block(d)

    def _q1_present(self, sql: str, args: tuple):
        """``_q1`` for rows that never change once written (a confirmed tx by hash): a row already in
        SQL is the answer, so the materialiser is only waited for when the row is not there yet. (Rows
        leave ``transactions`` only through rollback, which runs on the Python connection after a full
        settle.)"""
        with self.lock:
            r = self._conn.execute(sql, args).fetchone()
        return r if r is not None else self._q1(sql, args)

    @staticmethod
    async def _off_loop(fn, *args):
        """Run a blocking SQL read on the SQL reader threads, not on the calling event loop: a read that
        waits on the disk (or behind a WAL checkpoint of its file) then stalls no HTTP request."""
        global _SQL_READERS
        if _SQL_READERS is None:
            from concurrent.futures import ThreadPoolExecutor
            _SQL_READERS = ThreadPoolExecutor(max_workers=2, thread_name_prefix='upow-sql-read')
        return await asyncio.get_running_loop().run_in_executor(_SQL_READERS, fn, *args)

    async def get_transaction(self, tx_hash: str, check_signatures: bool = True):
        res = await self._off_loop(self._q1_present, 'SELECT tx_hex, block_hash FROM transactions WHERE tx_hash = ?',
                                   (tx_hash,))
        if res is None:
            return None
        tx = await Transaction.from_hex(res['tx_hex'], check_signatures)
        tx.block_hash = res['block_hash']
        return tx

    @staticmethod
    def _info_row(row) -> dict:
        d = dict(row)
        d['inputs_addresses'] = _arr(d['inputs_addresses'])
        d['outputs_addresses'] = _arr(d['outputs_addresses'])
        d['outputs_amounts'] = _arr(d['outputs_amounts'])
        d['fees'] = Decimal(d['fees'])
        return d

    INFO_CACHE = 8192

    def _cache_info(self, h: str, info: dict):
        c = self._info_cache
        c[h] = info
        if len(c) > self.INFO_CACHE:
            c.popitem(last=False)

    async def get_transaction_info(self, tx_hash: str) -> Optional[dict]:
        hit = self._info_cache.get(tx_hash)
        if hit is not None:
            return hit
        res = await self._off_loop(self._q1_present, 'SELECT * FROM transactions WHERE tx_hash = ?', (tx_hash,))
        if res is None:
            return None
        info = self._info_row(res)
        self._cache_info(tx_hash, info)
        return info

    async def get_transactions_info(self, tx_hashes: List[str]) -> Dict[str, dict]:
        out = {}
        hashes = list(dict.fromkeys(tx_hashes))
        if len(hashes) <= 32:  # a pushed tx's funding txs: as _q1_present, without a settle when all are in
            cache = self._info_cache
            miss = []
            for h in hashes:
                hit = cache.get(h)
                if hit is not None:
                    out[h] = hit
                else:
                    miss.append(h)
            if miss:
                def read(miss=miss):
                    with self.lock:
                        return self._conn.execute(f'SELECT * FROM transactions WHERE tx_hash IN '
                                                  f'({",".join("?" * len(miss))})', miss).fetchall()
                for r in await self._off_loop(read):
                    info = out[r['tx_hash']] = self._info_row(r)
                    self._cache_info(r['tx_hash'], info)
            if len(out) == len(hashes):
                return out
            hashes = [h for h in hashes if h not in out]
        for k in range(0, len(hashes), 500):
            chunk = hashes[k:k + 500]
            for r in self._q(f'SELECT * FROM transactions WHERE tx_hash IN ({",".join("?" * len(chunk))})', chunk):
                out[r['tx_hash']] = self._info_row(r)
        return out

    async def get_pending_transaction(self, tx_hash: str, check_signatures: bool = True):
        res = self._q1('SELECT tx_hex FROM pending_transactions WHERE tx_hash = ?', (tx_hash,))
        return await Transaction.from_hex(res['tx_hex'], check_signatures) if res is not None else None

    async def get_pending_transactions_by_hash(self, hashes: List[str], check_signatures: bool = True):
        return [await Transaction.from_hex(h, check_signatures) for h in await self.get_pending_transactions_hex_by_hash(hashes)]

    async def get_pending_transactions_hex_by_hash(self, hashes: List[str]) -> List[str]:
        """tx hex of the pending txs among ``hashes``, in mempool (table) order like database.py:297-301."""
        return self.pending_hex_by_hash(hashes)

    def pending_hex_by_hash(self, hashes: List[str]) -> List[str]:
        """Synchronous :meth:`get_pending_transactions_hex_by_hash` (callable from a worker thread)."""
        if not hashes:
            return []
        mp = self._mempool()
        if mp is not None:
            return mp.hex_in_order(hashes)
        want = set(hashes)
        self._settle(frozenset(('pending_transactions',)))
        with self.lock:
            cur = self._conn.cursor()
            cur.row_factory = None  # plain tuples: this scans the whole mempool
            rows = cur.execute('SELECT tx_hash, tx_hex FROM pending_transactions').fetchall()
        return [x for h, x in rows if h in want]

    async def get_transactions(self, tx_hashes: List[str]):
        infos = await self.get_transactions_info(tx_hashes)
        return {sha256(i['tx_hex']): await Transaction.from_hex(i['tx_hex']) for i in infos.values()}

    async def get_transaction_hash_by_contains_multi(self, contains: List[str], ignore: str = None):
        for r in self._q('SELECT tx_hash, tx_hex FROM transactions'):
            if ignore is not None and r['tx_hash'] == ignore:
                continue
            if any(c in r['tx_hex'] for c in contains):
                return r['tx_hash']
        return None

    async def get_pending_transactions_by_contains(self, contains: str):
        rows = self._q('SELECT tx_hash, tx_hex FROM pending_transactions')
        return [await Transaction.from_hex(r['tx_hex']) for r in rows
                if contains in r['tx_hex'] and r['tx_hash'] != contains]

    async def remove_pending_transactions_by_contains(self, search: List[str]) -> None:
        with self.transaction():
            rows = self.conn.execute('SELECT tx_hash, tx_hex FROM pending_transactions').fetchall()
            deleted = [r['tx_hash'] for r in rows if any(c in r['tx_hex'] for c in search)]
            self.conn.executemany('DELETE FROM pending_transactions WHERE tx_hash = ?', [(h,) for h in deleted])
        if deleted:
            logger.info(f'remove_pending_transactions_by_contains: removed {len(deleted)} transactions '
                        f'deleted_tx_hashes: {deleted}')
        else:
            logger.info(f'remove_pending_transactions_by_contains: no transactions matched patterns {search}')

    async def get_pending_transaction_by_contains_multi(self, contains: List[str], ignore: str = None):
        for r in self._q('SELECT tx_hash, tx_hex FROM pending_transactions'):
            if ignore is not None and r['tx_hash'] == ignore:
                continue
            if any(c in r['tx_hex'] for c in contains):
                return await Transaction.from_hex(r['tx_hex'])
        return None

    def _last_block_row(self) -> Optional[dict]:
        """The tip row, from the chain-tip cache the native block path keeps (no wait for the SQL
        materialiser) or from SQL."""
        if self._lean_tip is not None:
            return dict(self._lean_tip)
        tip = self._tip_cache
        if tip is None:
            gen = self._tip_gen
            tip = self._block_row(self._q1('SELECT * FROM blocks ORDER BY id DESC LIMIT 1'))
            if gen == self._tip_gen:  # no block landed or was removed meanwhile
                self._tip_cache = tip
        return dict(tip) if tip is not None else None

    async def get_last_block(self) -> Optional[dict]:
        return self._last_block_row()

    async def get_next_block_id(self) -> int:
        tip = self._last_block_row()
        return (tip['id'] if tip is not None else 0) + 1

    async def get_block(self, block_hash: str) -> Optional[dict]:
        if block_hash in self._lean_by_hash:
            return dict(self._lean_rows[self._lean_by_hash[block_hash]])
        return self._block_row(self._q1('SELECT * FROM blocks WHERE hash = ?', (block_hash,)))

    async def get_blocks(self, offset: int, limit: int, tx_details: bool = False) -> list:
        blocks = self._q('SELECT * FROM blocks WHERE id >= ? ORDER BY id LIMIT ?', (offset, limit))
        index = {b['hash']: [] for b in blocks}
        index_tx_hash = {b['hash']: [] for b in blocks}
        if blocks:
            for t in self._txs_of_blocks([b['hash'] for b in blocks], 'tx_hex, tx_hash, block_hash'):
                if t['block_hash'] in index:
                    index[t['block_hash']].append(t['tx_hex'])
                    index_tx_hash[t['block_hash']].append(t['tx_hash'])
        result, size = [], 0
        for b in blocks:
            block = self._block_row(b)
            txs = index[block['hash']]
            size += sum(len(tx) for tx in txs)
            if size > MAX_BLOCK_SIZE_HEX * 8:
                break
            result.append({'block': block,
                           'transactions': txs if not tx_details else
                           [await self.get_nice_transaction(h) for h in index_tx_hash[block['hash']]]})
        return result

    RECENT_ROWS = 256

    def _remember_row(self, row: dict):
        rr = self._recent_rows
        rr[int(row['id'])] = row
        while len(rr) > self.RECENT_ROWS:
            del rr[next(iter(rr))]

    async def get_block_by_id(self, block_id: int) -> Optional[dict]:
        # calculate_difficulty passes `id - BLOCKS_COUNT + 1` as a Decimal (manager.py:95-97)
        row = self._lean_rows.get(int(block_id))
        if row is None:
            row = self._recent_rows.get(int(block_id))
        if row is not None:
            return dict(row)
        tip = self._tip_cache
        if tip is not None and tip['id'] == int(block_id):
            return dict(tip)
        return self._block_row(self._q1('SELECT * FROM blocks WHERE id = ?', (int(block_id),)))

    def block_hash_at(self, block_id: int) -> Optional[str]:
        """The hash of block ``block_id`` (lean header rows first, then SQL); None when there is none."""
        if not block_id:
            return None
        row = self._lean_rows.get(int(block_id))
        if row is not None:
            return row['hash']
        r = self._q1('SELECT hash FROM blocks WHERE id = ?', (int(block_id),))
        return r[0] if r else None

    def block_tx_hexes(self, block_hash: str) -> List[str]:
        """The block's tx hex strings in block order (synchronous: callable from a worker thread)."""
        return [r[0] for r in self._q('SELECT tx_hex FROM transactions WHERE block_hash = ? ORDER BY rowid',
                                      (block_hash,))]

    async def get_block_transactions(self, block_hash: str, check_signatures: bool = True, hex_only: bool = False):
        if hex_only:
            return self.block_tx_hexes(block_hash)
        rows = self._q('SELECT tx_hex FROM transactions WHERE block_hash = ? ORDER BY rowid', (block_hash,))
        return [r['tx_hex'] if hex_only else await Transaction.from_hex(r['tx_hex'], check_signatures) for r in rows]

    async def get_block_transactions_hashes(self, block_hash: str) -> List[str]:
        return [r[0] for r in self._q('SELECT tx_hash FROM transactions WHERE block_hash = ? ORDER BY rowid',
                                      (block_hash,))]

    async def get_block_transaction_hashes(self, block_hash: str) -> List[str]:
        """Hashes of the block's non-coinbase txs (the coinbase hex contains the block hash)."""
        rows = self._q('SELECT tx_hash, tx_hex FROM transactions WHERE block_hash = ? ORDER BY rowid', (block_hash,))
        return [r['tx_hash'] for r in rows if block_hash not in r['tx_hex']]

    async def get_block_nice_transactions(self, block_hash: str) -> List[dict]:
        rows = self._q('SELECT tx_hash, inputs_addresses FROM transactions WHERE block_hash = ? ORDER BY rowid',
                       (block_hash,))
        return [{'hash': r['tx_hash'], 'is_coinbase': not _arr(r['inputs_addresses'])} for r in rows]

    # ------------------------------------------------------------------ outputs (database.py:439-580)
    async def add_unspent_outputs(self, outputs: List[tuple], index: bool = True) -> None:
        if not outputs:
            return
        payload = None
        if len(outputs[0]) == 2:
            # restored outpoints: address is re-derived from the creating tx (database.py:500-505)
            rows = []
            infos = await self.get_transactions_info([h for h, _ in outputs])
            amounts, addrs = [], []
            for h, i in outputs:
                info = infos.get(h)
                addr = _at(info['outputs_addresses'], i) if info else None
                rows.append((h, i, addr, None))
                amounts.append(_at(info['outputs_amounts'], i) if info else None)
                addrs.append(_addr_bytes(addr))
            payload = make_payload(amounts, addrs)
        else:
            rows = [(o[0], o[1], o[2], None if o[3] is None else int(bool(o[3]))) for o in outputs]
            if len(outputs[0]) >= 5:  # (tx_hash, index, address, is_stake, amount in smallest units)
                payload = make_payload([o[4] for o in outputs], [_addr_bytes(o[2]) for o in outputs],
                                       [r[3] == 1 for r in rows])
        self._xm('INSERT INTO unspent_outputs (tx_hash, "index", address, is_stake) VALUES (?, ?, ?, ?)', rows)
        if self.gov is not None:
            self.gov.added(STAKE, [(r[0], r[1]) for r in rows if r[3] == 1])
        if not index:
            return
        if payload is None:
            payload = await self._payload_from_ledger([(r[0], r[1]) for r in rows], [r[3] == 1 for r in rows])
        self.utxo.insert([(r[0], r[1]) for r in rows], TAG_BY_TABLE['unspent_outputs'], payload)

    @staticmethod
    def _key_order(in_keys: np.ndarray) -> np.ndarray:
        """Row order sorted by the leading 8 bytes of the tx hash: B-tree locality for bulk writes
        (the set of rows written, and so the result, does not depend on the order)."""
        return np.argsort(in_keys[:, :8].copy().view('>u8').ravel(), kind='stable').astype(np.int64)

    def _mempool_empty(self) -> bool:
        """Are both mempool tables empty? Cached until a Python-side write touches them."""
        mp = self._mp
        if mp is not None:
            return mp.empty()
        if self._pending_empty is None:
            self._pending_empty = self._q1('SELECT EXISTS(SELECT 1 FROM pending_transactions) OR '
                                           'EXISTS(SELECT 1 FROM pending_spent_outputs)')[0] == 0
        return self._pending_empty

    def apply_native_block(self, block_row: dict, coinbase_row: tuple, coinbase_outputs: list, n: int,
                           tx_cols: list, out_cols: tuple, in_keys: np.ndarray, spent_payload: np.ndarray,
                           gov: Optional[dict] = None, addr_pairs: Optional[tuple] = None,
                           cb_index: Optional[tuple] = None) -> int:
        """The ledger writes of one native-path block (reference manager.py:706-730: add_block,
        add_transaction(coinbase), add_transactions, add_transaction_outputs, remove_pending_transactions,
        remove_outputs, remove_pending_spent_outputs) as ONE journal batch, plus the HBM index update.

        ``tx_cols``: bulk column specs of the n tx rows (tx_hash, tx_hex, inputs_addresses,
        outputs_addresses, outputs_amounts, fees); ``out_cols``: (index int64, address text spec,
        txids n x 32, amounts u64, raw addresses n x 64, address lengths) of the REGULAR outputs;
        ``in_keys``: n x 40 spent outpoint records; ``spent_payload``: their index payloads (undo data).
        ``gov`` (blocks with governance txs, ledger/govcheck.py): per-output ``out_tag``/``out_type``, per-input
        ``in_tag`` (the table each input is spent from), ``out_tx``, ``gov_tx`` and the inputs_addresses arena:
        outputs land in their tables (stake flag from the output type), spends leave theirs, and the
        governance index follows from these columns — the object path's write set (apply_object_block) in
        the same statement order, so both paths leave identical tables.
        ``cb_index``: the coinbase outputs' index (records, payloads) when already built (a sync page's plan).
        Returns the journal sequence number (0 without the native writer: written synchronously)."""
        ts = [perf_counter()]  # stage clock: records, statements, encode, journal, index, mempool, governance
        names = ('apply:records', 'apply:stmts', 'apply:encode', 'apply:journal', 'apply:index', 'apply:mempool',
                 'apply:gov')
        roctx.push(names[0])

        def stamp():  # next stage (and its roctx range)
            ts.append(perf_counter())
            roctx.pop()
            if len(ts) <= len(names):
                roctx.push(names[len(ts) - 1])
        out_index, out_addr_spec, out_txid, out_amount, out_addr, out_len = out_cols
        n_out, n_in = len(out_index), len(in_keys)
        tag_u = TAG_BY_TABLE['unspent_outputs']
        out_tag = gov['out_tag'] if gov is not None else np.full(n_out, tag_u, dtype=np.uint32)
        # ---- index records: created outputs (block txs + coinbase) and spent inputs
        from ..ops.native import lib
        stake = (np.asarray(gov['out_type']) == int(OutputType.STAKE)).astype(np.uint8) if gov is not None \
            else np.zeros(0, np.uint8)
        rb, pb = lib().output_index_records(
            np.ascontiguousarray(out_txid, dtype=np.uint8), np.ascontiguousarray(out_index, dtype=np.int64),
            np.ascontiguousarray(out_tag, dtype=np.uint32), np.ascontiguousarray(out_amount, dtype=np.uint64),
            np.ascontiguousarray(out_addr, dtype=np.uint8), np.ascontiguousarray(out_len, dtype=np.uint8), stake)
        recs = np.frombuffer(rb, dtype=np.uint8).reshape(-1, 40)
        pay = np.frombuffer(pb, dtype=PAYLOAD_DTYPE)
        from .utxo import pack_records
        cb_keys = [(o[0], o[1]) for o in coinbase_outputs]
        if cb_index is not None:  # (records, payloads) of the coinbase outputs, built by a sync page's plan
            cb_recs, cb_pay = cb_index
        else:
            cb_recs = pack_records(cb_keys, tag_u)
            cb_pay = make_payload([o[4] for o in coinbase_outputs], [_addr_bytes(o[2]) for o in coinbase_outputs],
                                  [bool(o[3]) for o in coinbase_outputs])
        in_keys = np.ascontiguousarray(in_keys, dtype=np.uint8).reshape(-1, 40)
        in_tag = gov['in_tag'].astype(np.uint32) if gov is not None else np.full(n_in, tag_u, dtype=np.uint32)
        sb, ib = lib().spent_index_records(in_keys, np.ascontiguousarray(in_tag, dtype=np.uint32))
        spent = np.frombuffer(sb, dtype=np.uint8).reshape(-1, 40)
        in_idx = np.frombuffer(ib, dtype=np.int64)
        # the spends' key order (B-tree locality) is computed by the materialiser ('key': a stable sort of the
        # statement's rows by the leading 8 bytes of column 0, so a row selection keeps the global key order)
        in_order = 'key'
        stamp()

        # ---- statements (schema.sql write set of one block)
        b = block_row
        # the coinbase row first, then the block's txs (insertion order)
        tx_base = self._tx_rowids(n + 1)
        stmts = [
            ('INSERT INTO blocks (id, hash, content, address, random, difficulty, reward, timestamp) '
             'VALUES (?, ?, ?, ?, ?, ?, ?, ?)',
             [int(b['id']), b['hash'], b['content'], b['address'], int(b['random']), b['difficulty'], b['reward'],
              int(b['timestamp'])], 1, None, None, None),
            (self._TX_INSERT, [coinbase_row[1], coinbase_row[0], *coinbase_row[2:], tx_base], 1, None, None, None),
        ]
        self.checkpoint('block')
        stmts.append((self._TX_INSERT, [tx_cols[0], b['hash'], *tx_cols[1:],
                                        np.arange(tx_base + 1, tx_base + 1 + n, dtype=np.int64)], n, None, None, None))
        self.checkpoint('transactions')
        # explicit row ids from the ledger-wide counter: the rows land in several files (see UTXO_FILES_DEFAULT)
        ins_u = 'INSERT INTO unspent_outputs (tx_hash, "index", address, is_stake, rowid) VALUES (?, ?, ?, ?, ?)'
        if gov is None:
            if n_out:
                base = self._utxo_rowids(n_out)
                stmts.append((ins_u, [('hex32', np.ascontiguousarray(out_txid), 32, 0),
                                      np.ascontiguousarray(out_index, dtype=np.int64), out_addr_spec, 0,
                                      np.arange(base, base + n_out, dtype=np.int64)],
                              n_out, None, None, None))
        else:
            out_txid_c = np.ascontiguousarray(out_txid)
            sel = np.nonzero(out_tag == tag_u)[0]
            if len(sel):
                base = self._utxo_rowids(len(sel))
                stake = (gov['out_type'][sel] == int(OutputType.STAKE)).astype(np.int64)
                stmts.append((ins_u, [('hex32', out_txid_c, 32, 0, sel), np.ascontiguousarray(out_index[sel], dtype=np.int64),
                                      (*out_addr_spec, sel), stake,
                                      np.arange(base, base + len(sel), dtype=np.int64)],
                              len(sel), None, None, None))
        if coinbase_outputs:
            base = self._utxo_rowids(len(coinbase_outputs))
            stmts.append((ins_u, [[o[0] for o in coinbase_outputs], np.array([o[1] for o in coinbase_outputs], np.int64),
                                  [o[2] for o in coinbase_outputs],
                                  [None if o[3] is None else str(int(bool(o[3]))) for o in coinbase_outputs],
                                  np.arange(base, base + len(coinbase_outputs), dtype=np.int64)],
                          len(coinbase_outputs), None, None, None))
        tables = {'blocks', 'transactions', 'unspent_outputs'}
        gov_spent = {}
        if gov is not None:
            for table in self._GOV_INSERT_ORDER:
                sel = np.nonzero(out_tag == TAG_BY_TABLE[table])[0]
                if len(sel):
                    stmts.append((f'INSERT INTO {table} (tx_hash, "index", address) VALUES (?, ?, ?)',
                                  [('hex32', out_txid_c, 32, 0, sel), np.ascontiguousarray(out_index[sel], dtype=np.int64),
                                   (*out_addr_spec, sel)],
                                  len(sel), None, None, None))
                    tables.add(table)
            for table in self._SPEND_ORDER:
                if table == 'unspent_outputs':
                    continue
                sel = np.nonzero(in_tag == TAG_BY_TABLE[table])[0]
                if len(sel):
                    gov_spent[table] = sel
                    tables.add(table)
        self.checkpoint('outputs')
        mempool = n and not self._mempool_empty()
        if mempool:
            txids = np.ascontiguousarray(tx_cols[0][1], dtype=np.uint8).reshape(-1, 32)
            stmts.append(('DELETE FROM pending_transactions WHERE tx_hash = ?', [('hex32', txids, 32, 0)], n,
                          'key', 'SELECT EXISTS(SELECT 1 FROM pending_transactions)', None))

        def spend_stmt(table):
            sel = gov_spent[table]
            stmts.append((f'DELETE FROM {table} WHERE tx_hash = ? AND "index" = ?',
                          [('hex32', in_keys, 40, 0, sel), np.ascontiguousarray(in_idx[sel])], len(sel), None, None,
                          len(sel)))
        if 'inode_registration_output' in gov_spent:
            spend_stmt('inode_registration_output')
        sel_u = np.nonzero(in_tag == tag_u)[0] if gov is not None else None
        if gov is None and n_in:
            stmts.append(('DELETE FROM unspent_outputs WHERE tx_hash = ? AND "index" = ?',
                          [('hex32', in_keys, 40, 0), in_idx], n_in, in_order, None, n_in))
        elif gov is not None and len(sel_u):
            stmts.append(('DELETE FROM unspent_outputs WHERE tx_hash = ? AND "index" = ?',
                          [('hex32', in_keys, 40, 0, sel_u), np.ascontiguousarray(in_idx[sel_u])], len(sel_u),
                          'key', None, len(sel_u)))
        for table in self._SPEND_ORDER[2:]:
            if table in gov_spent:
                spend_stmt(table)
        if mempool and n_in:
            stmts.append(('DELETE FROM pending_spent_outputs WHERE tx_hash = ? AND "index" = ?',
                          [('hex32', in_keys, 40, 0), in_idx], n_in, in_order,
                          'SELECT EXISTS(SELECT 1 FROM pending_spent_outputs)', None))
            tables |= {'pending_transactions', 'pending_spent_outputs'}
        self.checkpoint('spent')
        # address index rows: the coinbase's, then the txs' (txcodec.address_pairs: blob, offsets, tx index)
        ca, ch = self.address_rows([coinbase_row])
        parts = [(ca, ch, len(ca))]
        if addr_pairs is not None:
            ab, ao, at = addr_pairs
            parts.append((('arena', ab, ao), ('hex32', tx_cols[0][1], 32, 0, np.frombuffer(at, dtype=np.int64)),
                          len(at) // 8))
        addr_stmts = self._address_index_stmts(b['hash'], int(b['id']), parts)
        stmts.extend(addr_stmts)
        tables |= {'address_transactions', 'address_index_state'}

        seq = 0
        stamp()
        if self.writer is not None:
            enc = self.encode_many(stmts)
            stamp()
            _commit_point()  # a cluster node: every replica votes to commit this block, now that nothing but the write can fail
            # the undo record as parts: the writer joins them in one copy off the GIL
            meta = [bytes.fromhex(b['hash']), struct.pack('<qII', int(b['id']), n_out + len(cb_keys), n_in), recs,
                    np.ascontiguousarray(cb_recs), spent, np.ascontiguousarray(spent_payload).view(np.uint8)]
            seq = self.submit_batch(enc, tables, meta, int(b['id']), defer_sync=True)
        else:
            stamp()
            _commit_point()
            with self.transaction(foreign_keys=False):
                for sql, cols, nn, order, guard, expect in stmts:
                    if guard is not None and not self._q1(guard)[0]:
                        continue
                    done = self.bulk(sql, cols, nn, order)
                    if expect is not None and done != expect:
                        logger.error(f'native block apply: {done} of {expect} rows changed [{sql[:40]}]')
        # ---- the index and the chain-tip cache follow the commit point
        stamp()
        if self.utxo_defer:
            # a sync page (ledger/pagesync.py): the page's index writes go to the device as one insert and one
            # erase launch when the page ends (or before anything reads the index)
            self.utxo.defer_block([(recs, pay), (cb_recs, cb_pay)], spent if n_in else spent[:0])
        else:
            # one H2D copy + insert + erase launch queued on the node stream, not waited for: the next block's
            # input lookup runs behind them on the same stream
            self.utxo.apply_block([(recs, pay), (cb_recs, cb_pay)], spent if n_in else spent[:0])
        stamp()
        tip = dict(b)
        tip['difficulty'], tip['reward'] = Decimal(tip['difficulty']), Decimal(tip['reward'])
        self._tip_gen += 1
        self._tip_cache = normalize_block(tip)
        self._remember_row(self._tip_cache)
        if mempool:
            self._pending_empty = None
            self._mempool_ver += 1
        if n:
            self._mempool_confirm(bool(mempool), txids=np.asarray(tx_cols[0][1]).reshape(-1, 32), in_keys=in_keys,
                                  block_seq=seq)
        stamp()
        if self.gov is not None and gov is not None:
            tg = perf_counter()
            _, blob, off = out_addr_spec
            off = np.frombuffer(off, dtype=np.int64) if isinstance(off, (bytes, bytearray)) else np.asarray(off, np.int64)
            # governance/stake outputs in, governance and staked spends out (csrc/gov_index.cpp apply_block),
            # on the governance apply thread: the block is committed, and every reader of the index (the next
            # block's rule check included) waits for this update through the index lock
            args = (np.ascontiguousarray(gov['out_type'], dtype=np.uint8), np.ascontiguousarray(tx_cols[0][1]),
                    np.ascontiguousarray(gov['out_tx'], dtype=np.int32), np.ascontiguousarray(gov['out_start'], np.int32),
                    np.ascontiguousarray(out_amount, dtype=np.uint64), np.ascontiguousarray(out_addr, dtype=np.uint8),
                    np.ascontiguousarray(out_len, dtype=np.uint8), blob, np.ascontiguousarray(off),
                    np.ascontiguousarray(gov['in_start'], np.int32), np.ascontiguousarray(spent_payload).view(np.uint8),
                    in_keys, np.ascontiguousarray(gov['in_tag'], dtype=np.uint8), gov['in_str'][0],
                    np.frombuffer(gov['in_str'][1], dtype=np.int64), n, int(b['timestamp']))
            g = self.gov

            def gov_apply():
                g.store.apply_block(*args)
                g.version += 1
                # the next block's coinbase needs the active inodes of this state: their emission cascade
                # (ballot terms, validator stakes) is evaluated here, off the block path, into the memo
                g.inodes_with_power(False)
            g.defer(gov_apply)
            self.last_gov_index_s = perf_counter() - tg
        elif self.gov is not None and n_in:
            hit = self._stake_spent(spent, spent_payload)
            if hit:
                self.gov.removed(STAKE, hit)
        stamp()
        self.last_apply_stages = dict(zip(('ap_records_s', 'ap_stmts_s', 'ap_encode_s', 'ap_journal_s', 'ap_index_s',
                                           'ap_mempool_s', 'ap_gov_s'), np.diff(ts).tolist()))
        return seq

    # ------------------------------------------------------------------ lean replica (ledger/lean.py)
    def enter_lean(self):
        """From now on blocks are applied lean (:meth:`apply_lean_block`): indexes, tip rows and the op log
        only. The SQL tables stay where they are until ``lean.materialise``."""
        from . import lean
        lean.open_log(self)
        self.flush()  # the tables hold every record journaled so far: lean blocks come after them
        self.lean = True

    def leave_lean(self):
        """Back to the SQL state: drop the lean tip rows and rebuild the HBM and governance indexes from the
        tables (a snapshot of exactly that state when one is there). ``lean.materialise`` then replays the op
        log on top of it."""
        self.utxo.settle()
        self.lean = False
        self._lean_rows.clear()
        self._lean_by_hash.clear()
        self._lean_tip = None
        self._invalidate_for(None)
        from . import manager
        manager.Manager.difficulty = None
        restored = False
        if self.path != ':memory:' and os.environ.get('UPOW_SNAPSHOT', '1') != '0':
            from . import snapshot
            restored = snapshot.try_restore(self)
        if not restored:
            self._rebuild_utxo_index()
        if self.gov is not None:
            self.gov.rebuild()

    def apply_lean_block(self, block_row: dict, coinbase_outputs: list, n: int, out_cols: tuple,
                         in_keys: np.ndarray, spent_payload: np.ndarray, txids: np.ndarray,
                         gov: Optional[dict] = None, cb_index: Optional[tuple] = None) -> int:
        """A lean follower's block apply (ledger/lean.py): what :meth:`apply_native_block` does to the indexes
        and the chain tip — the same index records (outputs, coinbase outputs, spends with their payloads),
        the same mempool confirm (its SQL deletes journaled: the pending tables stay the index's), the same
        governance-index update — and no block statements, no journal record, no SQL materialisation.
        The commit point (the cluster's vote) is where the journal write would be. Returns 0."""
        from ..ops.native import lib
        from .utxo import pack_records
        ts = [perf_counter()]
        out_index, out_addr_spec, out_txid, out_amount, out_addr, out_len = out_cols
        n_out, n_in = len(out_index), len(in_keys)
        tag_u = TAG_BY_TABLE['unspent_outputs']
        out_tag = gov['out_tag'] if gov is not None else np.full(n_out, tag_u, dtype=np.uint32)
        stake = (np.asarray(gov['out_type']) == int(OutputType.STAKE)).astype(np.uint8) if gov is not None \
            else np.zeros(0, np.uint8)
        rb, pb = lib().output_index_records(
            np.ascontiguousarray(out_txid, dtype=np.uint8), np.ascontiguousarray(out_index, dtype=np.int64),
            np.ascontiguousarray(out_tag, dtype=np.uint32), np.ascontiguousarray(out_amount, dtype=np.uint64),
            np.ascontiguousarray(out_addr, dtype=np.uint8), np.ascontiguousarray(out_len, dtype=np.uint8), stake)
        recs = np.frombuffer(rb, dtype=np.uint8).reshape(-1, 40)
        pay = np.frombuffer(pb, dtype=PAYLOAD_DTYPE)
        if cb_index is not None:
            cb_recs, cb_pay = cb_index
        else:
            cb_recs = pack_records([(o[0], o[1]) for o in coinbase_outputs], tag_u)
            cb_pay = make_payload([o[4] for o in coinbase_outputs], [_addr_bytes(o[2]) for o in coinbase_outputs],
                                  [bool(o[3]) for o in coinbase_outputs])
        in_keys = np.ascontiguousarray(in_keys, dtype=np.uint8).reshape(-1, 40)
        in_tag = gov['in_tag'].astype(np.uint32) if gov is not None else np.full(n_in, tag_u, dtype=np.uint32)
        sb, _ = lib().spent_index_records(in_keys, np.ascontiguousarray(in_tag, dtype=np.uint32))
        spent = np.frombuffer(sb, dtype=np.uint8).reshape(-1, 40)
        ts.append(perf_counter())
        _commit_point()
        ts.append(perf_counter())
        if self.utxo_defer:
            self.utxo.defer_block([(recs, pay), (cb_recs, cb_pay)], spent if n_in else spent[:0])
        else:
            self.utxo.apply_block([(recs, pay), (cb_recs, cb_pay)], spent if n_in else spent[:0])
        b = block_row
        tip = dict(b)
        tip['difficulty'], tip['reward'] = Decimal(tip['difficulty']), Decimal(tip['reward'])
        tip = normalize_block(tip)
        bid = int(b['id'])
        self._lean_rows[bid] = tip
        self._lean_by_hash[b['hash']] = bid
        self._lean_tip = tip
        self._tip_gen += 1
        self._tip_cache = tip
        ts.append(perf_counter())
        if n:
            self._mempool_confirm(False, txids=np.asarray(txids, np.uint8).reshape(-1, 32), in_keys=in_keys)
        ts.append(perf_counter())
        if self.gov is not None and gov is not None:
            _, blob, off = out_addr_spec
            off = np.frombuffer(off, dtype=np.int64) if isinstance(off, (bytes, bytearray)) else np.asarray(off, np.int64)
            args = (np.ascontiguousarray(gov['out_type'], dtype=np.uint8), np.ascontiguousarray(txids),
                    np.ascontiguousarray(gov['out_tx'], dtype=np.int32), np.ascontiguousarray(gov['out_start'], np.int32),
                    np.ascontiguousarray(out_amount, dtype=np.uint64), np.ascontiguousarray(out_addr, dtype=np.uint8),
                    np.ascontiguousarray(out_len, dtype=np.uint8), blob, np.ascontiguousarray(off),
                    np.ascontiguousarray(gov['in_start'], np.int32), np.ascontiguousarray(spent_payload).view(np.uint8),
                    in_keys, np.ascontiguousarray(gov['in_tag'], dtype=np.uint8), gov['in_str'][0],
                    np.frombuffer(gov['in_str'][1], dtype=np.int64), n, int(b['timestamp']))
            g = self.gov

            def gov_apply():
                g.store.apply_block(*args)
                g.version += 1
                g.inodes_with_power(False)
            g.defer(gov_apply)
        elif self.gov is not None and n_in:
            hit = self._stake_spent(spent, spent_payload)
            if hit:
                self.gov.removed(STAKE, hit)
        ts.append(perf_counter())
        self.last_apply_stages = dict(zip(('ap_records_s', 'ap_vote_s', 'ap_index_s', 'ap_mempool_s', 'ap_gov_s'),
                                          np.diff(ts).tolist()))
        return 0

    def _stake_spent(self, spent: np.ndarray, spent_payload: np.ndarray) -> List[Tuple[str, int]]:
        """Which of a block's spent outpoints (n x 40 records) are staked outputs: the stake flag their index
        payloads carry (FLAG_STAKE, set from unspent_outputs.is_stake), one vectorised test."""
        hit = np.nonzero(np.asarray(spent_payload['flags']) & FLAG_STAKE)[0]
        if not len(hit):
            return []
        idx = spent[hit, 32:36].copy().view(np.uint32).ravel()
        return [(bytes(spent[k, :32]).hex(), int(i)) for k, i in zip(hit.tolist(), idx.tolist())]

    # spend order and insert order of the object path's writes (manager._apply_block → remove_outputs,
    # add_transaction_outputs): kept so SQL row order (rowid) is the same on both write paths
    _GOV_INSERT_ORDER = ('inode_registration_output', 'validators_voting_power', 'delegates_voting_power',
                         'validator_registration_output', 'inodes_ballot', 'validators_ballot')
    _SPEND_ORDER = ('inode_registration_output', 'unspent_outputs', 'validators_voting_power',
                    'delegates_voting_power', 'inodes_ballot', 'validators_ballot')

    async def apply_object_block(self, block_row: dict, coinbase, transactions) -> int:
        """The object path's block writes (manager._apply_block; reference manager.py:706-730) as ONE journal
        batch — every table, governance ones included — plus the UTXO-index, governance-index and
        chain-tip updates from the same in-memory data, so a block with governance transactions commits
        like a native-path block (and carries undo records for rollback)."""
        b = block_row
        txs = [coinbase] + list(transactions)
        rows = [await self._tx_row(t, b['hash']) for t in txs]  # coinbase row first, as add_transaction did
        tx_base = self._tx_rowids(len(rows))
        stmts = [('INSERT INTO blocks (id, hash, content, address, random, difficulty, reward, timestamp) '
                  'VALUES (?, ?, ?, ?, ?, ?, ?, ?)',
                  [int(b['id']), b['hash'], b['content'], b['address'], int(b['random']), b['difficulty'], b['reward'],
                   int(b['timestamp'])], 1, None, None, None)]
        self.checkpoint('block')
        cols = [list(col) for col in zip(*rows)]
        stmts.append((self._TX_INSERT, [cols[1], cols[0], *cols[2:],
                                        np.arange(tx_base, tx_base + len(rows), dtype=np.int64)], len(rows), None, None,
                      None))
        self.checkpoint('transactions')
        outs = self.split_outputs(list(transactions) + [coinbase])
        created = []  # (table, key, payload fields) for the indexes
        u = outs['unspent_outputs']
        if u:
            base = self._utxo_rowids(len(u))
            stmts.append(('INSERT INTO unspent_outputs (tx_hash, "index", address, is_stake, rowid) VALUES (?, ?, ?, ?, ?)',
                          [[o[0] for o in u], np.array([o[1] for o in u], np.int64), [o[2] for o in u],
                           [None if o[3] is None else str(int(bool(o[3]))) for o in u],
                           np.arange(base, base + len(u), dtype=np.int64)], len(u), None, None, None))
        for table in self._GOV_INSERT_ORDER:
            g = outs[table]
            if g:
                stmts.append((f'INSERT INTO {table} (tx_hash, "index", address) VALUES (?, ?, ?)',
                              [[o[0] for o in g], np.array([o[1] for o in g], np.int64), [o[2] for o in g]],
                              len(g), None, None, None))
        self.checkpoint('outputs')
        tables = {'blocks', 'transactions', 'unspent_outputs', *self._GOV_INSERT_ORDER}
        spends = defaultdict(list)
        for t in transactions:
            spends[self.spend_table(t.transaction_type)].extend((i.tx_hash, int(i.index)) for i in t.inputs)
        mempool = bool(transactions) and not self._mempool_empty()
        if mempool:
            hashes = [t.hash() for t in transactions]
            stmts.append(('DELETE FROM pending_transactions WHERE tx_hash = ?', [hashes], len(hashes), None,
                          'SELECT EXISTS(SELECT 1 FROM pending_transactions)', None))
        for table in self._SPEND_ORDER:
            keys = spends.get(table)
            if keys:
                stmts.append((f'DELETE FROM {table} WHERE tx_hash = ? AND "index" = ?',
                              [[h for h, _ in keys], np.array([i for _, i in keys], np.int64)], len(keys), None,
                              None, len(keys)))
        all_in = [k for t in transactions for k in ((i.tx_hash, int(i.index)) for i in t.inputs)]
        if mempool and all_in:
            stmts.append(('DELETE FROM pending_spent_outputs WHERE tx_hash = ? AND "index" = ?',
                          [[h for h, _ in all_in], np.array([i for _, i in all_in], np.int64)], len(all_in), None,
                          'SELECT EXISTS(SELECT 1 FROM pending_spent_outputs)', None))
            tables |= {'pending_transactions', 'pending_spent_outputs'}
        self.checkpoint('spent')
        aa, ah = self.address_rows(rows)
        stmts.extend(self._address_index_stmts(b['hash'], int(b['id']), [(aa, ah, len(aa))]))
        tables |= {'address_transactions', 'address_index_state'}

        # ---- index records: created outputs (per table) and spent outpoints with their current payloads
        from .utxo import pack_records
        ins_recs, ins_pay = [], []
        if u:
            ins_recs.append(pack_records([(o[0], o[1]) for o in u], TAG_BY_TABLE['unspent_outputs']))
            ins_pay.append(make_payload([o[4] for o in u], [_addr_bytes(o[2]) for o in u], [o[3] for o in u]))
        for table in self._GOV_INSERT_ORDER:
            g = outs[table]
            if g:
                ins_recs.append(pack_records([(o[0], o[1]) for o in g], TAG_BY_TABLE[table]))
                ins_pay.append(make_payload([o[3] for o in g], [_addr_bytes(o[2]) for o in g]))
        created_recs = np.concatenate(ins_recs) if ins_recs else np.zeros((0, 40), np.uint8)
        created_pay = np.concatenate(ins_pay) if ins_pay else np.zeros(0, PAYLOAD_DTYPE)
        sp_recs, sp_pay = [], []
        for table in self._SPEND_ORDER:
            keys = spends.get(table)
            if keys:
                tags, pay = self.utxo.lookup(keys)
                present = tags == TAG_BY_TABLE[table]
                keys = [k for k, ok in zip(keys, present) if ok]
                if keys:
                    sp_recs.append(pack_records(keys, TAG_BY_TABLE[table]))
                    sp_pay.append(np.ascontiguousarray(pay[present]))
        spent_recs = np.concatenate(sp_recs) if sp_recs else np.zeros((0, 40), np.uint8)
        spent_pay = np.concatenate(sp_pay) if sp_pay else np.zeros(0, PAYLOAD_DTYPE)

        enc = [self.encode(*st) for st in stmts]
        meta = bytes.fromhex(b['hash']) + struct.pack('<qII', int(b['id']), len(created_recs), len(spent_recs)) + \
            created_recs.tobytes() + spent_recs.tobytes() + spent_pay.tobytes()
        _commit_point()
        seq = self.submit_batch(enc, tables, meta, int(b['id']))
        # ---- the indexes and the chain-tip cache follow the commit point
        if len(spent_recs):
            self.utxo.erase_records(spent_recs)
        if len(created_recs):
            self.utxo.insert_records(created_recs, created_pay)
        if self.gov is not None:
            self._gov_apply_block(rows, outs, spends, int(b['timestamp']))
        tip = dict(b)
        tip['difficulty'], tip['reward'] = Decimal(tip['difficulty']), Decimal(tip['reward'])
        self._tip_gen += 1
        self._tip_cache = normalize_block(tip)
        self._remember_row(self._tip_cache)
        if mempool:
            self._pending_empty = None
            self._mempool_ver += 1
        if transactions:
            self._mempool_confirm(mempool, hashes=[t.hash() for t in transactions], inputs=all_in, block_seq=seq)
        return seq

    def _gov_apply_block(self, rows, outs, spends, block_ts: int):
        """Governance-index update for one object-path block from its own rows: what GovernanceIndex.added
        would read back through the SQL joins (address; amount = outputs_amounts[index]; voter =
        inputs_addresses[index]; the block's timestamp)."""
        ia = {r[1]: _arr(r[3]) for r in rows}
        am = {r[1]: _arr(r[5]) for r in rows}
        g = self.gov
        with g.lock:
            for table in self._SPEND_ORDER:
                keys = spends.get(table)
                if keys:
                    g.removed(STAKE if table == 'unspent_outputs' else table, keys)
            for table in (STAKE, *self._GOV_INSERT_ORDER):
                src = outs['unspent_outputs'] if table == STAKE else outs[table]
                batch = [_gov_row((o[0], o[1]), o[2], _at(am[o[0]], o[1]), _at(ia[o[0]], o[1]), block_ts)
                         for o in src if table != STAKE or o[3] is True or o[3] == 1]
                if batch:
                    g.store.add_rows(GOV_TID[table], batch)
            g.version += 1

    def _undo_blocks_in_index(self, from_id: int, tip: int):
        """Roll the UTXO index back from ``tip`` to ``from_id - 1`` with the undo log's records (created
        outpoints erased, spent outpoints re-inserted, newest block first). Returns the created outpoints
        (for the governance index), or None when a block in the range has no undo record or its record
        belongs to another block with that id (applied before a rollback whose tombstone was lost): the
        caller rebuilds the index instead.

        Spent outpoints come back the way ``remove_blocks`` restores them in SQL (reference
        database.py:146-169 → add_unspent_outputs): as ``unspent_outputs`` rows with ``is_stake`` NULL,
        whatever table they were spent from — so the index stays record-for-record equal to a rebuild."""
        if self.writer is None or tip < from_id:
            return [] if tip < from_id else None
        hashes = {int(r[0]): r[1] for r in self._q('SELECT id, hash FROM blocks WHERE id >= ? AND id <= ?',
                                                  (from_id, tip))}
        metas = []
        for i in range(tip, from_id - 1, -1):
            m = self.writer.journal_meta(i)
            if m is None or len(m) < 48 or hashes.get(i) is None or m[:32] != bytes.fromhex(hashes[i]):
                return None
            metas.append(m)
        tag_u = TAG_BY_TABLE['unspent_outputs']
        created_all = []
        for m in metas:
            _, n_created, n_spent = struct.unpack_from('<qII', m, 32)
            o = 48
            created = np.frombuffer(m, dtype=np.uint8, count=40 * n_created, offset=o).reshape(-1, 40)
            o += 40 * n_created
            spent = np.frombuffer(m, dtype=np.uint8, count=40 * n_spent, offset=o).reshape(-1, 40)
            o += 40 * n_spent
            pay = np.frombuffer(m, dtype=PAYLOAD_DTYPE, count=n_spent, offset=o)
            if n_created:
                rec = created.copy()
                rec[:, 36:40] = np.full((n_created, 1), 0xFF, dtype=np.uint32).view(np.uint8)  # any table
                self.utxo.erase_records(rec)
                created_all.append(created)
            if n_spent:
                rec = spent.copy()
                rec[:, 36:40] = np.full((n_spent, 1), tag_u, dtype=np.uint32).view(np.uint8)
                p = pay.copy()
                p['flags'] &= np.uint32(~FLAG_STAKE & 0xFFFFFFFF)
                self.utxo.insert_records(rec, p)
        keys = []
        for c in created_all:
            idx = c[:, 32:36].copy().view(np.uint32).ravel()
            keys.extend(zip((bytes(r).hex() for r in c[:, :32]), idx.tolist()))
        return keys

    async def _add_gov_outputs(self, table: str, outputs: List[tuple]):
        if not outputs:
            return
        rows = [(o[0], o[1], o[2] if len(o) > 2 else None) for o in outputs]
        self._xm(f'INSERT INTO {table} (tx_hash, "index", address) VALUES (?, ?, ?)', rows)
        if self.gov is not None:
            self.gov.added(table, [(r[0], r[1]) for r in rows])
        if len(outputs[0]) >= 4:  # (tx_hash, index, address, amount in smallest units)
            payload = make_payload([o[3] for o in outputs], [_addr_bytes(o[2]) for o in outputs])
        else:
            payload = await self._payload_from_ledger([(r[0], r[1]) for r in rows])
        self.utxo.insert([(r[0], r[1]) for r in rows], TAG_BY_TABLE[table], payload)

    async def add_inode_registration_outputs(self, outputs):
        await self._add_gov_outputs('inode_registration_output', outputs)

    async def add_validator_registration_outputs(self, outputs):
        await self._add_gov_outputs('validator_registration_output', outputs)

    async def add_validator_voting_power(self, outputs):
        await self._add_gov_outputs('validators_voting_power', outputs)

    async def add_delegates_voting_power(self, outputs):
        await self._add_gov_outputs('delegates_voting_power', outputs)

    async def add_vote_to_inode_ballots(self, outputs):
        await self._add_gov_outputs('inodes_ballot', outputs)

    async def add_vote_to_validators_ballot(self, outputs):
        await self._add_gov_outputs('validators_ballot', outputs)

    async def add_pending_spent_outputs(self, outputs: List[Tuple[str, int]]) -> None:
        self._xm('INSERT INTO pending_spent_outputs (tx_hash, "index") VALUES (?, ?)', outputs)

    async def add_transactions_pending_spent_outputs(self, transactions: List[Transaction]) -> None:
        outputs = [(i.tx_hash, i.index) for t in transactions for i in t.inputs]
        try:
            self._xm('INSERT INTO pending_spent_outputs (tx_hash, "index") VALUES (?, ?)', outputs)
        except sqlite3.IntegrityError as e:  # FK: spent output must belong to a confirmed tx
            raise ForeignKeyViolationError(str(e)) from e

    @staticmethod
    def split_outputs(transactions) -> Dict[str, list]:
        """Bucket every output into its table (database.py:524-580)."""
        b = {t: [] for t in OUTPUT_TABLES}
        gov = {OutputType.INODE_REGISTRATION: 'inode_registration_output',
               OutputType.VALIDATOR_REGISTRATION: 'validator_registration_output',
               OutputType.VALIDATOR_VOTING_POWER: 'validators_voting_power',
               OutputType.DELEGATE_VOTING_POWER: 'delegates_voting_power',
               OutputType.VOTE_AS_VALIDATOR: 'inodes_ballot', OutputType.VOTE_AS_DELEGATE: 'validators_ballot'}
        for tx in transactions:
            h = tx.hash()
            for index, o in enumerate(tx.outputs):
                t = o.transaction_type
                amount = int(o.amount * SMALLEST)
                if t in (OutputType.REGULAR, OutputType.STAKE, OutputType.UN_STAKE):
                    b['unspent_outputs'].append((h, index, o.address, o.is_stake, amount))
                elif t in gov:
                    b[gov[t]].append((h, index, o.address, amount))
        return b

    async def add_transaction_outputs(self, transactions):
        b = self.split_outputs(transactions)
        await self.add_unspent_outputs(b['unspent_outputs'])
        await self.add_inode_registration_outputs(b['inode_registration_output'])
        await self.add_validator_voting_power(b['validators_voting_power'])
        await self.add_delegates_voting_power(b['delegates_voting_power'])
        await self.add_validator_registration_outputs(b['validator_registration_output'])
        await self.add_vote_to_inode_ballots(b['inodes_ballot'])
        await self.add_vote_to_validators_ballot(b['validators_ballot'])

    async def add_unspent_transactions_outputs(self, transactions) -> None:
        await self.add_unspent_outputs([(t.hash(), i, o.address, o.is_stake)
                                        for t in transactions for i, o in enumerate(t.outputs)])

    @staticmethod
    def spend_table(tx_type) -> str:
        """Which table a tx type spends from (database.py:589-621)."""
        return {TransactionType.INODE_DE_REGISTRATION: 'inode_registration_output',
                TransactionType.VOTE_AS_VALIDATOR: 'validators_voting_power',
                TransactionType.VOTE_AS_DELEGATE: 'delegates_voting_power',
                TransactionType.REVOKE_AS_VALIDATOR: 'inodes_ballot',
                TransactionType.REVOKE_AS_DELEGATE: 'validators_ballot'}.get(tx_type, 'unspent_outputs')

    async def remove_outputs(self, transactions):
        by_table = defaultdict(list)
        for t in transactions:
            by_table[self.spend_table(t.transaction_type)].append(t)
        for table in ('inode_registration_output', 'unspent_outputs', 'validators_voting_power',
                      'delegates_voting_power', 'inodes_ballot', 'validators_ballot'):
            if by_table[table]:
                if table == 'unspent_outputs':
                    await self.remove_unspent_outputs(by_table[table])
                else:
                    self._remove_table_inputs(table, by_table[table])

    def _remove_table_inputs(self, table, transactions):
        inputs = [(i.tx_hash, i.index) for t in transactions for i in t.inputs]
        self._delete_outpoints(table, inputs)
        if self.gov is not None:
            self.gov.removed(table, inputs)
        self.utxo.erase(inputs)

    async def remove_unspent_outputs(self, transactions, max_retries: int = 3) -> bool:
        """database.py:589-621: delete the spent outpoints and report whether every one was there.
        Like the reference (which returns from inside its transaction block, i.e. commits), the
        deletions that did happen stand — blocks in ``double_spend_dict`` rely on this."""
        start = perf_counter()
        inputs = [(i.tx_hash, i.index) for t in transactions for i in t.inputs]
        if not inputs:
            return True
        with self.transaction():
            n = self._xm('DELETE FROM unspent_outputs WHERE tx_hash = ? AND "index" = ?',
                         [(h, int(i)) for h, i in inputs]).rowcount
        self.utxo.erase(inputs, TAG_BY_TABLE['unspent_outputs'])
        if self.gov is not None:
            self.gov.removed(STAKE, inputs)
        if n != len(inputs):
            logger.error(f'Failed to delete all UTXOs: {n} of {len(inputs)} deleted')
            return False
        logger.info(f'Successfully removed {len(inputs)} unspent outputs in {perf_counter() - start:.3f} seconds')
        return True

    async def remove_inode_registration_output(self, transactions):
        self._remove_table_inputs('inode_registration_output', transactions)

    async def remove_validators_voting_power(self, transactions):
        self._remove_table_inputs('validators_voting_power', transactions)

    async def remove_delegates_voting_power(self, transactions):
        self._remove_table_inputs('delegates_voting_power', transactions)

    async def remove_inode_ballot_votes(self, transactions):
        self._remove_table_inputs('inodes_ballot', transactions)

    async def remove_validator_ballot_votes(self, transactions):
        self._remove_table_inputs('validators_ballot', transactions)

    async def remove_pending_spent_outputs(self, transactions) -> None:
        self._delete_outpoints('pending_spent_outputs', [(i.tx_hash, i.index) for t in transactions for i in t.inputs])

    async def remove_pending_spent_outputs_by_tuple(self, inputs: List[Tuple[str, int]], max_retries: int = 3) -> bool:
        if not inputs:
            return True
        start = perf_counter()
        with self.transaction():
            n = self._xm('DELETE FROM pending_spent_outputs WHERE tx_hash = ? AND "index" = ?',
                         [(h, int(i)) for h, i in inputs]).rowcount
        if n != len(inputs):
            logger.error(f'Failed to delete all pending_spent_outputs: {n} of {len(inputs)} deleted')
            return False
        logger.info(f'Successfully removed {len(inputs)} pending_spent_outputs in {perf_counter() - start:.3f} seconds')
        return True

    # lookups (database.py:788-825): a block's outpoints go to the HBM/host index in one batch; a
    # handful of them (one tx at /push_tx) on the GPU backend go to SQLite's outpoint index instead —
    # a device round trip costs ~1 ms when the card is busy (a co-located miner keeps every CU
    # occupied), an indexed probe ~5 us, and both hold the same set once the table is materialised.
    # While the materialiser is still writing a just-committed block into the table, the index
    # (current at the commit point) answers: waiting for the table would cost tens of ms.
    SMALL_LOOKUP = 16

    def _filter_outputs(self, table: str, outputs):
        if (self.lean or len(outputs) > self.SMALL_LOOKUP or self.utxo.backend_name != 'gpu'
                or not self._fresh(table)):
            return self.utxo.filter(outputs, TAG_BY_TABLE[table])
        uniq = list(dict.fromkeys((h, int(i)) for h, i in outputs))
        found = set(self._select_outpoints(table, uniq))
        return [k for k in uniq if k in found]  # the index's answer order: unique, first seen

    async def _outputs(self, table: str, outputs):
        """``_filter_outputs``; a /push_tx admission on the GPU backend instead joins the event loop's
        batched HBM-index probe (utils/coalesce.py): one device round trip for the concurrent requests,
        on an executor thread, so the event loop neither blocks on the device nor on SQLite."""
        if (coalesce.ADMISSION.get() and self.utxo.backend_name == 'gpu' and len(outputs) <= self.SMALL_LOOKUP
                and os.environ.get('UPOW_ADMISSION_HBM_PROBE', '1') != '0'):
            uniq = list(dict.fromkeys((h, int(i)) for h, i in outputs))
            found = await coalesce.coalescer('utxo-probe', _probe_batch).submit((self, TAG_BY_TABLE[table], uniq))
            return [k for k in uniq if k in found]
        return self._filter_outputs(table, outputs)

    async def get_unspent_outputs(self, outputs):
        return await self._outputs('unspent_outputs', outputs)

    async def get_inode_outputs(self, outputs):
        return await self._outputs('inode_registration_output', outputs)

    async def get_validator_voting_power_outputs(self, outputs):
        return await self._outputs('validators_voting_power', outputs)

    async def get_delegates_voting_power_outputs(self, outputs):
        return await self._outputs('delegates_voting_power', outputs)

    async def get_inodes_ballot_outputs(self, outputs):
        return await self._outputs('inodes_ballot', outputs)

    async def get_validators_ballot_outputs(self, outputs):
        return await self._outputs('validators_ballot', outputs)

    async def get_unspent_outputs_hash(self) -> str:
        """database.py:827-830: SHA256 over (tx_hash bytes || index byte) sorted by (tx_hash, index).

        From the UTXO index (K12 on the device for the HBM table: compaction + radix sort + gather, host
        hash tail), which is current at the commit point; ``UPOW_UTXO_HASH_SQL=1`` forces the SQL
        ORDER BY form."""
        if os.environ.get('UPOW_UTXO_HASH_SQL', '0') != '1':
            return self.utxo.set_hash(TAG_BY_TABLE['unspent_outputs'])
        return self.sql_unspent_outputs_hash()

    def sql_unspent_outputs_hash(self) -> str:
        rows = self._q('SELECT tx_hash, "index" FROM unspent_outputs ORDER BY tx_hash, "index"')
        return sha256(''.join(r[0] + bytes([r[1]]).hex() for r in rows))

    async def get_pending_spent_outputs(self, outputs):
        mp = self._mempool()
        if mp is not None:
            return mp.spent_of(outputs)
        return self._select_outpoints('pending_spent_outputs', outputs)

    async def set_unspent_outputs_addresses(self):
        rows = self._q('SELECT rowid, tx_hash, "index" FROM unspent_outputs WHERE address IS NULL')
        infos = await self.get_transactions_info([r['tx_hash'] for r in rows])
        self._xm('UPDATE unspent_outputs SET address = ? WHERE rowid = ?',
                 [(_at(infos[r['tx_hash']]['outputs_addresses'], r['index'])
                   if r['tx_hash'] in infos else None, r['rowid']) for r in rows])

    async def get_unspent_outputs_from_all_transactions(self):
        """database.py:846-862: replay every tx in block order (UTXO rebuild tool)."""
        outputs = set()
        blocks = [r[0] for r in self._q('SELECT hash FROM blocks ORDER BY id ASC')]
        for tx_hex in (h for b in blocks for h in self._txs_of_blocks([b], 'tx_hex')):
            tx_hash = sha256(tx_hex)
            tx = await Transaction.from_hex(tx_hex, check_signatures=False)
            if isinstance(tx, Transaction):
                outputs = outputs.difference({(i.tx_hash, i.index) for i in tx.inputs})
            outputs.update({(tx_hash, index) for index in range(len(tx.outputs))})
        return list(outputs)

    # ------------------------------------------------------------------ address queries
    @staticmethod
    def _forms(address: str) -> List[str]:
        return codec.address_forms(address)

    @staticmethod
    def _search(address: str) -> List[str]:
        return codec.address_search_hex(address)

    def _pending_matching(self, address: str, include_inputs: bool = True) -> List[sqlite3.Row]:
        search, forms = self._search(address), set(self._forms(address))
        out = []
        for r in self._q('SELECT tx_hash, tx_hex, inputs_addresses FROM pending_transactions ORDER BY rowid'):
            if any(s in r['tx_hex'] for s in search) or (include_inputs and forms & set(_arr(r['inputs_addresses']))):
                out.append(r)
        return out

    async def get_address_transactions(self, address: str, check_pending_txs: bool = False,
                                       check_signatures: bool = False, limit: int = 50, offset: int = 0):
        self.index_addresses()
        forms = self._forms(address)
        ph = ','.join('?' * len(forms))
        key = 'a.tx_hash'
        rows = self._q(f'SELECT tx_hex, block_no, rid FROM (SELECT DISTINCT a.tx_hash, {self._txq("tx_hex", key)} AS tx_hex, '
                       f'{self._txq("rowid", key)} AS rid, (SELECT b.id FROM blocks b WHERE b.hash = '
                       f'{self._txq("block_hash", key)}) AS block_no FROM address_transactions a '
                       f'WHERE a.address IN ({ph})) WHERE tx_hex IS NOT NULL AND block_no IS NOT NULL '
                       f'ORDER BY block_no DESC, rid LIMIT ? OFFSET ?', (*forms, limit, offset))
        txs = [r['tx_hex'] for r in rows]
        if check_pending_txs:
            txs = [r['tx_hex'] for r in self._pending_matching(address)] + txs
        return [await Transaction.from_hex(t, check_signatures) for t in txs]

    async def get_address_pending_transactions(self, address: str, check_signatures: bool = False):
        return [await Transaction.from_hex(r['tx_hex'], check_signatures) for r in self._pending_matching(address)]

    async def get_address_pending_spent_outputs(self, address: str, check_signatures: bool = False):
        txs = [await Transaction.from_hex(r['tx_hex'], check_signatures) for r in self._pending_matching(address)]
        return [{'tx_hash': i.tx_hash, 'index': i.index} for tx in txs for i in tx.inputs]

    def _amount_rows(self, table: str, forms: List[str], where: str = '', check_pending: bool = False,
                     args: tuple = ()):
        """``SELECT t.tx_hash, index, transactions.outputs_amounts[index + 1] FROM t JOIN transactions``."""
        ph = ','.join('?' * len(forms))
        rows = self._q(f'SELECT {table}.tx_hash AS tx_hash, {table}."index" AS idx, '
                       f'{self._txq("outputs_amounts", table + ".tx_hash")} AS am '
                       f'FROM {table} WHERE {table}.address IN ({ph}) {where} ORDER BY {table}.rowid', (*forms, *args))
        pend = self._pending_spent_set() if check_pending else set()
        out = []
        for r in rows:
            if r['am'] is None or (r['tx_hash'], r['idx']) in pend:  # (INNER JOIN transactions)
                continue
            out.append((r['tx_hash'], r['idx'], _at(_arr(r['am']), r['idx'])))
        return out

    def _index_address_rows(self, address: str, stake_sel: int, check_pending: bool) -> List[Tuple[str, int, int]]:
        """(tx_hash, index, amount) of the live ``unspent_outputs`` entries owned by ``address`` (either byte
        form), from the UTXO index (K14: one HBM scan per form on a GPU node, an owner map on the host)
        in canonical (tx_hash, index) order. The reference's ``address = ANY($1)`` over unspent_outputs
        (database.py:909-937) has no defined row order; the index answers at the commit point, without
        waiting for the SQL materialiser and without an address B-tree to maintain per block."""
        pend = (self.gov.pending_spent(True) if self.gov is not None else self._pending_spent_set()) \
            if check_pending else set()
        out = []
        for h in codec.address_search_hex(address):
            recs, pay, _ = self.utxo.address_outputs(bytes.fromhex(h), (TAG_BY_TABLE['unspent_outputs'],), stake_sel)
            idx = recs[:, 32:36].copy().view('<u4').ravel()
            for k in range(len(recs)):
                key = (bytes(recs[k, :32]).hex(), int(idx[k]))
                if key not in pend:
                    out.append((key[0], key[1], int(pay['amount'][k])))
        out.sort(key=lambda r: (r[0], r[1]))
        return out

    async def get_spendable_outputs(self, address: str, check_pending_txs: bool = False) -> List[TransactionInput]:
        point = string_to_point(address)
        if self.address_queries_from_index:
            from .utxo import STAKE_EXCLUDE
            return [TransactionInput(h, i, amount=Decimal(a) / SMALLEST, public_key=point)
                    for h, i, a in self._index_address_rows(address, STAKE_EXCLUDE, check_pending_txs)]
        forms = list(reversed(self._forms(address)))
        if self._q1('SELECT tx_hash FROM unspent_outputs WHERE address IS NULL LIMIT 1') is not None:
            await self.set_unspent_outputs_addresses()
        rows = self._amount_rows('unspent_outputs', forms,
                                 'AND (unspent_outputs.is_stake IS NULL OR unspent_outputs.is_stake = 0)',
                                 check_pending_txs)
        return [TransactionInput(h, i, amount=Decimal(a) / SMALLEST, public_key=point) for h, i, a in rows]

    async def get_stake_outputs(self, address: str, check_pending_txs: bool = False) -> List[TransactionInput]:
        point = string_to_point(address)
        forms = list(reversed(self._forms(address)))
        if self.gov is not None:
            return [TransactionInput(h, i, amount=Decimal(a) / SMALLEST, public_key=point)
                    for h, i, a in self.gov.amount_rows(STAKE, forms, check_pending_txs)]
        if self._q1('SELECT tx_hash FROM unspent_outputs WHERE address IS NULL LIMIT 1') is not None:
            await self.set_unspent_outputs_addresses()
        rows = self._amount_rows('unspent_outputs', forms, 'AND (unspent_outputs.is_stake = 1)', check_pending_txs)
        return [TransactionInput(h, i, amount=Decimal(a) / SMALLEST, public_key=point) for h, i, a in rows]

    async def _table_inputs(self, table: str, address: str, check_pending_txs: bool) -> List[TransactionInput]:
        point = string_to_point(address)
        forms = list(reversed(self._forms(address)))
        if self.gov is not None:
            rows = self.gov.amount_rows(table, forms, check_pending_txs)
        else:
            rows = self._amount_rows(table, forms, '', check_pending_txs)
        return [TransactionInput(h, i, amount=Decimal(a) / SMALLEST, public_key=point) for h, i, a in rows]

    async def get_inode_registration_outputs(self, address: str, check_pending_txs: bool = False):
        return await self._table_inputs('inode_registration_output', address, check_pending_txs)

    async def get_validator_registration_outputs(self, address: str, check_pending_txs: bool = False):
        return await self._table_inputs('validator_registration_output', address, check_pending_txs)

    async def get_validators_voting_power(self, address: str, check_pending_txs: bool = False):
        return await self._table_inputs('validators_voting_power', address, check_pending_txs)

    async def get_delegates_voting_power(self, address: str, check_pending_txs: bool = False):
        return await self._table_inputs('delegates_voting_power', address, check_pending_txs)

    async def is_inode_registered(self, address: str, check_pending_txs: bool = False) -> bool:
        return len(await self.get_inode_registration_outputs(address, check_pending_txs)) > 0

    async def is_validator_registered(self, address: str, check_pending_txs: bool = False) -> bool:
        return len(await self.get_validator_registration_outputs(address, check_pending_txs)) > 0

    def _spent_votes(self, table: str, address: str, check_pending: bool) -> List[TransactionInput]:
        """Ballots cast by ``address``: ``transactions.inputs_addresses[index + 1] = ANY(forms)``
        (database.py:1479-1500, 1526-1547; the ballot *output* index subscripts the inputs array)."""
        point = string_to_point(address)
        forms = set(self._forms(address))
        if self.gov is not None:
            return [TransactionInput(h, i, amount=Decimal(a) / SMALLEST, public_key=point)
                    for (h, i), a in self.gov.spent_votes(table, forms, check_pending)]
        pend = self._pending_spent_set() if check_pending else set()
        key = f'{table}.tx_hash'
        rows = self._q(f'SELECT {table}.tx_hash AS tx_hash, {table}."index" AS idx, {self._txq("outputs_amounts", key)} AS am, '
                       f'{self._txq("inputs_addresses", key)} AS ia FROM {table} ORDER BY {table}.rowid')
        out = []
        for r in rows:
            if r['am'] is None:  # (INNER JOIN transactions)
                continue
            if _at(_arr(r['ia']), r['idx']) in forms and (r['tx_hash'], r['idx']) not in pend:
                out.append(TransactionInput(r['tx_hash'], r['idx'], amount=Decimal(_at(_arr(r['am']), r['idx'])) / SMALLEST,
                                            public_key=point))
        return out

    async def get_validators_spent_votes(self, address: str, check_pending_txs: bool = False):
        return self._spent_votes('inodes_ballot', address, check_pending_txs)

    async def get_delegates_spent_votes(self, address: str, check_pending_txs: bool = False):
        return self._spent_votes('validators_ballot', address, check_pending_txs)

    async def get_delegates_all_power(self, address: str, check_pending_txs: bool = False):
        unspent = await self.get_delegates_voting_power(address, check_pending_txs)
        unspent.extend(await self.get_delegates_spent_votes(address, check_pending_txs))
        return unspent

    # ------------------------------------------------------------------ ballots (database.py:939-1136)
    def _ballot_rows(self, table: str, receiver_forms: Optional[List[str]], check_pending: bool,
                     limit: Optional[int] = None, offset: int = 0, voter_forms: Optional[Set[str]] = None,
                     order: bool = True):
        if self.gov is not None:
            out = self.gov.ballot_rows(table, receiver_forms, check_pending, voter_forms, order)
            return out[offset:offset + limit] if limit is not None else out
        where, args = '', []
        if receiver_forms is not None:
            where = f'WHERE {table}.address IN ({",".join("?" * len(receiver_forms))})'
            args = list(receiver_forms)
        key = f'{table}.tx_hash'
        rows = self._q(f'SELECT {table}.tx_hash AS tx_hash, {table}.address AS receiver, {table}."index" AS idx, '
                       f'{self._txq("outputs_amounts", key)} AS am, {self._txq("inputs_addresses", key)} AS ia '
                       f'FROM {table} {where} ORDER BY {(table + ".tx_hash, ") if order else ""}{table}.rowid', args)
        pend = self._pending_spent_set() if check_pending else set()
        out = []
        for r in rows:
            if r['am'] is None or (r['tx_hash'], r['idx']) in pend:  # (INNER JOIN transactions)
                continue
            voter = _at(_arr(r['ia']), r['idx'])
            if voter_forms is not None and voter not in voter_forms:
                continue
            vote = _at(_arr(r['am']), r['idx'])
            out.append((r['tx_hash'], r['receiver'], Decimal(vote) / SMALLEST if vote is not None else None,
                        voter, r['idx']))
        if limit is not None:
            out = out[offset:offset + limit]
        return out

    async def get_inode_ballot(self, offset: int, limit: int, check_pending_txs: bool = False):
        return self._ballot_rows('inodes_ballot', None, check_pending_txs, limit, offset)

    async def get_inode_ballot_by_address(self, offset: int, limit: int, inode: str, check_pending_txs: bool = False):
        return self._ballot_rows('inodes_ballot', self._forms(inode), check_pending_txs, limit, offset)

    async def get_inode_ballot_input_by_address(self, validator_address: str, vote_receiver_address: str,
                                                check_pending_txs: bool = False) -> List[TransactionInput]:
        point = string_to_point(validator_address)
        rows = self._ballot_rows('inodes_ballot', list(reversed(self._forms(vote_receiver_address))), check_pending_txs,
                                 voter_forms=set(self._forms(validator_address)), order=False)
        return [TransactionInput(h, i, amount=v, public_key=point) for h, _, v, _, i in rows]

    async def get_validator_ballot_input_by_address(self, delegate_address: str, vote_receiver_address: str,
                                                    check_pending_txs: bool = False) -> List[TransactionInput]:
        point = string_to_point(delegate_address)
        rows = self._ballot_rows('validators_ballot', list(reversed(self._forms(vote_receiver_address))),
                                 check_pending_txs, voter_forms=set(self._forms(delegate_address)), order=False)
        return [TransactionInput(h, i, amount=v, public_key=point) for h, _, v, _, i in rows]

    async def get_validator_ballot(self, offset: int, limit: int, check_pending_txs: bool = False):
        return self._ballot_rows('validators_ballot', None, check_pending_txs, limit, offset)

    async def get_validator_ballot_by_address(self, offset: int, limit: int, validator: str,
                                              check_pending_txs: bool = False):
        return self._ballot_rows('validators_ballot', self._forms(validator), check_pending_txs, limit, offset)

    async def get_transaction_time(self, tx_hash) -> datetime:
        r = self._q1('SELECT timestamp FROM blocks WHERE hash = '
                     '(SELECT block_hash FROM transactions WHERE tx_hash = ?)', (tx_hash,))
        assert r is not None
        return _dt(r[0])

    async def is_revoke_valid(self, tx_hash) -> bool:
        return _utcnow() - await self.get_transaction_time(tx_hash) >= timedelta(hours=48)

    async def get_validators_stake(self, validator: str, check_pending_txs: bool = False):
        if self.gov is not None:
            return self.gov.validators_stake(self._forms(validator), check_pending_txs)
        ballot = await self.get_validator_ballot_by_address(0, 100000, validator=validator,
                                                            check_pending_txs=check_pending_txs)
        ratio = [(vote * await self.get_address_stake(delegate)) / 10 for _, _, vote, delegate, _ in ballot]
        return round_up_decimal(sum(ratio, Decimal(0)))

    async def get_address_balance(self, address: str, check_pending_txs: bool = False) -> Decimal:
        forms = self._forms(address)
        balance = sum([i.amount for i in await self.get_spendable_outputs(address, check_pending_txs)], Decimal(0))
        if check_pending_txs:
            search = self._search(address)
            for r in self._q('SELECT tx_hex FROM pending_transactions ORDER BY rowid'):
                if not any(s in r['tx_hex'] for s in search):
                    continue
                tx = await Transaction.from_hex(r['tx_hex'], check_signatures=False)
                for o in tx.outputs:
                    if o.address in forms and o.transaction_type is OutputType.REGULAR and \
                            (o.is_stake is False or o.is_stake is None):
                        balance += o.amount
        return balance

    async def get_pending_stake_transaction(self, address: str):
        search = self._search(address)
        out = []
        for r in self._q('SELECT tx_hex FROM pending_transactions ORDER BY rowid'):
            if not any(s in r['tx_hex'] for s in search):
                continue
            tx = await Transaction.from_hex(r['tx_hex'], check_signatures=False)
            for o in tx.outputs:
                if o.address == address and o.transaction_type is OutputType.STAKE:
                    out.append(tx)
        assert len(out) < 2
        return out

    async def get_pending_vote_as_delegate_transaction(self, address: str):
        search = self._search(address)
        out = []
        for r in self._q('SELECT tx_hex FROM pending_transactions ORDER BY rowid'):
            if not any(s in r['tx_hex'] for s in search):
                continue
            tx = await Transaction.from_hex(r['tx_hex'], check_signatures=False)
            if tx.transaction_type == TransactionType.VOTE_AS_DELEGATE and await tx.inputs[0].get_address() == address:
                out.append(tx)
        return out

    async def get_address_stake(self, address: str, check_pending_txs: bool = False) -> Decimal:
        forms = self._forms(address)
        if self.gov is not None:
            return self.gov.address_stake(forms, check_pending_txs)
        stake = sum([i.amount for i in await self.get_stake_outputs(address, check_pending_txs)], Decimal(0))
        if check_pending_txs:
            search = self._search(address)
            for r in self._q('SELECT tx_hex FROM pending_transactions ORDER BY rowid'):
                if not any(s in r['tx_hex'] for s in search):
                    continue
                tx = await Transaction.from_hex(r['tx_hex'], check_signatures=False)
                for o in tx.outputs:
                    if o.address in forms and o.is_stake is True:
                        stake += o.amount
        return stake

    async def get_multiple_address_stakes(self, addresses: Set[str], check_pending_txs: bool = False
                                          ) -> Dict[str, Decimal]:
        if not addresses:
            return {}
        data = {a: {'formats': self._forms(a), 'searches': self._search(a)} for a in addresses}
        all_forms = [f for d in data.values() for f in d['formats']]
        if self.gov is not None:
            stake_map = defaultdict(Decimal)
            for h, i, a, address in self.gov.address_rows(STAKE, all_forms, check_pending_txs):
                original = next(k for k, d in data.items() if address in d['formats'])
                stake_map[original] += Decimal(a) / SMALLEST
            if check_pending_txs:
                pstake = self.gov._overlay()[2]
                for original, d in data.items():
                    for f in d['formats']:
                        if f in pstake:
                            stake_map[original] += pstake[f]
            return dict(stake_map)
        if self._q1('SELECT tx_hash FROM unspent_outputs WHERE address IS NULL LIMIT 1') is not None:
            await self.set_unspent_outputs_addresses()
        rows = self._amount_rows('unspent_outputs', all_forms, 'AND unspent_outputs.is_stake = 1', check_pending_txs)
        addr_of = {}
        for r in self._q(f'SELECT tx_hash, "index", address FROM unspent_outputs WHERE address IN '
                         f'({",".join("?" * len(all_forms))}) AND is_stake = 1', all_forms):
            addr_of[(r[0], r[1])] = r[2]
        stake_map = defaultdict(Decimal)
        for h, i, a in rows:
            address = addr_of.get((h, i))
            original = next(k for k, d in data.items() if address in d['formats'])
            stake_map[original] += Decimal(a) / SMALLEST
        if check_pending_txs:
            searches = [s for d in data.values() for s in d['searches']]
            for r in self._q('SELECT tx_hex FROM pending_transactions ORDER BY rowid'):
                if not any(s in r['tx_hex'] for s in searches):
                    continue
                tx = await Transaction.from_hex(r['tx_hex'], check_signatures=False)
                for o in tx.outputs:
                    if o.is_stake:
                        for original, d in data.items():
                            if o.address in d['formats']:
                                stake_map[original] += o.amount
        return dict(stake_map)

    # ------------------------------------------------------------------ inodes (database.py:1348-1438)
    async def get_genesis_block(self):
        if self._genesis_cache is None and 1 in self._lean_rows:
            return self._lean_rows[1]['content']
        if self._genesis_cache is None:
            r = self._q1('SELECT content FROM blocks WHERE id = 1')
            self._genesis_cache = r[0] if r else None
        return self._genesis_cache

    async def get_all_registered_inode(self, check_pending_txs: bool = False):
        if self.gov is not None:
            return [(a, _dt(ts)) for a, ts in self.gov.registered_inodes(check_pending_txs)]
        t = 'inode_registration_output'
        rows = self._q(f'SELECT {t}.address AS address, {t}.tx_hash AS h, {t}."index" AS idx, '
                       f'(SELECT b.timestamp FROM blocks b WHERE b.hash = {self._txq("block_hash", t + ".tx_hash")}) AS ts '
                       f'FROM {t} ORDER BY {t}.rowid')
        pend = self._pending_spent_set() if check_pending_txs else set()
        # (INNER JOIN transactions, blocks: rows without both have no timestamp)
        return [(r['address'], _dt(r['ts'])) for r in rows if r['ts'] is not None and (r['h'], r['idx']) not in pend]

    async def get_active_inodes(self, check_pending_txs: bool = False):
        codec.getting_active_inodes = True
        try:
            inode_with_vote = await self.get_all_registered_inode_with_vote(check_pending_txs)
            total_power = sum(item['power'] for item in inode_with_vote)
            now = _utcnow()
            for item in inode_with_vote:
                item['emission'] = (item['power'] / total_power) * 100 if total_power > 0 else item['power']
                item['emission'] = round_up_decimal(item['emission'], round_up_length='0.01')
                item['is_active'] = item['emission'] >= 1 or now - item['registered_at'] <= timedelta(hours=48)
            return [item for item in inode_with_vote if item['is_active'] is True]
        finally:
            codec.getting_active_inodes = False

    async def get_inode_vote_ratio_by_address(self, address: str, check_pending_txs: bool = False):
        if self.gov is not None:
            return self.gov.inode_power(list(reversed(self._forms(address))), check_pending_txs)
        rows = self._ballot_rows('inodes_ballot', list(reversed(self._forms(address))), check_pending_txs,
                                 order=False)
        votes = [(vote, validator) for _, _, vote, validator, _ in rows]
        ratio = [(vote * await self.get_validators_stake(validator)) / 10 for vote, validator in votes]
        return round_up_decimal(sum(ratio, Decimal(0)))

    async def get_all_registered_inode_with_vote(self, check_pending_txs: bool = False):
        if self.gov is not None:
            return [{'wallet': a, 'power': p, 'registered_at': _dt(ts)}
                    for a, p, ts in self.gov.inodes_with_power(check_pending_txs)]
        return [{'wallet': address, 'power': await self.get_inode_vote_ratio_by_address(address, check_pending_txs),
                 'registered_at': ts} for address, ts in await self.get_all_registered_inode(check_pending_txs)]

    async def get_inode_count(self, check_pending_txs: bool = False):
        if self.gov is not None:
            return [{'count': self.gov.inode_count(check_pending_txs)}]
        rows = self._q('SELECT tx_hash, "index" FROM inode_registration_output')
        pend = self._pending_spent_set() if check_pending_txs else set()
        return [{'count': sum(1 for r in rows if (r[0], r[1]) not in pend)}]

    async def get_address_spendable_outputs_delta(self, address: str, block_no: int):
        point = string_to_point(address)
        forms = self._forms(address)
        ph = ','.join('?' * len(forms))
        if self.address_queries_from_index:
            from .utxo import STAKE_ANY
            hits = self._index_address_rows(address, STAKE_ANY, False)
            recent = set()
            hashes = sorted({h for h, _, _ in hits})
            for k in range(0, len(hashes), 500):
                chunk = hashes[k:k + 500]
                recent.update(r[0] for r in self._q(
                    f'SELECT t.tx_hash FROM transactions t WHERE t.tx_hash IN ({",".join("?" * len(chunk))}) '
                    f'AND (SELECT b.id FROM blocks b WHERE b.hash = t.block_hash) >= ?', (*chunk, block_no)))
            unspent = [TransactionInput(h, i, amount=Decimal(a) / SMALLEST, public_key=point)
                       for h, i, a in hits if h in recent]
        else:
            key = 'unspent_outputs.tx_hash'
            rows = self._q(f'SELECT unspent_outputs.tx_hash AS h, unspent_outputs."index" AS idx, '
                           f'{self._txq("outputs_amounts", key)} AS am FROM unspent_outputs '
                           f'WHERE unspent_outputs.address IN ({ph}) AND (SELECT b.id FROM blocks b WHERE b.hash = '
                           f'{self._txq("block_hash", key)}) >= ? ORDER BY unspent_outputs.rowid', (*forms, block_no))
            unspent = [TransactionInput(r['h'], r['idx'], amount=Decimal(_at(_arr(r['am']), r['idx'])) / SMALLEST,
                                        public_key=point) for r in rows]
        srows = self._txs_of_blocks([r[0] for r in self._q('SELECT hash FROM blocks WHERE id >= ?', (block_no,))],
                                    'tx_hex, inputs_addresses AS ia')
        spending = [await Transaction.from_hex(r['tx_hex'], False) for r in srows if address in _arr(r['ia'])][:block_no]
        return unspent, [i for tx in spending for i in tx.inputs]

    async def get_nice_transaction(self, tx_hash: str, address: str = None):
        """database.py:1606-1654."""
        is_confirm = True
        res = self._q1('SELECT t.tx_hex AS tx_hex, t.tx_hash AS tx_hash, t.block_hash AS block_hash, '
                       't.inputs_addresses AS inputs_addresses, b.id AS block_no, b.timestamp AS timestamp '
                       'FROM (SELECT tx_hex, tx_hash, block_hash, inputs_addresses FROM transactions WHERE tx_hash = ?) t '
                       'INNER JOIN blocks b ON t.block_hash = b.hash', (tx_hash,))
        if res is None:
            res = self._q1('SELECT tx_hex, tx_hash, inputs_addresses FROM pending_transactions WHERE tx_hash = ?',
                           (tx_hash,))
            is_confirm = False
        if res is None:
            return None
        res = dict(res)
        inputs_addresses = _arr(res['inputs_addresses'])
        ts = _dt(res['timestamp']) if res.get('timestamp') is not None else None
        tx = await Transaction.from_hex(res['tx_hex'], False)
        if isinstance(tx, CoinbaseTransaction):
            transaction = {'is_coinbase': True, 'hash': res['tx_hash'], 'block_hash': res.get('block_hash'),
                           'block_no': res.get('block_no'), 'datetime': ts}
        else:
            delta = None
            if address is not None:
                public_key = string_to_point(address)
                delta = 0
                for i, tx_input in enumerate(tx.inputs):
                    if string_to_point(inputs_addresses[i]) == public_key:
                        delta -= await tx_input.get_amount()
                for o in tx.outputs:
                    if o.public_key == public_key:
                        delta += o.amount
            transaction = {'is_coinbase': False, 'hash': res['tx_hash'], 'block_hash': res.get('block_hash'),
                           'block_no': res.get('block_no'), 'datetime': ts,
                           'message': tx.message.hex() if tx.message is not None else None,
                           'transaction_type': tx.transaction_type.name, 'is_confirm': is_confirm,
                           'inputs': [], 'delta': delta, 'fees': await tx.get_fees()}
            for i, tx_input in enumerate(tx.inputs):
                transaction['inputs'].append({'index': tx_input.index, 'tx_hash': tx_input.tx_hash,
                                              'address': _at(inputs_addresses, i),
                                              'amount': await tx_input.get_amount()})
        transaction['outputs'] = [{'address': o.address, 'amount': o.amount, 'type': o.transaction_type.name}
                                  for o in tx.outputs]
        return transaction


class _Rollback(Exception):
    pass


class UniqueViolationError(Exception):
    """Stand-in for asyncpg.UniqueViolationError (reference main.py:10,455)."""


class ForeignKeyViolationError(Exception):
    pass
