"""UTXO-index snapshots: checkpoint / resume of the HBM outpoint table (SURVEY.md §5 "Checkpoint / resume").

The reference keeps all state in PostgreSQL and has no snapshots: a restart re-reads the tables, a
damaged UTXO set is rebuilt by replaying every transaction (create_unspent_outputs.py:9-45). Here the
SQLite ledger stays authoritative and durable; what a restart has to rebuild is the GPU index
(every row of the seven output tables → HBM). A snapshot is the index itself:

    line 1   JSON header {magic, version, height, tip_hash, count, utxo_hash, payload_sha256}
    then     count × 40-byte records {txid 32 B, u32 index, u32 table tag}, canonical (txid, index) order
    then     count × 80-byte payloads {u64 amount, u32 address length, pad, address[64]} (same order)

written atomically (tmp file + rename) at the tip. On start, :func:`try_restore` loads it only when
the snapshot's (height, tip hash) equals the ledger's tip, the payload checksum matches and the
per-table row counts match the SQL tables; the index's K12 hash (``UtxoIndex.set_hash``) must equal
the header's. Anything else — another chain, a partial write, a stale height — falls back to the
full rebuild from SQL, so a bad snapshot can cost time but never correctness.
"""
from __future__ import annotations

import hashlib
import json
import os
from typing import Optional

import numpy as np

from ..utils.logger import get_logger
from .utxo import PAYLOAD_DTYPE, TAG_BY_TABLE

logger = get_logger(__name__)
MAGIC, VERSION = 'upow-utxo-snapshot', 3  # v3: payload flags (is_stake)
FILE_NAME = 'utxo_snapshot.bin'


def default_path(db) -> Optional[str]:
    if db.path == ':memory:':
        return None
    return os.environ.get('UPOW_SNAPSHOT_PATH') or os.path.join(os.path.dirname(os.path.abspath(db.path)), FILE_NAME)


def _tip(db):
    row = db._last_block_row()  # the chain-tip cache: committed blocks, materialised or not
    return (int(row['id']), row['hash']) if row else (0, '')


_POOL = None
_pending: dict = {}  # snapshot path -> the background save in flight (a Future)


def save(db, path: Optional[str] = None, background: bool = False):
    """Write the index at the current tip. Returns the header; with ``background`` the Future of it (None when
    skipped).

    Only the dump of the index (one D2H copy on the GPU backend) happens under the ledger's lock, at the tip
    it is taken for; the canonical sort, the K12 hash of those very records, the checksum and the file write
    follow on the caller's thread or, with ``background``, on a snapshot thread, so the block path does not
    wait for them (a 5 M-outpoint index is ~600 MB to sort, hash and write). A background save finding the
    previous one still running is skipped: the next period takes it."""
    global _POOL
    path = path or default_path(db)
    if path is None:
        raise ValueError('in-memory ledger: give an explicit snapshot path')
    prev = _pending.get(path)
    if background and prev is not None and not prev.done():
        return None
    with db.lock:
        height, tip = _tip(db)
        recs, pay = db.utxo.records_payload(sort=False)
    if not background:
        return _write(path, height, tip, recs, pay)
    if _POOL is None:
        from concurrent.futures import ThreadPoolExecutor
        _POOL = ThreadPoolExecutor(max_workers=1, thread_name_prefix='upow-snapshot')
    fut = _pending[path] = _POOL.submit(_write, path, height, tip, recs, pay)  # fresh arrays of the dump: no copy
    return fut


def wait_pending(timeout: Optional[float] = None, path: Optional[str] = None):
    """The last background save (of ``path``, or of any ledger), finished: its header, or None when there was
    none."""
    futs = [_pending[path]] if path in _pending else ([] if path else list(_pending.values()))
    out = None
    for f in futs:
        out = f.result(timeout)
    return out


def _k12(recs: np.ndarray) -> str:
    """K12 (reference database.py:827-830) of canonically ordered records: SHA-256 over (txid || index byte)
    of the unspent_outputs entries — what ``UtxoIndex.set_hash`` gives for the same index."""
    tags = recs[:, 36:40].copy().view(np.uint32).ravel()
    m = recs[tags == TAG_BY_TABLE['unspent_outputs']]
    return hashlib.sha256(np.ascontiguousarray(np.concatenate([m[:, :32], m[:, 32:33]], axis=1)).tobytes()).hexdigest()


def _write(path: str, height: int, tip: str, recs: np.ndarray, pay: np.ndarray) -> dict:
    from .utxo import sort_order
    order = sort_order(np.ascontiguousarray(recs))
    recs, pay = np.ascontiguousarray(recs[order]), np.ascontiguousarray(pay[order])
    payload = recs.tobytes() + pay.tobytes()
    header = {'magic': MAGIC, 'version': VERSION, 'height': height, 'tip_hash': tip, 'count': int(len(recs)),
              'utxo_hash': _k12(recs), 'payload_sha256': hashlib.sha256(payload).hexdigest()}
    tmp = path + '.tmp'
    with open(tmp, 'wb') as f:
        f.write(json.dumps(header, separators=(',', ':')).encode() + b'\n')
        f.write(payload)
        f.flush()
        os.fsync(f.fileno())
    os.replace(tmp, path)
    return header


def read(path: str):
    """-> (header, records, payloads) after checking the checksum; raises ValueError on a bad file."""
    with open(path, 'rb') as f:
        header = json.loads(f.readline().decode())
        payload = f.read()
    if header.get('magic') != MAGIC or header.get('version') != VERSION:
        raise ValueError('not a uPow UTXO snapshot')
    n = header['count']
    if len(payload) != 120 * n or hashlib.sha256(payload).hexdigest() != header['payload_sha256']:
        raise ValueError('snapshot payload truncated or corrupted')
    recs = np.frombuffer(payload[:40 * n], dtype=np.uint8).reshape(-1, 40)
    return header, recs, np.frombuffer(payload[40 * n:], dtype=PAYLOAD_DTYPE)


def try_restore(db, path: Optional[str] = None) -> bool:
    """Load the snapshot into ``db.utxo`` if it matches the ledger tip; False (index untouched) otherwise."""
    path = path or default_path(db)
    if not path or not os.path.exists(path):
        return False
    try:
        header, recs, pay = read(path)
    except (ValueError, OSError, json.JSONDecodeError) as e:
        logger.warning(f'ignoring UTXO snapshot {path}: {e}')
        return False
    if (header['height'], header['tip_hash']) != _tip(db):
        logger.info(f'UTXO snapshot at height {header["height"]} does not match the ledger tip; rebuilding')
        return False
    tags = recs[:, 36:40].copy().view(np.uint32).ravel()
    for table, tag in TAG_BY_TABLE.items():
        if int((tags == tag).sum()) != int(db._q1(f'SELECT COUNT(*) FROM {table}')[0]):
            logger.warning(f'UTXO snapshot row count differs from table {table}; rebuilding')
            return False
    db.utxo.reset_records(recs, pay)
    if db.utxo.set_hash(TAG_BY_TABLE['unspent_outputs']) != header['utxo_hash']:
        logger.warning('UTXO snapshot hash mismatch after load; rebuilding')
        return False
    return True


def verify(db) -> dict:
    """Full audit: index vs SQL (K12 hash of the unspent table + per-table outpoint sets)."""
    sql_hash = db._q('SELECT tx_hash, "index" FROM unspent_outputs ORDER BY tx_hash, "index"')
    want = hashlib.sha256(b''.join(bytes.fromhex(r[0]) + bytes([r[1]]) for r in sql_hash)).hexdigest()
    got = db.utxo.set_hash(TAG_BY_TABLE['unspent_outputs'])
    recs = db.utxo.records()
    idx = recs[:, 32:36].copy().view(np.uint32).ravel()
    tags = recs[:, 36:40].copy().view(np.uint32).ravel()
    index_sets = {}
    for n in range(len(recs)):
        index_sets.setdefault(int(tags[n]), set()).add((bytes(recs[n, :32]).hex(), int(idx[n])))
    mismatched = [t for t, tag in TAG_BY_TABLE.items()
                  if index_sets.get(tag, set()) != {(r[0], int(r[1])) for r in db._q(f'SELECT tx_hash, "index" FROM {t}')}]
    # payloads: amount + address bytes of every entry against the creating tx's JSON columns
    from .database import _addr_bytes
    recs_p, pay = db.utxo.records_payload()
    idx_p = recs_p[:, 32:36].copy().view(np.uint32).ravel()
    bad_payload = 0
    for n in range(len(recs_p)):
        h, i = bytes(recs_p[n, :32]).hex(), int(idx_p[n])
        row = db._q1('SELECT json_extract(outputs_amounts, ?), json_extract(outputs_addresses, ?) FROM transactions '
                     'WHERE tx_hash = ?', (f'$[{i}]', f'$[{i}]', h))
        want_addr = _addr_bytes(row[1]) if row else None
        if row is None or row[0] is None or want_addr is None:
            bad_payload += int(pay['len'][n] != 0)
            continue
        ln = int(pay['len'][n])
        bad_payload += int(int(pay['amount'][n]) != int(row[0]) or bytes(pay['addr'][n][:ln]) != want_addr)
    return {'ok': want == got and not mismatched and bad_payload == 0, 'sql_hash': want, 'index_hash': got,
            'mismatched_tables': mismatched, 'payload_mismatches': bad_payload, 'entries': int(len(recs))}


__all__ = ['save', 'wait_pending', 'read', 'try_restore', 'verify', 'default_path']
