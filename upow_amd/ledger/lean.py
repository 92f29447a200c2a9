"""Lean cluster followers: HBM replicas that keep no SQL materialisation (SURVEY.md §2.6 "State replication").

The reference keeps ONE store (one asyncpg pool on one PostgreSQL, upow/database.py:36-43). A G-GPU cluster
node (parallel/cluster.py) replicates the ledger state in every GPU's HBM so every replica can validate
and vote on every block; but only the leader (rank 0) serves SQL-backed HTTP queries. A follower that ran
the whole host block path — apply strings, statement encoding, a journal record of ~8 MB per 2 MB block
and ten SQLite materialiser threads — would spend the host CPU the leader needs, and on one 8-GPU host
those seven copies share the same cores. So a follower is *lean*:

  keeps      the HBM UTXO index (and its payloads), the governance index, the mempool index (its pending
             rows stay journaled: they are small), the chain-tip header rows (difficulty retargets and the
             genesis rule read them), and an *op log*: the leader's state-changing ops exactly as they
             arrived (raw frames, ~the block's raw size) each followed by a tip marker (height, hash);
  skips      apply strings, statement encoding, the block's journal record and every SQL materialiser
             write of it, the UTXO snapshot cadence and the K12 log line (the leader logs it).

The SQL files of a lean follower stay at the height where it last materialised. ``materialise`` brings them
to the tip: the HBM and governance indexes are rebuilt from that SQL state and every logged op is applied
again through the full block path (full validation, full ledger writes), up to the tip the follower had
reached; then the log is cleared. It runs
  * when a follower restarts (``node/__main__._follow``) — after a crash the ops past the last tip marker are
    dropped; the leader's resync re-sends whatever the follower is missing,
  * when a follower's ledger is opened as a standalone node's (promotion, ``node/main.py`` startup) or by
    ``python -m upow_amd.tools materialise``,
  * online, before a follower runs anything that needs its SQL tables: a rollback or chain deletion, a fork
    window, a deep status audit, and a block the native path hands to the object path (that path resolves
    inputs from the SQL transactions table). The block being validated then continues in full mode.

Size: the log holds the raw ops since the last materialisation, about the raw size of those blocks (a full
replica's SQL files hold three to four times that); a long-running follower's restart replays all of it, so an
operator can materialise a follower at a quiet time with ``python -m upow_amd.tools materialise``.

Durability: the leader is the durable copy. The op log is written (page cache) before an op is applied and
fdatasync'd at status / quit / every ``SYNC_BYTES``; a torn tail is dropped on open (record lengths, and a
CRC over each record's header and the first and last 4 KB of its body). A replayed op is validated in full
(PoW, merkle root, signatures), so a damaged body stops the replay instead of entering the ledger.
"""
from __future__ import annotations

import os
import struct
import zlib
from typing import List, Optional, Tuple

from ..utils.logger import get_logger

logger = get_logger(__name__)

MAGIC = 0x314C5055  # "UPL1"
KIND_OP, KIND_TIP = 1, 2
_HDR = struct.Struct('<IIIIqQ')  # magic, kind, crc, reserved, aux, body length
_EDGE = 4096
SYNC_BYTES = int(os.environ.get('UPOW_LEAN_SYNC_MB', '64')) << 20


def enabled() -> bool:
    """Followers run lean unless ``UPOW_CLUSTER_LEAN=0`` (the full replica of rounds 1-5)."""
    return os.environ.get('UPOW_CLUSTER_LEAN', '1') != '0'


def _crc(kind: int, aux: int, n: int, head, tail) -> int:
    """CRC-32 of a record's header fields and the first and last 4 KB of its body (``head`` =
    body[:4096], ``tail`` = body[max(4096, n - 4096):]): a torn or zero-filled tail fails it, and the body's
    middle is checked where it matters, by the full validation of a replayed block."""
    c = zlib.crc32(struct.pack('<IqQ', kind, aux, n))
    return zlib.crc32(tail, zlib.crc32(head, c))


def _edges(mv, n: int):
    return mv[:_EDGE], mv[max(_EDGE, n - _EDGE):n]


class OpLog:
    """Append-only log of (op frame, tip marker) records next to the ledger (``<ledger>.oplog``)."""

    def __init__(self, path: str):
        self.path = path
        self.fd = os.open(path, os.O_RDWR | os.O_CREAT | os.O_APPEND | os.O_CLOEXEC, 0o644)
        self.records: List[Tuple[int, int, int, int]] = []  # (kind, aux, body offset, body length)
        self.size = 0
        self.unsynced = 0
        self.appended_bytes = 0
        self._scan()

    def _scan(self):
        end = os.fstat(self.fd).st_size
        at = 0
        while at + _HDR.size <= end:
            magic, kind, crc, _, aux, n = _HDR.unpack(os.pread(self.fd, _HDR.size, at))
            if magic != MAGIC or kind not in (KIND_OP, KIND_TIP) or at + _HDR.size + n > end:
                break
            t0 = max(_EDGE, n - _EDGE)
            head = os.pread(self.fd, min(n, _EDGE), at + _HDR.size)
            tail = os.pread(self.fd, n - t0, at + _HDR.size + t0) if n > t0 else b''
            if _crc(kind, aux, n, head, tail) != crc:
                break
            self.records.append((kind, aux, at + _HDR.size, n))
            at += _HDR.size + n
        if at != end:
            logger.warning(f'op log {self.path}: dropping a torn tail of {end - at} bytes')
            os.ftruncate(self.fd, at)
        self.size = at

    def append(self, kind: int, aux: int, body) -> None:
        mv = memoryview(body).cast('B')
        hdr = _HDR.pack(MAGIC, kind, _crc(kind, int(aux), len(mv), *_edges(mv, len(mv))), 0, int(aux), len(mv))
        os.writev(self.fd, [hdr, mv])
        self.records.append((kind, int(aux), self.size + _HDR.size, len(mv)))
        self.size += _HDR.size + len(mv)
        self.unsynced += _HDR.size + len(mv)
        self.appended_bytes += _HDR.size + len(mv)
        if self.unsynced >= SYNC_BYTES:
            self.sync()

    def op(self, raw) -> None:
        self.append(KIND_OP, 0, raw)

    def tip(self, height: int, tip_hash: Optional[str]) -> None:
        self.append(KIND_TIP, height, bytes.fromhex(tip_hash) if tip_hash else b'')

    def sync(self):
        if self.unsynced:
            os.fdatasync(self.fd)
            self.unsynced = 0

    def read(self, off: int, n: int) -> bytes:
        return os.pread(self.fd, n, off)

    def last_tip(self) -> Optional[Tuple[int, str]]:
        for kind, aux, off, n in reversed(self.records):
            if kind == KIND_TIP:
                return aux, self.read(off, n).hex()
        return None

    def ops(self, start_height: int):
        """The logged ops that moved the tip, one at a time (a log holds a long run of blocks): an op whose
        tip marker equals the previous one changed nothing (a rejected block) and is skipped; an op with no
        marker after it (the one being applied, online) is yielded."""
        prev = start_height
        recs = self.records
        for k, (kind, _, off, n) in enumerate(recs):
            if kind != KIND_OP:
                if kind == KIND_TIP:
                    prev = recs[k][1]
                continue
            nxt = recs[k + 1] if k + 1 < len(recs) else None  # every record is an op or a tip marker
            if nxt is not None and nxt[0] == KIND_TIP and nxt[1] == prev:
                continue
            yield self.read(off, n)

    def __len__(self) -> int:
        return len(self.records)

    def clear(self):
        os.ftruncate(self.fd, 0)
        os.fsync(self.fd)
        self.records.clear()
        self.size = self.unsynced = 0

    def close(self):
        if self.fd >= 0:
            self.sync()
            os.close(self.fd)
            self.fd = -1


def log_path(db) -> str:
    return db.file + '.oplog'


def open_log(db) -> OpLog:
    if db.lean_log is None:
        db.lean_log = OpLog(log_path(db))
    return db.lean_log


def pending(db) -> bool:
    """Does this ledger have logged ops its SQL tables do not hold yet?"""
    if db.lean_log is not None:
        return len(db.lean_log) > 0
    p = log_path(db)
    return os.path.exists(p) and os.path.getsize(p) > 0


def parse_frame(raw: bytes) -> dict:
    """A cluster op frame (parallel/cluster.py ``Cluster.send``): u32 header length, JSON header, payload."""
    import json
    n = int.from_bytes(raw[:4], 'little')
    msg = json.loads(raw[4:4 + n].decode())
    msg['_payload'] = raw[4 + n:]
    return msg


async def apply_op(db, msg: dict, stop_at: Optional[int] = None) -> None:
    """One state-changing op ('block', 'page', 'replay_block') on the full block path; blocks above height
    ``stop_at`` are not applied (a replay ends where the follower had stopped)."""
    from ..models.transaction import Transaction
    from ..parallel.cluster import Cluster, _split_coinbase, unpack_txs
    from . import fastpath, pagesync
    op = msg['op']
    tip = db._tip_id()
    if stop_at is not None and tip >= stop_at:
        return
    if op == 'block':
        cb = await Transaction.from_hex(msg['cb']) if msg.get('cb') else None
        await fastpath.create_block_from_hex(msg['content'], unpack_txs(msg['_payload']), coinbase=cb, mirror=False)
    elif op == 'replay_block':
        if int(msg['h']) <= tip:
            return
        hexes, cb = await _split_coinbase(unpack_txs(msg['_payload']))
        if cb is None:
            raise RuntimeError(f'block {msg["h"]} has no coinbase transaction')
        if not await fastpath.create_block_from_hex(msg['content'], hexes, coinbase=cb,
                                                    last_block=await db.get_last_block(), mirror=False):
            raise RuntimeError(f'block {msg["h"]} rejected')
    elif op == 'page':
        blocks = [b for b in Cluster.unpack_page(msg)
                  if int(b['block']['id']) > tip and (stop_at is None or int(b['block']['id']) <= stop_at)]
        if blocks:
            await pagesync.create_blocks(blocks, mirror=False)
    else:  # pragma: no cover
        raise RuntimeError(f'op {op} is not a logged ledger op')


async def materialise(db, online: bool = False) -> int:
    """Bring a lean ledger's SQL tables (and the indexes built from them) to the follower's tip; see the
    module docstring. ``online``: the follower is running (its in-memory tip is the target, the op being
    applied is already logged); otherwise the last tip marker of the log is. Returns the blocks replayed."""
    from ..parallel import cluster
    log = open_log(db)
    if online:
        target = (db._tip_id(), db.block_hash_at(db._tip_id()))
    else:
        target = log.last_tip()
    was_lean = db.lean
    if not len(log) or target is None:
        if not online and len(log):
            logger.info(f'op log {log.path}: no tip marker, nothing to replay')
        log.clear()
        if was_lean:
            db.leave_lean()
        return 0
    c = cluster.get()
    replaying = c.replaying if c is not None else None
    if c is not None:
        c.replaying = True  # no commit votes, no sharded verify: this replica alone replays its own history
    try:
        if was_lean:
            db.leave_lean()  # back to the SQL state (a restarted ledger is there already)
        start = db._tip_id()
        logger.info(f'materialising the op log ({len(log)} records) into the SQL ledger: height {start} -> '
                    f'{target[0]}')
        for raw in log.ops(start):
            if db._tip_id() >= target[0]:
                break
            await apply_op(db, parse_frame(raw), stop_at=target[0])
        got = (db._tip_id(), db.block_hash_at(db._tip_id()))
        if got != tuple(target):
            raise RuntimeError(f'op log replay from height {start} reached {got}, expected {tuple(target)}: the '
                               f'lean replica and its SQL tables disagree')
        db.wait_durable(force=True)
        log.clear()
        return got[0] - start
    finally:
        if c is not None:
            c.replaying = replaying


__all__ = ['OpLog', 'enabled', 'open_log', 'pending', 'parse_frame', 'apply_op', 'materialise', 'log_path']
