"""Nonce-space data parallelism across GPUs (one rank per MI355X).

reference: miner.py:126-156 forks N CPU workers that stride one 2^32 nonce space and signal a find
by exiting. Here every rank owns a disjoint slice of the (timestamp, nonce) search space:

* rank r mines the header with timestamp ``ts0 - r`` (the nonce field is only 32 bits and one
  MI355X sweeps all 2^32 nonces in ~0.1 s, so a per-rank timestamp is the natural partition; it
  stays consensus-valid as long as ``ts0 - world`` > the previous block's timestamp,
  upow/manager.py:445-460);
* each step every rank sweeps ``count`` nonce words of its header on its GPU;
* the winner is agreed with ONE all-reduce(MIN) of ``rank if found else world`` and the winning
  108-byte header is broadcast from it over RCCL/xGMI; every rank re-checks it on the host.
"""
from __future__ import annotations

import hashlib
from dataclasses import dataclass
from typing import Callable, List, Optional

from ..models.block import PowTarget, header_prefix
from ..ops.pow import NONCE_SPACE, PowJob, search
from .dist import DistContext


@dataclass
class StepResult:
    winner: int                 # rank that found the chosen header (world if none)
    header: Optional[bytes]     # agreed header (None if no rank found one)
    local_hits: int             # exact-checked solutions found by this rank
    global_hits: int            # summed over ranks
    searched: int               # nonces searched by this rank


class DataParallelMiner:
    def __init__(self, ctx: DistContext, prev_hash: str, address: str, merkle_root: str, ts0: int, difficulty,
                 device: Optional[str] = None, search_fn: Callable = search, **search_kw):
        self.ctx = ctx
        self.target = PowTarget.from_difficulty(prev_hash, difficulty)
        self.ts = ts0 - ctx.rank
        self.job = PowJob.create(header_prefix(prev_hash, address, merkle_root, self.ts, difficulty), self.target)
        self.device = device
        self.search_fn = search_fn
        self.search_kw = search_kw
        self.next_word = 0

    def roll(self):
        """Move to the next timestamp slot once this rank exhausted its nonce space."""
        self.ts -= self.ctx.world
        # timestamp is the 4 bytes before difficulty(2)+nonce(4): bytes [-10:-6] of the full header
        hdr = bytearray(self.job.header)
        hdr[-10:-6] = int(self.ts).to_bytes(4, 'little')
        self.job = PowJob.create(bytes(hdr[:-4]), self.target)
        self.next_word = 0

    def step(self, count: int = NONCE_SPACE) -> StepResult:
        if self.next_word + count > NONCE_SPACE:
            self.roll()
        res = self.search_fn(self.job, self.next_word, count, device=self.device, **self.search_kw)
        local_header = self.job.header_with_nonce(res.nonces[0]) if res.nonces else None
        self.next_word += count
        if self.next_word >= NONCE_SPACE:
            self.roll()
        ctx = self.ctx
        # ONE all-reduce(SUM) per step: a found-flag slot per rank (the lowest set slot is the winner)
        # followed by this rank's solution count
        vec = [0] * (ctx.world + 1)
        if local_header is not None:
            vec[ctx.rank] = 1
        vec[ctx.world] = len(res.nonces)
        red = ctx.allreduce_sum_vec(vec)
        winner = next((r for r in range(ctx.world) if red[r]), ctx.world)
        global_hits = red[ctx.world]
        header = None
        if winner < ctx.world:
            header = ctx.broadcast_bytes(local_header if ctx.rank == winner else None, src=winner)
            if not self.target.check_hex(hashlib.sha256(header).hexdigest()):
                raise RuntimeError('broadcast header failed the PoW re-check')
        return StepResult(winner, header, len(res.nonces), global_hits, res.searched)

    def mine_until_found(self, count: int = 1 << 28, max_steps: int = 1 << 20) -> StepResult:
        for _ in range(max_steps):
            r = self.step(count)
            if r.header is not None:
                return r
        raise TimeoutError('no block found')


class ClusterMiner:
    """Real-network nonce-space DP (used by the miner CLI).

    Work units are header variants (timestamp in ``[ts_min, ts_max]`` newest first, then — only with
    ``extranonce=True`` — the unchecked u16 difficulty field). Every unit's 2^32 nonce words are
    split into ``world`` contiguous slices, one per rank; the ranks sweep their slice in ``chunk``
    pieces and after each piece agree on a winner (all-reduce MIN) and broadcast its header.
    """

    def __init__(self, ctx: DistContext, prev_hash: str, address: str, merkle_root: str, difficulty,
                 ts_max: int, ts_min: int, extranonce: bool = False, device: Optional[str] = None,
                 chunk: int = 1 << 28, search_fn: Callable = search, **search_kw):
        from ..models.block import header_prefix_raw
        self.ctx = ctx
        self.prev_hash, self.address, self.merkle = prev_hash, address, merkle_root
        self.target = PowTarget.from_difficulty(prev_hash, difficulty)
        self.dfield = int(float(difficulty) * 10)
        self.ts_max, self.ts_min = int(ts_max), int(ts_min)
        self.extranonce = extranonce
        self.device = device
        self.chunk = chunk
        self.search_fn = search_fn
        self.search_kw = search_kw
        self._hp = header_prefix_raw
        self.hashes = 0
        self.stopped = False  # the last mine() ended on should_stop (not on a swept space or a block)

    def units(self):
        for ts in range(self.ts_max, self.ts_min - 1, -1):
            yield ts, self.dfield
        if self.extranonce:
            for ts in range(self.ts_max, self.ts_min - 1, -1):
                for d in range(1 << 16):
                    if d != self.dfield:
                        yield ts, d

    def mine(self, should_stop: Callable[[], bool] = lambda: False) -> Optional[bytes]:
        ctx = self.ctx
        self.stopped = False
        slice_len = NONCE_SPACE // ctx.world
        lo = ctx.rank * slice_len
        hi = NONCE_SPACE if ctx.rank == ctx.world - 1 else lo + slice_len
        for ts, d in self.units():
            job = PowJob.create(self._hp(self.prev_hash, self.address, self.merkle, ts, d), self.target)
            pos = lo
            while True:
                n = min(self.chunk, hi - pos)
                nonces = []
                if n > 0:
                    res = self.search_fn(job, pos, n, device=self.device, **self.search_kw)
                    nonces = res.nonces
                    self.hashes += n
                    pos += n
                local = job.header_with_nonce(nonces[0]) if nonces else None
                # one fused all-reduce(MIN) per chunk: [lowest finder rank | world, any rank asked to
                # stop -> 0, every rank's slice exhausted -> 1]
                winner, keep_going, all_done = ctx.allreduce_min_vec(
                    [ctx.rank if local is not None else ctx.world, 0 if should_stop() else 1, 1 if pos >= hi else 0])
                if winner < ctx.world:
                    header = ctx.broadcast_bytes(local if ctx.rank == winner else None, src=winner)
                    if not self.target.check_hex(hashlib.sha256(header).hexdigest()):
                        raise RuntimeError('broadcast header failed the PoW re-check')
                    return header
                if keep_going == 0:
                    self.stopped = True
                    return None
                if all_done == 1:
                    break
        return None
