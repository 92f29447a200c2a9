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
        winner = ctx.allreduce_min(ctx.rank if local_header is not None else ctx.world)
        global_hits = ctx.allreduce_sum(len(res.nonces))
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
