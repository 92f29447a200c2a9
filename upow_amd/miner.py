"""GPU miner CLI — same argv as the reference ``miner.py <address> [workers] [node_url]``.

reference: miner.py:126-156 (fetch /get_mining_info, fork N CPU workers striding the nonce space,
POST /push_block, refresh every <= 100 s).

MI355X version:
* one process per GPU. Single GPU: ``python -m upow_amd.miner ADDRESS``. A node with 8 GPUs:
  ``torchrun --nproc-per-node 8 -m upow_amd.miner ADDRESS`` — rank 0 fetches the job and broadcasts it
  over RCCL, every rank sweeps its slice of the nonce space on its GPU (``csrc/pow_search.hip``), the
  winner's header is agreed by all-reduce and broadcast, and rank 0 submits it;
* ``workers`` is accepted for argv compatibility and ignored on GPUs (the kernel already runs one
  nonce per lane); on a CPU-only host it is the host-search thread count;
* the job is refreshed every ``--refresh`` seconds (default 90, like the reference's window), and
  earlier as soon as the node's tip moves: rank 0 polls ``/get_mining_info`` every ``--poll`` seconds
  (default 3 s, inside the endpoint's 30/min limit) and the ranks agree to drop the stale job — one
  GPU sweeps a timestamp's whole 2^32 nonces in ~0.12 s, so mining on an old tip for up to 90 s
  would waste almost all of the work after a competing block arrives;
* a job whose whole space was swept without a block (the header is fixed but for the timestamp, which
  may not run ahead of the clock, and the nonce) is followed by a FRESH space, never the same one again
  (:class:`JobPlanner`): only the timestamps not yet swept, and once the tip is ``--trim-after`` seconds
  old (default 8), the template minus its last transaction (the merkle root is over the sorted hash set,
  so only a different SET gives a new root; the dropped transactions, at most half the template, wait
  one block). With an unchanged
  mempool a re-fetched job used to re-sweep the timestamps it had already failed on, leaving ~2^32 fresh
  nonces per wall second: at difficulty 9 the last block of a soak took 13-40 s instead of ~2 s
  (profiles/r4/node_soak_inclusion_tail_r4ac.json). Dropping at once instead would starve the newest
  transaction: right after a block the window is one or two timestamps, which a GPU sweeps in 0.2 s.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

import httpx

from .constants import GENESIS_PREV_HASH
from .models.block import miner_merkle_root
from .utils.codec import timestamp


def fetch_mining_info(node_url: str) -> dict:
    r = httpx.get(node_url + 'get_mining_info', timeout=5)
    return r.json()['result']


class TipWatcher:
    """Background poll of the node's tip (rank 0 only). ``moved(prev)`` is True once the node reports
    a last block whose hash differs from the job's previous hash."""

    def __init__(self, node_url: str, interval: float, fetch=fetch_mining_info):
        self.node_url, self.interval, self.fetch = node_url, interval, fetch
        self.tip = None
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, name='upow-tip-watch', daemon=True)
        self._t.start()

    def _run(self):
        while not self._stop.wait(self.interval):
            try:
                self.tip = self.fetch(self.node_url)['last_block'].get('hash', GENESIS_PREV_HASH)
            except Exception:
                pass

    def moved(self, prev: str) -> bool:
        return self.tip is not None and self.tip != prev

    def close(self):
        self._stop.set()
        self._t.join(timeout=5)


class JobPlanner:
    """Rank 0's choice of (transactions, lowest timestamp) for the next job, so that a job never repeats
    a search space an earlier job of the same template swept in full."""

    def __init__(self, trim_after_s: float = 8.0):
        self.trim_after_s = trim_after_s
        self.key = None
        self.trim = 0  # trailing template transactions left out
        self.swept_to = None  # highest timestamp swept with the current transaction set
        self.exhausted = False
        self.last_ts_max = None

    def plan(self, job: dict, now: int):
        last = job['last_block']
        hashes = job['pending_transactions_hashes']
        key = (last.get('hash', GENESIS_PREV_HASH), hash(tuple(hashes)))
        if key != self.key:
            self.key, self.trim, self.swept_to, self.exhausted = key, 0, None, False
        elif self.exhausted:
            old = now - last.get('timestamp', now) >= self.trim_after_s
            # at most half the template is held back: a one-transaction template is never mined empty
            if old and self.trim < len(hashes) // 2:
                self.trim += 1  # a new merkle root: the whole timestamp window is fresh again
                self.swept_to = None
            else:
                self.swept_to = self.last_ts_max  # only the timestamps the clock has added since
        self.exhausted = False
        use = hashes[:len(hashes) - self.trim] if self.trim else hashes
        ts_min = last.get('timestamp', now - 60) + 1
        if self.swept_to is not None:
            ts_min = max(ts_min, self.swept_to + 1)
        return use, ts_min

    def finished(self, exhausted: bool, ts_max: int):
        """The job ended: ``exhausted`` = its whole space was swept (not stopped, no block found)."""
        self.exhausted, self.last_ts_max = exhausted, ts_max


def submit(node_url: str, header: bytes, hashes, block_no: int) -> dict:
    r = httpx.post(node_url + 'push_block', json={'block_content': header.hex(), 'txs': hashes, 'block_no': block_no},
                   timeout=20 + int((len(hashes) or 1) / 3))
    return r.json()


def main(argv=None):
    ap = argparse.ArgumentParser(description='uPow MI355X miner')
    ap.add_argument('address')
    ap.add_argument('workers', nargs='?', type=int, default=1)
    ap.add_argument('node_url', nargs='?', default=None)
    ap.add_argument('--device', choices=['gpu', 'cpu'], default=None)
    ap.add_argument('--refresh', type=float, default=90.0)
    ap.add_argument('--trim-after', type=float, default=8.0,
                    help='tip age (s) after which a swept-out template is retried without its last transaction')
    ap.add_argument('--poll', type=float, default=3.0, help='tip poll period in seconds (0 = off)')
    ap.add_argument('--chunk', type=int, default=1 << 28)
    ap.add_argument('--extranonce', action='store_true',
                    help='also vary the (unchecked) header difficulty field once timestamps are exhausted')
    ap.add_argument('--blocks', type=int, default=0, help='stop after this many accepted blocks (0 = forever)')
    ap.add_argument('--dispatch-log2', type=int, default=int(os.environ.get('UPOW_POW_DISPATCH_LOG2', '23')),
                    help='nonces per GPU dispatch (log2). 23 (~0.25 ms) lets a node sharing the GPU run its block '
                         'kernels between dispatches (its GPU stages ~1.2x their idle time) at a ~2%% hashrate '
                         'cost; 28 for a dedicated GPU (docs/PERF.md §3)')
    a = ap.parse_args(argv)
    os.environ.setdefault('UPOW_FILE_LOG', '1')  # reference: logs/app.log always (my_logger.py:17-53)
    os.environ['UPOW_POW_DISPATCH_LOG2'] = str(a.dispatch_log2)
    from . import config
    node_url = (a.node_url or os.environ.get('UPOW_MINING_NODE_URL') or 'http://localhost:3006/').strip('/') + '/'

    from .ops.native import gpu_available, lib
    lib()
    from .parallel.dist import init_from_env, shutdown
    from .parallel.miner_dp import ClusterMiner
    ctx = init_from_env(want_gpu=a.device != 'cpu')
    device = a.device or ('gpu' if gpu_available() else 'cpu')
    kw = {} if device == 'gpu' else {'threads': max(1, a.workers)}
    accepted = 0
    watcher = TipWatcher(node_url, a.poll) if (ctx.is_main and a.poll > 0) else None
    planner = JobPlanner(a.trim_after)
    try:
        while True:
            job = None
            if ctx.is_main:
                while job is None:
                    try:
                        job = fetch_mining_info(node_url)
                    except Exception as e:
                        print(e, flush=True)
                        time.sleep(1)
                job['pending_transactions_hashes'], job['_ts_min'] = planner.plan(job, timestamp())
            job = json.loads(ctx.broadcast_bytes(json.dumps(job).encode() if ctx.is_main else None, src=0,
                                                 max_len=0).decode())
            last = job['last_block']
            prev = last.get('hash', GENESIS_PREV_HASH)
            block_no = last.get('id', 0) + 1
            hashes = job['pending_transactions_hashes']
            merkle = miner_merkle_root(hashes)
            now = timestamp()
            ts_min = job['_ts_min']
            if ts_min > now:  # the previous block (or the last swept timestamp) is from this very second
                time.sleep(ts_min - now)
                now = timestamp()
            if ctx.is_main:
                print(f"difficulty: {job['difficulty']}\nblock number: {last.get('id', 0)}\n"
                      f"Confirming {len(hashes)} transactions", flush=True)
            miner = ClusterMiner(ctx, prev, a.address, merkle, job['difficulty'], ts_max=now, ts_min=ts_min,
                                 extranonce=a.extranonce, device=device, chunk=a.chunk, **kw)
            t0 = time.time()
            if watcher is not None:
                watcher.tip = None  # only polls made during this job count
            header = miner.mine(should_stop=lambda: time.time() - t0 > a.refresh or
                                (watcher is not None and watcher.moved(prev)))
            planner.finished(header is None and not miner.stopped, now)
            dt = max(time.time() - t0, 1e-9)
            per_rank = [float(x) / dt for x in ctx.all_gather_bytes(str(miner.hashes).encode())]
            rate = sum(per_rank)
            if ctx.is_main:
                print(f'{rate / 1e6:.1f} MH/s ({ctx.world} x {device})', flush=True)
                if ctx.world > 1 or ctx.forced:
                    print('per-rank MH/s: ' + json.dumps([round(r / 1e6, 1) for r in per_rank]), flush=True)
                if header is not None:
                    print(header.hex())
                    print(','.join(hashes))
                    try:
                        result = submit(node_url, header, hashes, block_no)
                    except Exception as e:
                        result = {'ok': False, 'error': str(e)}
                    print(result, flush=True)
                    if result.get('ok'):
                        print('BLOCK MINED\n', flush=True)
                        accepted += 1
            accepted = ctx.allreduce_sum(accepted if ctx.is_main else 0)
            if a.blocks and accepted >= a.blocks:
                break
    finally:
        if watcher is not None:
            watcher.close()
        shutdown(ctx)


if __name__ == '__main__':
    sys.exit(main())
