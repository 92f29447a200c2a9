#!/usr/bin/env python3
"""Headline benchmark: whole-node SHA-256 PoW hashrate (MH/s) on N MI355X (BASELINE.json metric).

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N>1 it is launched by
``torch.distributed.run`` with one rank per GPU (RCCL over xGMI). One *step* = every rank sweeps the
full 2^32 nonce space of its own synthetic v2 header (108 B, difficulty 6.3, per-rank timestamp:
nonce-space data parallelism, upow_amd/parallel/miner_dp.py), exact-checks every candidate on the
host, then the ranks agree on a winner with an all-reduce(MIN) and broadcast the winning header over
RCCL; every rank re-verifies it. Nothing is skipped: every nonce of every step is hashed.

Weak scaling: per-GPU work (2^32 nonces/step) is fixed as N grows; ``value`` is the aggregate MH/s
of all N GPUs. ``vs_baseline`` divides by BASELINE.md's 0.99 MH/s (the reference miner.py inner loop,
one process, measured in the survey sandbox — the reference publishes no number).

The default (mine) run then also measures the second BASELINE metric in the same process on every
rank — tx-verify/s over 2 MB blocks (8,300 signed txs each) through the native push_block path into a
file-backed ledger — and reports it as extra keys (``verify_tx_per_s`` aggregated over ranks,
``ecdsa_sig_per_s``, per-block commit latency); ``--verify-steps 0`` skips it. Then chain sync:
``sync_tx_per_s`` of one chain of 200-tx blocks replayed from /get_blocks pages (page-batched,
ledger/pagesync.py); with N ranks the N GPUs form one cluster node syncing that chain (``--sync-steps 0``
skips it).
``--mode verify`` runs that measurement alone (default 10 blocks); ``--mode sync`` the chain-sync
throughput of the same blocks replayed from a ``/get_blocks`` page.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

BASELINE_MHS = 0.99  # miner.py-style loop, 1 process (measured; nothing published)


def _synthetic_job(seed: int = 2026):
    import random

    from upow_amd.utils import p256
    from upow_amd.utils.codec import AddressFormat, point_to_string
    rng = random.Random(seed)
    prev_hash = hashlib.sha256(rng.randbytes(32)).hexdigest()
    d = rng.randrange(1, p256.N)
    address = point_to_string(p256.get_public_key(d), AddressFormat.COMPRESSED)
    tx_hashes = sorted(hashlib.sha256(rng.randbytes(250)).hexdigest() for _ in range(10))
    merkle = hashlib.sha256(b''.join(bytes.fromhex(h) for h in tx_hashes)).hexdigest()
    return prev_hash, address, merkle


def bench_mine(args, ctx):
    from upow_amd.ops.native import gpu_available
    from upow_amd.ops.pow import NONCE_SPACE
    from upow_amd.parallel.miner_dp import DataParallelMiner

    device = 'gpu' if gpu_available() else 'cpu'
    count = args.nonces if args.nonces else (NONCE_SPACE if device == 'gpu' else 1 << 22)
    prev_hash, address, merkle = _synthetic_job()
    ts0 = 1_790_000_000
    miner = DataParallelMiner(ctx, prev_hash, address, merkle, ts0, args.difficulty, device=device,
                              variant=args.variant)
    for _ in range(args.warmup):
        miner.step(count)
    ctx.barrier()
    ctx.synchronize()
    t0 = time.perf_counter()
    hits = 0
    winners = 0
    for _ in range(args.steps):
        r = miner.step(count)
        hits += r.global_hits
        winners += r.header is not None
    ctx.synchronize()
    ctx.barrier()
    dt = time.perf_counter() - t0
    dt = ctx.allreduce_max_f(dt)
    total_hashes = count * args.steps * ctx.world
    mhs = total_hashes / dt / 1e6
    return {
        'metric': 'sha256_pow_hashrate_MH/s',
        'value': round(mhs, 3),
        'unit': 'MH/s',
        'n_gpus': ctx.world if device == 'gpu' else 0,
        'world': ctx.world,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': round(dt * 1000 / max(1, args.steps), 3),
        'higher_is_better': True,
        'scaling': 'weak',
        'vs_baseline': round(mhs / BASELINE_MHS, 1),
        'dtype': 'uint32',
        'data': 'synthetic (random prev-hash, random P-256 miner key, 10 random tx hashes)',
        'config': {
            'model': 'upow v2 block header PoW (108 B, single SHA-256, nibble-prefix target)',
            'difficulty': float(args.difficulty),
            'global_batch': total_hashes // max(1, args.steps),
            'seq_len': 108,
            'parallelism': f'dp{ctx.world}',
            'nonces_per_rank_step': count,
            'device': device,
            'kernel_variant': args.variant,
        },
        'solutions_found': hits,
        'steps_with_block': winners,
    }


def bench_verify(args, ctx):
    from upow_amd.bench_verify import run_cluster_verify_bench, run_verify_bench
    # N ranks validate ONE chain as a cluster node (replicas + sharded ECDSA), not N private chains
    return run_cluster_verify_bench(args, ctx) if ctx.is_distributed else run_verify_bench(args, ctx)


def _verify_once(args, ctx, keys: str, segments: int = 1) -> dict:
    import shutil
    import tempfile
    from upow_amd.bench_verify import run_cluster_verify_bench, run_verify_bench
    tmp = tempfile.mkdtemp(prefix='upow_bench_verify_')
    try:
        v = argparse.Namespace(**{**vars(args), 'steps': args.verify_steps, 'warmup': args.verify_warmup, 'ledger': tmp,
                                  'object_path': False, 'from_mempool': False, 'governance': False,
                                  'governance_txs': 0.0, 'age_txs': 0, 'keys': keys, 'grouped_txs': 0.0,
                                  'segments': segments})
        return run_cluster_verify_bench(v, ctx) if ctx.is_distributed else run_verify_bench(v, ctx)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def _verify_side_metrics(args, ctx) -> dict:
    """BASELINE metric 2 next to the hashrate: ``--verify-steps`` timed 2 MB blocks (+2 warmup) through the
    native push_block path on this rank's GPU, file-backed ledger in a temporary directory, as the median of
    ``--verify-segments`` consecutive segments (each ending with its own SQL drain). The reported
    number uses distinct keys (a fresh key pair per tx, fresh output addresses: BASELINE's random-keypair
    data); the 256-key pool run follows as a labelled second number (``verify_pool256_*``)."""
    r = _verify_once(args, ctx, 'distinct', args.verify_segments)
    out = {'verify_tx_per_s': r['value'], 'verify_ms_per_block': r['ms_per_step'],
           **({'verify_segments_tx_per_s': r['segments_tx_per_s'], 'verify_segment_diag': r.get('segment_diag')}
              if 'segments_tx_per_s' in r else {}),
           'verify_commit_latency_ms': r['commit_latency_ms'], 'validate_tx_per_s': r['validate_tx_per_s'],
           'ecdsa_sig_per_s': r['ecdsa_sig_per_s'], 'verify_stage_ms_avg': r['stage_ms_avg'],
           'verify_config': {'metric': r['metric'], 'unit': r['unit'], 'steps': args.verify_steps,
                             'warmup': args.verify_warmup,
                             'txs_per_block': r['config']['seq_len'], 'ledger': r['config']['ledger'],
                             'block_path': r['config']['block_path'], 'scaling': r['scaling'],
                             'layout': r['config']['parallelism'], 'keys': 'distinct', 'data': r['data']}}
    if args.verify_pool256:
        p = _verify_once(args, ctx, 'pool256')
        out.update({'verify_pool256_tx_per_s': p['value'], 'verify_pool256_ms_per_block': p['ms_per_step'],
                    'verify_pool256_data': p['data']})
    return out


def _sync_side_metrics(args, ctx) -> dict:
    """Chain sync next to the hashrate: ``--sync-steps`` 200-tx blocks (+5 warmup) replayed from /get_blocks
    pages into a file-backed ledger (ledger/pagesync.py). With N ranks it is ONE chain synced by an N-GPU
    cluster node (every page's signatures sharded over the GPUs, every block agreed before commit), so the
    per-N values of the scaling runs compare one chain's sync rate at 1, 2, 4 and 8 GPUs."""
    import shutil
    import tempfile
    from upow_amd.bench_verify import run_cluster_sync_bench, run_sync_bench
    tmp = tempfile.mkdtemp(prefix='upow_bench_sync_')
    try:
        v = argparse.Namespace(**{**vars(args), 'steps': args.sync_steps, 'warmup': 5, 'txs': 200, 'txs_range': None,
                                  'ledger': tmp, 'keys': 'distinct', 'age_txs': 0, 'sync_page_blocks': 1000})
        r = run_cluster_sync_bench(v, ctx) if ctx.is_distributed else run_sync_bench(v, ctx)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    return {'sync_tx_per_s': r['value'], 'sync_blocks_per_s': r.get('blocks_per_s'),
            'sync_ms_per_block': r['ms_per_step'],
            'sync_config': {'metric': r['metric'], 'unit': r['unit'], 'blocks': args.sync_steps, 'warmup': 5,
                            'txs_per_block': 200, 'scaling': r['scaling'], 'layout': r['config']['parallelism'],
                            'path': 'page', 'data': r['data']}}


def _guarded_side_metric(args, ctx, headline: dict) -> dict:
    """The sync side metric must never cost the headline its one JSON line. With N ranks a failure on one rank
    would leave the others waiting in a collective, so every rank arms the same deadline after a barrier: if
    the side metric has not finished by then, rank 0 prints the headline (with ``sync_error``) and every rank
    exits 0. A Python error on a rank is reported the same way."""
    import threading
    deadline = float(os.environ.get('UPOW_BENCH_SIDE_DEADLINE_S', '420'))
    ctx.barrier()

    def fire():
        if ctx.is_main:
            print(json.dumps({**headline, 'sync_error': f'side metric unfinished after {deadline:.0f} s'}), flush=True)
        os._exit(0)
    timer = threading.Timer(deadline, fire)
    timer.daemon = True
    timer.start()
    fatal, ctx.fatal = ctx.fatal, False  # a failed collective raises here instead of exiting with status 70
    try:
        res = _sync_side_metrics(args, ctx)
    except Exception as e:
        if not ctx.is_distributed:
            timer.cancel()
            return {'sync_error': f'{type(e).__name__}: {e}'[:300]}
        if ctx.is_main:  # the other ranks may be waiting in a collective: report and leave together
            print(json.dumps({**headline, 'sync_error': f'{type(e).__name__}: {e}'[:300]}), flush=True)
        os._exit(0)
    finally:
        ctx.fatal = fatal
    timer.cancel()
    return res


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _launch_ranks(n: int, argv) -> int:
    """``python bench.py --gpus N`` without a torchrun environment: start ``torch.distributed.run`` with N
    ranks (one per GPU, 127.0.0.1 rendezvous) as a CHILD process — this process has not touched the GPU
    (no HIP call, no ``torch.cuda`` query), so nothing is exec'd from a GPU-initialised process. The
    children inherit stdout: rank 0's JSON line is the only thing printed there."""
    import subprocess
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={n}',
           '--master-addr', '127.0.0.1', '--master-port', str(_free_port()), os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')  # dmabuf IPC (RCCL across processes on this host)
    env.setdefault('OMP_NUM_THREADS', '1')
    return subprocess.call(cmd, env=env)


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--warmup', type=int, default=2)
    ap.add_argument('--mode', choices=['mine', 'verify', 'sync'], default='mine')
    ap.add_argument('--difficulty', default='6.3')
    ap.add_argument('--nonces', type=int, default=0, help='nonce words per rank per step (default 2^32)')
    ap.add_argument('--variant', type=int, default=int(os.environ.get('UPOW_POW_VARIANT', '0')))
    ap.add_argument('--txs', type=int, default=8300, help='verify mode: txs per block')
    ap.add_argument('--object-path', action='store_true', help='verify mode: Transaction-object path (A/B)')
    ap.add_argument('--ledger', default=None, help='verify mode: directory for a file-backed (WAL) ledger')
    ap.add_argument('--from-mempool', action='store_true',
                    help='verify mode: block txs are in the mempool and pushed as hashes (the miner path)')
    ap.add_argument('--governance', action='store_true',
                    help='verify mode: seed 12 inodes, 200 validators, 5,000 delegates with ballots before the blocks')
    ap.add_argument('--governance-txs', default='0',
                    help="verify mode: fraction of each block's txs that are governance txs, e.g. 5%% or 0.05")
    ap.add_argument('--grouped-txs', default='0',
                    help="verify mode (distinct keys): fraction of each block's txs with 2 signatures over 4 inputs of "
                         "two keys (signature grouping by owner key), e.g. 10%%")
    ap.add_argument('--age-txs', type=int, default=0,
                    help='verify/sync modes: first age the ledger with N confirmed txs (2N UTXO rows), e.g. 2500000')
    ap.add_argument('--keys', choices=['distinct', 'pool256'], default='distinct',
                    help='verify/sync modes: a fresh key pair per tx (default) or a 256-key pool (cache-friendly)')
    ap.add_argument('--verify-pool256', type=int, default=1,
                    help='mine mode: also report the 256-key-pool verify number as a labelled second value')
    ap.add_argument('--txs-range', default=None,
                    help='sync mode: per-block tx count uniform in LO-HI (e.g. 0-20, mainnet-shaped) instead of --txs')
    ap.add_argument('--sync-page-blocks', type=int, default=1000, help='sync mode: blocks per /get_blocks page')
    ap.add_argument('--sync-steps', type=int, default=500,
                    help='mine mode: blocks of the chain-sync side measurement (200-tx blocks; 0: skip; GPU only)')
    ap.add_argument('--sync-path', choices=['page', 'block'], default='page',
                    help='sync mode: page-batched (ledger/pagesync.py, default) or the per-block pipeline (A/B)')
    ap.add_argument('--verify-segments', type=int, default=3,
                    help='mine mode: the verify side metric is the median of this many consecutive segments of '
                         '--verify-steps blocks (one setup, one process)')
    ap.add_argument('--segments', type=int, default=1, help='verify mode: median of this many segments of --steps blocks')
    ap.add_argument('--verify-warmup', type=int, default=2,
                    help='mine mode: untimed 2 MB blocks before the verify side metric\'s segments')
    ap.add_argument('--verify-steps', type=int, default=10,
                    help='mine mode: timed 2 MB blocks of the tx-verify side measurement (0: skip; GPU only)')
    args = ap.parse_args(argv)
    g = str(args.governance_txs).strip()
    args.governance_txs = float(g[:-1]) / 100 if g.endswith('%') else float(g)
    g = str(args.grouped_txs).strip()
    args.grouped_txs = float(g[:-1]) / 100 if g.endswith('%') else float(g)

    # rank launch: the driver either starts N ranks itself (torchrun sets WORLD_SIZE) or runs
    # ``bench.py --gpus N`` plainly, in which case this process becomes the launcher of N ranks
    if 'WORLD_SIZE' not in os.environ and args.gpus > 1:
        sys.exit(_launch_ranks(args.gpus, argv))
    world = int(os.environ.get('WORLD_SIZE', '1'))
    if world != args.gpus:
        print(json.dumps({'error': f'--gpus {args.gpus} but WORLD_SIZE={world}: refusing to report a '
                                   f'{world}-rank number as {args.gpus} GPUs'}), file=sys.stderr, flush=True)
        sys.exit(2)

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    # log lines go through the native console writer, as in a node process (upow_amd/utils/logger.py)
    os.environ.setdefault('UPOW_NATIVE_CONSOLE', '1')
    from upow_amd.ops.native import lib
    lib()  # loads torch's HIP runtime first, then the extension (fails loudly if not built)
    from upow_amd.utils.cpus import presize_fd_table, tune_malloc
    tune_malloc()  # as the node process does (upow_amd/node/__main__.py)
    presize_fd_table()
    from upow_amd.parallel.dist import init_from_env, shutdown
    ctx = init_from_env()
    try:
        if args.mode == 'mine':
            out = bench_mine(args, ctx)
            if ctx.world > 1:
                # the multi-GPU runs report the hashrate scaling curve; the verify side metric is the 1-GPU
                # config (BASELINE config 4), and a cluster verify here would put RCCL collectives of a second
                # workload between the headline measurement and its one JSON line
                out['verify_side_metrics'] = 'single-GPU runs (bench.py --mode verify --gpus N for the cluster)'
            elif args.verify_steps > 0 and out['config']['device'] == 'gpu':
                try:
                    out.update(_verify_side_metrics(args, ctx))
                except Exception as e:  # the headline number stands on its own; say why the extra is missing
                    out['verify_error'] = f'{type(e).__name__}: {e}'[:300]
            if args.sync_steps > 0 and out['config']['device'] == 'gpu':
                out.update(_guarded_side_metric(args, ctx, out))
        elif args.mode == 'verify':
            out = bench_verify(args, ctx)
        else:
            from upow_amd.bench_verify import run_cluster_sync_bench, run_sync_bench
            from upow_amd.ledger import pagesync
            pagesync.ENABLED = args.sync_path == 'page'
            # N ranks sync ONE chain as a cluster node (replicas + sharded page verify), not N private chains
            out = run_cluster_sync_bench(args, ctx) if ctx.is_distributed else run_sync_bench(args, ctx)
        if ctx.is_main:
            print(json.dumps(out), flush=True)
    finally:
        shutdown(ctx)


if __name__ == '__main__':
    main()
