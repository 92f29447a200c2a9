"""Multi-process (gloo, world_size 2) tests of the nonce-space data parallelism and collectives.

The same code runs over RCCL on MI355X ranks; here every rank uses the host C++ search."""
import hashlib
import os
import socket

import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update({'RANK': str(rank), 'WORLD_SIZE': str(world), 'LOCAL_RANK': str(rank),
                       'MASTER_ADDR': '127.0.0.1', 'MASTER_PORT': str(port), 'UPOW_DISABLE_GPU': '1'})
    try:
        from upow_amd.models.block import PowTarget
        from upow_amd.parallel.dist import init_from_env, shutdown
        from upow_amd.parallel.miner_dp import ClusterMiner, DataParallelMiner
        ctx = init_from_env(backend='gloo', want_gpu=False)
        assert ctx.world == world and ctx.rank == rank
        # collectives
        assert ctx.allreduce_min(10 + rank) == 10
        assert ctx.allreduce_sum(1) == world
        assert ctx.broadcast_bytes(b'x' * 300 if rank == 1 else None, src=1, max_len=0) == b'x' * 300
        got = ctx.all_gather_bytes(bytes([rank]) * (rank + 1))
        assert got == [bytes([r]) * (r + 1) for r in range(world)]
        prev = hashlib.sha256(b'p').hexdigest()
        addr = 'DgQKikeDqS2Fzue23KuA36L4eJSFh649zA9jJ6zwbzUMp'
        merkle = hashlib.sha256(b'm').hexdigest()
        # weak-scaling bench miner: per-rank timestamps, agreed winner header
        m = DataParallelMiner(ctx, prev, addr, merkle, 1_700_000_000, '2.5', device='cpu', threads=2)
        r = m.step(1 << 14)
        assert r.header is not None and r.winner < world
        assert PowTarget.from_difficulty(prev, '2.5').check_hex(hashlib.sha256(r.header).hexdigest())
        # roll to the next timestamp slot at the end of the nonce space
        m.next_word = (1 << 32) - (1 << 10)
        ts_before = m.ts
        m.step(1 << 10)
        assert m.ts == ts_before - world
        # CLI miner: nonce-slice partition, everyone returns the same header
        cm = ClusterMiner(ctx, prev, addr, merkle, '3.0', ts_max=1_700_000_100, ts_min=1_700_000_090, device='cpu',
                          chunk=1 << 12, threads=2)
        h = cm.mine()
        hs = ctx.all_gather_bytes(h)
        assert len(set(hs)) == 1 and PowTarget.from_difficulty(prev, '3.0').check_hex(hashlib.sha256(h).hexdigest())
        shutdown(ctx)
        q.put((rank, 'ok'))
    except Exception as e:  # pragma: no cover
        import traceback
        q.put((rank, traceback.format_exc()))


def test_dp_miner_gloo_world2():
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(60)
    assert results == {0: 'ok', 1: 'ok'}, results
