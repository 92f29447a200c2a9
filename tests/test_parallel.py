"""Multi-process (gloo, world_size 2 and 4) tests of the nonce-space data parallelism, the collectives,
sharded verification and the multi-GPU node's replica op stream.

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
        # fused per-chunk agreement of ClusterMiner: element-wise MIN in one collective
        assert ctx.allreduce_min_vec([rank if rank % 2 else world, 0 if rank == world - 1 else 1, 1]) == \
            [1 if world > 1 else world, 0, 1]
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


def _spawn(target, world, *args):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, *args, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(60)
    return results


@pytest.mark.parametrize('world', [2, 4])
def test_dp_miner_gloo(world):
    results = _spawn(_worker, world)
    assert results == {r: 'ok' for r in range(world)}, results


def test_shard_bounds_partition():
    from upow_amd.parallel.verify_dp import shard_bounds
    for n in (0, 1, 7, 8300):
        for world in (1, 2, 3, 8):
            spans = [shard_bounds(n, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            assert max(h - l for l, h in spans) - min(h - l for l, h in spans) <= 1


def _replica_worker(rank, world, port, tmp, q):
    os.environ.update({'RANK': str(rank), 'WORLD_SIZE': str(world), 'LOCAL_RANK': str(rank),
                       'MASTER_ADDR': '127.0.0.1', 'MASTER_PORT': str(port), 'UPOW_DISABLE_GPU': '1',
                       'UPOW_START_DIFFICULTY': '1.0', 'UPOW_CORE_URL': '',
                       'UPOW_CLUSTER_SHARD_MIN': '1'})  # shard even tiny blocks: the sharded path is under test
    try:
        import asyncio
        import hashlib as hl

        from upow_amd import devnet
        from upow_amd.ledger import validate
        from upow_amd.ledger.database import Database
        from upow_amd.models.transaction import Transaction
        from upow_amd.ops import p256 as op
        from upow_amd.parallel.dist import init_from_env, shutdown
        from upow_amd.parallel import verify_dp
        from upow_amd.wallet.builders import address_of, create_transaction

        ctx = init_from_env(backend='gloo', want_gpu=False)
        # sharded raw-record verify: one bad signature in the last shard
        d = 0x1234567
        qpt = op.public_key(d)
        recs = []
        for i in range(9):
            dig = hl.sha256(b'm%d' % i).digest()
            r, s = op.sign(b'm%d' % i, d)
            recs.append(op.record(qpt, (r, s + (1 if i == 7 else 0)), dig))
        st = verify_dp.verify_records_dp(ctx, b''.join(recs))
        assert list(st) == [1] * 7 + [0, 1], list(st)
        assert verify_dp.verify_shard_first_failure(ctx, b''.join(recs)) == 7
        assert verify_dp.verify_shard_first_failure(ctx, b''.join(recs[:7])) == -1
        async def replicate(content, txs):
            # the harness's replication: rank 0's block to every rank, each applies it with the
            # signature batch sharded across the ranks, and all verdicts must agree
            import json as js
            from upow_amd.ledger import manager
            raw = ctx.broadcast_bytes(js.dumps({'b': content, 't': txs or []}).encode() if rank == 0 else None,
                                      src=0, max_len=0)
            obj = js.loads(raw.decode())
            ok = await manager.create_block(obj['b'], [await Transaction.from_hex(h) for h in obj['t']])
            assert ctx.allreduce_sum(1 if ok else 0) in (0, ctx.world)
            return ok

        async def go():
            db = await Database.create(path=os.path.join(tmp, f'r{rank}.sqlite3'), utxo_backend='host')
            validate.set_dist_context(ctx)
            key = 0x61
            addr = address_of(key)
            base = 1_700_000_000
            for b in range(3):
                content = await devnet.mine_header(addr, [], ts=base + 60 * b, device='cpu') if rank == 0 else None
                assert await replicate(content, [])
            txs = []
            if rank == 0:
                for j in range(3):
                    tx = await create_transaction(key, address_of(0x100 + j), '1.5')
                    await db.add_pending_transaction(tx)
                    txs.append(tx)
            # a block whose last signature (rank 1's shard) is forged: both replicas reject it
            bad_hex = None
            if rank == 0:
                forged, _ = Transaction.parse(txs[-1].hex())
                r, s = forged.inputs[0].signed
                forged.inputs[0].signed = (r, s + 1 if s + 1 < op.oracle.N else s - 1)
                bad = txs[:-1] + [forged]
                bad_hex = [t.hex() for t in bad]
                content = await devnet.mine_header(addr, bad, ts=base + 60 * 3, device='cpu')
            assert not await replicate(content if rank == 0 else None, bad_hex)
            good = None
            if rank == 0:
                good = [t.hex() for t in txs]
                content = await devnet.mine_header(addr, txs, ts=base + 60 * 3, device='cpu')
            assert await replicate(content if rank == 0 else None, good)
            h = await db.get_unspent_outputs_hash()
            hs = ctx.all_gather_bytes(h.encode())
            assert len(set(hs)) == 1 and (await db.get_next_block_id()) == 5
            db.close()
        asyncio.run(go())
        shutdown(ctx)
        q.put((rank, 'ok'))
    except Exception:  # pragma: no cover
        import traceback
        q.put((rank, traceback.format_exc()))


@pytest.mark.parametrize('world', [2, 4])
def test_sharded_verify_and_replicated_ledger_gloo(tmp_path, world):
    results = _spawn(_replica_worker, world, str(tmp_path))
    assert results == {r: 'ok' for r in range(world)}, results


def _cluster_worker(rank, world, port, tmp, q):
    """The multi-GPU node's op stream (parallel/cluster.py): the leader applies blocks (each broadcast as a
    binary frame, signatures sharded over the ranks, verdict agreed), admits mempool txs, rolls a block
    back and re-applies it; every follower replica must end at the same height and UTXO-set hash."""
    os.environ.update({'RANK': str(rank), 'WORLD_SIZE': str(world), 'LOCAL_RANK': str(rank),
                       'MASTER_ADDR': '127.0.0.1', 'MASTER_PORT': str(port), 'UPOW_DISABLE_GPU': '1',
                       'UPOW_START_DIFFICULTY': '1.0', 'UPOW_CORE_URL': ''})
    try:
        import asyncio

        from upow_amd import devnet
        from upow_amd.ledger import fastpath, validate
        from upow_amd.ledger.database import Database
        from upow_amd.parallel import cluster
        from upow_amd.parallel.dist import init_from_env, shutdown
        from upow_amd.wallet.builders import address_of, create_transaction

        ctx = init_from_env(backend='gloo', want_gpu=False)
        c = cluster.init(ctx)

        async def go():
            db = await Database.create(path=os.path.join(tmp, f'c{rank}.sqlite3'), utxo_backend='host')
            if rank != 0:
                await cluster.follower_main(c, db)
                res = (db._tip_id(), await db.get_unspent_outputs_hash())
                db.close()
                return res
            key = 0x71
            addr = address_of(key)
            base = 1_700_000_000
            await cluster.leader_start(db)
            assert validate._dist_ctx is ctx
            for b in range(5):
                content = await devnet.mine_header(addr, [], ts=base + 60 * b, device='cpu')
                assert await fastpath.create_block_from_hex(content, [])
            txs = []
            for j in range(4):
                tx = await create_transaction(key, address_of(0x200 + j), '1.25')
                assert await db.add_pending_transaction(tx)  # replicated through db.on_admit
                txs.append(tx)
            cluster.flush_txs()
            c.send('status')
            st = c.status(db)
            assert {x['mempool'] for x in st} == {4}, st
            content = await devnet.mine_header(addr, txs, ts=base + 60 * 5, device='cpu')
            assert await fastpath.create_block_from_hex(content, [t.hex() for t in txs])
            assert fastpath.last_path == 'native'
            c.send('status')
            st = c.status(db)
            assert len({(x['height'], x['utxo_hash']) for x in st}) == 1 and st[0]['height'] == 6, st
            await cluster.mirror_rollback(db, 6)
            c.send('status')
            st = c.status(db)
            assert len({(x['height'], x['utxo_hash']) for x in st}) == 1 and st[0]['height'] == 5, st
            assert await fastpath.create_block_from_hex(content, [t.hex() for t in txs])
            res = (db._tip_id(), await db.get_unspent_outputs_hash())
            await cluster.leader_quit()
            db.close()
            return res

        res = asyncio.run(go())
        hs = ctx.all_gather_bytes(repr(res).encode())
        assert len(set(hs)) == 1 and res[0] == 6, hs
        shutdown(ctx)
        q.put((rank, 'ok'))
    except Exception:  # pragma: no cover
        import traceback
        q.put((rank, traceback.format_exc()))


def test_cluster_op_stream_replicas_and_rollback_gloo_world4(tmp_path):
    results = _spawn(_cluster_worker, 4, str(tmp_path))
    assert results == {r: 'ok' for r in range(4)}, results
