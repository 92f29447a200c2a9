"""Collective self-check over RCCL (run under torch.distributed.run; UPOW_FORCE_DIST=1 makes a
1-GPU job use a real process group). Exercises every DistContext collective plus the sharded
signature verify, mempool all-gather and block broadcast of parallel/verify_dp.py on cuda tensors."""
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from upow_amd.ops.native import lib  # noqa: E402


def main():
    lib()
    from upow_amd.ops import p256 as op
    from upow_amd.parallel import verify_dp
    from upow_amd.parallel.dist import init_from_env, shutdown
    ctx = init_from_env()
    from upow_amd.ops.native import gpu_available
    dev = 'gpu' if gpu_available() else 'cpu'
    assert ctx.is_distributed, 'set UPOW_FORCE_DIST=1 or run with >1 rank'
    assert ctx.allreduce_min(5 + ctx.rank) == 5
    assert ctx.allreduce_sum(2) == 2 * ctx.world
    assert ctx.allreduce_min_vec([ctx.rank, 1, 0]) == [0, 1, 0]  # ClusterMiner's fused per-chunk agreement
    assert ctx.broadcast_bytes(b'h' * 108 if ctx.rank == 0 else None, src=0) == b'h' * 108
    big = bytes(range(256)) * 9000  # ~2.3 MB block-sized payload
    assert ctx.broadcast_bytes(big if ctx.rank == 0 else None, src=0, max_len=0) == big
    d = 0xC0FFEE
    q = op.public_key(d)
    recs, want = [], []
    for i in range(4096):
        m = b'tx%d' % i
        r, s = op.sign(m, d)
        bad = i % 997 == 5
        recs.append(op.record(q, (r, s ^ 1 if bad else s), hashlib.sha256(m).digest()))
        want.append(0 if bad else 1)
    st = verify_dp.verify_records_dp(ctx, b''.join(recs), device=dev)
    assert list(st) == want
    assert verify_dp.verify_shard_first_failure(ctx, b''.join(recs), device=dev) == 5
    # the multi-GPU node's op frame (parallel/cluster.py): JSON header + raw tx bytes, over RCCL
    from upow_amd.parallel import cluster
    c = cluster.Cluster(ctx)
    txs = [bytes([k]) * (100 + k) for k in range(50)]
    if ctx.rank == 0:
        c.send('block', cluster.pack_txs([t.hex() for t in txs]), content='ee' * 108)
    msg = c.recv() if ctx.rank != 0 else None
    if ctx.rank != 0:
        assert msg['op'] == 'block' and cluster.unpack_txs(msg['_payload']) == [t.hex() for t in txs]
    ctx.barrier()
    if ctx.rank == 0:
        print(json.dumps({'rccl_selfcheck': 'ok', 'world': ctx.world, 'backend': ctx.backend}))
    shutdown(ctx)
    return 0


if __name__ == '__main__':
    sys.exit(main())
