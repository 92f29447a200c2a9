"""Latency of the cluster node's collectives (parallel/dist.py) over the job's backend: the per-block commit
vote (split-phase all-gather: start to outcome, and the host time of queueing it), an 8-byte all-reduce, an idle op frame and a 64 KB frame (one fixed-capacity broadcast), a block-sized
frame (two broadcasts), the fixed-size state all-gather. Run under torch.distributed.run (UPOW_FORCE_DIST=1
for a single-rank RCCL group on one GPU). Prints one JSON line from rank 0: median microseconds per call."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _issue(ctx, med):
    """Host time of queueing one vote (its outcome collected outside the timed call)."""
    pending = []

    def one():
        if pending:
            ctx.vote_finish(pending.pop())
        pending.append(ctx.vote_start(1))
    # time only the start: finish the previous vote first, outside the clock
    import time
    for _ in range(20):
        one()
    ts = []
    for _ in range(int(os.environ.get('LAT_ITERS', '400'))):
        if pending:
            ctx.vote_finish(pending.pop())
        t0 = time.perf_counter()
        pending.append(ctx.vote_start(1))
        ts.append(time.perf_counter() - t0)
    ctx.vote_finish(pending.pop())
    ts.sort()
    return round(ts[len(ts) // 2] * 1e6, 1)


def main():
    from upow_amd.ops.native import lib
    lib()
    from upow_amd.parallel.dist import init_from_env, shutdown
    ctx = init_from_env()
    assert ctx.is_distributed, 'set UPOW_FORCE_DIST=1 or run with >1 rank'
    ctx.bind_owner()
    n = int(os.environ.get('LAT_ITERS', '400'))

    def med(fn):
        for _ in range(20):
            fn()
        ts = []
        for _ in range(n):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        ts.sort()
        return round(ts[len(ts) // 2] * 1e6, 1)
    me = ctx.rank == 0
    frame64 = b'x' * (60 << 10)
    block = b'y' * (2 << 20)
    out = {
        'backend': ctx.backend, 'world': ctx.world,
        'allreduce_sum_us': med(lambda: ctx.allreduce_sum(1)),
        'vote_us': med(lambda: ctx.vote_finish(ctx.vote_start(1))),  # the commit vote, start to outcome
        'vote_native': ctx.__dict__.get('_nv') is not None,
        'vote_issue_us': _issue(ctx, med),
        'allreduce_min_vec_us': med(lambda: ctx.allreduce_min_vec([1, -1])),
        'frame_ping_us': med(lambda: ctx.broadcast_frame(b'{"op":"ping"}' if me else None, src=0)),
        'frame_60k_us': med(lambda: ctx.broadcast_frame(frame64 if me else None, src=0)),
        'frame_2mb_us': med(lambda: ctx.broadcast_frame(block if me else None, src=0)),
        'all_gather_fixed_48b_us': med(lambda: ctx.all_gather_fixed(b'z' * 48)),
        'all_gather_bytes_us': med(lambda: ctx.all_gather_bytes(b'z' * 300)),
    }
    if me:
        print(json.dumps(out), flush=True)
    shutdown(ctx)


if __name__ == '__main__':
    main()
