"""``python -m upow_amd.node [--host H] [--port P] [--data DIR] [--db PATH]`` (reference: run_node.py,
upow/node/run.py — uvicorn on port 3006)."""
import argparse
import os


def parse_cpus(spec: str):
    """'0-15,32,40-43' -> sorted CPU list."""
    out = set()
    for part in spec.split(','):
        part = part.strip()
        if not part:
            continue
        if '-' in part:
            lo, hi = part.split('-', 1)
            out.update(range(int(lo), int(hi) + 1))
        else:
            out.add(int(part))
    return sorted(out)


def pin_cpus(spec: str):
    """Process CPU affinity before any thread starts (``UPOW_CPU_AFFINITY``): 'off' (default), an explicit
    CPU list, or 'auto' = as many CPUs as the cgroup CPU quota grants, taken from the current affinity set.
    A node whose quota is far below the host's core count otherwise spreads its threads over every core,
    and CFS bandwidth control hands quota to each core in slices: a burst then exhausts the period's quota
    and freezes every thread of the node (the HTTP loop included) until the next period."""
    if not spec or spec == 'off':
        return None
    cur = sorted(os.sched_getaffinity(0))
    if spec == 'auto':
        from ..ledger.fastpath import cpu_budget
        q = cpu_budget()
        if q >= len(cur):
            return None
        want = cur[:q]
    else:
        want = [c for c in parse_cpus(spec) if c in set(cur)]
    if want:
        os.sched_setaffinity(0, want)
    return want


def server_protocol() -> dict:
    """uvicorn keyword arguments for the node's HTTP/WebSocket protocol (``node/http.py``: native request
    framing, WebSocket served in place); ``UPOW_NATIVE_HTTP=0`` keeps uvicorn's own h11 protocol."""
    if os.environ.get('UPOW_NATIVE_HTTP', '1') == '0':
        return {}
    from .http import NodeHttpProtocol
    return {'http': NodeHttpProtocol}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument('--host', default='0.0.0.0')
    ap.add_argument('--port', type=int, default=3006)
    ap.add_argument('--data', default=None, help='data directory (ledger, peers.json, ip_config.json)')
    ap.add_argument('--db', default=None, help='SQLite ledger path')
    ap.add_argument('--core-url', default=None, help='bootstrap peer (empty string disables)')
    ap.add_argument('--log-level', default='info')
    ap.add_argument('--cluster', action='store_true',
                    help='multi-GPU node under torchrun: rank 0 serves the API, other ranks are HBM replicas')
    a = ap.parse_args(argv)
    pin_cpus(os.environ.get('UPOW_CPU_AFFINITY', 'off'))
    from ..utils.cpus import presize_fd_table, tune_malloc
    tune_malloc()
    presize_fd_table()
    if a.data:
        os.environ['UPOW_DATA_DIR'] = a.data
    if a.db:
        os.environ['UPOW_DATABASE_PATH'] = a.db
    if a.core_url is not None:
        os.environ['UPOW_CORE_URL'] = a.core_url
    os.environ.setdefault('UPOW_FILE_LOG', '1')  # reference: logs/app.log always (my_logger.py:17-53)
    import uvicorn
    if a.cluster and (int(os.environ.get('WORLD_SIZE', '1')) > 1 or os.environ.get('UPOW_FORCE_DIST') == '1'):
        return _run_cluster(a)  # UPOW_FORCE_DIST=1: a single-rank cluster (the op stream over RCCL on one GPU)
    prof_out = os.environ.get('UPOW_PROFILE_OUT')  # cProfile of the serving process (load tests)
    if prof_out:
        import cProfile
        import signal
        import sys
        prof = cProfile.Profile()

        def dump(*_):
            prof.disable()
            prof.dump_stats(prof_out)
            sys.exit(0)

        # uvicorn re-raises the SIGTERM it caught once the graceful shutdown is done: dump there
        signal.signal(signal.SIGTERM, dump)
        prof.enable()
        uvicorn.run('upow_amd.node.main:app', host=a.host, port=a.port, log_level=a.log_level, **server_protocol())
        dump()
    uvicorn.run('upow_amd.node.main:app', host=a.host, port=a.port, log_level=a.log_level, **server_protocol())


def _run_cluster(a):
    """One process per GPU (parallel/cluster.py): rank 0 runs the node, the others replicate it."""
    import asyncio

    from ..ops.native import lib
    from ..parallel import cluster
    from ..parallel.dist import init_from_env, op_context, shutdown
    lib()  # the extension binds to torch's HIP runtime before the process group exists
    # a replica's block submit may wait on its SQL materialisers (writer backpressure); that wait must stay well
    # inside the op group's collective timeout, or a slow disk would end the whole cluster (parallel/dist.py)
    op_timeout = float(os.environ.setdefault('UPOW_DIST_TIMEOUT_S', '120'))
    throttle = float(os.environ.get('UPOW_WRITER_THROTTLE_TIMEOUT', '300'))
    os.environ['UPOW_WRITER_THROTTLE_TIMEOUT'] = str(min(throttle, op_timeout / 4))
    ctx = init_from_env()
    c = cluster.init(op_context(ctx), ctx)  # op traffic on a short-timeout group, start-up on the default one
    try:
        if ctx.rank == 0:
            import uvicorn
            from . import main as node_main
            uvicorn.run(node_main.app, host=a.host, port=a.port, log_level=a.log_level, **server_protocol())
        else:
            asyncio.run(_follow(c))
    finally:
        shutdown(ctx)


def follower_ledger_path(rank: int) -> str:
    """A follower's durable replica: ``<data dir>/rank<N>/ledger.sqlite3`` with its own journal, undo
    segments and UTXO snapshot (``UPOW_CLUSTER_FOLLOWER_DB=:memory:`` keeps the old ephemeral replica)."""
    from .. import config
    spec = os.environ.get('UPOW_CLUSTER_FOLLOWER_DB')
    if spec:
        return spec if spec == ':memory:' else spec.replace('{rank}', str(rank))
    return config.data_path(f'rank{rank}', 'ledger.sqlite3')


async def _follow(c):
    import signal

    from ..ledger.database import Database
    from ..parallel import cluster
    # a stop signal reaches every rank of the job at once: the follower keeps applying the op stream until
    # the leader's graceful shutdown sends 'quit' (then it snapshots and closes its ledger); if the leader
    # is gone instead, the op group's collective timeout ends this process (parallel/dist.py)
    signal.signal(signal.SIGTERM, lambda *_: None)
    signal.signal(signal.SIGINT, lambda *_: None)
    db = await Database.create(path=follower_ledger_path(c.ctx.rank))
    try:
        # a lean replica (ledger/lean.py) first materialises what its previous run logged
        await cluster.follower_main(c, db)
    finally:
        from ..ledger import lean
        # a lean replica's index is ahead of its SQL tables: the next start materialises its op log instead
        if db.path != ':memory:' and os.environ.get('UPOW_SNAPSHOT', '1') != '0' and not lean.pending(db):
            try:  # the next start restores the index from here instead of rebuilding it from SQL
                from ..ledger import snapshot
                snapshot.save(db)
            except Exception as e:
                from ..utils.logger import get_logger
                get_logger(__name__).error(f'follower UTXO snapshot failed: {e}')
        db.close()


if __name__ == '__main__':
    main()
