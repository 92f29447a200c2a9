"""Host CPU budget of this process (thread-pool sizing for the codec, host verify and admission)."""
import os


def cpu_budget(per_rank: bool = True) -> int:
    """CPUs this process can actually use: its affinity, capped by a cgroup CPU quota (a GPU box gives a
    node 16 CPUs' worth of time on a 256-core host; threads beyond that are throttled, not parallel).
    ``per_rank``: one share of it per local rank (``LOCAL_WORLD_SIZE`` under torchrun) when the ranks of a
    node share one affinity set, so 8 ranks do not each size their host pools for the whole machine."""
    try:
        aff = os.sched_getaffinity(0)
        avail = len(aff)
    except (AttributeError, OSError):
        aff, avail = None, os.cpu_count() or 1
    try:
        with open('/sys/fs/cgroup/cpu.max') as f:
            quota, period = f.read().split()[:2]
        if quota != 'max':
            avail = min(avail, max(1, int(quota) // int(period)))
    except (OSError, ValueError):
        pass
    local = int(os.environ.get('LOCAL_WORLD_SIZE', '1') or 1)
    if per_rank and local > 1 and (aff is None or len(aff) >= (os.cpu_count() or 1) // 2):
        # not pinned per rank: split the node's budget. By role (UPOW_CPU_ROLE_SPLIT, default on): local rank 0
        # — a cluster node's leader, the one rank that renders, encodes and materialises the SQL ledger and
        # serves HTTP — takes half, the lean followers (ledger/lean.py: decode, index updates, their verify
        # shard) share the other half; an equal split gave the leader 1/8 of an 8-GPU host for 8x the host work
        if os.environ.get('UPOW_CPU_ROLE_SPLIT', '1') != '0':
            lead = max(1, avail // 2)
            if int(os.environ.get('LOCAL_RANK', '0') or 0) == 0:
                return lead
            return max(1, (avail - lead) // (local - 1))
        avail = max(1, avail // local)
    return avail


def tune_malloc() -> bool:
    """Fixed glibc allocator thresholds for a block-processing process (``UPOW_MALLOC_TUNE=0`` leaves the
    defaults): 256 MB mmap threshold and 1 GB trim threshold, so the multi-megabyte column buffers every
    2 MB block allocates are reused heap pages instead of fresh mappings faulted in again on each block
    (csrc/bindings.cpp ``malloc_tune``). The process keeps its peak heap mapped: tens of MB for a node,
    nothing next to a GPU host's RAM."""
    if os.environ.get('UPOW_MALLOC_TUNE', '1') == '0':
        return False
    from ..ops.native import lib
    return bool(lib().malloc_tune(256 << 20, 1 << 30))


def presize_fd_table(n: int = 16384) -> int:
    """Grow this process's file-descriptor table to ``n`` slots now, while it is cheap (``UPOW_FD_PRESIZE=0``
    skips). The kernel grows the table by doubling when an open/accept needs a slot past its end, and in a
    multithreaded process each growth waits for an RCU grace period before the old table can go; every
    other thread opening a descriptor meanwhile waits too. A node crossing a size boundary mid-run (ledger
    files x connections x WAL/shm files, plus sockets) froze its HTTP event loop in ``accept4`` for
    150-200 ms at a time: soak probe samples showed the loop in ``__wait_rcu_gp`` and the other threads in
    ``expand_files`` (profiles/r4/node_soak_fdtable_r4z.json). The soft RLIMIT_NOFILE is raised to ``n``
    when the hard limit allows. Returns the table size reached (/proc/self/status FDSize), 0 if skipped."""
    if os.environ.get('UPOW_FD_PRESIZE', '1') == '0':
        return 0
    import resource
    soft, hard = resource.getrlimit(resource.RLIMIT_NOFILE)
    if soft != resource.RLIM_INFINITY and soft < n and (hard == resource.RLIM_INFINITY or hard >= n):
        resource.setrlimit(resource.RLIMIT_NOFILE, (n, hard))
        soft = n
    top = (n if soft == resource.RLIM_INFINITY else min(n, soft)) - 1
    fd = os.open(os.devnull, os.O_RDONLY)
    try:
        if fd < top:
            os.dup2(fd, top, inheritable=False)  # the table is sized to fit the highest descriptor
            os.close(top)
    finally:
        os.close(fd)
    try:
        with open('/proc/self/status') as f:
            for line in f:
                if line.startswith('FDSize:'):
                    return int(line.split()[1])
    except OSError:
        pass
    return top + 1

