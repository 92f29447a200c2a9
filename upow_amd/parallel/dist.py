"""Process-group bootstrap: one process per GPU, ``torch.distributed`` over RCCL (backend "nccl").

MI355X topology: 8 GPUs per node, fully connected by 7 xGMI links each. Every collective this
framework issues is small and latency-bound (8-byte flags, 108-byte headers, <=2 MB blocks,
mempool deltas), so there is no bucketing: each exchange is one RCCL call on the
default stream, and the messages ride the LL/LL128 protocols over the direct links.

Tests use the same code with the ``gloo`` backend on CPU (world_size > 1 on one host).

Failure model. A collective that one rank never joins (a replica that diverged onto another code path, a
rank that died) must not hang the node forever:

* every collective of a cluster node runs on ONE owner thread per process (``bind_owner``; the leader's
  ledger thread, the follower's op loop). A call from any other thread raises before touching the
  communicator, so two threads can never interleave their collective sequences;
* the cluster's op traffic runs on a process group created with a timeout (``UPOW_DIST_TIMEOUT_S``, 60 s
  by default, 120 s for a ``--cluster`` node; the leader's idle heartbeat keeps followers inside it), and a
  collective that fails or times out ends the process loudly with a non-zero status (``UPOW_DIST_FATAL=0``
  raises instead, for tests). Anything a rank may legitimately wait on between two ops is kept well inside
  that timeout: the ledger writer's backpressure wait is capped at a quarter of it on cluster ranks
  (node/__main__.py), and the full-table ``/cluster_info?deep=true`` audit gathers on the long group;
* start-up (ledger open and replica resync, acknowledged every few replayed blocks) uses the default group
  with a long timeout (``UPOW_DIST_INIT_TIMEOUT_S``, 1 h).
"""
from __future__ import annotations

import os
import threading
import time
from dataclasses import dataclass, field
from typing import Optional

EXIT_COLLECTIVE_FAILED = 70


@dataclass
class DistContext:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    backend: Optional[str] = None
    device: str = 'cpu'

    comm_device: str = 'cpu'  # where collective tensors live: cuda:N for RCCL, cpu for gloo
    forced: bool = False  # run collectives even for world == 1 (exercises the RCCL path on one GPU)
    group: object = None  # process group of the collectives (None: the default group)
    owner: Optional[int] = None  # thread ident allowed to issue collectives (None: any thread)
    fatal: bool = field(default_factory=lambda: os.environ.get('UPOW_DIST_FATAL', '1') != '0')
    collectives: int = 0  # issued so far (tests, /cluster_info)
    vote_call_s: float = 0.0  # host time inside the native vote's start calls (/cluster_info)

    @property
    def is_distributed(self) -> bool:
        return self.world > 1 or self.forced

    @property
    def is_main(self) -> bool:
        return self.rank == 0

    # ---------------------------------------------------------------- ownership and failure
    def bind_owner(self, ident: Optional[int] = None):
        """From now on only thread ``ident`` (default: the calling thread) may issue collectives."""
        self.owner = threading.get_ident() if ident is None else ident

    def _enter(self, what: str):
        if self.owner is not None and threading.get_ident() != self.owner:
            raise RuntimeError(f'collective {what} issued from thread {threading.current_thread().name}, '
                               f'not the owner thread: ranks would see interleaved collective sequences')
        self.collectives += 1

    def _failed(self, what: str, e: BaseException):
        """A collective failed or timed out: the ranks' sequences no longer line up, so nothing later can
        be trusted. Exit loudly (the launcher tears the other ranks down) unless UPOW_DIST_FATAL=0."""
        msg = f'rank {self.rank}/{self.world}: collective {what} failed ({type(e).__name__}: {e})'
        if not self.fatal:
            raise RuntimeError(msg) from e
        import sys
        try:
            from ..utils.logger import get_logger
            get_logger(__name__).critical(msg)
        finally:
            print(msg, file=sys.stderr, flush=True)
            os._exit(EXIT_COLLECTIVE_FAILED)

    def _run(self, what: str, fn, *args, **kw):
        self._enter(what)
        try:
            return fn(*args, group=self.group, **kw)
        except Exception as e:
            self._failed(what, e)

    # ---------------------------------------------------------------- collectives (thin wrappers)
    def _t(self, values, dtype=None):
        import torch
        return torch.tensor(values, dtype=dtype or torch.int64, device=self.comm_device)

    def _reduce(self, values, op, dtype=None, what: str = 'all_reduce') -> list:
        """All-reduce of a short vector through buffers kept for the process (a pinned host staging vector
        and its device twin for RCCL): no allocation and no pageable copy per call. The per-block commit
        vote of a cluster node is one of these, so its fixed cost is what a block pays for agreement."""
        import torch
        import torch.distributed as dist
        dtype = dtype or torch.int64
        key = (dtype, len(values))
        bufs = self.__dict__.setdefault('_rbuf', {})
        pair = bufs.get(key)
        if pair is None:
            gpu = self.comm_device != 'cpu'
            host = torch.zeros(len(values), dtype=dtype, pin_memory=gpu)
            pair = bufs[key] = (host, torch.zeros(len(values), dtype=dtype, device=self.comm_device) if gpu else host)
        host, dev = pair
        h = host.numpy()
        h[:] = values
        if dev is not host:
            dev.copy_(host, non_blocking=True)
        self._run(what, dist.all_reduce, dev, op=op)
        if dev is not host:
            host.copy_(dev, non_blocking=True)
            torch.cuda.current_stream().synchronize()
        return h.tolist()

    def vote_start(self, v: int):
        """Split-phase agreement on one small int (the cluster's per-block commit vote): every rank's value is
        gathered (``all_gather_into_tensor`` from a constant device tensor: no host-to-device copy; the
        device-to-host copy of the gathered vector into pinned memory and an event are queued behind it) and
        the host goes on; :meth:`vote_finish` waits and returns the SUM. Every rank votes through this pair,
        ready or not, so the collectives pair up. Nothing else may be issued in between."""
        if not self.is_distributed:
            return ('done', int(v))
        nv = self._native_vote()
        if nv is not None:  # RCCL: the native communicator of csrc/rccl_vote.hip
            L, h = nv
            self._enter('vote')
            t0 = time.perf_counter()
            try:
                L.rccl_vote_start(h, 1 if v else 0)
            except Exception as e:
                self._failed('vote', e)
            self.vote_call_s += time.perf_counter() - t0  # the native call alone (cluster info: vote_call_us)
            return ('native', L, h)
        import torch
        import torch.distributed as dist
        st = self.__dict__.get('_vote')
        if st is None:
            gpu = self.comm_device != 'cpu'
            consts = {k: torch.full((1,), k, dtype=torch.int64, device=self.comm_device) for k in (0, 1)}
            out = torch.zeros(self.world, dtype=torch.int64, device=self.comm_device)
            host = torch.zeros(self.world, dtype=torch.int64, pin_memory=gpu) if gpu else out
            ev = torch.cuda.Event() if gpu else None
            st = self._vote = (consts, out, host, ev)
        consts, out, host, ev = st
        src = consts.get(int(v))
        if src is None:
            src = torch.full((1,), int(v), dtype=torch.int64, device=self.comm_device)
        self._run('all_gather(vote)', dist.all_gather_into_tensor, out, src)
        if ev is None:  # gloo: synchronous
            return ('done', int(host.sum()))
        host.copy_(out, non_blocking=True)
        ev.record()
        return ('pending', host, ev)

    def _native_vote(self):
        """(lib, handle) of this context's native vote communicator on an RCCL job (created at the first
        vote: rank 0's unique id goes out in one broadcast on this context's group, then every rank joins),
        None on gloo or with UPOW_NATIVE_VOTE=0."""
        nv = self.__dict__.get('_nv', False)
        if nv is not False:
            return nv
        nv = None
        if self.comm_device != 'cpu' and os.environ.get('UPOW_NATIVE_VOTE', '1') != '0':
            from ..ops.native import lib
            L = lib()
            uid = self.broadcast_bytes(L.rccl_unique_id() if self.rank == 0 else None, src=0, max_len=128)
            self._enter('vote communicator')
            try:
                nv = (L, L.rccl_vote_create(uid, self.world, self.rank))
            except Exception as e:
                self._failed('vote communicator', e)
        self._nv = nv
        return nv

    def vote_finish(self, handle) -> int:
        if handle[0] == 'done':
            return handle[1]
        if handle[0] == 'native':
            _, L, h = handle
            n = L.rccl_vote_finish(h, float(os.environ.get('UPOW_DIST_TIMEOUT_S', '60')))
            if n < 0:
                self._failed('vote', TimeoutError('no outcome within UPOW_DIST_TIMEOUT_S'))
            return int(n)
        _, host, ev = handle
        try:
            ev.synchronize()
        except Exception as e:
            self._failed('all_gather(vote)', e)
        return int(host.numpy().sum())

    def allreduce_min(self, v: int) -> int:
        if not self.is_distributed:
            return int(v)
        import torch.distributed as dist
        return int(self._reduce([int(v)], dist.ReduceOp.MIN, what='all_reduce(min)')[0])

    def allreduce_min_vec(self, values) -> list:
        """Element-wise MIN of a short int vector: several per-step agreements in ONE collective."""
        if not self.is_distributed:
            return [int(v) for v in values]
        import torch.distributed as dist
        return [int(x) for x in self._reduce([int(v) for v in values], dist.ReduceOp.MIN, what='all_reduce(min vec)')]

    def allreduce_sum_vec(self, values) -> list:
        """Element-wise SUM of a short int vector in ONE collective."""
        if not self.is_distributed:
            return [int(v) for v in values]
        import torch.distributed as dist
        return [int(x) for x in self._reduce([int(v) for v in values], dist.ReduceOp.SUM, what='all_reduce(sum vec)')]

    def allreduce_max_f(self, v: float) -> float:
        if not self.is_distributed:
            return float(v)
        import torch
        import torch.distributed as dist
        return float(self._reduce([float(v)], dist.ReduceOp.MAX, dtype=torch.float64, what='all_reduce(max)')[0])

    def allreduce_sum(self, v: int) -> int:
        if not self.is_distributed:
            return int(v)
        import torch.distributed as dist
        return int(self._reduce([int(v)], dist.ReduceOp.SUM, what='all_reduce(sum)')[0])

    def broadcast_bytes(self, data: Optional[bytes], src: int, max_len: int = 256) -> bytes:
        """Broadcast a byte string from ``src``. Payloads up to ``max_len`` (e.g. the 108-byte header)
        take ONE fixed-size RCCL broadcast; longer ones (a mining job with thousands of tx hashes)
        first broadcast their length."""
        if not self.is_distributed:
            return bytes(data or b'')
        import torch
        import torch.distributed as dist
        me = self.rank == src
        n_src = len(data) if (me and data is not None) else 0
        size = max_len
        if max_len <= 0:
            t = self._t([n_src])
            self._run('broadcast(len)', dist.broadcast, t, src=src)
            size = n_src if me else int(t.item())  # the source knows its length: no host sync there
        if me:
            assert data is not None and len(data) <= size, 'payload larger than max_len (use max_len=0)'
            # the frame goes out from a pinned staging copy, asynchronously on the communicator's stream:
            # the source returns as soon as the broadcast is queued (a later host sync, e.g. the block
            # verdict's all-reduce, orders it) and never reads its own payload back
            import numpy as np
            host, slot = self._staging(size + 4)
            h = host.numpy()
            h[:4] = np.frombuffer(len(data).to_bytes(4, 'little'), np.uint8)
            h[4:4 + len(data)] = np.frombuffer(data, np.uint8)
            h[4 + len(data):size + 4] = 0
            if self.comm_device != 'cpu':
                buf = host[:size + 4].to(self.comm_device, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record()  # the staging slot is free again once the copy has read it
                slot[1] = ev
            else:
                buf = host[:size + 4].clone()
            self._run('broadcast(bytes)', dist.broadcast, buf, src=src)
            return bytes(data)
        buf = torch.empty(size + 4, dtype=torch.uint8, device=self.comm_device)
        self._run('broadcast(bytes)', dist.broadcast, buf, src=src)
        raw = bytes(buf.cpu().numpy().tobytes())
        n = int.from_bytes(raw[:4], 'little')
        return raw[4:4 + n]

    FRAME_CAP = int(os.environ.get('UPOW_DIST_FRAME_KB', '64')) << 10

    def broadcast_frame(self, data: Optional[bytes], src: int) -> bytes:
        """One op frame from ``src`` in ONE fixed-capacity broadcast when it fits (``FRAME_CAP``, 64 KB: the
        cluster's status, ping, heartbeat and mempool-batch ops), two for larger frames (a block): the first
        carries the total length and the head of the payload, the second the exact remainder. Receivers keep
        one device-resident frame buffer across ops (no allocation per op)."""
        if not self.is_distributed:
            return bytes(data or b'')
        import numpy as np
        import torch
        import torch.distributed as dist
        cap = self.FRAME_CAP
        me = self.rank == src
        if me:
            data = bytes(data or b'')
            total = len(data)
            head = data[:cap - 4]
            host, slot = self._staging(cap)
            h = host.numpy()
            h[:4] = np.frombuffer(total.to_bytes(4, 'little'), np.uint8)
            h[4:4 + len(head)] = np.frombuffer(head, np.uint8)
            if self.comm_device != 'cpu':
                buf = host[:cap].to(self.comm_device, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record()
                slot[1] = ev
            else:
                buf = host[:cap].clone()
            self._run('broadcast(frame)', dist.broadcast, buf, src=src)
            if total > cap - 4:
                rest = data[cap - 4:]
                host2, slot2 = self._staging(len(rest))
                host2.numpy()[:len(rest)] = np.frombuffer(rest, np.uint8)
                if self.comm_device != 'cpu':
                    buf2 = host2[:len(rest)].to(self.comm_device, non_blocking=True)
                    ev2 = torch.cuda.Event()
                    ev2.record()
                    slot2[1] = ev2
                else:
                    buf2 = host2[:len(rest)].clone()
                self._run('broadcast(frame tail)', dist.broadcast, buf2, src=src)
            return data
        buf = self.__dict__.get('_frame_rx')
        if buf is None or buf.numel() != cap:
            buf = torch.empty(cap, dtype=torch.uint8, device=self.comm_device)
            self.__dict__['_frame_rx'] = buf
        self._run('broadcast(frame)', dist.broadcast, buf, src=src)
        raw = buf.cpu().numpy()
        total = int.from_bytes(raw[:4].tobytes(), 'little')
        if total <= cap - 4:
            return raw[4:4 + total].tobytes()
        tail = torch.empty(total - (cap - 4), dtype=torch.uint8, device=self.comm_device)
        self._run('broadcast(frame tail)', dist.broadcast, tail, src=src)
        return raw[4:].tobytes() + tail.cpu().numpy().tobytes()

    def all_gather_fixed(self, data: bytes) -> list:
        """All-gather of a byte string every rank sends with the SAME length: one collective."""
        if not self.is_distributed:
            return [bytes(data)]
        import torch
        import torch.distributed as dist
        buf = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(self.comm_device)
        outs = [torch.empty_like(buf) for _ in range(self.world)]
        self._run('all_gather(fixed)', dist.all_gather, outs, buf)
        return [o.cpu().numpy().tobytes() for o in outs]

    def _staging(self, n: int):
        """A pinned host buffer of at least ``n`` bytes and its slot ``[buffer, copy-done event]``, reused
        across broadcasts: two slots alternate, and a slot is written again only after the async copy of
        its previous frame has completed (its event)."""
        import torch
        slots = self.__dict__.setdefault('_stage', [[None, None], [None, None]])
        k = self.__dict__.get('_stage_k', 0) ^ 1
        self.__dict__['_stage_k'] = k
        slot = slots[k]
        if slot[1] is not None:
            slot[1].synchronize()
            slot[1] = None
        if slot[0] is None or slot[0].numel() < n:
            slot[0] = torch.empty(max(n, 1 << 16), dtype=torch.uint8, pin_memory=self.comm_device != 'cpu')
        return slot[0], slot

    def all_gather_bytes(self, data: bytes) -> list:
        """Variable-length all-gather (size all-gather, then a padded all-gather)."""
        if not self.is_distributed:
            return [bytes(data)]
        import torch
        import torch.distributed as dist
        n = self._t([len(data)])
        sizes = [torch.zeros_like(n) for _ in range(self.world)]
        self._run('all_gather(len)', dist.all_gather, sizes, n)
        mx = max(int(s.item()) for s in sizes)
        buf = torch.zeros(max(mx, 1), dtype=torch.uint8, device=self.comm_device)
        if data:
            buf[:len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(self.comm_device)
        outs = [torch.zeros_like(buf) for _ in range(self.world)]
        self._run('all_gather(bytes)', dist.all_gather, outs, buf)
        return [bytes(o.cpu().numpy().tobytes()[:int(s.item())]) for o, s in zip(outs, sizes)]

    def barrier(self):
        if self.is_distributed:
            import torch.distributed as dist
            if self.backend == 'nccl':
                import torch
                self._run('barrier', dist.barrier, device_ids=[torch.cuda.current_device()])
            else:
                self._run('barrier', dist.barrier)

    def synchronize(self):
        if self.device.startswith('cuda'):
            import torch
            torch.cuda.synchronize()


def init_from_env(backend: Optional[str] = None, want_gpu: bool = True) -> DistContext:
    """Initialise from torchrun's RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* (127.0.0.1 rendezvous)."""
    rank = int(os.environ.get('RANK', '0'))
    world = int(os.environ.get('WORLD_SIZE', '1'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    ctx = DistContext(rank=rank, world=world, local_rank=local)
    gpu = False
    if want_gpu:
        try:
            import torch
            gpu = torch.cuda.is_available()
            if gpu:
                torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
                ctx.device = f'cuda:{torch.cuda.current_device()}'
        except Exception:
            gpu = False
        if gpu:
            # node-side native GPU calls from any thread of this rank (ledger worker, executors) go to
            # the rank's GPU, not to the device 0 a fresh thread starts on
            from ..ops.native import lib
            lib().set_node_device(int(ctx.device.split(':')[1]))
    force = os.environ.get('UPOW_FORCE_DIST', '0') == '1' and 'MASTER_PORT' in os.environ
    if world > 1 or force:
        ctx.forced = world == 1
        import torch.distributed as dist
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        # UPOW_DIST_BACKEND=gloo: host collectives with GPU compute (several ranks sharing one GPU, e.g. a
        # multi-rank cluster measured on a one-GPU box; RCCL needs one GPU per rank)
        be = backend or os.environ.get('UPOW_DIST_BACKEND') or ('nccl' if gpu else 'gloo')
        from datetime import timedelta
        init_timeout = timedelta(seconds=float(os.environ.get('UPOW_DIST_INIT_TIMEOUT_S', '3600')))
        if not dist.is_initialized():
            if be == 'nccl':
                import torch
                dist.init_process_group(be, rank=rank, world_size=world, timeout=init_timeout,
                                        device_id=torch.device(ctx.device))
            else:
                dist.init_process_group(be, rank=rank, world_size=world, timeout=init_timeout)
        ctx.backend = be
        ctx.comm_device = ctx.device if be == 'nccl' else 'cpu'
    return ctx


def op_context(ctx: DistContext) -> DistContext:
    """A copy of ``ctx`` whose collectives run on a new process group with the short op timeout
    (``UPOW_DIST_TIMEOUT_S``): the cluster's steady-state op traffic. Collective (every rank calls it)."""
    if not ctx.is_distributed:
        return ctx
    import dataclasses
    from datetime import timedelta

    import torch.distributed as dist
    t = timedelta(seconds=float(os.environ.get('UPOW_DIST_TIMEOUT_S', '60')))
    ctx._enter('new_group')
    try:
        g = dist.new_group(ranks=list(range(ctx.world)), timeout=t, backend=ctx.backend)
    except Exception as e:
        ctx._failed('new_group', e)
    return dataclasses.replace(ctx, group=g, collectives=0)


def shutdown(ctx: DistContext):
    if ctx.is_distributed:
        import torch.distributed as dist
        if dist.is_initialized():
            dist.destroy_process_group()
