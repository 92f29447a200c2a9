"""Process-group bootstrap: one process per GPU, ``torch.distributed`` over RCCL (backend "nccl").

MI355X topology: 8 GPUs per node, fully connected by 7 xGMI links each. Every collective this
framework issues is small and latency-bound (8-byte flags, 108-byte headers, <=2 MB blocks,
mempool deltas), so there is no bucketing: each exchange is one RCCL call on the
default stream, and the messages ride the LL/LL128 protocols over the direct links.

Tests use the same code with the ``gloo`` backend on CPU (world_size > 1 on one host).
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Optional


@dataclass
class DistContext:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    backend: Optional[str] = None
    device: str = 'cpu'

    comm_device: str = 'cpu'  # where collective tensors live: cuda:N for RCCL, cpu for gloo
    forced: bool = False  # run collectives even for world == 1 (exercises the RCCL path on one GPU)

    @property
    def is_distributed(self) -> bool:
        return self.world > 1 or self.forced

    @property
    def is_main(self) -> bool:
        return self.rank == 0

    # ---------------------------------------------------------------- collectives (thin wrappers)
    def _t(self, values, dtype=None):
        import torch
        return torch.tensor(values, dtype=dtype or torch.int64, device=self.comm_device)

    def allreduce_min(self, v: int) -> int:
        if not self.is_distributed:
            return int(v)
        import torch.distributed as dist
        t = self._t([v])
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return int(t.item())

    def allreduce_min_vec(self, values) -> list:
        """Element-wise MIN of a short int vector: several per-step agreements in ONE collective."""
        if not self.is_distributed:
            return [int(v) for v in values]
        import torch.distributed as dist
        t = self._t(list(values))
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return [int(x) for x in t.tolist()]

    def allreduce_sum_vec(self, values) -> list:
        """Element-wise SUM of a short int vector in ONE collective."""
        if not self.is_distributed:
            return [int(v) for v in values]
        import torch.distributed as dist
        t = self._t(list(values))
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return [int(x) for x in t.tolist()]

    def allreduce_max_f(self, v: float) -> float:
        if not self.is_distributed:
            return float(v)
        import torch
        import torch.distributed as dist
        t = self._t([v], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def allreduce_sum(self, v: int) -> int:
        if not self.is_distributed:
            return int(v)
        import torch.distributed as dist
        t = self._t([v])
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return int(t.item())

    def broadcast_bytes(self, data: Optional[bytes], src: int, max_len: int = 256) -> bytes:
        """Broadcast a byte string from ``src``. Payloads up to ``max_len`` (e.g. the 108-byte header)
        take ONE fixed-size RCCL broadcast; longer ones (a mining job with thousands of tx hashes)
        first broadcast their length."""
        if not self.is_distributed:
            return bytes(data or b'')
        import torch
        import torch.distributed as dist
        n_src = len(data) if (self.rank == src and data is not None) else 0
        size = max_len
        if max_len <= 0:
            t = self._t([n_src])
            dist.broadcast(t, src=src)
            size = int(t.item())
        buf = torch.zeros(size + 4, dtype=torch.uint8, device=self.comm_device)
        if self.rank == src:
            assert data is not None and len(data) <= size, 'payload larger than max_len (use max_len=0)'
            payload = len(data).to_bytes(4, 'little') + data
            buf[:len(payload)] = torch.frombuffer(bytearray(payload), dtype=torch.uint8).to(self.comm_device)
        dist.broadcast(buf, src=src)
        raw = bytes(buf.cpu().numpy().tobytes())
        n = int.from_bytes(raw[:4], 'little')
        return raw[4:4 + n]

    def all_gather_bytes(self, data: bytes) -> list:
        """Variable-length all-gather (size all-gather, then a padded all-gather)."""
        if not self.is_distributed:
            return [bytes(data)]
        import torch
        import torch.distributed as dist
        n = self._t([len(data)])
        sizes = [torch.zeros_like(n) for _ in range(self.world)]
        dist.all_gather(sizes, n)
        mx = max(int(s.item()) for s in sizes)
        buf = torch.zeros(max(mx, 1), dtype=torch.uint8, device=self.comm_device)
        if data:
            buf[:len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(self.comm_device)
        outs = [torch.zeros_like(buf) for _ in range(self.world)]
        dist.all_gather(outs, buf)
        return [bytes(o.cpu().numpy().tobytes()[:int(s.item())]) for o, s in zip(outs, sizes)]

    def barrier(self):
        if self.is_distributed:
            import torch.distributed as dist
            if self.backend == 'nccl':
                import torch
                dist.barrier(device_ids=[torch.cuda.current_device()])
            else:
                dist.barrier()

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
        be = backend or ('nccl' if gpu else 'gloo')
        if not dist.is_initialized():
            if be == 'nccl':
                import torch
                dist.init_process_group(be, rank=rank, world_size=world,
                                        device_id=torch.device(ctx.device))
            else:
                dist.init_process_group(be, rank=rank, world_size=world)
        ctx.backend = be
        ctx.comm_device = ctx.device if be == 'nccl' else 'cpu'
    return ctx


def shutdown(ctx: DistContext):
    if ctx.is_distributed:
        import torch.distributed as dist
        if dist.is_initialized():
            dist.destroy_process_group()
