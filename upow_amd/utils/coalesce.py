"""Per-event-loop request coalescing for /push_tx admission.

reference: every ``/push_tx`` runs its checks one at a time on the node's event loop (upow/node/main.py
push_tx -> database.add_pending_transaction -> transaction.verify_pending): a signature verify and an
outpoint lookup per request, each blocking the loop for its duration.

Here the handlers of concurrent requests hand those checks to a :class:`Coalescer`: whatever arrives
while a batch is in flight forms the next batch, which runs on an executor thread (the native calls it
makes release the GIL), so the event loop never blocks on a check and, under load, one GPU launch or one
HBM-index round trip serves many requests. Requests opt in through the :data:`ADMISSION` context
variable (set by the node's /push_tx handler for its own task only), so block validation and tools keep
their synchronous calls.
"""
from __future__ import annotations

import asyncio
import contextvars
import threading
import weakref
from concurrent.futures import ThreadPoolExecutor
from typing import Any, Callable, Dict, List, Sequence

ADMISSION = contextvars.ContextVar('upow_admission_batching', default=False)

_pools: Dict[str, ThreadPoolExecutor] = {}
_pools_lock = threading.Lock()


def executor(name: str) -> ThreadPoolExecutor:
    """One single-thread executor per coalescer kind (batches of one kind run in order)."""
    with _pools_lock:
        ex = _pools.get(name)
        if ex is None:
            ex = _pools[name] = ThreadPoolExecutor(max_workers=1, thread_name_prefix=f'upow-{name}')
        return ex


class Coalescer:
    """``await c.submit(item)`` -> the item's result from ``batch_fn(items) -> results`` (same length),
    where ``batch_fn`` runs on the kind's executor thread over everything submitted meanwhile."""

    def __init__(self, loop: asyncio.AbstractEventLoop, name: str, batch_fn: Callable[[List[Any]], Sequence[Any]]):
        self.loop = loop
        self.name = name
        self.fn = batch_fn
        self.pending: List[tuple] = []
        self.running = False
        self.batches = 0
        self.items = 0

    def submit(self, item) -> asyncio.Future:
        fut = self.loop.create_future()
        self.pending.append((item, fut))
        if not self.running:
            self.running = True
            self.loop.create_task(self._drain())
        return fut

    async def _drain(self):
        try:
            while self.pending:
                batch, self.pending = self.pending, []
                try:
                    res = await self.loop.run_in_executor(executor(self.name), self.fn, [it for it, _ in batch])
                except Exception as e:  # noqa: BLE001 - handed to every waiter
                    for _, f in batch:
                        if not f.done():
                            f.set_exception(e)
                    continue
                self.batches += 1
                self.items += len(batch)
                for (_, f), v in zip(batch, res):
                    if not f.done():
                        f.set_result(v)
        finally:
            self.running = False


_registry: 'weakref.WeakKeyDictionary' = weakref.WeakKeyDictionary()


def coalescer(name: str, batch_fn: Callable[[List[Any]], Sequence[Any]]) -> Coalescer:
    """The running loop's coalescer of this kind (created on first use)."""
    loop = asyncio.get_running_loop()
    per = _registry.get(loop)
    if per is None:
        per = _registry[loop] = {}
    c = per.get(name)
    if c is None:
        c = per[name] = Coalescer(loop, name, batch_fn)
    return c


def stats() -> Dict[str, Dict[str, int]]:
    out: Dict[str, Dict[str, int]] = {}
    for per in list(_registry.values()):
        for name, c in per.items():
            s = out.setdefault(name, {'batches': 0, 'items': 0})
            s['batches'] += c.batches
            s['items'] += c.items
    return out


__all__ = ['ADMISSION', 'Coalescer', 'coalescer', 'executor', 'stats']
