"""Ledger worker: block validation and application on a thread of its own, off the HTTP event loop.

reference: ``POST /push_block`` awaits ``create_block`` on the node's single asyncio loop
(upow/node/main.py:521-652 → manager.py:650-757); while a block is checked and written, every other
request (``/push_tx``, ``/get_mining_info``, ``/ws`` traffic) waits for the loop. Here the node hands
block work to one dedicated thread running its own event loop: the HTTP loop awaits a future and keeps
serving, while the ledger thread decodes, launches the GPU passes and commits (the native calls
release the GIL). All block mutations (push, sync, rollback) run on that one loop, so ``ledger_lock``
still serialises them in arrival order.

``UPOW_LEDGER_THREAD=0`` runs the same coroutines inline on the caller's loop.
"""
from __future__ import annotations

import asyncio
import os
import threading
from typing import Awaitable, Callable, Optional

from ..utils.logger import get_logger

logger = get_logger(__name__)


class LedgerWorker:
    def __init__(self, name: str = 'upow-ledger'):
        self.loop = asyncio.new_event_loop()
        self._ready = threading.Event()
        self.thread = threading.Thread(target=self._main, name=name, daemon=True)
        self.thread.start()
        self._ready.wait()
        self.busy_s = 0.0
        self.jobs = 0

    def _main(self):
        asyncio.set_event_loop(self.loop)
        self.loop.call_soon(self._ready.set)
        self.loop.run_forever()
        # drain callbacks scheduled during shutdown, then close
        self.loop.run_until_complete(asyncio.sleep(0))
        self.loop.close()

    def on_thread(self) -> bool:
        return threading.current_thread() is self.thread

    async def run(self, fn: Callable[..., Awaitable], *args, **kwargs):
        """``await fn(*args, **kwargs)`` on the ledger thread (inline when already on it)."""
        if self.on_thread():
            return await fn(*args, **kwargs)
        import time

        async def timed():
            t0 = time.perf_counter()
            try:
                return await fn(*args, **kwargs)
            finally:
                self.busy_s += time.perf_counter() - t0
                self.jobs += 1
        fut = asyncio.run_coroutine_threadsafe(timed(), self.loop)
        return await asyncio.wrap_future(fut)

    def stop(self, timeout: float = 30.0):
        if not self.thread.is_alive():
            return
        self.loop.call_soon_threadsafe(self.loop.stop)
        self.thread.join(timeout)


_worker: Optional[LedgerWorker] = None
_lock = threading.Lock()


def enabled() -> bool:
    return os.environ.get('UPOW_LEDGER_THREAD', '1') != '0'


def start() -> Optional[LedgerWorker]:
    global _worker
    with _lock:
        if _worker is None and enabled():
            # the GIL changes hands every switch interval when both threads run Python: at CPython's
            # 5 ms default a request arriving during a block's Python stages waits up to 5 ms per turn, and
            # the HTTP loop gives the GIL away at every socket call (recv, send, epoll), so each request
            # can pay that wait several times. 0.25 ms: soaks at 1,200 tx/s measured lower push latency
            # during block apply than at 1 ms, with no slower block apply (docs/PERF.md §3)
            import sys
            sys.setswitchinterval(float(os.environ.get('UPOW_SWITCH_INTERVAL_MS', '0.25')) / 1000.0)
            _worker = LedgerWorker()
            logger.info('ledger worker thread started')
        return _worker


def stop():
    global _worker
    with _lock:
        w, _worker = _worker, None
    if w is not None:
        w.stop()


def get() -> Optional[LedgerWorker]:
    return _worker


async def on_ledger(fn: Callable[..., Awaitable], *args, **kwargs):
    """Run a ledger coroutine function on the ledger thread when the worker is running, inline otherwise."""
    w = _worker
    if w is None:
        return await fn(*args, **kwargs)
    return await w.run(fn, *args, **kwargs)


__all__ = ['LedgerWorker', 'on_ledger', 'start', 'stop', 'get', 'enabled']
