"""Admission, channel registry, fan-out and housekeeping for ``/ws`` sessions.

- Admission: at most ``limits.max_sockets`` live sessions; an extra client is refused before the
  handshake completes (reference socket_manager.py:63-68 raises before ``accept``, which ends in the
  same HTTP 403 denial).
- Registry: ``channel -> WeakSet[Session]``. A session that disappears without unsubscribing cannot
  leak into a channel.
- Publish: the event is encoded ONCE and handed to every member's outbox with ``put_nowait``; the
  publisher never awaits a client (see session.py).
- One housekeeping task for all sessions (instead of two timers per socket): heartbeats every
  ``limits.heartbeat`` s, idle close (1001, "Connection timeout") after ``limits.idle_close`` s
  without a valid client frame, and a stats line every ``limits.stats_every`` s
  (reference behaviour: socket_connection.py:327-351, socket_manager.py:333-372).
"""
from __future__ import annotations

import asyncio
import time
import uuid
import weakref
from typing import Any, Dict, Optional

from ..utils.logger import get_logger
from . import protocol
from .config import CHANNELS, Limits, client_verbs
from .session import Session

logger = get_logger(__name__)


class Hub:
    def __init__(self, limits: Optional[Limits] = None):
        self.limits = limits or Limits.from_env()
        self.verbs = client_verbs()
        self.sessions: Dict[str, Session] = {}
        self.members: Dict[str, weakref.WeakSet] = {c: weakref.WeakSet() for c in CHANNELS}
        self.refused = 0
        self.published = 0
        self._chores: Optional[asyncio.Task] = None

    # ------------------------------------------------------------------ sessions
    async def serve(self, socket) -> None:
        if len(self.sessions) >= self.limits.max_sockets:
            self.refused += 1
            logger.warning(f'ws: refusing client, {len(self.sessions)} sockets open (cap {self.limits.max_sockets})')
            await socket.close(code=1013)
            return
        await socket.accept()
        client = getattr(socket, 'client', None)
        s = Session(self, socket, uuid.uuid4().hex, f'{client.host}:{client.port}' if client else '')
        self.sessions[s.sid] = s
        logger.info(f'ws {s.sid} open ({s.peer}); {len(self.sessions)} sockets')
        try:
            await s.serve()
        finally:
            self.sessions.pop(s.sid, None)
            for ch in list(s.channels):
                self.leave(s, ch)
            logger.info(f'ws {s.sid} closed {s.shut_with}; {len(self.sessions)} sockets')

    def join(self, s: Session, channel: str) -> bool:
        group = self.members.get(channel)
        if group is None:
            return False
        group.add(s)
        s.channels.add(channel)
        return True

    def leave(self, s: Session, channel: str) -> bool:
        if channel not in s.channels:
            return False
        s.channels.discard(channel)
        group = self.members.get(channel)
        if group is not None:
            group.discard(s)
        return True

    # ------------------------------------------------------------------ fan-out
    def listening(self, channel: str) -> bool:
        """Whether any session is subscribed to ``channel`` (callers skip building unsent events)."""
        return bool(self.members.get(channel))

    def publish(self, channel: str, kind: str, data: Any) -> int:
        """Queue ``{"type": kind, "data": data}`` for every member of ``channel``; returns how many
        sessions accepted it. Never awaits a client."""
        group = self.members.get(channel)
        if not group:
            return 0
        text = protocol.encode(protocol.event_frame(kind, data))
        if len(text.encode('utf-8')) > self.limits.frame_bytes:
            logger.warning(f'ws: {kind} event of {len(text)} B exceeds the frame limit, not sent')
            return 0
        self.published += 1
        return sum(1 for s in list(group) if s.offer(text))

    # ------------------------------------------------------------------ housekeeping
    def sweep(self, now: Optional[float] = None) -> None:
        now = time.monotonic() if now is None else now
        lim = self.limits
        for s in list(self.sessions.values()):
            if s.shut_with is not None:
                continue
            if now - s.last_seen > lim.idle_close:
                logger.info(f'ws {s.sid}: idle for {now - s.last_seen:.0f} s, closing')
                s.shut(1001, 'Connection timeout')
            elif now - s.last_beat >= lim.heartbeat:
                s.last_beat = now
                s.reply(protocol.beat_frame('ping'))

    async def _chore_loop(self):
        last_stats = time.monotonic()
        while True:
            await asyncio.sleep(self.limits.tick)
            try:
                self.sweep()
                now = time.monotonic()
                if now - last_stats >= self.limits.stats_every:
                    last_stats = now
                    st = self.stats()
                    logger.info(f"ws stats: {st['sockets']} sockets, channels {st['channels']}, "
                                f"{st['published']} events published, {st['refused']} refused")
            except Exception as e:
                logger.error(f'ws housekeeping: {e}')

    async def start(self):
        if self._chores is None or self._chores.done():
            self._chores = asyncio.ensure_future(self._chore_loop())

    async def stop(self):
        if self._chores is not None:
            self._chores.cancel()
            await asyncio.gather(self._chores, return_exceptions=True)
            self._chores = None
        for s in list(self.sessions.values()):
            s.shut(1001, 'Server shutting down')

    def stats(self, detail: bool = False) -> dict:
        out = {'sockets': len(self.sessions), 'channels': {c: len(g) for c, g in self.members.items()},
               'published': self.published, 'refused': self.refused, 'timestamp': protocol.utc_stamp()}
        if detail:
            out['sessions'] = [s.summary() for s in self.sessions.values()]
        return out
