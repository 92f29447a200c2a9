"""One ``/ws`` client: a reader task, a writer task and a bounded outbox between them.

Design (independent of the reference's per-connection object): the socket is owned by two tasks.

- ``_read``: takes a token from the client's bucket, awaits the next frame, validates it
  (:func:`protocol.decode_client_frame`) and runs the verb. Replies never touch the socket: they
  are queued.
- ``_write``: drains the outbox to the socket and performs the close handshake when the session is
  shut. A broadcast therefore costs one ``put_nowait`` per subscriber, and a slow or dead client can
  only fill its own outbox — when it overflows the client is dropped (1008) instead of stalling the
  publisher (the reference awaits every subscriber's send in turn, socket_manager.py:214-224).

Client-visible behaviour kept from the reference (websocket/socket_connection.py:149-268,
socket_handlers.py:67-143): a pong per ping; ``subscribe_block`` answers with two success frames;
``unsubscribe_block`` when not subscribed answers ``NOT_SUBSCRIBED`` followed by the generic success;
every rejected frame gets one error frame and the socket is closed (1000); the rate check runs
before each receive, so the frame after a full burst is refused.
"""
from __future__ import annotations

import asyncio
import time

from ..utils.logger import get_logger
from . import protocol

logger = get_logger(__name__)

_SHUT = object()  # outbox sentinel: close the socket after what is queued before it


class TokenBucket:
    """``burst`` tokens, refilled continuously at burst/window per second."""

    __slots__ = ('burst', 'rate', 'level', 'stamp', 'clock')

    def __init__(self, burst: int, window: float, clock=time.monotonic):
        self.burst = float(burst)
        self.rate = burst / window if window > 0 else float('inf')
        self.level = float(burst)
        self.clock = clock
        self.stamp = clock()

    def take(self) -> bool:
        now = self.clock()
        self.level = min(self.burst, self.level + (now - self.stamp) * self.rate)
        self.stamp = now
        if self.level >= 1.0:
            self.level -= 1.0
            return True
        return False


class Session:
    def __init__(self, hub, socket, sid: str, peer: str = ''):
        self.hub = hub
        self.socket = socket
        self.sid = sid
        self.peer = peer
        lim = hub.limits
        self.bucket = TokenBucket(lim.burst, lim.burst_window)
        self.outbox: asyncio.Queue = asyncio.Queue()  # bounded by hand in offer(): _SHUT must always fit
        self.channels: set = set()
        now = time.monotonic()
        self.opened = self.last_seen = self.last_beat = now
        self.shut_with = None        # (code, reason) once closing was requested
        self.peer_gone = False       # the client closed first: no close handshake to send
        self.frames_in = self.frames_out = self.bytes_in = self.bytes_out = self.dropped = 0

    # ------------------------------------------------------------------ outbound
    def offer(self, text: str) -> bool:
        """Queue an encoded frame (never blocks). False if the session is closing or overflowed."""
        if self.shut_with is not None:
            return False
        if self.outbox.qsize() >= self.hub.limits.outbox:
            self.dropped += 1
            logger.warning(f'ws {self.sid}: outbox full ({self.hub.limits.outbox} frames), dropping slow client')
            self.shut(1008, 'Send queue overflow', flush=False)
            return False
        self.outbox.put_nowait(text)
        return True

    def reply(self, frame: dict) -> bool:
        return self.offer(protocol.encode(frame))

    def shut(self, code: int = 1000, reason: str = 'Connection closed', flush: bool = True):
        if self.shut_with is not None:
            return
        self.shut_with = (code, reason)
        if not flush:
            while not self.outbox.empty():
                self.outbox.get_nowait()
        self.outbox.put_nowait(_SHUT)

    async def _write(self):
        try:
            while True:
                item = await self.outbox.get()
                if item is _SHUT:
                    break
                await self.socket.send_text(item)
                self.frames_out += 1
                self.bytes_out += len(item)
        except Exception as e:  # socket already gone
            self.peer_gone = True
            logger.debug(f'ws {self.sid}: send failed: {e}')
        finally:
            if not self.peer_gone:
                code, reason = self.shut_with or (1000, 'Connection closed')
                try:
                    await self.socket.close(code=code, reason=reason)
                except Exception:
                    pass

    # ------------------------------------------------------------------ inbound
    async def _read(self):
        lim = self.hub.limits
        verbs = self.hub.verbs
        while self.shut_with is None:
            if not self.bucket.take():
                self.reply(protocol.error_frame('RATE_LIMIT_EXCEEDED', 'Too many messages sent'))
                self.shut()
                return
            event = await self.socket.receive()
            if event['type'] == 'websocket.disconnect':
                self.peer_gone = True
                self.shut(event.get('code', 1000), 'client closed', flush=False)
                return
            raw = event.get('text')
            if raw is None:
                raw = event.get('bytes') or b''
            try:
                msg, size = protocol.decode_client_frame(raw, lim.frame_bytes, verbs)
            except protocol.Reject as r:
                self.reply(protocol.error_frame(r.code, r.text))
                self.shut()
                return
            self.frames_in += 1
            self.bytes_in += size
            self.last_seen = time.monotonic()
            self._run_verb(msg['type'])

    def _run_verb(self, verb: str):
        # verbs are "<action>" or "<action>_<channel>" (ping, pong, subscribe_block, ...)
        action, _, channel = verb.partition('_')
        if action == 'ping':
            self.reply(protocol.beat_frame('pong'))
        elif action == 'subscribe':
            self.hub.join(self, channel)
            self.reply(protocol.success_frame(f'Subscribed to {channel}', {'channel': channel}))
            self.reply(protocol.success_frame(f'Subscribed to {channel} updates', {'type': f'{channel}_subscription'}))
        elif action == 'unsubscribe':
            if self.hub.leave(self, channel):
                self.reply(protocol.success_frame(f'Unsubscribed from {channel}', {'channel': channel}))
            else:
                self.reply(protocol.error_frame('NOT_SUBSCRIBED', f"Not subscribed to channel '{channel}'"))
            self.reply(protocol.success_frame(f'Unsubscribed from {channel} updates',
                                              {'type': f'{channel}_unsubscription'}))
        # 'pong' only refreshes last_seen (done by the caller)

    # ------------------------------------------------------------------ lifetime
    async def serve(self):
        """Run until either side closes. Returns when both tasks are done."""
        reader = asyncio.ensure_future(self._read())
        writer = asyncio.ensure_future(self._write())
        try:
            done, _ = await asyncio.wait({reader, writer}, return_when=asyncio.FIRST_COMPLETED)
            if writer in done:          # closed by the server side (idle, overflow, shutdown)
                reader.cancel()
            else:                       # client left or broke the protocol: let the outbox drain
                if reader.exception() is not None and self.shut_with is None:
                    self.peer_gone = True
                    self.shut(1011, 'internal error', flush=False)
                await asyncio.wait({writer}, timeout=5.0)
                writer.cancel()
        finally:
            for t in (reader, writer):
                if not t.done():
                    t.cancel()
            await asyncio.gather(reader, writer, return_exceptions=True)

    def summary(self) -> dict:
        return {'id': self.sid, 'peer': self.peer, 'channels': sorted(self.channels),
                'age_s': round(time.monotonic() - self.opened, 1), 'frames_in': self.frames_in,
                'frames_out': self.frames_out, 'bytes_in': self.bytes_in, 'bytes_out': self.bytes_out,
                'queued': self.outbox.qsize(), 'dropped': self.dropped}
