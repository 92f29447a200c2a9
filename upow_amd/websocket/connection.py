"""One client connection: send/receive with size + rate limits, heartbeat, idle expiry.

reference: websocket/socket_connection.py:31-368 (same message shapes and error codes).
"""
from __future__ import annotations

import asyncio
import json
import time
import uuid
from dataclasses import dataclass, field
from datetime import datetime, timezone
from decimal import Decimal
from typing import Any, Dict, Optional, Set

from ..utils.logger import get_logger
from . import config as C

logger = get_logger(__name__)


def _now() -> str:
    return datetime.now(timezone.utc).isoformat()


class UUIDEncoder(json.JSONEncoder):
    """UUID -> str, Decimal -> float, datetime -> ISO (socket_connection.py:31-39)."""

    def default(self, obj):
        if isinstance(obj, uuid.UUID):
            return str(obj)
        if isinstance(obj, Decimal):
            return float(obj)
        if isinstance(obj, datetime):
            return obj.isoformat()
        return super().default(obj)


@dataclass
class ConnectionStats:
    connected_at: datetime = field(default_factory=lambda: datetime.now(timezone.utc))
    last_activity: datetime = field(default_factory=lambda: datetime.now(timezone.utc))
    messages_sent: int = 0
    messages_received: int = 0
    bytes_sent: int = 0
    bytes_received: int = 0
    reconnect_count: int = 0


class RateLimiter:
    """Sliding window: at most ``max_messages`` per ``window`` seconds."""

    def __init__(self, max_messages: int = C.RATE_LIMIT_MESSAGES_PER_MINUTE, window: int = C.RATE_LIMIT_WINDOW):
        self.max_messages = max_messages
        self.window = window
        self.message_times = []

    def is_allowed(self) -> bool:
        now = time.time()
        self.message_times = [t for t in self.message_times if now - t < self.window]
        if len(self.message_times) >= self.max_messages:
            return False
        self.message_times.append(now)
        return True


class WebSocketConnection:
    def __init__(self, websocket, connection_id: str, user_id: Optional[int] = None):
        self.websocket = websocket
        self.connection_id = connection_id
        self.user_id = user_id
        self.is_authenticated = False
        self.subscriptions: Set[str] = set()
        self.stats = ConnectionStats()
        self.rate_limiter = RateLimiter()
        self.is_alive = True
        self.last_heartbeat = time.time()
        self._heartbeat_task: Optional[asyncio.Task] = None
        self._cleanup_task: Optional[asyncio.Task] = None

    async def accept(self):
        await self.websocket.accept()
        self.stats.connected_at = self.stats.last_activity = datetime.now(timezone.utc)
        self._heartbeat_task = asyncio.create_task(self._heartbeat_loop())
        self._cleanup_task = asyncio.create_task(self._cleanup_loop())
        if C.LOG_CONNECTION_EVENTS:
            logger.info(f'WebSocket connection accepted: {self.connection_id}')

    async def send_message(self, message: Dict[str, Any]) -> bool:
        if not self.is_alive:
            return False
        try:
            text = json.dumps(message, cls=UUIDEncoder)
            size = len(text.encode('utf-8'))
            if size > C.MESSAGE_SIZE_LIMIT:
                logger.warning(f'Message too large for connection {self.connection_id}: {size} bytes')
                return False
            await self.websocket.send_text(text)
            self.stats.messages_sent += 1
            self.stats.bytes_sent += size
            self.stats.last_activity = datetime.now(timezone.utc)
            return True
        except Exception as e:
            logger.error(f'Error sending message to {self.connection_id}: {e}')
            await self.close()
            return False

    async def receive_message(self) -> Optional[Dict[str, Any]]:
        if not self.is_alive:
            return None
        try:
            if not self.rate_limiter.is_allowed():
                await self.send_error('RATE_LIMIT_EXCEEDED', 'Too many messages sent')
                return None
            data = await self.websocket.receive_text()
            size = len(data.encode('utf-8'))
            if size > C.MESSAGE_SIZE_LIMIT:
                await self.send_error('MESSAGE_TOO_LARGE', f'Message size exceeds {C.MESSAGE_SIZE_LIMIT} bytes')
                return None
            message = json.loads(data)
            if not isinstance(message, dict) or 'type' not in message:
                await self.send_error('INVALID_MESSAGE', "Message must be JSON object with 'type' field")
                return None
            if message['type'] not in C.ALLOWED_MESSAGE_TYPES:
                await self.send_error('INVALID_MESSAGE_TYPE', f"Message type '{message['type']}' not allowed")
                return None
            self.stats.messages_received += 1
            self.stats.bytes_received += size
            self.stats.last_activity = datetime.now(timezone.utc)
            self.last_heartbeat = time.time()
            return message
        except json.JSONDecodeError:
            await self.send_error('INVALID_JSON', 'Message must be valid JSON')
            return None
        except Exception as e:
            logger.info(f'Receive ended for {self.connection_id}: {type(e).__name__}')
            await self.close()
            return None

    async def send_error(self, error_code: str, message: str):
        await self.send_message({'type': 'error', 'error_code': error_code, 'message': message, 'timestamp': _now()})

    async def send_success(self, message: str, data: Optional[Dict] = None):
        await self.send_message({'type': 'success', 'message': message, 'data': data or {}, 'timestamp': _now()})

    async def subscribe(self, channel: str) -> bool:
        if channel not in C.SUBSCRIPTION_CHANNELS:
            await self.send_error('INVALID_CHANNEL', f"Channel '{channel}' not available")
            return False
        self.subscriptions.add(channel)
        await self.send_success(f'Subscribed to {channel}', {'channel': channel})
        return True

    async def unsubscribe(self, channel: str) -> bool:
        if channel in self.subscriptions:
            self.subscriptions.remove(channel)
            await self.send_success(f'Unsubscribed from {channel}', {'channel': channel})
            return True
        await self.send_error('NOT_SUBSCRIBED', f"Not subscribed to channel '{channel}'")
        return False

    def authenticate(self, user_id: int):
        self.user_id = user_id
        self.is_authenticated = True

    def is_subscribed_to(self, channel: str) -> bool:
        return channel in self.subscriptions

    def is_expired(self) -> bool:
        return time.time() - self.last_heartbeat > C.CONNECTION_TIMEOUT

    async def ping(self):
        await self.send_message({'type': 'ping', 'timestamp': _now()})

    async def pong(self):
        await self.send_message({'type': 'pong', 'timestamp': _now()})

    async def close(self, code: int = 1000, reason: str = 'Connection closed'):
        if not self.is_alive:
            return
        self.is_alive = False
        current = asyncio.current_task()
        for t in (self._heartbeat_task, self._cleanup_task):
            if t and t is not current:
                t.cancel()
        try:
            await self.websocket.close(code=code, reason=reason)
        except Exception:
            pass
        if C.LOG_CONNECTION_EVENTS:
            logger.info(f'WebSocket connection closed: {self.connection_id} (reason: {reason})')

    async def _heartbeat_loop(self):
        try:
            while self.is_alive:
                await asyncio.sleep(C.HEARTBEAT_INTERVAL)
                if self.is_alive:
                    await self.ping()
        except asyncio.CancelledError:
            pass

    async def _cleanup_loop(self):
        try:
            while self.is_alive:
                await asyncio.sleep(30)
                if self.is_expired():
                    await self.close(code=1001, reason='Connection timeout')
                    break
        except asyncio.CancelledError:
            pass

    def get_stats(self) -> Dict[str, Any]:
        uptime = datetime.now(timezone.utc) - self.stats.connected_at
        return {'connection_id': self.connection_id, 'user_id': self.user_id,
                'is_authenticated': self.is_authenticated, 'subscriptions': sorted(self.subscriptions),
                'uptime_seconds': uptime.total_seconds(), 'messages_sent': self.stats.messages_sent,
                'messages_received': self.stats.messages_received, 'bytes_sent': self.stats.bytes_sent,
                'bytes_received': self.stats.bytes_received, 'is_alive': self.is_alive}
