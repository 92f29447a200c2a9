"""Connection registry, channel subscriptions and broadcast (reference: websocket/socket_manager.py:23-406)."""
from __future__ import annotations

import asyncio
import uuid
from collections import defaultdict
from datetime import datetime, timezone
from typing import Any, Dict, List, Optional, Set

from ..utils.logger import get_logger
from . import config as C
from .connection import WebSocketConnection

logger = get_logger(__name__)


class WebSocketManager:
    def __init__(self):
        self.connections: Dict[str, WebSocketConnection] = {}
        self.user_connections: Dict[int, Set[str]] = defaultdict(set)
        self.channel_subscribers: Dict[str, Set[str]] = defaultdict(set)
        self._cleanup_task: Optional[asyncio.Task] = None
        self._stats_task: Optional[asyncio.Task] = None
        self._tasks_started = False

    async def start_background_tasks(self):
        if self._tasks_started:
            return
        self._cleanup_task = asyncio.create_task(self._cleanup_loop())
        self._stats_task = asyncio.create_task(self._stats_loop())
        self._tasks_started = True

    async def add_connection(self, websocket, user_id: Optional[int] = None) -> WebSocketConnection:
        if len(self.connections) >= C.MAX_TOTAL_CONNECTIONS:
            raise Exception('Maximum connections reached')
        if user_id and len(self.user_connections[user_id]) >= C.MAX_CONNECTIONS_PER_IP:
            raise Exception('Maximum connections per user reached')
        connection_id = str(uuid.uuid4())
        connection = WebSocketConnection(websocket, connection_id, user_id)
        self.connections[connection_id] = connection
        if user_id:
            self.user_connections[user_id].add(connection_id)
            connection.authenticate(user_id)
        await connection.accept()
        return connection

    async def remove_connection(self, connection_id: str):
        connection = self.connections.get(connection_id)
        if connection is None:
            return
        if connection.user_id:
            self.user_connections[connection.user_id].discard(connection_id)
            if not self.user_connections[connection.user_id]:
                del self.user_connections[connection.user_id]
        for channel in connection.subscriptions.copy():
            await self._unsubscribe_connection(connection_id, channel)
        await connection.close()
        self.connections.pop(connection_id, None)

    async def subscribe_connection(self, connection_id: str, channel: str) -> bool:
        connection = self.connections.get(connection_id)
        if connection is None:
            return False
        if await connection.subscribe(channel):
            self.channel_subscribers[channel].add(connection_id)
            return True
        return False

    async def add_channel_subscriber(self, connection_id: str, channel: str) -> bool:
        if channel not in C.SUBSCRIPTION_CHANNELS:
            return False
        return await self.subscribe_connection(connection_id, channel)

    async def _unsubscribe_connection(self, connection_id: str, channel: str):
        self.channel_subscribers[channel].discard(connection_id)
        if not self.channel_subscribers[channel]:
            del self.channel_subscribers[channel]

    async def unsubscribe_connection(self, connection_id: str, channel: str) -> bool:
        connection = self.connections.get(connection_id)
        if connection is None:
            return False
        if await connection.unsubscribe(channel):
            await self._unsubscribe_connection(connection_id, channel)
            return True
        return False

    async def remove_channel_subscriber(self, connection_id: str, channel: str) -> bool:
        if channel not in C.SUBSCRIPTION_CHANNELS:
            return False
        return await self.unsubscribe_connection(connection_id, channel)

    async def broadcast_to_channel(self, channel: str, message: Dict[str, Any],
                                   exclude_connection: Optional[str] = None) -> int:
        if channel not in self.channel_subscribers:
            return 0
        sent, failed = 0, []
        for cid in self.channel_subscribers[channel].copy():
            if cid == exclude_connection or cid not in self.connections:
                continue
            if await self.connections[cid].send_message(message):
                sent += 1
            else:
                failed.append(cid)
        for cid in failed:
            await self.remove_connection(cid)
        return sent

    async def send_to_connection(self, connection_id: str, message: Dict[str, Any]) -> bool:
        connection = self.connections.get(connection_id)
        if connection is None:
            return False
        ok = await connection.send_message(message)
        if not ok:
            await self.remove_connection(connection_id)
        return ok

    def get_channel_subscribers(self, channel: str) -> List[WebSocketConnection]:
        return [self.connections[c] for c in self.channel_subscribers.get(channel, set()) if c in self.connections]

    def get_stats(self) -> Dict[str, Any]:
        total = len(self.connections)
        auth = len([c for c in self.connections.values() if c.is_authenticated])
        return {'total_connections': total, 'authenticated_connections': auth,
                'anonymous_connections': total - auth,
                'channel_subscribers': {ch: len(self.channel_subscribers.get(ch, set()))
                                        for ch in C.SUBSCRIPTION_CHANNELS},
                'user_stats': {'total_users': len(self.user_connections),
                               'max_connections_per_user': max([len(v) for v in self.user_connections.values()] + [0])},
                'timestamp': datetime.now(timezone.utc).isoformat()}

    async def _cleanup_loop(self):
        try:
            while True:
                await asyncio.sleep(C.CLEANUP_INTERVAL)
                dead = [cid for cid, c in self.connections.items() if not c.is_alive or c.is_expired()]
                for cid in dead:
                    await self.remove_connection(cid)
        except asyncio.CancelledError:
            pass

    async def _stats_loop(self):
        try:
            while True:
                await asyncio.sleep(C.STATS_INTERVAL)
                logger.info(f'WebSocket stats: {self.get_stats()}')
        except asyncio.CancelledError:
            pass

    async def shutdown(self):
        for t in (self._cleanup_task, self._stats_task):
            if t:
                t.cancel()
        for cid in list(self.connections):
            await self.remove_connection(cid)
        self._tasks_started = False


websocket_manager = WebSocketManager()
