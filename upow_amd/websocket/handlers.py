"""Client message router (reference: websocket/socket_handlers.py:19-196)."""
from __future__ import annotations

from typing import Any, Dict

from ..utils.logger import get_logger
from .config import ALLOWED_MESSAGE_TYPES
from .connection import WebSocketConnection
from .manager import websocket_manager

logger = get_logger(__name__)


class WebSocketMessageHandler:
    def __init__(self, manager=None):
        self.manager = manager or websocket_manager
        self.handlers = {
            'ping': self.handle_ping,
            'pong': self.handle_pong,
            'subscribe_block': self.handle_subscribe_block,
            'unsubscribe_block': self.handle_unsubscribe_block,
            'subscribe_transaction': self.handle_subscribe_transaction,
            'unsubscribe_transaction': self.handle_unsubscribe_transaction,
        }

    async def handle_message(self, connection: WebSocketConnection, message: Dict[str, Any]) -> bool:
        message_type = message.get('type')
        if not message_type:
            await connection.send_error('INVALID_MESSAGE', 'Message type is required')
            return False
        if message_type not in ALLOWED_MESSAGE_TYPES:
            await connection.send_error('INVALID_MESSAGE_TYPE', f"Message type '{message_type}' not allowed")
            return False
        handler = self.handlers.get(message_type)
        if not handler:
            await connection.send_error('HANDLER_NOT_FOUND', f"No handler for message type '{message_type}'")
            return False
        try:
            return await handler(connection, message)
        except Exception as e:
            logger.error(f"Error handling message type '{message_type}': {e}")
            await connection.send_error('HANDLER_ERROR', f'Error processing {message_type} message')
            return False

    async def handle_ping(self, connection, message) -> bool:
        await connection.pong()
        return True

    async def handle_pong(self, connection, message) -> bool:
        return True

    async def _sub(self, connection, channel, ok_text, ok_type, err_code, err_text, subscribe=True) -> bool:
        try:
            if subscribe:
                await self.manager.add_channel_subscriber(connection.connection_id, channel)
            else:
                await self.manager.remove_channel_subscriber(connection.connection_id, channel)
            await connection.send_success(ok_text, {'type': ok_type})
            return True
        except Exception as e:
            logger.error(f'{err_text}: {e}')
            await connection.send_error(err_code, err_text)
            return False

    async def handle_subscribe_block(self, connection, message) -> bool:
        return await self._sub(connection, 'block', 'Subscribed to block updates', 'block_subscription',
                               'SUBSCRIPTION_ERROR', 'Error processing block subscription')

    async def handle_unsubscribe_block(self, connection, message) -> bool:
        return await self._sub(connection, 'block', 'Unsubscribed from block updates', 'block_unsubscription',
                               'UNSUBSCRIPTION_ERROR', 'Error processing block unsubscription', subscribe=False)

    async def handle_subscribe_transaction(self, connection, message) -> bool:
        return await self._sub(connection, 'transaction', 'Subscribed to transaction updates',
                               'transaction_subscription', 'SUBSCRIPTION_ERROR',
                               'Error processing transaction subscription')

    async def handle_unsubscribe_transaction(self, connection, message) -> bool:
        return await self._sub(connection, 'transaction', 'Unsubscribed from transaction updates',
                               'transaction_unsubscription', 'UNSUBSCRIPTION_ERROR',
                               'Error processing transaction unsubscription', subscribe=False)


message_handler = WebSocketMessageHandler()
