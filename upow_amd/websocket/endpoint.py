"""``/ws`` route and the broadcaster used by the node (reference: websocket/socket_endpoint.py:26-82,
websocket/socket_utils.py:14-74)."""
from __future__ import annotations

from datetime import datetime, timezone
from typing import Any, Dict

from fastapi import APIRouter, WebSocket, WebSocketDisconnect

from ..utils.logger import get_logger
from .handlers import WebSocketMessageHandler
from .manager import websocket_manager

logger = get_logger(__name__)
websocket_router = APIRouter()
message_handler = WebSocketMessageHandler()


@websocket_router.websocket('/ws')
async def websocket_endpoint(websocket: WebSocket):
    connection = None
    try:
        connection = await websocket_manager.add_connection(websocket)
        while True:
            message = await connection.receive_message()
            if message is None:  # invalid/over-limit message or disconnect: close (socket_endpoint.py:36-38)
                break
            await message_handler.handle_message(connection, message)
    except WebSocketDisconnect:
        pass
    except Exception as e:
        logger.error(f'WebSocket error: {e}')
    finally:
        if connection:
            await websocket_manager.remove_connection(connection.connection_id)


class WebSocketBroadcaster:
    @staticmethod
    async def broadcast_new_block(block_data: Dict[str, Any]) -> int:
        try:
            message = {'type': 'new_block', 'data': block_data, 'timestamp': datetime.now(timezone.utc).isoformat()}
            return await websocket_manager.broadcast_to_channel('block', message)
        except Exception as e:
            logger.error(f'Error broadcasting new block: {e}')
            return 0

    @staticmethod
    async def broadcast_new_transaction(tx_data: Dict[str, Any]) -> int:
        try:
            message = {'type': 'new_transaction', 'data': tx_data,
                       'timestamp': datetime.now(timezone.utc).isoformat()}
            return await websocket_manager.broadcast_to_channel('transaction', message)
        except Exception as e:
            logger.error(f'Error broadcasting new transaction: {e}')
            return 0


broadcaster = WebSocketBroadcaster()


async def broadcast_new_block(block_data, background_tasks=None):
    await broadcaster.broadcast_new_block(block_data)


async def broadcast_new_transaction(tx_data, background_tasks=None):
    await broadcaster.broadcast_new_transaction(tx_data)


async def start_websocket_manager():
    await websocket_manager.start_background_tasks()


async def shutdown_websocket_manager():
    await websocket_manager.shutdown()
