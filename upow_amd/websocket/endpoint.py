"""``/ws`` route and the publish helpers the node calls (wire behaviour: reference
websocket/socket_endpoint.py:26-82, socket_utils.py:14-74)."""
from __future__ import annotations

from fastapi import APIRouter, WebSocket

from ..utils.logger import get_logger
from .hub import Hub

logger = get_logger(__name__)
router = APIRouter()
hub = Hub()


@router.websocket('/ws')
async def ws_route(websocket: WebSocket):
    await hub.serve(websocket)


async def broadcast_new_block(block_data: dict, background_tasks=None) -> int:
    n = hub.publish('block', 'new_block', block_data)
    logger.info(f"New block broadcast: Block #{block_data.get('block_no')} - sent to {n} connections")
    return n


def transaction_listeners() -> bool:
    return hub.listening('transaction')


async def broadcast_new_transaction(tx_data: dict, background_tasks=None) -> int:
    return hub.publish('transaction', 'new_transaction', tx_data)


async def start_websocket_manager():
    await hub.start()


async def shutdown_websocket_manager():
    await hub.stop()
