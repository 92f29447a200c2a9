"""Frames of the ``/ws`` pub/sub protocol.

Wire behaviour (what a client sees) follows the reference: server frames are JSON objects with a
``type`` and an ISO-8601 UTC ``timestamp``; errors carry ``error_code`` + ``message``; successes
carry ``message`` + ``data``; events are ``new_block`` / ``new_transaction`` with a ``data`` payload
(reference websocket/socket_connection.py:213-302, socket_utils.py:29-33,57-61). Decimals go out as
JSON numbers, as the reference's encoder does (socket_connection.py:31-39).

A client frame that breaks the protocol raises :class:`Reject`; the session answers it with one
error frame and closes the socket (reference socket_endpoint.py:36-38: any rejected frame ends the
receive loop).
"""
from __future__ import annotations

import json
import uuid
from datetime import datetime, timezone
from decimal import Decimal
from typing import Any, Tuple


def utc_stamp() -> str:
    return datetime.now(timezone.utc).isoformat()


def _jsonable(o: Any):
    if isinstance(o, Decimal):
        return float(o)
    if isinstance(o, uuid.UUID):
        return str(o)
    raise TypeError(f'{type(o).__name__} is not JSON serialisable')


def encode(frame: dict) -> str:
    return json.dumps(frame, default=_jsonable)


class Reject(Exception):
    def __init__(self, code: str, text: str):
        super().__init__(code)
        self.code = code
        self.text = text


def decode_client_frame(raw, frame_bytes: int, verbs: Tuple[str, ...]) -> Tuple[dict, int]:
    """Validate one client frame; returns (message, size in bytes) or raises :class:`Reject`.
    Order of checks = order of the reference's error codes: size, JSON, shape, verb."""
    if isinstance(raw, (bytes, bytearray)):
        data = bytes(raw)
        try:
            text = data.decode('utf-8')
        except UnicodeDecodeError:
            raise Reject('INVALID_JSON', 'Message must be valid JSON')
    else:
        text = raw or ''
        data = text.encode('utf-8')
    if len(data) > frame_bytes:
        raise Reject('MESSAGE_TOO_LARGE', f'Message size exceeds {frame_bytes} bytes')
    try:
        msg = json.loads(text)
    except ValueError:
        raise Reject('INVALID_JSON', 'Message must be valid JSON')
    if not isinstance(msg, dict) or 'type' not in msg:
        raise Reject('INVALID_MESSAGE', "Message must be JSON object with 'type' field")
    verb = msg['type']
    if not isinstance(verb, str) or verb not in verbs:
        raise Reject('INVALID_MESSAGE_TYPE', f"Message type '{verb}' not allowed")
    return msg, len(data)


def error_frame(code: str, text: str) -> dict:
    return {'type': 'error', 'error_code': code, 'message': text, 'timestamp': utc_stamp()}


def success_frame(text: str, data: dict) -> dict:
    return {'type': 'success', 'message': text, 'data': data, 'timestamp': utc_stamp()}


def beat_frame(kind: str) -> dict:
    """``ping`` (server heartbeat) or ``pong`` (answer to a client ping)."""
    return {'type': kind, 'timestamp': utc_stamp()}


def event_frame(kind: str, data: Any) -> dict:
    return {'type': kind, 'data': data, 'timestamp': utc_stamp()}
