"""``/ws`` limits and protocol tables.

Values are the reference's wire contract (websocket/socket_config.py:7-43): 1000 sockets, 64 KiB
frames, 60 client frames per minute, 30 s server heartbeat, 300 s idle close. They are gathered in
one mutable :class:`Limits` record that the hub reads at run time, so an operator (env) or a test can
change them without patching module globals.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

# client verbs the server accepts; the reference's allow-list leaves the transaction channel
# unreachable from clients (socket_config.py:18-23), and so does this default.
# UPOW_WS_TX_CHANNEL=1 opens it (an extension: the server already publishes on it).
CLIENT_VERBS = ('ping', 'pong', 'subscribe_block', 'unsubscribe_block')
TX_CHANNEL_VERBS = ('subscribe_transaction', 'unsubscribe_transaction')
CHANNELS = ('block', 'transaction')


def _env_int(name: str, default: int) -> int:
    try:
        return int(os.environ.get(name, default))
    except ValueError:
        return default


@dataclass
class Limits:
    max_sockets: int = 1000          # admission cap (reference MAX_TOTAL_CONNECTIONS)
    frame_bytes: int = 64 * 1024     # largest client or server frame (MESSAGE_SIZE_LIMIT)
    burst: int = 60                  # client frames allowed per `burst_window` seconds
    burst_window: float = 60.0
    heartbeat: float = 30.0          # server -> client {"type": "ping"} period
    idle_close: float = 300.0        # close (1001) after this long without a valid client frame
    tick: float = 5.0                # housekeeping period (heartbeats, idle sweep)
    stats_every: float = 300.0       # log a one-line summary this often
    outbox: int = 256                # queued frames per socket before a slow client is dropped

    @classmethod
    def from_env(cls) -> 'Limits':
        return cls(max_sockets=_env_int('UPOW_WS_MAX_CONNECTIONS', 1000),
                   outbox=_env_int('UPOW_WS_OUTBOX', 256))


def client_verbs() -> tuple:
    if os.environ.get('UPOW_WS_TX_CHANNEL', '0') == '1':
        return CLIENT_VERBS + TX_CHANNEL_VERBS
    return CLIENT_VERBS


WEBSOCKET_LOG_LEVEL = os.getenv('WEBSOCKET_LOG_LEVEL', 'INFO')
