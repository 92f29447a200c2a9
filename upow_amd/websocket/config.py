"""WebSocket protocol constants (reference: websocket/socket_config.py:7-43)."""
import os

MAX_CONNECTIONS_PER_IP = 5
MAX_TOTAL_CONNECTIONS = 1000
HEARTBEAT_INTERVAL = 30
CONNECTION_TIMEOUT = 300
MESSAGE_SIZE_LIMIT = 64 * 1024
RATE_LIMIT_MESSAGES_PER_MINUTE = 60
RATE_LIMIT_WINDOW = 60
# the reference's allow-list omits the *_transaction types, so those handlers are unreachable
ALLOWED_MESSAGE_TYPES = ['ping', 'pong', 'subscribe_block', 'unsubscribe_block']
SUBSCRIPTION_CHANNELS = ['block', 'transaction']
WEBSOCKET_LOG_LEVEL = os.getenv('WEBSOCKET_LOG_LEVEL', 'INFO')
LOG_CONNECTION_EVENTS = True
LOG_MESSAGE_EVENTS = False
REQUIRE_AUTH = False
VALIDATE_ORIGIN = True
ENABLE_COMPRESSION = True
PING_INTERVAL = 20
PING_TIMEOUT = 10
CLEANUP_INTERVAL = 60
STATS_INTERVAL = 300
