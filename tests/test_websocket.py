"""/ws pub/sub hub: every wire error code, rate limit, heartbeat, idle close, admission cap and
slow-client isolation (behaviour reference: websocket/socket_connection.py:82-368,
socket_handlers.py:19-196, socket_manager.py:59-231)."""
import asyncio
import contextlib
import json
import time

import pytest
from starlette.testclient import TestClient
from starlette.websockets import WebSocketDisconnect

from upow_amd.websocket import protocol
from upow_amd.websocket.config import Limits
from upow_amd.websocket.hub import Hub
from upow_amd.websocket.session import Session, TokenBucket


def _app(**overrides):
    from fastapi import FastAPI, WebSocket

    hub = Hub(Limits(**overrides))

    @contextlib.asynccontextmanager
    async def lifespan(app):
        await hub.start()
        yield
        await hub.stop()

    app = FastAPI(lifespan=lifespan)

    @app.websocket('/ws')
    async def ws(websocket: WebSocket):
        await hub.serve(websocket)

    return app, hub


def _expect_error_then_close(ws, code):
    msg = ws.receive_json()
    assert msg['type'] == 'error' and msg['error_code'] == code, msg
    with pytest.raises(WebSocketDisconnect) as exc:
        ws.receive_json()
    assert exc.value.code == 1000


@pytest.mark.parametrize('frame,code', [
    ('{not json', 'INVALID_JSON'),
    ('[1, 2]', 'INVALID_MESSAGE'),
    ('{"kind": "ping"}', 'INVALID_MESSAGE'),
    ('{"type": "authenticate"}', 'INVALID_MESSAGE_TYPE'),
    ('{"type": ["ping"]}', 'INVALID_MESSAGE_TYPE'),
    ('{"type": "ping", "pad": "' + 'x' * (64 * 1024) + '"}', 'MESSAGE_TOO_LARGE'),
])
def test_rejected_frames_get_one_error_then_close(frame, code):
    app, hub = _app()
    with TestClient(app) as c, c.websocket_connect('/ws') as ws:
        ws.send_text(frame)
        _expect_error_then_close(ws, code)
    assert hub.sessions == {}


def test_bytes_frame_is_parsed_like_text():
    app, _ = _app()
    with TestClient(app) as c, c.websocket_connect('/ws') as ws:
        ws.send_bytes(b'{"type": "ping"}')
        assert ws.receive_json()['type'] == 'pong'
        ws.send_bytes(b'\xff\xfe')
        _expect_error_then_close(ws, 'INVALID_JSON')


def test_rate_limit_after_a_full_burst():
    app, _ = _app(burst=60, burst_window=60.0)
    with TestClient(app) as c, c.websocket_connect('/ws') as ws:
        for _ in range(60):
            ws.send_json({'type': 'ping'})
            assert ws.receive_json()['type'] == 'pong'
        # the 60 tokens are spent: the server refuses before the next frame arrives
        _expect_error_then_close(ws, 'RATE_LIMIT_EXCEEDED')


def test_token_bucket_refills():
    t = [0.0]
    b = TokenBucket(2, 2.0, clock=lambda: t[0])
    assert b.take() and b.take() and not b.take()
    t[0] += 1.0
    assert b.take() and not b.take()
    t[0] += 100.0
    assert b.take() and b.take() and not b.take()  # capped at the burst


def test_heartbeat_and_idle_close():
    app, hub = _app(heartbeat=0.1, idle_close=0.6, tick=0.05)
    with TestClient(app) as c, c.websocket_connect('/ws') as ws:
        assert ws.receive_json()['type'] == 'ping'  # server heartbeat
        ws.send_json({'type': 'pong'})
        t0 = time.monotonic()
        with pytest.raises(WebSocketDisconnect) as exc:
            while True:
                assert ws.receive_json()['type'] == 'ping'
        assert exc.value.code == 1001
        assert time.monotonic() - t0 >= 0.4


def test_admission_cap():
    assert Limits().max_sockets == 1000  # the reference's MAX_TOTAL_CONNECTIONS
    app, hub = _app(max_sockets=2)
    with TestClient(app) as c, c.websocket_connect('/ws') as a, c.websocket_connect('/ws') as b:
        for ws in (a, b):
            ws.send_json({'type': 'ping'})
            assert ws.receive_json()['type'] == 'pong'
        with pytest.raises(WebSocketDisconnect):
            with c.websocket_connect('/ws') as third:
                third.receive_json()
        assert hub.refused == 1 and len(hub.sessions) == 2
    # after the two leave, a new client is admitted again
    with TestClient(app) as c, c.websocket_connect('/ws') as ws:
        ws.send_json({'type': 'ping'})
        assert ws.receive_json()['type'] == 'pong'


def test_publish_reaches_only_subscribers_and_encodes_once():
    from decimal import Decimal
    app, hub = _app()
    with TestClient(app) as c, c.websocket_connect('/ws') as sub, c.websocket_connect('/ws') as other:
        sub.send_json({'type': 'subscribe_block'})
        sub.receive_json(), sub.receive_json()
        n = c.portal.call(lambda: hub.publish('block', 'new_block', {'block_no': 7, 'reward': Decimal('6.5')}))
        assert n == 1
        ev = sub.receive_json()
        assert ev['type'] == 'new_block' and ev['data'] == {'block_no': 7, 'reward': 6.5}
        other.send_json({'type': 'ping'})
        assert other.receive_json()['type'] == 'pong'  # nothing else was queued for it
        assert c.portal.call(lambda: hub.publish('transaction', 'new_transaction', {})) == 0
        big = {'blob': 'x' * (70 * 1024)}
        assert c.portal.call(lambda: hub.publish('block', 'new_block', big)) == 0  # over the frame limit


class _StuckSocket:
    """A client that never reads: every send blocks."""

    def __init__(self):
        self.closed = None
        self.gate = asyncio.Event()

    async def send_text(self, text):
        await self.gate.wait()

    async def receive(self):
        await asyncio.sleep(3600)

    async def close(self, code=1000, reason=''):
        self.closed = (code, reason)


def test_slow_client_is_dropped_without_stalling_publish():
    async def run():
        hub = Hub(Limits(outbox=8))
        fast_frames = []

        class _Fast(_StuckSocket):
            async def send_text(self, text):
                fast_frames.append(text)

        slow = Session(hub, _StuckSocket(), 'slow')
        fast = Session(hub, _Fast(), 'fast')
        tasks = [asyncio.ensure_future(s.serve()) for s in (slow, fast)]
        for s in (slow, fast):
            hub.sessions[s.sid] = s
            hub.join(s, 'block')
        await asyncio.sleep(0)
        t0 = time.perf_counter()
        counts = []
        for i in range(20):
            counts.append(hub.publish('block', 'new_block', {'i': i}))
            await asyncio.sleep(0)  # let the writers run between events
        assert time.perf_counter() - t0 < 0.5
        await asyncio.sleep(0.05)
        # slow: 1 frame in flight + 8 queued, then overflow -> shut 1008 and out of the fan-out
        assert slow.shut_with == (1008, 'Send queue overflow')
        assert counts[0] == 2 and counts[-1] == 1
        assert len(fast_frames) == 20 and [json.loads(f)['data']['i'] for f in fast_frames] == list(range(20))
        fast.shut()
        slow.socket.gate.set()
        await asyncio.wait_for(asyncio.gather(*tasks), 5)
        assert slow.socket.closed == (1008, 'Send queue overflow')

    asyncio.run(run())


def test_frame_helpers():
    msg, size = protocol.decode_client_frame('{"type": "ping"}', 100, ('ping',))
    assert msg == {'type': 'ping'} and size == 16
    with pytest.raises(protocol.Reject):
        protocol.decode_client_frame('{"type": "ping"}', 10, ('ping',))
    f = protocol.error_frame('X', 'y')
    assert set(f) == {'type', 'error_code', 'message', 'timestamp'}
