"""Peer table + peer HTTP client (reference: upow/node/nodes_manager.py:24-210).

Persistent peer list and last-seen map in ``nodes.json`` under a file lock; active window 7 days,
pruning after 90 days, at most 100 peers; streamed JSON fetch capped at 10x the max block hex size.
The httpx client is a class attribute so tests can route peers to in-process ASGI apps.
"""
from __future__ import annotations

import fcntl
import json
import os
import time
from contextlib import contextmanager
from random import sample
from typing import List, Optional

import httpx

from .. import config
from ..constants import MAX_BLOCK_SIZE_HEX
from ..utils.codec import timestamp
from ..utils.jsonstore import JsonStore

ACTIVE_NODES_DELTA = 60 * 60 * 24 * 7
INACTIVE_NODES_DELTA = 60 * 60 * 24 * 90
MAX_NODES_COUNT = 100


@contextmanager
def _file_lock(path: str):
    with open(path + '.lock', 'a+') as f:
        fcntl.flock(f, fcntl.LOCK_EX)
        try:
            yield
        finally:
            fcntl.flock(f, fcntl.LOCK_UN)


class NodesManager:
    last_messages: dict = None
    nodes: list = None
    db: JsonStore = None
    path: str = None
    timeout = httpx.Timeout(5)
    async_client: httpx.AsyncClient = None

    @staticmethod
    def _core_url() -> str:
        return (os.environ.get('UPOW_CORE_URL', config.CORE_URL) or '').rstrip('/')

    @staticmethod
    def client() -> httpx.AsyncClient:
        if NodesManager.async_client is None:
            NodesManager.async_client = httpx.AsyncClient(timeout=NodesManager.timeout, follow_redirects=True)
        return NodesManager.async_client

    _stamp = None   # (mtime_ns, size, inode) of nodes.json as last read or written by this process
    _written = None  # (nodes, last_messages) as last written by this process

    _stat_at = 0.0  # monotonic time of the last stat
    _stat_val = None
    STAT_PERIOD = 0.5  # seconds a stat result is reused (every /push_tx gossips through get_nodes)

    @staticmethod
    def _file_stamp(fresh: bool = False):
        now = time.monotonic()
        if not fresh and now - NodesManager._stat_at < NodesManager.STAT_PERIOD:
            return NodesManager._stat_val
        try:
            st = os.stat(NodesManager.path)
            val = st.st_mtime_ns, st.st_size, st.st_ino
        except OSError:
            val = None
        NodesManager._stat_at, NodesManager._stat_val = now, val
        return val

    @staticmethod
    def init(path: Optional[str] = None):
        """(Re)load nodes.json. The node calls this on every request (as the reference does with
        pickledb); the file is only re-read when it changed on disk since this process last read or
        wrote it (checked at most every ``STAT_PERIOD``), so another process sharing the peer table is
        seen within half a second."""
        if path is not None or NodesManager.path is None:
            NodesManager.path = path or config.data_path('nodes.json')
            NodesManager._stamp = None
        if NodesManager._stamp is not None and NodesManager.db is not None and \
                NodesManager._file_stamp() == NodesManager._stamp:
            return
        with _file_lock(NodesManager.path):
            NodesManager.db = JsonStore(NodesManager.path, auto_dump=False)
            core = NodesManager._core_url()
            NodesManager.nodes = NodesManager.db.get('nodes') or ([core] if core else [])
            NodesManager.last_messages = NodesManager.db.get('last_messages') or ({core: timestamp()} if core else {})
            NodesManager._stamp = NodesManager._file_stamp(fresh=True)

    @staticmethod
    def sync():
        """Write the peer table back, skipped when nothing changed since this process's last write."""
        state = (list(NodesManager.nodes), dict(NodesManager.last_messages))
        if state == NodesManager._written and NodesManager._file_stamp() == NodesManager._stamp:
            return
        with _file_lock(NodesManager.path):
            NodesManager.db.set('nodes', NodesManager.nodes)
            NodesManager.db.set('last_messages', NodesManager.last_messages)
            NodesManager.db.dump()
            NodesManager._stamp = NodesManager._file_stamp(fresh=True)
            NodesManager._written = state

    @staticmethod
    async def request(url: str, method: str = 'GET', **kwargs):
        res = ''
        async with NodesManager.client().stream(method, url, **kwargs) as response:
            async for chunk in response.aiter_text():
                res += chunk
                if len(res) > MAX_BLOCK_SIZE_HEX * 10:
                    break
        return json.loads(res)

    @staticmethod
    async def is_node_working(node: str) -> bool:
        try:
            await NodesManager.request(node)
            return True
        except Exception:
            return False

    @staticmethod
    def add_node(node: str):
        node = node.strip('/')
        if len(NodesManager.nodes) > MAX_NODES_COUNT or len(NodesManager.get_zero_nodes()) > 10:
            NodesManager.clear_old_nodes()
        if len(NodesManager.nodes) > MAX_NODES_COUNT:
            raise Exception('Too many nodes')
        NodesManager.init()
        NodesManager.nodes.append(node)
        NodesManager.sync()

    @staticmethod
    def get_nodes() -> List[str]:
        NodesManager.init()
        NodesManager.nodes.extend(NodesManager.last_messages.keys())
        NodesManager.nodes = list(dict.fromkeys(n.strip('/') for n in NodesManager.nodes if len(n)))
        NodesManager.sync()
        return NodesManager.nodes

    @staticmethod
    def get_recent_nodes() -> List[str]:
        full = {n: NodesManager.get_last_message(n) for n in NodesManager.get_nodes()}
        return [k for k, v in sorted(full.items(), key=lambda kv: kv[1], reverse=True)
                if v > timestamp() - ACTIVE_NODES_DELTA]

    @staticmethod
    def get_zero_nodes() -> List[str]:
        return [n for n in NodesManager.get_nodes() if NodesManager.get_last_message(n) == 0]

    @staticmethod
    def get_propagate_nodes() -> List[str]:
        active = NodesManager.get_recent_nodes()
        zero = NodesManager.get_zero_nodes()
        return (sample(active, k=10) if len(active) > 10 else active) + \
            (sample(zero, k=10) if len(zero) > 10 else zero)

    @staticmethod
    def clear_old_nodes():
        NodesManager.init()
        NodesManager.nodes = [n for n in NodesManager.get_nodes()
                              if NodesManager.get_last_message(n) > timestamp() - INACTIVE_NODES_DELTA]
        NodesManager.sync()

    @staticmethod
    def get_last_message(node_url: str) -> int:
        NodesManager.init()
        return NodesManager.last_messages.get(node_url, 0)

    @staticmethod
    def update_last_message(node_url: str):
        NodesManager.init()
        NodesManager.last_messages[node_url.strip('/')] = timestamp()
        NodesManager.sync()


class NodeInterface:
    def __init__(self, url: str):
        self.url = url.strip('/')
        self.base_url = self.url.replace('http://', '', 1).replace('https://', '', 1)

    async def get_block(self, block_no: int, full_transactions: bool = False):
        res = await self.request('get_block', {'block': block_no, 'full_transactions': full_transactions})
        return res['result']

    async def get_blocks(self, offset: int, limit: int):
        res = await self.request('get_blocks', {'offset': offset, 'limit': limit})
        if 'result' not in res:
            raise Exception(res['error'])
        return res['result']

    async def get_nodes(self):
        res = await self.request('get_nodes')
        return res['result']

    async def request(self, path: str, data: dict = None, sender_node: str = ''):
        data = data or {}
        headers = {'Sender-Node': sender_node}
        if path in ('push_block', 'push_tx'):
            return await NodesManager.request(f'{self.url}/{path}', method='POST', json=data, headers=headers,
                                              timeout=10)
        params = {k: (str(v).lower() if isinstance(v, bool) else v) for k, v in data.items()}
        return await NodesManager.request(f'{self.url}/{path}', params=params, headers=headers, timeout=10)
