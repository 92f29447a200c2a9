"""Peer registry and peer HTTP client.

Behaviour contract (reference upow/node/nodes_manager.py): a node remembers the peers it learned about
and when it last heard from each; peers heard from within 7 days are "recent" (most recent first);
peers never heard from are tried too; gossip goes to at most 10 random recent peers plus at most 10
random never-heard-from peers; a peer table of more than 100 entries (or more than 10 never-heard-from
peers) is pruned of everything silent for 90 days before a new peer is accepted, and a table still over
100 refuses the new peer ('Too many nodes'); a peer's JSON answer is read as a stream capped at 40 MB.

Design (not the reference's layout):

* one :class:`Peer` record per peer (url, first_seen, last_seen; last_seen 0 = never heard from), kept in
  an in-memory table guarded by a lock — /push_tx touches it for every gossiped tx;
* selection and pruning are pure policy functions over records (:func:`recent`, :func:`never_heard`,
  :func:`stale`, :func:`gossip_targets`), so they are testable without a node;
* persistence is write-behind: a change marks the table dirty and the file (``peers.json``, one list of
  records) is replaced atomically (write to a temporary file, fsync, rename) at most once per
  ``FLUSH_INTERVAL`` and on shutdown; another process sharing the file is merged in when the file
  changes on disk (newest ``last_seen`` per peer wins). A legacy ``nodes.json`` (``nodes`` +
  ``last_messages``) is imported once.
"""
from __future__ import annotations

import json
import os
import random
import threading
import time
from dataclasses import asdict, dataclass
from typing import Dict, Iterable, List, Optional

import httpx

from .. import config
from ..utils import hexspans
from ..utils.logger import get_logger
from ..constants import MAX_BLOCK_SIZE_HEX

logger = get_logger(__name__)

ACTIVE_WINDOW = 7 * 86_400      # recent peers (nodes_manager.py:24)
PRUNE_AFTER = 90 * 86_400       # silence after which a peer may be dropped (nodes_manager.py:25)
MAX_PEERS = 100                 # table cap (nodes_manager.py:26)
MAX_NEVER_HEARD = 10            # never-heard-from peers tolerated before a prune
GOSSIP_FANOUT = 10              # per class (recent / never heard from)
FETCH_CAP = MAX_BLOCK_SIZE_HEX * 10
FLUSH_INTERVAL = 1.0


def _now() -> int:
    return int(time.time())


def normalize(url: str) -> str:
    return (url or '').strip().strip('/')


@dataclass
class Peer:
    url: str
    first_seen: int
    last_seen: int = 0  # 0: never heard from


# ------------------------------------------------------------------------------------------ policies
def recent(peers: Iterable[Peer], now: int, window: int = ACTIVE_WINDOW) -> List[Peer]:
    """Peers heard from within ``window`` seconds, most recently heard first."""
    return sorted((p for p in peers if p.last_seen > now - window), key=lambda p: p.last_seen, reverse=True)


def never_heard(peers: Iterable[Peer]) -> List[Peer]:
    return [p for p in peers if p.last_seen == 0]


def stale(peers: Iterable[Peer], now: int, horizon: int = PRUNE_AFTER) -> List[Peer]:
    """Peers silent for at least ``horizon`` seconds (never-heard-from peers included)."""
    return [p for p in peers if p.last_seen <= now - horizon]


def gossip_targets(peers: Iterable[Peer], now: int, rng: random.Random = random, fanout: int = GOSSIP_FANOUT
                   ) -> List[str]:
    """Up to ``fanout`` random recent peers, then up to ``fanout`` random never-heard-from ones."""
    peers = list(peers)
    out = []
    for group in (recent(peers, now), never_heard(peers)):
        urls = [p.url for p in group]
        out.extend(rng.sample(urls, fanout) if len(urls) > fanout else urls)
    return out


# ------------------------------------------------------------------------------------------ registry
class PeerBook:
    def __init__(self, path: Optional[str], seed_url: str = ''):
        self.path = path
        self.seed_url = normalize(seed_url)
        self.lock = threading.RLock()
        self._peers: Dict[str, Peer] = {}
        self._dirty = False
        self._flushed_at = 0.0
        self._stamp = None       # (mtime_ns, size, inode) of the file as this process last saw it
        self._stat_at = 0.0
        self._pruned: Dict[str, int] = {}  # url -> last_seen when this process pruned it (merges skip it)
        self._wake = threading.Event()
        self._flush_mu = threading.Lock()
        self._flusher: Optional[threading.Thread] = None
        self.load()

    # ---- persistence
    def _file_stamp(self):
        try:
            st = os.stat(self.path)
            return st.st_mtime_ns, st.st_size, st.st_ino
        except (OSError, TypeError):
            return None

    def _read(self) -> List[Peer]:
        if not self.path or not os.path.exists(self.path):
            legacy = os.path.join(os.path.dirname(self.path), 'nodes.json') if self.path else None
            return self._read_legacy(legacy) if legacy and os.path.exists(legacy) else []
        try:
            with open(self.path) as f:
                raw = json.load(f)
            return [Peer(normalize(r['url']), int(r.get('first_seen', 0)), int(r.get('last_seen', 0)))
                    for r in raw.get('peers', []) if normalize(r.get('url', ''))]
        except (OSError, ValueError, KeyError, TypeError, AttributeError):
            return []  # a corrupt table starts over from the seed (nodes_manager.py:58-64)

    @staticmethod
    def _read_legacy(path: str) -> List[Peer]:
        try:
            with open(path) as f:
                raw = json.load(f)
        except (OSError, ValueError):
            return []
        seen = {normalize(k): int(v or 0) for k, v in (raw.get('last_messages') or {}).items()}
        urls = [normalize(u) for u in (raw.get('nodes') or [])] + list(seen)
        now = _now()
        return [Peer(u, now, seen.get(u, 0)) for u in dict.fromkeys(u for u in urls if u)]

    def load(self):
        with self.lock:
            self._peers = {}
            self._merge(self._read())
            if not self._peers and self.seed_url:
                self._peers[self.seed_url] = Peer(self.seed_url, _now(), _now())
                self._dirty = True
            self._stamp = self._file_stamp()

    def _merge(self, records: Iterable[Peer]):
        for r in records:
            gone = self._pruned.get(r.url)
            if gone is not None and r.last_seen <= gone:
                continue  # pruned here; only news of the peer (a later contact) brings it back
            mine = self._peers.get(r.url)
            if mine is None:
                self._peers[r.url] = Peer(r.url, r.first_seen, r.last_seen)
            elif r.last_seen > mine.last_seen:
                mine.last_seen = r.last_seen

    def _refresh(self):
        """Pick up another process's writes (checked at most twice a second)."""
        if not self.path:
            return
        t = time.monotonic()
        if t - self._stat_at < 0.5:
            return
        self._stat_at = t
        stamp = self._file_stamp()
        if stamp is not None and stamp != self._stamp:
            self._merge(self._read())
            self._stamp = stamp

    def flush(self, force: bool = True):
        """Write the table. Under an exclusive lock on ``<path>.lock`` (the reference's FileLock,
        nodes_manager.py:28-43) the file is re-read and merged first — newest last_seen wins, this process's
        prunes stay pruned — so peers another process added since our last look are kept."""
        if not self.path:
            return
        with self._flush_mu:  # one flush of this book at a time: a flush returns once its data is on disk
            self._flush(force)

    def _flush(self, force: bool):
        with self.lock:
            if not self._dirty:
                return
            if not force and time.monotonic() - self._flushed_at < FLUSH_INTERVAL:
                return
        import fcntl
        os.makedirs(os.path.dirname(os.path.abspath(self.path)), exist_ok=True)
        with open(self.path + '.lock', 'a') as lk:
            fcntl.flock(lk.fileno(), fcntl.LOCK_EX)
            try:
                disk = self._read()
                with self.lock:
                    self._merge(disk)
                    rows = [asdict(p) for p in self._peers.values()]
                    self._dirty = False
                tmp = f'{self.path}.{os.getpid()}.tmp'
                with open(tmp, 'w') as f:
                    json.dump({'peers': rows}, f)
                    f.flush()
                    os.fsync(f.fileno())
                os.replace(tmp, self.path)
                with self.lock:
                    self._stamp = self._file_stamp()
                    self._flushed_at = time.monotonic()
            finally:
                fcntl.flock(lk.fileno(), fcntl.LOCK_UN)

    def _changed(self):
        """Mark dirty; the write (file lock, re-read, fsync) happens on the book's flusher thread, never on
        the caller's (the HTTP event loop)."""
        self._dirty = True
        if not self.path:
            return
        if self._flusher is None or not self._flusher.is_alive():
            self._flusher = threading.Thread(target=self._flush_loop, name='upow-peers-flush', daemon=True)
            self._flusher.start()
        self._wake.set()

    def _flush_loop(self):
        while True:
            self._wake.wait()
            self._wake.clear()
            wait = FLUSH_INTERVAL - (time.monotonic() - self._flushed_at)
            if wait > 0:
                time.sleep(wait)
            try:
                self.flush(force=True)
            except Exception as e:  # pragma: no cover - disk trouble: keep serving, retry on the next change
                logger.error(f'peers flush failed: {e}')

    # ---- queries
    def records(self) -> List[Peer]:
        with self.lock:
            self._refresh()
            return list(self._peers.values())

    def urls(self) -> List[str]:
        return [p.url for p in self.records()]

    def recent_urls(self) -> List[str]:
        return [p.url for p in recent(self.records(), _now())]

    def gossip_urls(self) -> List[str]:
        return gossip_targets(self.records(), _now())

    def last_seen(self, url: str) -> int:
        p = self._peers.get(normalize(url))
        return p.last_seen if p is not None else 0

    # ---- updates
    def add(self, url: str) -> bool:
        """Learn a peer (never heard from yet). Prunes long-silent peers when the table is full or holds too
        many never-heard-from peers; raises when it is still full. False when already known."""
        url = normalize(url)
        if not url:
            return False
        with self.lock:
            self._refresh()
            if url in self._peers:
                return False
            now = _now()
            peers = list(self._peers.values())
            if len(peers) > MAX_PEERS or len(never_heard(peers)) > MAX_NEVER_HEARD:
                for p in stale(peers, now):
                    del self._peers[p.url]
                    self._pruned[p.url] = p.last_seen
                self._dirty = True
            if len(self._peers) > MAX_PEERS:
                self._changed()
                raise Exception('Too many nodes')
            self._peers[url] = Peer(url, now, 0)
            self._changed()
            return True

    def seen(self, url: str):
        """We heard from ``url`` just now (learning it if new)."""
        url = normalize(url)
        if not url:
            return
        with self.lock:
            p = self._peers.get(url)
            now = _now()
            if p is None:
                self._peers[url] = Peer(url, now, now)
            elif p.last_seen == now:
                return
            else:
                p.last_seen = now
            self._changed()


_book: Optional[PeerBook] = None


def book() -> PeerBook:
    global _book
    if _book is None:
        seed = os.environ.get('UPOW_CORE_URL', config.CORE_URL) or ''
        _book = PeerBook(config.data_path('peers.json'), seed)
    return _book


def reset():
    """Forget the process-wide registry (tests; a changed data directory)."""
    global _book
    if _book is not None:
        _book.flush()
    _book = None


# ------------------------------------------------------------------------------------------ client
_client: Optional[httpx.AsyncClient] = None


def client() -> httpx.AsyncClient:
    """The shared peer HTTP client (5 s timeout, redirects followed); tests may replace it."""
    global _client
    if _client is None:
        _client = httpx.AsyncClient(timeout=httpx.Timeout(5), follow_redirects=True)
    return _client


def set_client(c: Optional[httpx.AsyncClient]):
    global _client
    _client = c


async def fetch_json(url: str, method: str = 'GET', **kwargs):
    """A peer's JSON answer, read as a stream and cut at ``FETCH_CAP`` bytes. Tx arrays ('transactions' of a
    /get_blocks page, 'txs') stay inside the body bytes (utils/hexspans.py): the sync decoder reads them there."""
    parts, size = [], 0
    async with client().stream(method, url, **kwargs) as response:
        async for chunk in response.aiter_bytes():
            parts.append(chunk)
            size += len(chunk)
            if size > FETCH_CAP:
                break
    return hexspans.loads(b''.join(parts))


async def is_alive(url: str) -> bool:
    try:
        await fetch_json(url)
        return True
    except Exception:
        return False


class PeerClient:
    """Typed calls to one peer's REST API."""

    def __init__(self, url: str):
        self.url = normalize(url)
        self.host = self.url.replace('http://', '', 1).replace('https://', '', 1)

    async def call(self, path: str, data: dict = None, sender: str = ''):
        data = data or {}
        headers = {'Sender-Node': sender}
        if path in ('push_block', 'push_tx'):
            return await fetch_json(f'{self.url}/{path}', method='POST', json=data, headers=headers, timeout=10)
        params = {k: (str(v).lower() if isinstance(v, bool) else v) for k, v in data.items()}
        return await fetch_json(f'{self.url}/{path}', params=params, headers=headers, timeout=10)

    async def block(self, block_no: int, full_transactions: bool = False):
        return (await self.call('get_block', {'block': block_no, 'full_transactions': full_transactions}))['result']

    async def blocks(self, offset: int, limit: int):
        res = await self.call('get_blocks', {'offset': offset, 'limit': limit})
        if 'result' not in res:
            raise Exception(res['error'])
        return res['result']

    async def peers(self):
        return (await self.call('get_nodes'))['result']


__all__ = ['Peer', 'PeerBook', 'PeerClient', 'book', 'reset', 'fetch_json', 'is_alive', 'recent', 'never_heard',
           'stale', 'gossip_targets', 'client', 'set_client']
