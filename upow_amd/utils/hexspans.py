"""Request and response bodies whose transaction arrays stay inside the body bytes.

``loads(body)`` is ``json.loads(body)``, except that an array of plain ASCII strings under a key in
``SPAN_KEYS`` ('txs' of a /push_block body, 'transactions' of a /get_blocks page row) comes back as a
:class:`HexSpans`: a read-only sequence of str over (start, length) spans of the body
(csrc/jsonspan.cpp ``json_loads_spans``). The native block decoder reads such a sequence straight out of
the body (csrc/txcodec.cpp ``decode_block_spans``), so a full block's 8,300 txs never become Python str
objects on the push / sync path; an item becomes a str only when something indexes it.

Any body outside the plain subset the native parser takes (escapes aside, which it delegates) is parsed by
``json.loads`` itself, so the result -- or the error -- is always ``json.loads``'s. Reference:
/root/reference/upow/node/main.py:521-652 (the push_block body) and main.py:97-150 (get_blocks pages).
"""
from __future__ import annotations

import json
from collections.abc import Sequence
from typing import Iterable, List, Optional

import numpy as np

SPAN_KEYS = ('txs', 'transactions')


class HexSpans(Sequence):
    """Transaction hex strings as spans of one immutable body (``buf``), then ``extra`` str items.

    Behaves as a read-only ``list`` of str for indexing, slicing (a HexSpans again), iteration, ``len``,
    ``+`` (with a list or another HexSpans of the same body) and equality with a list."""
    __slots__ = ('buf', 'spans', 'extra')

    def __init__(self, buf: bytes, spans, extra: Iterable[str] = ()):
        self.buf = buf
        sp = np.frombuffer(spans, dtype='<i8') if isinstance(spans, (bytes, bytearray, memoryview)) else \
            np.asarray(spans, dtype=np.int64)
        self.spans = sp.reshape(-1, 2)
        self.extra = tuple(extra)

    @classmethod
    def from_list(cls, hexes: Iterable[str]) -> 'HexSpans':
        """A HexSpans over one new body holding ``hexes`` (tests; the cluster's replay)."""
        hexes = list(hexes)
        enc = [h.encode('ascii') for h in hexes]
        lens = np.fromiter(map(len, enc), dtype=np.int64, count=len(enc))
        starts = np.concatenate([[0], np.cumsum(lens)[:-1]]) if len(enc) else np.zeros(0, np.int64)
        return cls(b''.join(enc), np.stack([starts, lens], axis=1) if len(enc) else np.zeros((0, 2), np.int64))

    def __len__(self) -> int:
        return len(self.spans) + len(self.extra)

    def _one(self, k: int) -> str:
        ns = len(self.spans)
        if k < ns:
            st, ln = self.spans[k]
            return self.buf[st:st + ln].decode('ascii')
        return self.extra[k - ns]

    def __getitem__(self, k):
        if isinstance(k, slice):
            idx = range(*k.indices(len(self)))
            return self.take(np.arange(idx.start, idx.stop, idx.step, dtype=np.int64))
        n = len(self)
        k = int(k)
        if k < 0:
            k += n
        if not 0 <= k < n:
            raise IndexError('HexSpans index out of range')
        return self._one(k)

    def __iter__(self):
        buf = self.buf
        for st, ln in self.spans.tolist():
            yield buf[st:st + ln].decode('ascii')
        yield from self.extra

    def __add__(self, other):
        if isinstance(other, HexSpans):
            if other.buf is self.buf and not self.extra:
                return HexSpans(self.buf, np.concatenate([self.spans, other.spans]), other.extra)
            other = list(other)
        return HexSpans(self.buf, self.spans, self.extra + tuple(other))

    def __eq__(self, other):
        if isinstance(other, (list, tuple, HexSpans)):
            return len(self) == len(other) and all(a == b for a, b in zip(self, other))
        return NotImplemented

    def __ne__(self, other):
        r = self.__eq__(other)
        return r if r is NotImplemented else not r

    __hash__ = None

    def __repr__(self):
        return f'HexSpans({len(self)} txs)'

    @property
    def lengths(self) -> np.ndarray:
        """Character length of every item (spans, then extra)."""
        ex = np.fromiter(map(len, self.extra), dtype=np.int64, count=len(self.extra))
        return np.concatenate([self.spans[:, 1], ex]) if len(ex) else self.spans[:, 1].copy()

    def take(self, idx) -> 'HexSpans':
        """The items at ``idx`` (in that order) as a HexSpans: span items stay spans."""
        idx = np.asarray(idx, dtype=np.int64).reshape(-1)
        ns = len(self.spans)
        if len(idx) and np.all(idx < ns):
            return HexSpans(self.buf, self.spans[idx])
        sp = idx[idx < ns]
        if len(sp) and np.any(np.nonzero(idx < ns)[0] != np.arange(len(sp))):
            # span items after extra items: keep the order with str items
            return HexSpans(self.buf, np.zeros((0, 2), np.int64), [self._one(int(k)) for k in idx.tolist()])
        return HexSpans(self.buf, self.spans[sp], [self.extra[int(k) - ns] for k in idx[idx >= ns].tolist()])

    def without(self, k: int) -> 'HexSpans':
        """A copy without item ``k``."""
        keep = np.ones(len(self), dtype=bool)
        keep[k] = False
        return self.take(np.nonzero(keep)[0])

    def tail2(self) -> List[Optional[bytes]]:
        """The last two characters of every span item as bytes (the coinbase scan), without a str per item."""
        end = self.spans[:, 0] + self.spans[:, 1]
        b = self.buf
        return [b[e - 2:e] if ln >= 2 else None for e, ln in zip(end.tolist(), self.spans[:, 1].tolist())]

    def tolist(self) -> List[str]:
        return list(self)


def native_loads(body: bytes, span_keys=SPAN_KEYS):
    """The native parse, or ValueError (json.loads is then the authority)."""
    from ..ops.native import lib
    buf = bytes(body)
    return lib().json_loads_spans(buf, tuple(span_keys), lambda sp: HexSpans(buf, sp))


def loads(body, span_keys=SPAN_KEYS):
    """``json.loads(body)`` with the tx arrays as :class:`HexSpans` where the body allows."""
    try:
        raw = body.encode('utf-8') if isinstance(body, str) else body
        return native_loads(raw, span_keys)
    except (ValueError, ImportError):  # outside the native subset (UnicodeError is a ValueError), or no build
        return json.loads(body)


def to_json(obj):
    """``json.dumps`` default= hook: a HexSpans serialises as the list it stands for."""
    if isinstance(obj, HexSpans):
        return obj.tolist()
    raise TypeError(f'Object of type {type(obj).__name__} is not JSON serializable')


__all__ = ['HexSpans', 'SPAN_KEYS', 'loads', 'native_loads', 'to_json']
