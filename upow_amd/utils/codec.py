"""Byte-exact codecs and helpers (reference: upow/helpers.py:37-230).

Wire contract: integers little-endian, compressed address = ``[42|43] || x_LE``
(33 B, base58 string form), full address = ``x_LE || y_LE`` (64 B, hex string form). Address
strings are parsed as hex first and base58 second (helpers.py:183-188).

Point decompression is cached (addresses repeat heavily inside a ledger) and, for batches, is
done by the native/HIP path (:mod:`upow_amd.ops.p256`).
"""
from __future__ import annotations

import hashlib
import json
import sys
from datetime import datetime, timezone
from decimal import Decimal
from enum import Enum, IntEnum
from functools import lru_cache
from math import ceil
from typing import Union

from ..constants import ENDIAN, SMALLEST
from . import p256
from .p256 import Point

# Global node flags (helpers.py:21-22)
is_blockchain_syncing = False
getting_active_inodes = False

NOLOGS = '--nologs' in sys.argv

_B58 = '123456789ABCDEFGHJKLMNPQRSTUVWXYZabcdefghijkmnopqrstuvwxyz'
_B58_INDEX = {c: i for i, c in enumerate(_B58)}


_NATIVE = None


def _native():
    """Native codec (csrc/base58.cpp) when the extension is built; None -> pure Python."""
    global _NATIVE
    if _NATIVE is None:
        try:
            from ..ops.native import lib
            _NATIVE = lib()
        except Exception:
            _NATIVE = False
    return _NATIVE or None


_B58_CACHE: dict = {}


def b58encode(data: bytes) -> str:
    hit = _B58_CACHE.get(data)
    if hit is not None:
        return hit
    n = _native()
    s = n.b58encode(bytes(data)) if n is not None else _b58encode_py(data)
    if len(_B58_CACHE) > (1 << 20):
        _B58_CACHE.clear()
    _B58_CACHE[bytes(data)] = s
    return s


def _b58encode_py(data: bytes) -> str:
    n = int.from_bytes(data, 'big')
    out = []
    while n:
        n, r = divmod(n, 58)
        out.append(_B58[r])
    pad = len(data) - len(data.lstrip(b'\0'))
    return '1' * pad + ''.join(reversed(out))


def b58decode(s: Union[str, bytes]) -> bytes:
    if isinstance(s, bytes):
        s = s.decode('ascii')
    n = _native()
    if n is not None:
        return n.b58decode(s)
    return _b58decode_py(s)


def _b58decode_py(s: str) -> bytes:
    s = s.rstrip()
    n = 0
    for c in s:
        try:
            n = n * 58 + _B58_INDEX[c]
        except KeyError:
            raise ValueError(f'Invalid character {c!r}') from None
    pad = len(s) - len(s.lstrip('1'))
    body = n.to_bytes((n.bit_length() + 7) // 8, 'big') if n else b''
    return b'\0' * pad + body


def get_json(obj):
    return json.loads(json.dumps(obj, default=lambda o: getattr(o, 'as_dict', getattr(o, '__dict__', str(o)))))


def timestamp() -> int:
    return int(datetime.now(timezone.utc).timestamp())


def sha256(message: Union[str, bytes]) -> str:
    """Single SHA-256 hex digest; a ``str`` is hex-decoded first (helpers.py:41-44)."""
    if isinstance(message, str):
        message = bytes.fromhex(message)
    return hashlib.sha256(message).hexdigest()


def byte_length(i: int) -> int:
    return ceil(i.bit_length() / 8.0)


def normalize_block(block) -> dict:
    block = dict(block)
    block['address'] = block['address'].strip(' ')
    ts = block['timestamp']
    if isinstance(ts, datetime):
        ts = int(ts.replace(tzinfo=timezone.utc).timestamp())
    block['timestamp'] = int(ts)
    return block


def x_to_y(x: int, is_odd: bool = False) -> int:
    return p256.x_to_y(x, is_odd)


class AddressFormat(Enum):
    FULL_HEX = 'hex'
    COMPRESSED = 'compressed'


class TransactionType(IntEnum):
    REGULAR = 0
    INODE_DE_REGISTRATION = 4
    VALIDATOR_REGISTRATION = 5
    VOTE_AS_VALIDATOR = 6
    VOTE_AS_DELEGATE = 7
    REVOKE_AS_VALIDATOR = 8
    REVOKE_AS_DELEGATE = 9


class OutputType(IntEnum):
    REGULAR = 0
    STAKE = 1
    UN_STAKE = 2
    INODE_REGISTRATION = 3
    VALIDATOR_REGISTRATION = 5
    VOTE_AS_VALIDATOR = 6
    VOTE_AS_DELEGATE = 7
    VALIDATOR_VOTING_POWER = 8
    DELEGATE_VOTING_POWER = 9


class InputType(IntEnum):
    REGULAR = 0
    FEES = 10


_TX_TYPE_BY_STR = {str(t.value): t for t in TransactionType}


def simple_bytes_to_string(data: bytes):
    if data is None:
        return None
    try:
        return data.decode('utf-8')
    except UnicodeDecodeError:
        return data.hex()


def get_transaction_type_from_message(message: bytes) -> TransactionType:
    """helpers.py:97-112: the tx type is carried as ASCII digits in the message."""
    try:
        decoded = int(simple_bytes_to_string(message))
        return _TX_TYPE_BY_STR.get(str(decoded), TransactionType.REGULAR)
    except (UnicodeDecodeError, ValueError, TypeError):
        return TransactionType.REGULAR


def point_to_bytes(point: Point, address_format: AddressFormat = AddressFormat.FULL_HEX) -> bytes:
    if address_format is AddressFormat.FULL_HEX:
        return point.x.to_bytes(32, ENDIAN) + point.y.to_bytes(32, ENDIAN)
    elif address_format is AddressFormat.COMPRESSED:
        return bytes([42 if point.y % 2 == 0 else 43]) + point.x.to_bytes(32, ENDIAN)
    raise NotImplementedError()


_POINT_CACHE: dict = {}
_POINT_CACHE_MAX = 1 << 20


def _cache_put(key: bytes, value):
    if len(_POINT_CACHE) >= _POINT_CACHE_MAX:
        _POINT_CACHE.clear()
    _POINT_CACHE[key] = value


def _decode_point(point_bytes: bytes) -> Point:
    if len(point_bytes) == 64:
        return Point(int.from_bytes(point_bytes[:32], ENDIAN), int.from_bytes(point_bytes[32:], ENDIAN))
    specifier = point_bytes[0]
    x = int.from_bytes(point_bytes[1:], ENDIAN)
    return Point(x, p256.x_to_y(x, specifier == 43))


def bytes_to_point(point_bytes: bytes) -> Point:
    """helpers.py:135-144. Raises ValueError for off-curve coordinates (fastecdsa Point ctor)."""
    point_bytes = bytes(point_bytes)
    if len(point_bytes) not in (33, 64):
        raise NotImplementedError()
    hit = _POINT_CACHE.get(point_bytes)
    if hit is None:
        try:
            hit = _decode_point(point_bytes)
        except ValueError as e:
            hit = e
        _cache_put(point_bytes, hit)
    if isinstance(hit, Exception):
        raise ValueError(str(hit))
    return hit


def prefetch_points(addresses_bytes) -> None:
    """Batch-decompress every uncached 33-byte address (gfx950 kernel for large batches, host C++
    otherwise) so the per-tx validation code never runs a Python square root."""
    todo = []
    for b in addresses_bytes:
        b = bytes(b)
        if len(b) == 33 and b not in _POINT_CACHE:
            todo.append(b)
        elif len(b) == 64 and b not in _POINT_CACHE:
            try:
                _cache_put(b, _decode_point(b))
            except ValueError as e:
                _cache_put(b, e)
    todo = list(dict.fromkeys(todo))
    if not todo:
        return
    from ..ops.p256 import decompress
    for b, xy in zip(todo, decompress(todo)):
        if xy is None:
            _cache_put(b, ValueError('coordinates are not on curve P256'))
        else:
            _cache_put(b, Point(xy[0], xy[1], check=False))


def round_up_decimal(decimal: Decimal, round_up_length: str = '0.00000001'):
    round_up_length = Decimal(round_up_length)
    if (decimal * SMALLEST) % 1 != 0.0:
        decimal = decimal.quantize(round_up_length)
    return decimal


def round_up_decimal_new(decimal: Decimal, round_up_length: str = '0.00000001'):
    return decimal.quantize(Decimal(round_up_length))


def bytes_to_string(point_bytes: bytes) -> str:
    """Canonical address string of raw address bytes (helpers.py:160-168).

    For 33-byte addresses the string is base58 of ``[42|43] || x``: the specifier is normalised to
    42 unless it is 43 (the reference re-derives it from the parity of the decompressed y, which
    is exactly ``specifier == 43``), so no square root is needed to produce the string.
    """
    if len(point_bytes) == 64:
        return bytes(point_bytes).hex()
    elif len(point_bytes) == 33:
        spec = 43 if point_bytes[0] == 43 else 42
        return b58encode(bytes([spec]) + bytes(point_bytes[1:]))
    raise NotImplementedError()


def point_to_string(point: Point, address_format: AddressFormat = AddressFormat.COMPRESSED) -> str:
    if address_format is AddressFormat.FULL_HEX:
        return point_to_bytes(point).hex()
    elif address_format is AddressFormat.COMPRESSED:
        return b58encode(point_to_bytes(point, AddressFormat.COMPRESSED))
    raise NotImplementedError()


@lru_cache(maxsize=1 << 16)
def string_to_bytes(string: str) -> bytes:
    try:
        return bytes.fromhex(string)
    except ValueError:
        return b58decode(string)


def string_to_point(string: str) -> Point:
    return bytes_to_point(string_to_bytes(string))


def address_forms(address: str):
    """Both string forms of an address (FULL_HEX, COMPRESSED) — the reference's ``addresses`` list
    used by every address query (e.g. database.py:531)."""
    point = string_to_point(address)
    return [point_to_string(point, f) for f in AddressFormat]


def address_search_hex(address: str):
    """Both byte forms (hex) of an address — the reference's ``LIKE '%hex%'`` search patterns."""
    point = string_to_point(address)
    return [point_to_bytes(point, f).hex() for f in AddressFormat]
