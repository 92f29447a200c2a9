"""Block header codec, merkle root and the nibble-prefix PoW predicate.

reference: upow/manager.py:130-151 (check_block_is_valid), 365-378 (merkle), 385-419 (header
codec), miner.py:43-82 (miner-side predicate and header template).

Header v2 (108 B, 33-byte miner address)::

    0x02 | prev_hash 32 | address 33 | merkle 32 | timestamp u32 | difficulty*10 u16 | nonce u32

Header v1 (138 B) is the same without the version byte and with a 64-byte address.
"""
from __future__ import annotations

import hashlib
from dataclasses import dataclass
from decimal import Decimal
from io import BytesIO
from math import ceil, floor
from typing import Iterable, List, Optional, Sequence, Union

from ..constants import ENDIAN
from ..utils.codec import bytes_to_string, string_to_bytes


def block_to_bytes(last_block_hash: str, block: dict) -> bytes:
    """manager.py:385-398."""
    address_bytes = string_to_bytes(block['address'])
    version = bytes([]) if len(address_bytes) == 64 else bytes([2])
    return (version + bytes.fromhex(last_block_hash) + address_bytes + bytes.fromhex(block['merkle_tree'])
            + int(block['timestamp']).to_bytes(4, ENDIAN)
            + int(float(block['difficulty']) * 10).to_bytes(2, ENDIAN)
            + int(block['random']).to_bytes(4, ENDIAN))


def split_block_content(block_content: str):
    """manager.py:401-419 -> (previous_hash, address, merkle_tree, timestamp, difficulty, random)."""
    _bytes = bytes.fromhex(block_content)
    stream = BytesIO(_bytes)
    if len(_bytes) == 138:
        version = 1
    else:
        version = int.from_bytes(stream.read(1), ENDIAN)
        assert version > 1
        if version == 2:
            assert len(_bytes) == 108
        else:
            raise NotImplementedError()
    previous_hash = stream.read(32).hex()
    address = bytes_to_string(stream.read(64 if version == 1 else 33))
    merkle_tree = stream.read(32).hex()
    ts = int.from_bytes(stream.read(4), ENDIAN)
    difficulty = int.from_bytes(stream.read(2), ENDIAN) / Decimal(10)
    random = int.from_bytes(stream.read(4), ENDIAN)
    return previous_hash, address, merkle_tree, ts, difficulty, random


def _tx_bytes(tx) -> bytes:
    if isinstance(tx, (bytes, bytearray)):
        return bytes(tx)
    if isinstance(tx, str):
        return bytes.fromhex(tx)
    return bytes.fromhex(tx.hex())


def get_transactions_merkle_tree(transactions: Iterable) -> str:
    """manager.py:365-378: SHA256( concat over txs *sorted by raw bytes* of SHA256(tx) ).

    Batched leaf hashing runs natively (:func:`upow_amd.ops.sha256.merkle_root`) when the
    extension is present; this is the oracle form.
    """
    txs = [_tx_bytes(t) for t in transactions]
    if len(txs) >= 64:
        try:
            from ..ops.sha256 import merkle_root
            return merkle_root(txs)
        except ImportError:
            pass
    h = hashlib.sha256()
    for b in sorted(txs):
        h.update(hashlib.sha256(b).digest())
    return h.hexdigest()


def get_transactions_merkle_tree_ordered(transactions: Iterable) -> str:
    """manager.py:352-362 (legacy, insertion order)."""
    h = hashlib.sha256()
    for t in transactions:
        h.update(hashlib.sha256(_tx_bytes(t)).digest())
    return h.hexdigest()


def miner_merkle_root(tx_hashes: Sequence[str]) -> str:
    """miner.py:15-18: SHA256 over the concatenation of the (already sorted) tx hashes."""
    return hashlib.sha256(b''.join(bytes.fromhex(t) for t in tx_hashes)).hexdigest()


@dataclass(frozen=True)
class PowTarget:
    """The reference predicate compiled to bit masks over the 256-bit digest.

    ``hex(sha256(header)).startswith(prev_hash[-D:])`` and, if frac(d) > 0,
    ``hex_digest[D] in '0123456789abcdef'[:ceil(16*(1-frac))]``.

    ``words``/``masks`` are the 8 big-endian digest words and the bits that must equal them;
    ``frac_nibble`` is the nibble index D (or -1) whose value must be < ``frac_limit``.
    Note ``prev_hash[-0:]`` is the whole hash (the reference quirk for d < 1).
    """
    prefix: str
    frac_nibble: int
    frac_limit: int
    words: tuple
    masks: tuple

    @staticmethod
    def from_difficulty(prev_hash: str, difficulty) -> 'PowTarget':
        d = Decimal(str(difficulty)) if not isinstance(difficulty, Decimal) else difficulty
        dec = d % 1
        di = floor(d)
        prefix = prev_hash[-di:]
        frac_nibble, frac_limit = -1, 16
        if dec > 0:
            frac_nibble = di
            frac_limit = ceil(16 * (1 - dec))
        nib = [0] * 64
        msk = [0] * 64
        for i, c in enumerate(prefix[:64]):
            nib[i] = int(c, 16)
            msk[i] = 0xF
        words, masks = [], []
        for w in range(8):
            v = m = 0
            for k in range(8):
                v = (v << 4) | nib[w * 8 + k]
                m = (m << 4) | msk[w * 8 + k]
            words.append(v)
            masks.append(m)
        return PowTarget(prefix, frac_nibble, frac_limit, tuple(words), tuple(masks))

    def check_hex(self, digest_hex: str) -> bool:
        if not digest_hex.startswith(self.prefix):
            return False
        if self.frac_nibble >= 0:
            return int(digest_hex[self.frac_nibble], 16) < self.frac_limit
        return True


def check_pow(block_content: Union[str, bytes], prev_hash: Optional[str], difficulty) -> bool:
    """Pure form of manager.py:130-151 (no prev block => genesis => always valid)."""
    if isinstance(block_content, str):
        block_content = bytes.fromhex(block_content)
    if prev_hash is None:
        return True
    digest = hashlib.sha256(block_content).hexdigest()
    # the predicate of PowTarget.check_hex without building the search kernel's word/mask target
    d = Decimal(str(difficulty)) if not isinstance(difficulty, Decimal) else difficulty
    di = floor(d)
    if not digest.startswith(prev_hash[-di:]):
        return False
    dec = d % 1
    return int(digest[di], 16) < ceil(16 * (1 - dec)) if dec > 0 else True


def header_prefix(prev_hash: str, address: str, merkle_root: str, ts: int, difficulty) -> bytes:
    """Header without the trailing 4-byte nonce (miner.py:74-82)."""
    wallet = string_to_bytes(address)
    pre = (bytes.fromhex(prev_hash) + wallet + bytes.fromhex(merkle_root) + int(ts).to_bytes(4, ENDIAN)
           + int(float(difficulty) * 10).to_bytes(2, ENDIAN))
    if len(wallet) == 33:
        pre = bytes([2]) + pre
    return pre


def header_prefix_raw(prev_hash: str, address: str, merkle_root: str, ts: int, difficulty_field: int) -> bytes:
    """Like :func:`header_prefix` but with an explicit u16 difficulty field. The reference node parses
    but never checks that field (upow/manager.py:431), so miners may use it as an extra nonce."""
    wallet = string_to_bytes(address)
    pre = (bytes.fromhex(prev_hash) + wallet + bytes.fromhex(merkle_root) + int(ts).to_bytes(4, ENDIAN)
           + int(difficulty_field).to_bytes(2, ENDIAN))
    if len(wallet) == 33:
        pre = bytes([2]) + pre
    return pre
