"""Seed corpora for the libFuzzer targets (tools/sanitize_host.sh): valid HTTP requests and WebSocket
frames, and valid transactions of every shape the codec knows (regular, message, governance type, 64-byte
v1 addresses, one signature per input, coinbase), each in the fuzzers' input framing."""
import os
import random
import struct
import sys
from decimal import Decimal

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
os.environ.setdefault('UPOW_NO_TORCH', '1')


def http_seeds():
    reqs = [
        b'GET / HTTP/1.1\r\nHost: x\r\n\r\n',
        b'POST /push_tx HTTP/1.1\r\nHost: x\r\nContent-Length: 12\r\n\r\n{"tx_hex":1}',
        b'POST /push_tx HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\n5\r\nhello\r\n0\r\nX-T: 1\r\n\r\n',
        b'GET /get_block?block=1 HTTP/1.0\r\nConnection: keep-alive\r\n\r\nGET / HTTP/1.1\r\nConnection: close\r\n\r\n',
        b'POST /a HTTP/1.1\r\nExpect: 100-continue\r\nContent-Length: 3\r\n\r\nabc',
        b'GET /ws HTTP/1.1\r\nConnection: Upgrade\r\nUpgrade: websocket\r\nSec-WebSocket-Key: dGhlIHNhbXBsZSBub25jZQ==\r\n\r\n\x81\x85',
    ]
    out = [bytes([0, k * 37 % 256]) + r for k, r in enumerate(reqs)]

    def frame(op, payload, fin=True, mask=b'\x01\x02\x03\x04'):
        n = len(payload)
        head = bytes([(0x80 if fin else 0) | op])
        if n < 126:
            head += bytes([0x80 | n])
        elif n < 65536:
            head += bytes([0x80 | 126]) + struct.pack('>H', n)
        else:
            head += bytes([0x80 | 127]) + struct.pack('>Q', n)
        return head + mask + bytes(b ^ mask[i % 4] for i, b in enumerate(payload))
    frames = [frame(1, b'{"type":"ping"}'), frame(9, b''), frame(8, b'\x03\xe8'), frame(2, b'x' * 300),
              frame(1, b'ab', fin=False) + frame(0, b'cd'), frame(1, b'y' * 70000)]
    out += [bytes([1, k * 53 % 256]) + f for k, f in enumerate(frames)]
    return out


def tx_seeds():
    from upow_amd.models.transaction import CoinbaseTransaction, Transaction, TransactionInput, TransactionOutput
    from upow_amd.ops import p256 as op
    from upow_amd.utils.codec import OutputType, TransactionType, point_to_bytes, point_to_string, AddressFormat
    from upow_amd.wallet.builders import type_message
    rng = random.Random(3)
    keys = [rng.randrange(1, op.oracle.N) for _ in range(3)]
    pubs = [op.public_key(k) for k in keys]
    addrs = [point_to_string(p) for p in pubs]
    full = point_to_string(pubs[2], AddressFormat.FULL_HEX)

    def inputs(k, n):
        out = []
        for i in range(n):
            t = TransactionInput(rng.randbytes(32).hex(), i)
            t.public_key = pubs[k]
            out.append(t)
        return out
    txs = [Transaction(inputs(0, 2), [TransactionOutput(addrs[1], Decimal('1.5')), TransactionOutput(addrs[0], Decimal('0.25'))]).sign([keys[0]]),
           Transaction(inputs(1, 1), [TransactionOutput(addrs[0], Decimal('3'))], b'hello world').sign([keys[1]]),
           Transaction(inputs(1, 1), [TransactionOutput(addrs[0], Decimal('10'), OutputType.VOTE_AS_DELEGATE)],
                       type_message(TransactionType.VOTE_AS_DELEGATE)).sign([keys[1]]),
           Transaction(inputs(2, 1), [TransactionOutput(full, Decimal('2'))], version=1).sign([keys[2]])]
    two = inputs(0, 1) + inputs(1, 1)  # one signature per input
    txs.append(Transaction(two, [TransactionOutput(addrs[2], Decimal('1'))]).sign(keys[:2]))
    hexes = [t.hex() for t in txs] + [CoinbaseTransaction(rng.randbytes(32).hex(), addrs[0], Decimal(6)).hex()]
    out = []
    for h in hexes:
        raw = bytes.fromhex(h)
        out += [b'\x00' + raw, b'\x01' + raw, b'\x02' + h.encode()]
    return out


def json_seeds(tx_hexes):
    """Request and page bodies the span parser sees (csrc/jsonspan.cpp): /push_block bodies, /get_blocks
    pages, and JSON outside the plain subset (escapes, UTF-8, numbers, nesting, duplicate keys)."""
    import json
    hexes = [h[1:].hex() if h[:1] == b'\x00' else None for h in tx_hexes]
    hexes = [h for h in hexes if h]
    push = {'block_content': 'ab' * 108, 'txs': hexes, 'block_no': 7}
    page = {'ok': True, 'result': [{'block': {'id': 5, 'hash': 'cd' * 32, 'content': 'ef' * 108, 'address': 'D' * 45,
                                              'random': 0, 'difficulty': 6.3, 'reward': 6.0, 'timestamp': 1700000000},
                                    'transactions': hexes[:3]}, {'block': {'id': 6}, 'transactions': []}]}
    docs = [json.dumps(push).encode(), json.dumps(push, separators=(',', ':')).encode(), json.dumps(page).encode(),
            json.dumps(page, indent=2).encode(), b'{"txs": ["ab", "c\\"d"], "txs": ["x"]}',
            '{"k": "\u00e9\u2603", "txs": ["\u00e9"], "n": [-0.0, 1e400, 12345678901234567890, 1E-5]}'.encode(),
            b'[[[[[[{"transactions": [ ]}]]]]]]', b' {"a":true,"b":false,"c":null} ', b'{"txs": "ab"}',
            b'{"txs": [1, "a"]}', b'"\\ud800"', b'{"transactions": ["a" ,"b" , "c"]}']
    return docs


def main(out_dir):
    tx = tx_seeds()
    for name, seeds in (('http', http_seeds()), ('tx', tx), ('json', json_seeds(tx))):
        d = os.path.join(out_dir, name)
        os.makedirs(d, exist_ok=True)
        for k, s in enumerate(seeds):
            with open(os.path.join(d, f'seed_{k:03d}'), 'wb') as f:
                f.write(s)
    print(f'corpus seeds written under {out_dir}')


if __name__ == '__main__':
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, 'build', 'fuzz', 'corpus'))
