"""Second headline metric: tx-verify/s on a synthetic 2 MB block (BASELINE.json config 4).

Setup (untimed): an in-memory ledger with a funding block of P-256-owned outputs, then ``steps +
warmup`` full blocks of ~8,300 transactions (2 inputs of one random key, 2 outputs, 1 signature:
216 B each -> 1.79 MB per block, under the 2 MB cap). Every block header is mined at the chain's
difficulty (6.0) on the GPU.

Timed: for each block exactly what ``POST /push_block`` does with full tx hex — parse every tx
(``Transaction.from_hex``) and ``manager.create_block``: PoW/prev/timestamp/size checks, per-category
UTXO probes against the HBM index, batched point decompression, ONE batched P-256 verify launch
(+ ASCII-hex fallback pass), per-tx rule checks, merkle root, then the ledger writes and the UTXO
index insert/erase. Weak scaling: each rank validates its own chain on its own GPU.
"""
from __future__ import annotations

import asyncio
import hashlib
import json
import os
import random
import time
from typing import Optional
from decimal import Decimal

from .constants import SMALLEST
from .utils import hexspans


def batch_keys(n: int, rng, threads: int = 16):
    """``n`` random P-256 private keys, their public points (x, y little-endian) and 33-byte compressed
    addresses, computed in one native batch on host threads (csrc/bindings.cpp ``p256_pubkey_batch``)."""
    from .ops.native import lib
    from .utils.p256 import N
    keys = [rng.randrange(1, N) for _ in range(n)]
    pubs = lib().p256_pubkey_batch(b''.join(k.to_bytes(32, 'big') for k in keys), threads)
    addr33 = []
    for i in range(n):
        q = pubs[64 * i:64 * i + 64]
        addr33.append(bytes([43 if q[32] & 1 else 42]) + q[:32])
    return keys, pubs, addr33


def _amount_bytes(units: int) -> bytes:
    n = (units.bit_length() + 7) // 8
    return bytes([n]) + units.to_bytes(n, 'little')


def signed_spend_txs(spends, keys, owner33, recip33, amount_out=(1_250_000_000, 749_000_000), threads: int = 16):
    """Version-3 2-in/2-out regular txs, serialised and signed in bulk (the bytes ``Transaction.sign().hex()``
    produces: reference transaction.py:46-83 layout, RFC 6979 signature over SHA-256 of the unsigned part,
    one signature for both inputs). ``spends[j]`` = ((txid, index), (txid, index)) of tx ``j``, signed by
    ``keys[j]``; output 0 pays ``recip33[j]``, output 1 returns change to ``owner33[j]``."""
    from .ops.native import lib
    a0, a1 = _amount_bytes(amount_out[0]) + b'\x00', _amount_bytes(amount_out[1]) + b'\x00'
    unsigned, digests = [], []
    for j, ((h1, i1), (h2, i2)) in enumerate(spends):
        u = (b'\x03\x02' + bytes.fromhex(h1) + bytes([i1, 0]) + bytes.fromhex(h2) + bytes([i2, 0]) + b'\x02'
             + recip33[j] + a0 + owner33[j] + a1)
        unsigned.append(u)
        digests.append(hashlib.sha256(u).digest())
    sigs = lib().p256_sign_batch(b''.join(keys[j].to_bytes(32, 'big') for j in range(len(spends))), b''.join(digests),
                                 threads)
    return [(u + b'\x00' + sigs[64 * j:64 * j + 64]).hex() for j, u in enumerate(unsigned)]


def signed_grouped_txs(spends, keys_a, keys_b, owner33, recip33, amount_out=(1_250_000_000, 749_000_000),
                       threads: int = 16):
    """Version-3 4-in/2-out txs spending two outputs of key A then two of key B, with TWO signatures: the
    1 < k < n case whose signature -> input assignment groups the inputs by owner key (reference
    transaction.py:578-590), as a wallet produces when it spends coins of several keys together."""
    from .ops.native import lib
    a0, a1 = _amount_bytes(amount_out[0]) + b'\x00', _amount_bytes(amount_out[1]) + b'\x00'
    unsigned, digests = [], []
    for j, ins in enumerate(spends):
        u = b'\x03\x04' + b''.join(bytes.fromhex(h) + bytes([i, 0]) for h, i in ins) + b'\x02' + recip33[j] + a0 \
            + owner33[j] + a1
        unsigned.append(u)
        digests.append(hashlib.sha256(u).digest())
    dig = b''.join(digests)
    sa = lib().p256_sign_batch(b''.join(k.to_bytes(32, 'big') for k in keys_a), dig, threads)
    sb = lib().p256_sign_batch(b''.join(k.to_bytes(32, 'big') for k in keys_b), dig, threads)
    return [(u + b'\x00' + sa[64 * j:64 * j + 64] + sb[64 * j:64 * j + 64]).hex() for j, u in enumerate(unsigned)]


def _funding_tx(owner_addrs, amount: Decimal, rng):
    from .models.transaction import Transaction, TransactionInput, TransactionOutput
    inp = TransactionInput(rng.randbytes(32).hex(), 0)
    inp.signed = (1, 1)
    return Transaction([inp], [TransactionOutput(a, amount) for a in owner_addrs])


async def _setup(n_blocks: int, txs_per_block: int, seed: int, utxo_backend=None, device=None, base_ts=None,
                 make_blocks: bool = True, ledger_path: str = None, governance: bool = False, gov_txs: float = 0.0,
                 age_txs: int = 0, aging: dict = None, distinct_keys: bool = False, grouped_txs: float = 0.0,
                 tx_counts: list = None):
    """``gov_txs`` > 0: that fraction of every block's txs are governance txs (70 % delegate votes, 10 %
    validator votes, 20 % delegate revokes of seeded ballots, signed by the voters) on a seeded governance
    state; the chain starts four days back so the seeded ballots are past the 48 h revoke window.

    ``distinct_keys``: every plain tx slot gets its own fresh key pair (it owns the two funding outputs the
    tx spends) and pays a fresh recipient address — a 2 MB block then has ~8,300 distinct signers and
    ~16,600 distinct output addresses, as random-keypair traffic does. Default (False): a pool of 256 keys
    signs every tx and receives every output (cache-friendly: key dedup and the base58 memo hit).

    ``tx_counts``: a tx count per block (mainnet-shaped chains: most blocks carry 0-20 txs) instead of
    ``txs_per_block`` for every block."""
    from . import devnet
    from .ledger import manager
    from .ledger.database import Database
    from .models.transaction import CoinbaseTransaction, Transaction, TransactionInput, TransactionOutput
    from .ops import p256 as op
    from .utils.codec import point_to_string
    rng = random.Random(seed)
    db = await Database.create(ledger_path, utxo_backend=utxo_backend)
    manager.Manager.difficulty = None
    keys = [rng.randrange(1, op.oracle.N) for _ in range(256)]
    addrs = [point_to_string(op.public_key(k)) for k in keys]
    n_gov = int(round(gov_txs * txs_per_block)) if gov_txs > 0 else 0
    n_dv, n_vv = int(n_gov * 0.7), int(n_gov * 0.1)
    n_rv = n_gov - n_dv - n_vv
    if base_ts is None:
        base_ts = int(time.time()) - (4 * 86_400 if n_gov else 0) - max(10_000, SPACING_S * (n_blocks + 10))
    genesis_addr = addrs[0]
    await devnet.mine_block(genesis_addr, ts=base_ts, device=device)
    if age_txs:
        info = age_ledger(db, age_txs, random.Random(seed ^ 0xA6ED))  # own stream: funding stays seed-identical
        if aging is not None:
            aging.update(info)
    # funding block written straight into the ledger (trusted setup, not part of the measurement)
    # grouped txs (distinct keys only) spend two key slots each: size the funding for the extra slots
    n_grp = int(round(grouped_txs * txs_per_block)) if (grouped_txs > 0 and distinct_keys) else 0
    counts = list(tx_counts) if tx_counts is not None else [txs_per_block] * n_blocks
    n_out = (sum(counts) + n_blocks * n_grp) * 2
    if distinct_keys:
        # own streams, so the funding set is identical whether or not this rank builds the blocks
        from .utils.codec import bytes_to_string
        t_keys = time.perf_counter()
        tx_keys, _, tx_owner33 = batch_keys(n_out // 2, random.Random(seed * 7919 + 17))
        owner_addr = [bytes_to_string(a) for a in tx_owner33]
        fund_addrs = [owner_addr[i // 2] for i in range(n_out)]  # tx slot j owns outputs 2j and 2j+1
        if aging is not None:
            aging['distinct_key_setup_s'] = round(time.perf_counter() - t_keys, 2)
    else:
        owners = [(i // 2) % 256 for i in range(n_out)]  # outputs 2j and 2j+1 share an owner
        fund_addrs = [addrs[o] for o in owners]
    funding = []
    for k in range(0, n_out, 255):
        funding.append(_funding_tx(fund_addrs[k:k + 255], Decimal(10), rng))
    block_hash = rng.randbytes(32).hex()
    last = await db.get_last_block()
    await db.add_block(2, block_hash, last['content'], genesis_addr, 0, Decimal('6.0'), Decimal(6), base_ts + 1)
    cb = CoinbaseTransaction(block_hash, genesis_addr, Decimal(6))
    await db.add_transaction(cb, block_hash)
    rows = []
    for t in funding:
        rows.append((block_hash, t.hash(), t.hex(), '[]', __import__('json').dumps([o.address for o in t.outputs]),
                     __import__('json').dumps([int(o.amount * SMALLEST) for o in t.outputs]), '0.000000'))
    db.insert_transaction_rows(rows)
    await db.add_transaction_outputs(funding + [cb])
    seeded = None
    if governance or n_gov:
        blocks_n = n_blocks if make_blocks else 0
        seeded = _seed_governance(db, rng, block_hash, n_validators=max(200, blocks_n * n_vv + 1),
                                  n_delegates=max(5000, blocks_n * (n_dv + n_rv) + 1))
    outpoints = [(t.hash(), i) for t in funding for i in range(len(t.outputs))]
    # spending blocks
    blocks = []
    j = 0
    gov_next = {'d': 0, 'v': 0}
    if distinct_keys and make_blocks:
        _, _, recip33 = batch_keys(n_out // 2, random.Random(seed * 7919 + 29))
    for b in range(n_blocks if make_blocks else 0):
        txs = []
        if n_gov:
            txs.extend(_governance_txs(seeded, gov_next, n_dv, n_vv, n_rv, rng))
        if distinct_keys:
            n_plain = counts[b] - len(txs) - n_grp
            slots = range(j, j + n_plain)
            txs.extend(signed_spend_txs([(outpoints[2 * s], outpoints[2 * s + 1]) for s in slots],
                                        [tx_keys[s] for s in slots], [tx_owner33[s] for s in slots],
                                        [recip33[s] for s in slots]))
            j += n_plain
            if n_grp:  # slot pairs (A, B): A's two outputs then B's, signed by A and B
                pairs = [(j + 2 * q, j + 2 * q + 1) for q in range(n_grp)]
                txs.extend(signed_grouped_txs(
                    [[outpoints[2 * a], outpoints[2 * a + 1], outpoints[2 * b], outpoints[2 * b + 1]] for a, b in pairs],
                    [tx_keys[a] for a, _ in pairs], [tx_keys[b] for _, b in pairs], [tx_owner33[a] for a, _ in pairs],
                    [recip33[a] for a, _ in pairs]))
                j += 2 * n_grp
            if n_gov or n_grp:
                rng.shuffle(txs)
            blocks.append(txs)
            continue
        for _ in range(counts[b] - len(txs)):
            (h1, i1), (h2, i2) = outpoints[2 * j], outpoints[2 * j + 1]
            owner = owners[2 * j]
            j += 1
            ins = [TransactionInput(h1, i1, amount=Decimal(10)), TransactionInput(h2, i2, amount=Decimal(10))]
            for i in ins:
                i.public_key = op.public_key(keys[owner])
            outs = [TransactionOutput(addrs[rng.randrange(256)], Decimal('12.5')),
                    TransactionOutput(addrs[owner], Decimal('7.49'))]
            tx = Transaction(ins, outs)
            tx.sign([keys[owner]])
            txs.append(tx.hex())
        if n_gov:
            rng.shuffle(txs)
        blocks.append(txs)
    return db, genesis_addr, blocks, base_ts


SPACING_S = 45  # verify benches: block timestamps 45 s apart, so every 100-block retarget raises the difficulty


async def premine_headers(db, addr: str, blocks, base_ts: int, device, spacing: int = SPACING_S):
    """Headers for ``blocks`` on top of ``db``'s tip, timestamps ``spacing`` apart, each mined at the difficulty
    the chain will require of it (``manager.difficulty_schedule``: calculate_difficulty's retarget arithmetic
    over the planned timestamps), so a run longer than 100 blocks crosses retargets like a real chain.
    Returns (headers, difficulties)."""
    from . import devnet
    from .ledger import manager
    from .models.block import get_transactions_merkle_tree
    rows = db._q('SELECT timestamp, difficulty FROM blocks ORDER BY id')
    chain = [(int(r[0]), r[1]) for r in rows]
    ts = [base_ts + spacing * (b + 1) for b in range(len(blocks))]
    ts = [max(t, chain[-1][0] + 1 + b) for b, t in enumerate(ts)] if chain else ts
    diffs = manager.difficulty_schedule(chain, ts)
    prev = (await db.get_last_block())['hash']
    headers = []
    for b, txs_hex in enumerate(blocks):
        content = devnet.mine_header_raw(prev, addr, get_transactions_merkle_tree(txs_hex), ts[b], diffs[b],
                                         device=device)
        headers.append(content)
        prev = hashlib.sha256(bytes.fromhex(content)).hexdigest()
    return headers, diffs


def _io_write_mb() -> Optional[float]:
    """Bytes this process has caused to be written to storage so far (/proc/self/io write_bytes), in MB."""
    try:
        with open('/proc/self/io') as f:
            for line in f:
                if line.startswith('write_bytes:'):
                    return int(line.split()[1]) / 2**20
    except OSError:
        pass
    return None


def _governance_txs(seeded, nxt, n_dv, n_vv, n_rv, rng):
    """One block's governance txs (wallet/builders.py shapes): delegate votes spending a seeded delegate
    voting-power output, validator votes spending a validator voting-power output, and delegate revokes of
    seeded ballots; every delegate/validator is used once per run."""
    from .models.transaction import Transaction, TransactionInput, TransactionOutput
    from .ops import p256 as op
    from .utils.codec import OutputType as O, TransactionType as T
    from .wallet.builders import type_message
    out = []

    def tx(key, inputs, outputs, t):
        ins = [TransactionInput(h, i) for h, i in inputs]
        pub = op.public_key(key)
        for i in ins:
            i.public_key = pub
        return Transaction(ins, outputs, type_message(t)).sign([key]).hex()
    for _ in range(n_dv):
        d = seeded['delegates'][nxt['d']]
        nxt['d'] += 1
        v = rng.randint(1, 10)
        target = seeded['validators'][rng.randrange(len(seeded['validators']))]['addr']
        outs = [TransactionOutput(target, Decimal(v), O.VOTE_AS_DELEGATE)]
        if v < 10:
            outs.append(TransactionOutput(d['addr'], Decimal(10 - v), O.DELEGATE_VOTING_POWER))
        out.append(tx(d['key'], [d['dvp']], outs, T.VOTE_AS_DELEGATE))
    for _ in range(n_vv):
        val = seeded['validators'][nxt['v']]
        nxt['v'] += 1
        v = rng.randint(1, 10)
        target = seeded['inodes'][rng.randrange(len(seeded['inodes']))]
        outs = [TransactionOutput(target, Decimal(v), O.VOTE_AS_VALIDATOR)]
        if v < 10:
            outs.append(TransactionOutput(val['addr'], Decimal(10 - v), O.VALIDATOR_VOTING_POWER))
        out.append(tx(val['key'], [val['vvp']], outs, T.VOTE_AS_VALIDATOR))
    for _ in range(n_rv):
        d = seeded['delegates'][nxt['d']]
        nxt['d'] += 1
        out.append(tx(d['key'], [d['ballot']], [TransactionOutput(d['addr'], Decimal(d['vote']), O.DELEGATE_VOTING_POWER)],
                      T.REVOKE_AS_DELEGATE))
    return out


def age_ledger(db, n_txs: int, rng, chunk: int = 250_000) -> dict:
    """Trusted bulk aging (untimed setup): ``n_txs`` synthetic confirmed transactions attached to the genesis
    block, each with two unspent outputs owned by a pool of 1,024 addresses — ``n_txs`` transaction rows and
    ``2 * n_txs`` UTXO rows in the SQL tables (both UTXO files) and in the UTXO index, the size a long-running
    mainnet node's ledger has. Rows go through sqlite's executemany in large transactions; the index is
    loaded in one batch from the same arrays (no SQL read-back)."""
    import numpy as np
    from .ledger.utxo import PAYLOAD_DTYPE, TAG_BY_TABLE
    from .ops import p256 as op
    from .utils.codec import point_to_string, string_to_bytes
    t0 = time.perf_counter()
    genesis = db._q1('SELECT hash FROM blocks WHERE id = 1')[0]
    pool = [point_to_string(op.public_key(rng.randrange(1, op.oracle.N))) for _ in range(1024)]
    pool_raw = [string_to_bytes(a) for a in pool]
    nrng = np.random.default_rng(rng.randrange(1 << 32))
    recs_all, pay_all = [], []
    done = 0
    while done < n_txs:
        n = min(chunk, n_txs - done)
        hashes = nrng.integers(0, 256, size=(n, 32), dtype=np.uint8)
        hexes = [bytes(h).hex() for h in hashes]
        owners = nrng.integers(0, len(pool), size=(n, 2))
        amounts = nrng.integers(1, 10 ** 10, size=(n, 2))
        body = nrng.integers(0, 256, size=(n, 110), dtype=np.uint8)
        tx_rows, u_rows = [], []
        for k in range(n):
            a0, a1 = pool[owners[k, 0]], pool[owners[k, 1]]
            x0, x1 = int(amounts[k, 0]), int(amounts[k, 1])
            tx_rows.append((genesis, hexes[k], bytes(body[k]).hex(), '[]', f'["{a0}","{a1}"]', f'[{x0},{x1}]',
                            '0.000000'))
            u_rows.append((hexes[k], 0, a0, None))
            u_rows.append((hexes[k], 1, a1, None))
        with db.transaction(foreign_keys=False, invalidate=False):
            ins_tx = ('INSERT INTO transactions (block_hash, tx_hash, tx_hex, inputs_addresses, outputs_addresses, '
                      'outputs_amounts, fees) VALUES (?, ?, ?, ?, ?, ?, ?)')
            if db._split_target(ins_tx):
                db._routed_exec('transactions', ins_tx, tx_rows)
            else:
                db._conn.executemany(ins_tx, tx_rows)
            db._routed_exec('unspent_outputs', 'INSERT INTO unspent_outputs (tx_hash, "index", address, is_stake) '
                            'VALUES (?, ?, ?, ?)', u_rows)
        recs = np.zeros((2 * n, 40), dtype=np.uint8)
        recs[:, :32] = np.repeat(hashes, 2, axis=0)
        recs[:, 32:36] = np.tile(np.array([[0, 0, 0, 0], [1, 0, 0, 0]], np.uint8), (n, 1))
        recs[:, 36:40] = np.frombuffer(np.uint32(TAG_BY_TABLE['unspent_outputs']).tobytes(), np.uint8)
        pay = np.zeros(2 * n, dtype=PAYLOAD_DTYPE)
        pay['amount'] = amounts.reshape(-1).astype(np.uint64)
        own = owners.reshape(-1)
        raw = np.zeros((len(pool), 64), np.uint8)
        lens = np.zeros(len(pool), np.uint32)
        for i, r in enumerate(pool_raw):
            raw[i, :len(r)] = np.frombuffer(r, np.uint8)
            lens[i] = len(r)
        pay['addr'] = raw[own]
        pay['len'] = lens[own]
        recs_all.append(recs)
        pay_all.append(pay)
        done += n
    t1 = time.perf_counter()
    live, live_pay = db.utxo.records_payload()
    db.utxo.reset_records(np.concatenate([live] + recs_all), np.concatenate([live_pay] + pay_all))
    db._info_cache.clear()
    return {'aged_txs': n_txs, 'aged_utxos': 2 * n_txs, 'sql_insert_s': round(t1 - t0, 1),
            'index_load_s': round(time.perf_counter() - t1, 1), 'utxo_index_entries': len(db.utxo)}


def _admit_untimed(db, txs_hex):
    """Put a block's txs into the mempool tables as if each had gone through /push_tx earlier
    (trusted bulk insert, outside the timed region): pending_transactions rows + one
    pending_spent_outputs row per input."""
    now = int(time.time())
    rows, spent = [], []
    for h in txs_hex:
        raw = bytes.fromhex(h)
        rows.append((hashlib.sha256(raw).hexdigest(), h, '[]', '0.000000', now))
        n_in = raw[1]
        for k in range(n_in):
            rec = raw[2 + 34 * k: 2 + 34 * (k + 1)]
            spent.append((rec[:32].hex(), rec[32]))
    with db.transaction():
        db.conn.executemany('INSERT INTO pending_transactions (tx_hash, tx_hex, inputs_addresses, fees, '
                            'propagation_time) VALUES (?, ?, ?, ?, ?)', rows)
        db.conn.executemany('INSERT INTO pending_spent_outputs (tx_hash, "index") VALUES (?, ?)', spent)


def _seed_governance(db, rng, block_hash: str, n_inodes: int = 12, n_validators: int = 200,
                     n_delegates: int = 5000):
    """Trusted setup of a governance-heavy chain state inside the funding block (written straight into the
    ledger like the funding outputs; not part of the measurement): every validator and delegate has a
    staked output and a voting-power output, validators and inodes are registered, each delegate votes for
    one validator and each validator for two inodes. Row layout as the reference's output tables
    (database.py:524-580): a ballot carries the vote in ``outputs_amounts[index]`` and the voter in
    ``inputs_addresses[index]`` of its tx. Returns the keys and outpoints per role."""
    import json
    from .ops import p256 as op
    from .utils.codec import point_to_string
    keys = [rng.randrange(1, op.oracle.N) for _ in range(n_inodes + n_validators + n_delegates)]
    addrs = [point_to_string(op.public_key(k)) for k in keys]
    inodes = addrs[:n_inodes]
    validators = addrs[n_inodes:n_inodes + n_validators]
    delegates = addrs[n_inodes + n_validators:]
    tx_rows = []
    tables = {t: [] for t in ('unspent_outputs', 'inode_registration_output', 'validator_registration_output',
                              'validators_voting_power', 'delegates_voting_power', 'validators_ballot',
                              'inodes_ballot')}

    def tx(voter, receiver, amount):
        h = rng.randbytes(32).hex()
        tx_rows.append((block_hash, h, rng.randbytes(120).hex(), json.dumps([voter]), json.dumps([receiver]),
                        json.dumps([amount]), '0.000000'))
        return h
    out = {'inodes': inodes, 'validators': [], 'delegates': []}
    for a in validators + delegates:  # staked outputs (unspent_outputs.is_stake = 1)
        tables['unspent_outputs'].append((tx(a, a, 10 * SMALLEST), 0, a, 1))
    for a in inodes:
        tables['inode_registration_output'].append((tx(a, a, 1000 * SMALLEST), 0, a))
    for k, a in enumerate(validators):
        tables['validator_registration_output'].append((tx(a, a, 100 * SMALLEST), 0, a))
        vvp = tx(a, a, 10 * SMALLEST)
        tables['validators_voting_power'].append((vvp, 0, a))
        out['validators'].append({'key': keys[n_inodes + k], 'addr': a, 'vvp': (vvp, 0)})
        for _ in range(2):
            target = inodes[rng.randrange(n_inodes)]
            tables['inodes_ballot'].append((tx(a, target, rng.randint(1, 5) * SMALLEST), 0, target))
    for k, a in enumerate(delegates):
        dvp = tx(a, a, 10 * SMALLEST)
        tables['delegates_voting_power'].append((dvp, 0, a))
        target = validators[rng.randrange(n_validators)]
        vote = rng.randint(1, 10)
        ballot = tx(a, target, vote * SMALLEST)
        tables['validators_ballot'].append((ballot, 0, target))
        out['delegates'].append({'key': keys[n_inodes + n_validators + k], 'addr': a, 'dvp': (dvp, 0),
                                 'ballot': (ballot, 0), 'vote': vote})
    db.insert_transaction_rows(tx_rows)
    db._xm('INSERT INTO unspent_outputs (tx_hash, "index", address, is_stake) VALUES (?, ?, ?, ?)',
           tables.pop('unspent_outputs'))
    for t, rows in tables.items():
        db._xm(f'INSERT INTO {t} (tx_hash, "index", address) VALUES (?, ?, ?)', rows)
    db._rebuild_utxo_index()  # index + governance index from the tables
    return out


async def _governance_probe(db) -> dict:
    """get_active_inodes on the seeded chain: the first (index build of the aggregates) and the
    per-block steady-state call (memoised until a governance write), and the SQL cascade's cost for
    one validator's stake (database.py:1127-1136 + 1189-1205, the per-ballot N+1) for comparison."""
    t0 = time.perf_counter()
    first = await db.get_active_inodes()
    t1 = time.perf_counter()
    n = 200
    for _ in range(n):
        await db.get_active_inodes()
    t2 = time.perf_counter()
    db.gov.version += 1  # force one full recomputation of the aggregates
    await db.get_active_inodes()
    t3 = time.perf_counter()
    validator = db.gov.ballot_rows('inodes_ballot', None, False)[0][3]
    gov, db.gov = db.gov, None
    try:
        t4 = time.perf_counter()
        sql_stake = await db.get_validators_stake(validator)
        t5 = time.perf_counter()
    finally:
        db.gov = gov
    idx_stake = await db.get_validators_stake(validator)
    t = db.gov.tables
    return {'inodes': len(t['inode_registration_output']), 'validators': len(t['validator_registration_output']),
            'delegates_ballots': len(t['validators_ballot']), 'inode_ballots': len(t['inodes_ballot']),
            'stake_rows': len(t['stake']), 'active_inodes': len(first),
            'get_active_inodes_first_ms': round((t1 - t0) * 1e3, 3),
            'get_active_inodes_per_block_ms': round((t2 - t1) * 1e3 / n, 4),
            'get_active_inodes_recompute_ms': round((t3 - t2) * 1e3, 3),
            'one_validator_stake_sql_ms': round((t5 - t4) * 1e3, 2), 'stake_matches_sql': sql_stake == idx_stake}


def _dump_profile(prof, path: str):
    import io
    import pstats
    prof.disable()
    out = io.StringIO()
    st = pstats.Stats(prof, stream=out)
    st.sort_stats('cumulative').print_stats(70)
    st.sort_stats('tottime').print_stats(40)
    with open(path, 'w') as f:
        f.write(out.getvalue())


def _distinct(args) -> bool:
    return getattr(args, 'keys', 'distinct') == 'distinct'


def _data_label(args) -> str:
    if _distinct(args):
        return ('synthetic 2 MB blocks: a fresh random P-256 key pair per tx (~8,300 distinct signers) paying a '
                'fresh address (~16,600 distinct output addresses per block), 2-in/2-out signed txs, funding UTXOs')
    return ('synthetic 2 MB blocks: 256 random P-256 keys sign every tx and own every output (cache-friendly), '
            '2-in/2-out signed txs, funding UTXOs')


def _ledger_path(args, ctx):
    """``--ledger DIR``: a file-backed ledger (WAL, synchronous=NORMAL — what a node runs with) in a
    fresh per-rank directory; default is an in-memory SQLite ledger."""
    base = getattr(args, 'ledger', None)
    if not base:
        return None
    import os
    import tempfile
    os.makedirs(base, exist_ok=True)
    return os.path.join(tempfile.mkdtemp(prefix=f'bench_r{ctx.rank}_', dir=base), 'ledger.sqlite3')


async def _run(args, ctx, device, utxo_backend):
    from . import devnet
    from .ledger import fastpath, manager, validate
    from .models.transaction import Transaction
    segments = max(1, int(getattr(args, 'segments', 1) or 1))
    n_blocks = args.steps * segments + args.warmup
    gov = getattr(args, 'governance', False)
    gov_txs = float(getattr(args, 'governance_txs', 0.0) or 0.0)
    aging = {}
    db, addr, blocks, base_ts = await _setup(n_blocks, args.txs, 1234 + ctx.rank, utxo_backend, device,
                                             ledger_path=_ledger_path(args, ctx), governance=gov, gov_txs=gov_txs,
                                             age_txs=int(getattr(args, 'age_txs', 0) or 0), aging=aging,
                                             distinct_keys=_distinct(args),
                                             grouped_txs=float(getattr(args, 'grouped_txs', 0.0) or 0.0))
    key_setup = aging.pop('distinct_key_setup_s', None)
    if aging:
        db.flush()
    # (untimed) the txs as a node holds them: parsed from a /push_block JSON body (node/main.py _json_body),
    # which leaves the tx array inside the body bytes (utils/hexspans.py); the parse itself is timed apart
    bodies = [json.dumps({'block_content': '', 'txs': b}).encode() for b in blocks]
    extra_parse = _body_parse_ms(bodies[0]) if bodies else None
    blocks = [(json.loads if _TX_LISTS else hexspans.loads)(body)['txs'] for body in bodies]
    del bodies
    gov_probe = await _governance_probe(db) if gov else None
    # mine every header up front (untimed), each at the difficulty the chain will require of it
    headers, difficulties = await premine_headers(db, addr, blocks, base_ts, device)
    stages = []
    paths = set()
    total_txs = 0
    prof = None
    if os.environ.get('UPOW_BENCH_PROFILE'):
        import cProfile
        prof = cProfile.Profile()
    from_mempool = getattr(args, 'from_mempool', False)
    queue_trace = []  # (journal records not yet in SQL, bytes queued) after each timed block
    untimed = 0.0  # mempool admission of the next block's txs happens inside the wall-clock window
    seg_walls, seg_txs = [], []  # per segment of ``steps`` blocks, each ending with its own SQL drain
    seg_diag = []  # per segment: where its wall time went (the spread between segments of one run)

    def writer_snapshot():
        if db.writer is None:
            return None
        import resource
        w = db.writer.stats()
        ru = resource.getrusage(resource.RUSAGE_SELF)
        return {'t': time.perf_counter(), 'submitted': w['submitted'], 'applied': w['applied'],
                'throttle_s': w['throttle_s'], 'fdatasync_s': w['fdatasync_s'],
                'io': [w.get(k, 0.0) for k in ('io_queue_s', 'io_crc_s', 'io_write_s', 'io_undo_wait_s')],
                'apply': [sh['apply_s'] for sh in w['shards']], 'commit': [sh['commit_s'] for sh in w['shards']],
                'cpu_s': ru.ru_utime + ru.ru_stime, 'nivcsw': ru.ru_nivcsw, 'write_mb': _io_write_mb()}

    def end_segment():
        lag = None
        w0 = seg[3]
        if db.writer is not None:
            st = db.writer.stats()
            lag = st['submitted'] - st['applied']
        tf = time.perf_counter()
        db.flush()
        ctx.synchronize()
        te = time.perf_counter()
        seg_walls.append(te - seg[0] - (untimed - seg[1]))
        seg_txs.append(total_txs - seg[2])
        blocks_in = stages[seg[4]:]
        d = {'wall_ms': round(seg_walls[-1] * 1000, 2), 'tx_per_s': round(seg_txs[-1] / seg_walls[-1], 1),
             'commit_latency_ms': round(1000 * sum(x['block_s'] for x in blocks_in) / max(1, len(blocks_in)), 3),
             'drain_ms': round((te - tf) * 1000, 2), 'lag_records_before_drain': lag}
        for k in ('decode_s', 'utxo_s', 'ecdsa_s', 'apply_commit_s'):
            vals = [x[k] for x in blocks_in if isinstance(x.get(k), float)]
            if vals:
                d[k.replace('_s', '_ms')] = round(1000 * sum(vals) / len(vals), 3)
        w1 = writer_snapshot()
        if w0 is not None and w1 is not None:
            nb = max(1, len(blocks_in))
            ap = [(b - a) * 1000 / nb for a, b in zip(w0['apply'], w1['apply'])]
            cm = [(b - a) * 1000 / nb for a, b in zip(w0['commit'], w1['commit'])]
            wall = w1['t'] - w0['t']
            d.update({'throttle_ms': round((w1['throttle_s'] - w0['throttle_s']) * 1000, 2),
                      'fdatasync_ms_per_block': round((w1['fdatasync_s'] - w0['fdatasync_s']) * 1000 / nb, 3),
                      # the journal I/O thread per block: queue wait, checksum, write, undo-writer wait
                      'journal_io_ms_per_block': dict(zip(('queue', 'crc', 'write', 'undo_wait'),
                                                          [round((b - a) * 1000 / nb, 3) for a, b in zip(w0['io'], w1['io'])])),
                      'materialiser_busy_ms_per_block': [round(a + c, 2) for a, c in zip(ap, cm)],
                      'materialiser_apply_ms_per_block': round(max(ap[1:] or ap), 2),
                      'materialiser_commit_ms_per_block': round(max(cm[1:] or cm), 2),
                      'process_cores_busy': round((w1['cpu_s'] - w0['cpu_s']) / wall, 2) if wall > 0 else None,
                      'involuntary_switches': w1['nivcsw'] - w0['nivcsw'],
                      'write_mb_per_block': round((w1['write_mb'] - w0['write_mb']) / nb, 2)
                      if w1['write_mb'] is not None and w0['write_mb'] is not None else None})
        seg_diag.append(d)
    seg = None
    for b, txs_hex in enumerate(blocks):
        if from_mempool:
            ta = time.perf_counter()
            _admit_untimed(db, txs_hex)
            hashes = [hashlib.sha256(bytes.fromhex(h)).hexdigest() for h in txs_hex]  # the miner's request
            if b > args.warmup:
                untimed += time.perf_counter() - ta
        if b == args.warmup:
            ctx.barrier()
            ctx.synchronize()
            if prof is not None:
                prof.enable()
            t_start = time.perf_counter()
            unix_start = time.time()
        if b >= args.warmup and (b - args.warmup) % args.steps == 0:
            if seg is not None:
                end_segment()
            seg = (time.perf_counter(), untimed, total_txs, writer_snapshot(), len(stages))
        t0 = time.perf_counter()
        errors = []
        if from_mempool:
            # what POST /push_block does with a miner's tx-hash list (node/main.py): resolve the hex
            # from the mempool, then validate + apply (which also clears the confirmed txs and their
            # pending spends from the mempool tables)
            txs_hex = await db.get_pending_transactions_hex_by_hash(hashes)
            assert len(txs_hex) == len(hashes)
            t_resolve = time.perf_counter() - t0
        if args.object_path:
            txs = [await Transaction.from_hex(h) for h in txs_hex]
            ok = await manager.create_block(headers[b], txs, error_list=errors)
        else:
            ok = await fastpath.create_block_from_hex(headers[b], txs_hex, error_list=errors)
        if not ok:
            raise RuntimeError(f'synthetic block rejected: {errors}')
        t2 = time.perf_counter()
        if b >= args.warmup:
            total_txs += len(txs_hex)
            if db.writer is not None:
                wst = db.writer.stats()
                queue_trace.append((wst['submitted'] - wst['applied'], wst['queued_bytes']))
            stages.append({'block_s': t2 - t0, **({'resolve_s': t_resolve} if from_mempool else {}),
                           **manager.last_block_timings,
                           **{k: v for k, v in validate.timings.items() if k.endswith('_s')},
                           **({} if args.object_path else fastpath.timings)})
            paths.add('object' if args.object_path else fastpath.last_path)
    # the timed region ends when the SQL tables hold every block (the journal is the commit point;
    # the materialiser must have caught up too)
    td = time.perf_counter()
    end_segment()
    drain = time.perf_counter() - td
    ctx.barrier()
    wall = time.perf_counter() - t_start - untimed
    if prof is not None:  # UPOW_BENCH_PROFILE=PATH: cProfile of the timed blocks only (text report)
        _dump_profile(prof, os.environ['UPOW_BENCH_PROFILE'])
    wall = ctx.allreduce_max_f(wall)
    writer = db.writer.stats() if db.writer is not None else None
    if writer is not None:
        writer = {k: (round(v, 4) if isinstance(v, float) else v) for k, v in writer.items() if k != 'error'}
    extra = {'body_parse': extra_parse, 'drain_s': drain, 'writer': writer, 'window_unix': [unix_start, time.time()],
             'governance': gov_probe,
             'difficulties': sorted({str(d) for d in difficulties}),
             'segments': [(t, w) for t, w in zip(seg_txs, seg_walls)], 'segment_diag': seg_diag,
             'aging': aging or None, 'queue_trace': queue_trace, 'key_setup_s': key_setup}
    if gov_probe is not None:
        gov_probe['active_inodes_after'] = len(await db.get_active_inodes())
        gov_probe['coinbase_outputs_last_block'] = len(json.loads(
            db._q1('SELECT outputs_addresses FROM transactions WHERE tx_hex LIKE ? LIMIT 1',
                   ('%' + (await db.get_last_block())['hash'] + '%',))[0]))
    return total_txs, wall, stages, len(blocks[0]), sorted(paths), extra


# A/B switch: hold the txs as json.loads' str lists (the form before the span parse) instead of body spans
_TX_LISTS = os.environ.get('UPOW_BENCH_TX_LISTS', '0') == '1'


def _as_fetched(page: list) -> list:
    """(untimed) /get_blocks rows as a syncing node holds them: parsed by peers.fetch_json from the JSON
    body, each row's tx array left inside the body bytes (utils/hexspans.py)."""
    from fastapi.encoders import jsonable_encoder  # what the /get_blocks answer goes through (Decimal -> number)
    body = json.dumps(jsonable_encoder(page)).encode()
    return json.loads(body) if _TX_LISTS else hexspans.loads(body)


def _body_parse_ms(body: bytes, reps: int = 5) -> dict:
    """Median ms to parse one /push_block body: json.loads (what the framework did) against the native
    parse that keeps the tx array in the body (utils/hexspans.py)."""
    def med(fn):
        ts = []
        for _ in range(reps):
            t = time.perf_counter()
            fn(body)
            ts.append(time.perf_counter() - t)
        return round(sorted(ts)[len(ts) // 2] * 1000, 3)
    return {'body_mb': round(len(body) / 2**20, 2), 'json_loads': med(json.loads), 'native_spans': med(hexspans.loads)}


def run_verify_bench(args, ctx):
    from .ops.native import gpu_available
    device = 'gpu' if gpu_available() else 'cpu'
    utxo_backend = 'gpu' if device == 'gpu' else 'host'
    if not hasattr(args, 'object_path'):
        args.object_path = False
    total_txs, wall, stages, txs_per_block, paths, extra = asyncio.run(_run(args, ctx, device, utxo_backend))
    gov_txs = float(getattr(args, 'governance_txs', 0.0) or 0.0)
    if gov_txs:
        args_cfg = (f'governance txs: {gov_txs:.0%} of every block (70% delegate votes, 10% validator votes, '
                    f'20% delegate revokes) on a seeded state (12 inodes, validators, delegates with stakes, '
                    f'voting power and ballots)')
    elif getattr(args, 'governance', False):
        args_cfg = 'governance: 12 inodes, 200 validators, 5000 delegates'
    elif float(getattr(args, 'grouped_txs', 0.0) or 0.0):
        args_cfg = (f'grouped-signature txs: {float(args.grouped_txs):.0%} of every block are 4-in txs of two keys '
                    f'with two signatures (inputs grouped by owner key, reference transaction.py:578-590)')
    else:
        args_cfg = None
    total = ctx.allreduce_sum(total_txs)
    segs = extra.get('segments') or []
    if len(segs) > 1:
        # the median of the run's segments (each ``steps`` blocks ending in its own SQL drain): separate runs
        # on the pool's boxes differ by up to +-15 %, interleaved segments of one run far less
        seg_tps = sorted(ctx.allreduce_sum(t) / ctx.allreduce_max_f(w) for t, w in segs)
        tps = seg_tps[len(seg_tps) // 2]
        ms = round(1000 * (total / len(segs)) / tps / max(1, args.steps), 2) if tps else 0.0
    else:
        seg_tps = None
        tps = total / wall
        ms = round(wall * 1000 / max(1, args.steps), 2)
    avg = {k: round(sum(s[k] for s in stages) / len(stages) * 1000, 2) for k in stages[0]
           if isinstance(stages[0][k], float)}
    return {
        'metric': 'block_tx_verify_per_s',
        'value': round(tps, 1),
        'unit': 'tx/s',
        'n_gpus': ctx.world if device == 'gpu' else 0,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': ms,
        **({'segments_tx_per_s': [round(x, 1) for x in seg_tps], 'segment_blocks': args.steps,
            'segment_diag': extra.get('segment_diag')} if seg_tps else {}),
        'higher_is_better': True,
        'scaling': 'weak',
        'vs_baseline': None,
        'dtype': 'uint32',
        'data': _data_label(args),
        'config': {'model': 'upow block validation + apply (push_block path)', 'keys': getattr(args, 'keys', 'distinct'), 'global_batch': total // max(1, args.steps),
                   'seq_len': txs_per_block, 'parallelism': f'dp{ctx.world}', 'device': device,
                   'utxo_backend': utxo_backend, 'block_path': '+'.join(paths),
                   'ledger': 'file (WAL)' if getattr(args, 'ledger', None) else 'memory',
                   'txs_from': 'mempool (hashes)' if getattr(args, 'from_mempool', False) else 'block body (hex)',
                   **({'chain_state': args_cfg} if args_cfg else {})},
        'stage_ms_avg': avg,
        # the same run split by stage: validation alone (decode, HBM UTXO pass, decompression, ECDSA —
        # everything before the ledger writes) and the signature kernel alone, per 2 MB block
        'validate_tx_per_s': round(txs_per_block / max(1e-9, (avg.get('decode_to_checks_s', 0) + avg.get('utxo_s', 0)
                                                             + avg.get('verify_s', 0)) / 1000), 1),
        'ecdsa_sig_per_s': round(txs_per_block / max(1e-9, avg.get('ecdsa_s', 0) / 1000), 1),
        # commit-point latency of one block (validation + journal append + HBM update), and the SQL
        # materialiser's catch-up after the last block (inside the timed region)
        'commit_latency_ms': avg.get('block_s'),
        'final_drain_ms': round(extra['drain_s'] * 1000, 2),
        **({'push_body_parse_ms': extra['body_parse']} if extra.get('body_parse') else {}),
        'ledger_writer': extra['writer'],
        'window_unix': extra['window_unix'],
        'difficulties': extra.get('difficulties'),
        **({'key_setup_s': extra['key_setup_s']} if extra.get('key_setup_s') is not None else {}),
        **({'governance': extra['governance']} if extra['governance'] else {}),
        **({'aged_ledger': extra['aging'], 'writer_lag_after_block': extra['queue_trace']} if extra['aging'] else {}),
    }


async def _run_cluster(args, ctx, device, utxo_backend):
    """ONE chain on a G-rank cluster node (parallel/cluster.py): every rank holds a replica built from the
    same seed; rank 0 (the leader) pushes each block through ``fastpath.create_block_from_hex``, which
    broadcasts it to the followers as a cluster ``block`` op; every rank validates it with the signature
    batch sharded across the GPUs (validate.set_dist_context), applies it to its own ledger + HBM index,
    and an all-reduce checks that all replicas agree. The timed region is the leader's block loop plus
    every replica's SQL drain; the reported tx/s is the CHAIN's (not a sum over ranks)."""
    from . import devnet
    from .constants import START_DIFFICULTY
    from .ledger import fastpath, manager, validate
    from .models.block import get_transactions_merkle_tree
    from .parallel import cluster
    from .parallel.cluster import unpack_txs
    n_blocks = args.steps + args.warmup
    base_ts = ctx.allreduce_min(int(time.time()) - max(10_000, SPACING_S * (n_blocks + 10)))
    db, addr, blocks, _ = await _setup(n_blocks, args.txs, 1234, utxo_backend, device, base_ts=base_ts,
                                       make_blocks=ctx.rank == 0, ledger_path=_ledger_path(args, ctx),
                                       distinct_keys=_distinct(args))
    c = cluster.init(ctx)
    st = c.status(db)
    if any((s['height'], s['utxo_hash']) != (st[0]['height'], st[0]['utxo_hash']) for s in st):
        raise RuntimeError(f'cluster bench: replicas differ after setup: {st}')
    validate.set_dist_context(ctx)
    headers = []
    if c.leader:
        headers, _ = await premine_headers(db, addr, blocks, base_ts, device)
    stages = []
    total_txs = 0
    try:
        for b in range(n_blocks):
            if b == args.warmup:
                ctx.barrier()
                ctx.synchronize()
                t_start = time.perf_counter()
            t0 = time.perf_counter()
            errors = []
            if c.leader:
                ok = await fastpath.create_block_from_hex(headers[b], blocks[b], error_list=errors)
                n_tx = len(blocks[b])
            else:
                msg = c.recv()
                assert msg['op'] == 'block', msg['op']
                txs = unpack_txs(msg['_payload'])
                ok = await fastpath.create_block_from_hex(msg['content'], txs, error_list=errors, mirror=False)
                n_tx = len(txs)
            if not ok:
                raise RuntimeError(f'cluster bench: block {b} rejected on rank {ctx.rank}: {errors}')
            if b >= args.warmup:
                total_txs += n_tx
                stages.append({'block_s': time.perf_counter() - t0, **manager.last_block_timings,
                               **{k: v for k, v in validate.timings.items() if k.endswith('_s')},
                               **fastpath.timings})
        db.flush()
        ctx.synchronize()
        ctx.barrier()
        wall = ctx.allreduce_max_f(time.perf_counter() - t_start)
        st = c.status(db)
        agree = all((s['height'], s['utxo_hash']) == (st[0]['height'], st[0]['utxo_hash']) for s in st)
        if not agree:
            raise RuntimeError(f'cluster bench: replicas diverged: {st}')
    finally:
        validate.set_dist_context(None)
        cluster.init(type(ctx)())  # a world-1 context: no cluster
    writer = db.writer.stats() if db.writer is not None else None
    if writer is not None:
        writer = {k: (round(v, 4) if isinstance(v, float) else v) for k, v in writer.items() if k != 'error'}
    return total_txs, wall, stages, args.txs, [fastpath.last_path], {
        'drain_s': 0.0, 'writer': writer, 'window_unix': None, 'governance': None,
        'replicas': [{'rank': s['rank'], 'height': s['height'], 'utxo_hash': s['utxo_hash']} for s in st]}


def run_cluster_verify_bench(args, ctx):
    """tx-verify/s of ONE chain on the cluster node (all ranks; the same numbers on every rank)."""
    from .ops.native import gpu_available
    device = 'gpu' if gpu_available() else 'cpu'
    utxo_backend = 'gpu' if device == 'gpu' else 'host'
    total_txs, wall, stages, txs_per_block, paths, extra = asyncio.run(_run_cluster(args, ctx, device, utxo_backend))
    avg = {k: round(sum(s[k] for s in stages) / len(stages) * 1000, 2) for k in stages[0]
           if isinstance(stages[0][k], float)}
    return {
        'metric': 'block_tx_verify_per_s',
        'value': round(total_txs / wall, 1),
        'unit': 'tx/s',
        'n_gpus': ctx.world if device == 'gpu' else 0,
        'world': ctx.world,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': round(wall * 1000 / max(1, args.steps), 2),
        'higher_is_better': True,
        'scaling': 'strong',
        'vs_baseline': None,
        'dtype': 'uint32',
        'data': _data_label(args),
        'config': {'model': 'upow cluster node: one chain, G replicas, sharded ECDSA (push_block path)',
                   'keys': getattr(args, 'keys', 'distinct'),
                   'global_batch': txs_per_block, 'seq_len': txs_per_block, 'parallelism': f'replica{ctx.world}+sigshard',
                   'device': device, 'utxo_backend': utxo_backend, 'block_path': '+'.join(p for p in paths if p),
                   'ledger': 'file (WAL)' if getattr(args, 'ledger', None) else 'memory',
                   'txs_from': 'block body (hex)'},
        'stage_ms_avg': avg,
        'validate_tx_per_s': round(txs_per_block / max(1e-9, (avg.get('decode_to_checks_s', 0) + avg.get('utxo_s', 0)
                                                             + avg.get('verify_s', 0)) / 1000), 1),
        'ecdsa_sig_per_s': round(txs_per_block / max(1e-9, avg.get('ecdsa_s', 0) / 1000), 1),
        'commit_latency_ms': avg.get('block_s'),
        'final_drain_ms': 0.0,
        'ledger_writer': extra['writer'],
        'window_unix': extra['window_unix'],
        'replicas': extra['replicas'],
    }


async def _run_sync(args, ctx, device, utxo_backend):
    """Sync throughput: a source ledger applies ``steps + warmup`` full blocks through push_block; a
    second ledger with the same genesis + funding then replays them the way a syncing node does
    (``node.main.create_blocks`` over a ``/get_blocks`` page: trusted coinbase, native block path,
    decode of block k+1 overlapped with the apply of block k). Only the replay is timed."""
    from . import devnet
    from .constants import START_DIFFICULTY
    from .ledger import manager
    from .ledger.database import Database
    from .models.block import get_transactions_merkle_tree
    from .ledger import fastpath
    n_blocks = args.steps + args.warmup
    # one block per target interval (60 s, manager.py:26): long chains keep the start difficulty at every
    # 100-block retarget, as a real chain at equilibrium does; every header is mined at the difficulty the
    # chain computes for it, so a run of more than 100 blocks crosses retargets
    base_ts = int(time.time()) - 60 * (n_blocks + 10) - 1_000
    seed = 4321 + ctx.rank
    counts = _tx_counts(args, n_blocks, seed)
    src, addr, blocks, _ = await _setup(n_blocks, args.txs, seed, utxo_backend, device, base_ts=base_ts,
                                        distinct_keys=_distinct(args), tx_counts=counts)
    prev = (await src.get_last_block())['hash']
    for b, txs_hex in enumerate(blocks):
        manager.Manager.difficulty = None
        difficulty, _ = await manager.calculate_difficulty()
        content = devnet.mine_header_raw(prev, addr, get_transactions_merkle_tree(txs_hex), base_ts + 60 * (b + 1),
                                         difficulty, device=device)
        errors = []
        if not await fastpath.create_block_from_hex(content, txs_hex, error_list=errors):
            raise RuntimeError(f'source block rejected: {errors}')
        prev = hashlib.sha256(bytes.fromhex(content)).hexdigest()
    page = []  # /get_blocks caps a response at 8 x the max block hex (database.get_blocks): several pages
    while len(page) < n_blocks:
        part = await src.get_blocks(3 + len(page), n_blocks - len(page))
        assert part, 'source ledger returned an empty page'
        page += part
    page = _as_fetched(page)
    assert len(page) == n_blocks and all(len(p['transactions']) == counts[b] + 1 for b, p in enumerate(page))
    retargets = sorted({str(b['block']['difficulty']) for b in page})
    src.close()
    aging = {}
    dst, _, _, _ = await _setup(n_blocks, args.txs, seed, utxo_backend, device, base_ts=base_ts, make_blocks=False,
                                ledger_path=_ledger_path(args, ctx), age_txs=int(getattr(args, 'age_txs', 0) or 0),
                                aging=aging, distinct_keys=_distinct(args), tx_counts=counts)
    aging.pop('distinct_key_setup_s', None)
    dst.flush()
    Database.instance = dst
    manager.Manager.difficulty = None
    from .node.main import create_blocks
    if args.warmup:
        if not await create_blocks(page[:args.warmup]):
            raise RuntimeError('sync warmup rejected')
    ctx.barrier()
    ctx.synchronize()
    prof = None
    if os.environ.get('UPOW_BENCH_PROFILE'):  # cProfile of the timed replay only (text report)
        import cProfile
        prof = cProfile.Profile()
        prof.enable()
    cpu0 = _thread_cpu()
    t0 = time.perf_counter()
    errors = []
    per_page = max(1, int(getattr(args, 'sync_page_blocks', 1000) or 1000))  # /get_blocks returns <= 1,000
    timed = page[args.warmup:]
    for a in range(0, len(timed), per_page):
        if not await create_blocks(timed[a:a + per_page], errors):
            raise RuntimeError(f'sync rejected: {errors}')
    dst.flush()  # the SQL tables hold every block (the journal is the commit point)
    ctx.synchronize()
    ctx.barrier()
    wall_local = time.perf_counter() - t0
    threads_cpu = _thread_cpu_delta(cpu0, _thread_cpu(), wall_local)
    wall = ctx.allreduce_max_f(wall_local)
    if prof is not None:
        _dump_profile(prof, os.environ['UPOW_BENCH_PROFILE'])
    assert (await dst.get_last_block())['hash'] == page[-1]['block']['hash']
    writer = dst.writer.stats() if dst.writer is not None else {}
    from .ledger import pagesync
    return sum(counts[args.warmup:]), wall, fastpath.last_path, {
        'blocks_per_s': round(args.steps / wall, 1), 'tx_counts': _counts_label(args, counts[args.warmup:]),
        'difficulties': retargets, 'blocks_per_page': per_page,
        'aged_ledger': aging or None, 'journal_rotations': writer.get('rotations'),
        'writer_throttle_s': writer.get('throttle_s'), 'undo_blocks': writer.get('undo_blocks'),
        'sync_path': 'page' if pagesync.ENABLED else 'per-block',
        'page': ({k: (round(v, 4) if isinstance(v, float) else v) for k, v in pagesync.stats.items()}
                 if pagesync.ENABLED else None),
        'journal_fdatasyncs': writer.get('fdatasyncs'), 'journal_group_records': writer.get('group_records'),
        'utxo_deferred_flushes': dst.utxo.deferred_flushes, 'threads_cpu': threads_cpu}


def _thread_cpu() -> dict:
    """CPU seconds (user + system) per thread of this process, keyed by 'name/tid' (/proc/self/task)."""
    out = {}
    tick = os.sysconf('SC_CLK_TCK')
    try:
        for tid in os.listdir('/proc/self/task'):
            try:
                with open(f'/proc/self/task/{tid}/stat') as f:
                    st = f.read()
                with open(f'/proc/self/task/{tid}/comm') as f:
                    name = f.read().strip()
            except OSError:
                continue
            fields = st[st.rindex(')') + 2:].split()
            out[f'{name}/{tid}'] = (int(fields[11]) + int(fields[12])) / tick
    except OSError:
        pass
    return out


def _thread_cpu_delta(before: dict, after: dict, wall: float, top: int = 12) -> dict:
    """The threads that used the most CPU over a timed region: {name: cpu seconds}, plus the total as a
    multiple of the wall time (how many cores the process kept busy)."""
    d = {k: round(after[k] - before.get(k, 0.0), 3) for k in after}
    agg = {}
    for k, v in d.items():
        name = k.rsplit('/', 1)[0]
        agg[name] = round(agg.get(name, 0.0) + v, 3)
    busy = sorted(agg.items(), key=lambda kv: -kv[1])[:top]
    return {'cores_busy': round(sum(d.values()) / wall, 2) if wall > 0 else None, 'top_threads_cpu_s': dict(busy)}


def _sync_data_label(args) -> str:
    rng = getattr(args, 'txs_range', None) or f'{args.txs}'
    keys = 'a fresh random P-256 key pair per tx' if _distinct(args) else 'a 256-key pool'
    return (f'synthetic chain of {rng}-tx blocks (2-in/2-out signed txs, {keys}), headers mined at the '
            f'difficulty the chain computes, replayed from /get_blocks pages (coinbase included)')


def _tx_counts(args, n_blocks: int, seed: int) -> list:
    """Per-block tx counts: ``--txs`` for every block, or uniform in ``--txs-range LO-HI`` (seeded)."""
    spec = getattr(args, 'txs_range', None)
    if not spec:
        return [args.txs] * n_blocks
    lo, hi = (int(x) for x in str(spec).split('-'))
    rng = random.Random(seed ^ 0x5EED)
    return [rng.randint(lo, hi) for _ in range(n_blocks)]


def _counts_label(args, counts) -> dict:
    return {'range': getattr(args, 'txs_range', None) or f'{args.txs}-{args.txs}', 'total': sum(counts),
            'mean': round(sum(counts) / max(1, len(counts)), 2), 'empty_blocks': sum(1 for c in counts if c == 0)}


def run_sync_bench(args, ctx):
    from .ops.native import gpu_available
    device = 'gpu' if gpu_available() else 'cpu'
    utxo_backend = 'gpu' if device == 'gpu' else 'host'
    txs, wall, path, extra = asyncio.run(_run_sync(args, ctx, device, utxo_backend))
    total = ctx.allreduce_sum(txs)
    return {
        'metric': 'sync_tx_per_s',
        'value': round(total / wall, 1),
        'unit': 'tx/s',
        'n_gpus': ctx.world if device == 'gpu' else 0,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': round(wall * 1000 / max(1, args.steps), 2),
        'higher_is_better': True,
        'scaling': 'weak',
        'vs_baseline': None,
        'dtype': 'uint32',
        'data': _sync_data_label(args),
        'config': {'model': 'upow chain sync (node.main.create_blocks, trusted coinbase)',
                   'global_batch': total // max(1, args.steps), 'seq_len': extra['tx_counts']['mean'],
                   'parallelism': f'dp{ctx.world}', 'device': device, 'utxo_backend': utxo_backend,
                   'block_path': path, 'ledger': 'file (WAL)' if getattr(args, 'ledger', None) else 'memory'},
        **{k: v for k, v in extra.items() if v is not None},
    }


async def _run_cluster_sync(args, ctx, device, utxo_backend):
    """Chain sync on a G-rank cluster node: ONE chain, G replicas. Rank 0 builds the source chain (untimed);
    every rank opens an identical destination ledger (same seed: genesis + funding); the leader then syncs the
    chain page by page through ``node.main.create_blocks`` — each page one 'page' op to the followers, every
    chunk's signatures sharded over the G GPUs (one all-gather of status bytes), every block agreed before it
    commits. The timed region is the leader's page loop plus a final status op that every replica answers
    after applying the last page; the reported tx/s is the chain's."""
    from . import devnet
    from .ledger import manager
    from .ledger.database import Database
    from .models.block import get_transactions_merkle_tree
    from .ledger import fastpath, pagesync
    from .parallel import cluster
    n_blocks = args.steps + args.warmup
    base_ts = ctx.allreduce_min(int(time.time()) - 60 * (n_blocks + 10) - 1_000)
    seed = 4321
    counts = _tx_counts(args, n_blocks, seed)
    page = None
    if ctx.rank == 0:
        src, addr, blocks, _ = await _setup(n_blocks, args.txs, seed, utxo_backend, device, base_ts=base_ts,
                                            distinct_keys=_distinct(args), tx_counts=counts)
        prev = (await src.get_last_block())['hash']
        for b, txs_hex in enumerate(blocks):
            manager.Manager.difficulty = None
            difficulty, _ = await manager.calculate_difficulty()
            content = devnet.mine_header_raw(prev, addr, get_transactions_merkle_tree(txs_hex),
                                             base_ts + 60 * (b + 1), difficulty, device=device)
            errors = []
            if not await fastpath.create_block_from_hex(content, txs_hex, error_list=errors):
                raise RuntimeError(f'source block rejected: {errors}')
            prev = hashlib.sha256(bytes.fromhex(content)).hexdigest()
        page = []
        while len(page) < n_blocks:
            part = await src.get_blocks(3 + len(page), n_blocks - len(page))
            page += part
        page = _as_fetched(page)
        src.close()
    dst, _, _, _ = await _setup(n_blocks, args.txs, seed, utxo_backend, device, base_ts=base_ts, make_blocks=False,
                                ledger_path=_ledger_path(args, ctx), distinct_keys=_distinct(args), tx_counts=counts)
    dst.flush()
    Database.instance = dst
    manager.Manager.difficulty = None
    c = cluster.init(ctx)
    per_page = max(1, int(getattr(args, 'sync_page_blocks', 1000) or 1000))
    if not c.leader:
        fprof = None
        if os.environ.get('UPOW_BENCH_PROFILE_FOLLOWER') and ctx.rank == 1:  # cProfile of one follower's op loop
            import cProfile
            fprof = cProfile.Profile()
            fprof.enable()
        await cluster.follower_main(c, dst)
        if fprof is not None:
            _dump_profile(fprof, os.environ['UPOW_BENCH_PROFILE_FOLLOWER'])
        wall = ctx.allreduce_max_f(0.0)
        st = None
    else:
        from .node.main import create_blocks
        await cluster.leader_start(dst)
        if args.warmup and not await create_blocks(page[:args.warmup]):
            raise RuntimeError('cluster sync warmup rejected')
        c.send('status')
        st0 = c.status(dst)  # every replica's process CPU seconds at the start of the timed region
        prof = None
        if os.environ.get('UPOW_BENCH_PROFILE'):  # cProfile of the leader's timed sync (text report)
            import cProfile
            prof = cProfile.Profile()
            prof.enable()
        cpu0 = _thread_cpu()
        t0 = time.perf_counter()
        errors = []
        timed = page[args.warmup:]
        for a in range(0, len(timed), per_page):
            if not await create_blocks(timed[a:a + per_page], errors):
                raise RuntimeError(f'cluster sync rejected: {errors}')
        dst.flush()
        c.send('status')
        st = c.status(dst)  # every replica has applied the last page when it answers
        wall = time.perf_counter() - t0
        threads_cpu = _thread_cpu_delta(cpu0, _thread_cpu(), wall)
        if prof is not None:
            _dump_profile(prof, os.environ['UPOW_BENCH_PROFILE'])
        await cluster.leader_quit()
        wall = ctx.allreduce_max_f(wall)
        if any((s['height'], s['utxo_hash']) != (st[0]['height'], st[0]['utxo_hash']) for s in st):
            raise RuntimeError(f'cluster sync: replicas diverged: {st}')
        # host CPU per synced block of every replica (process time of all its threads over the timed region)
        rank_cpu = [round((b['cpu_s'] - a['cpu_s']) * 1000 / max(1, args.steps), 3) for a, b in zip(st0, st)]
        # the same without the page plans' P-256 work (key decompression, curve checks, the rank's verify shard):
        # host CPU on a CPU-only node, GPU kernels on an MI355X node
        ex = [round(c - (b['crypto_cpu_s'] - a['crypto_cpu_s']) * 1000 / max(1, args.steps), 3)
              for c, a, b in zip(rank_cpu, st0, st)]
        many = len(st) > 1
        cpu = {'rank_cpu_ms_per_block': rank_cpu, 'rank_cpu_ms_per_block_ex_p256': ex,
               'lean_followers': all(s['lean'] for s in st[1:]) if many else None,
               'follower_cpu_vs_leader': round(max(rank_cpu[1:]) / rank_cpu[0], 3) if many and rank_cpu[0] else None,
               'follower_cpu_vs_leader_ex_p256': round(max(ex[1:]) / ex[0], 3) if many and ex[0] > 0 else None}
    info = c.info()
    cluster.init(type(ctx)())  # a world-1 context: no cluster
    dst.close()
    return sum(counts[args.warmup:]), wall, {
        'blocks_per_s': round(args.steps / wall, 1), 'tx_counts': _counts_label(args, counts[args.warmup:]),
        'blocks_per_page': per_page, 'sync_path': 'page', 'op_stream': info,
        'threads_cpu': threads_cpu if c.leader else None, **(cpu if c.leader else {}),
        'page': {k: (round(v, 4) if isinstance(v, float) else v) for k, v in pagesync.stats.items()},
        'replicas': [{'rank': x['rank'], 'height': x['height'], 'utxo_hash': x['utxo_hash']} for x in st] if st else None}


def _gpus_used(ctx) -> int:
    """Distinct GPUs under the job's ranks (a multi-rank cluster may share one GPU over host collectives)."""
    import torch
    return min(ctx.world, max(1, torch.cuda.device_count()))


def run_cluster_sync_bench(args, ctx):
    """sync tx/s of ONE chain on a G-rank cluster node (strong scaling: the chain is fixed as G grows)."""
    from .ops.native import gpu_available
    device = 'gpu' if gpu_available() else 'cpu'
    utxo_backend = 'gpu' if device == 'gpu' else 'host'
    txs, wall, extra = asyncio.run(_run_cluster_sync(args, ctx, device, utxo_backend))
    return {
        'metric': 'sync_tx_per_s',
        'value': round(txs / wall, 1),
        'unit': 'tx/s',
        'n_gpus': _gpus_used(ctx) if device == 'gpu' else 0,
        'world': ctx.world,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': round(wall * 1000 / max(1, args.steps), 3),
        'higher_is_better': True,
        'scaling': 'strong',
        'vs_baseline': None,
        'dtype': 'uint32',
        'data': _sync_data_label(args),
        'config': {'model': 'upow cluster node chain sync: one chain, G replicas, page plans with sharded ECDSA',
                   'global_batch': txs // max(1, args.steps), 'seq_len': extra['tx_counts']['mean'],
                   'parallelism': f'replica{ctx.world}+sigshard', 'device': device, 'utxo_backend': utxo_backend,
                   'ledger': 'file (WAL)' if getattr(args, 'ledger', None) else 'memory'},
        **{k: v for k, v in extra.items() if v is not None},
    }
