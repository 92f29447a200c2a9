"""Consensus manager: difficulty, emission, block validation/application, mempool GC.

reference: upow/manager.py:26-904. Same rules, same constants, same consensus exception tables.
The per-transaction validation loop of ``check_block`` (manager.py:628-632) is replaced by
:func:`upow_amd.ledger.validate.verify_block_transactions`, which runs every signature of the block
as ONE batched P-256 verify on the GPU (with the reference's raw-bytes-then-ASCII-hex fallback),
prefetches all point decompressions in one kernel, and still runs each tx's rule checks in order.
"""
from __future__ import annotations

import asyncio
import contextvars
import decimal
import os
import weakref
from datetime import datetime, timedelta
from decimal import Decimal
from math import ceil, floor, log
from time import perf_counter
from typing import List, Optional, Tuple, Union

from ..constants import (BLOCK_TIME, BLOCKS_COUNT, HALVING_INTERVAL, LAST_BLOCK_FOR_GENESIS_KEY, MAX_BLOCK_SIZE_HEX,
                         MAX_SUPPLY, NINE_HALVING_INTERVAL, START_DIFFICULTY)
from ..models.block import (block_to_bytes, check_pow, get_transactions_merkle_tree,
                            get_transactions_merkle_tree_ordered, split_block_content)
from ..models.transaction import CoinbaseTransaction, Transaction, TransactionOutput
from ..utils import codec, metrics, roctx
from ..utils.codec import TransactionType, round_up_decimal, round_up_decimal_new, sha256, timestamp
from ..utils.logger import get_logger
from .database import Database

logger = get_logger(__name__)

cache: dict = {}
cache_expiration = timedelta(minutes=5)
cache_updating = False

# stage timers of the last validated block (tracing)
last_block_timings: dict = {}


class Manager:
    difficulty: Optional[Tuple[Decimal, dict]] = None


# ---------------------------------------------------------------------------------------------- difficulty
def difficulty_to_hashrate_old(difficulty: Decimal) -> Decimal:
    decimal_ = difficulty % 1 or 1 / 16
    return Decimal(16 ** int(difficulty) * (16 * decimal_))


def difficulty_to_hashrate(difficulty: Decimal) -> Decimal:
    """manager.py:44-46."""
    decimal_ = difficulty % 1
    return Decimal(16 ** int(difficulty) * (16 / ceil(16 * (1 - decimal_))))


def hashrate_to_difficulty_old(hashrate: int) -> Decimal:
    difficulty = int(log(hashrate, 16))
    if hashrate == 16 ** difficulty:
        return Decimal(difficulty)
    return Decimal(difficulty + (hashrate / Decimal(16) ** difficulty) / 16)


def hashrate_to_difficulty(hashrate) -> Decimal:
    """manager.py:67-80 (quantised to 0.1)."""
    difficulty = int(log(hashrate, 16))
    ratio = hashrate / 16 ** difficulty
    for i in range(0, 10):
        coeff = 16 / ceil(16 * (1 - i / 10))
        if coeff > ratio:
            return Decimal(difficulty + (i - 1) / Decimal(10))
        if coeff == ratio:
            return Decimal(difficulty + i / Decimal(10))
    return Decimal(difficulty) + Decimal('0.9')


async def calculate_difficulty() -> Tuple[Decimal, dict]:
    """manager.py:83-121: retarget every 100 blocks toward 60 s."""
    database = Database.instance
    last_block = await database.get_last_block()
    if last_block is None:
        return START_DIFFICULTY, dict()
    last_block = dict(last_block)
    last_block['address'] = last_block['address'].strip(' ')
    if last_block['id'] < BLOCKS_COUNT:
        return START_DIFFICULTY, last_block
    if last_block['id'] % BLOCKS_COUNT == 0:
        last_adjust_block = await database.get_block_by_id(last_block['id'] - BLOCKS_COUNT + 1)
        new_difficulty = retarget(last_block['id'], last_block['difficulty'], last_block['timestamp'],
                                  last_adjust_block['timestamp'])
        logger.info(f'calculate_difficulty hashrate_to_difficulty block {last_block["id"]}, '
                    f'new_difficulty {new_difficulty}')
        return new_difficulty, last_block
    return last_block['difficulty'], last_block


def retarget(last_id: int, last_difficulty, last_ts: int, window_first_ts: int) -> Decimal:
    """The retarget arithmetic of manager.py:83-121 at a block id divisible by BLOCKS_COUNT: the next
    difficulty from the last one and the timestamps of the window's first and last blocks."""
    average_per_block = (last_ts - window_first_ts) / BLOCKS_COUNT
    hashrate = difficulty_to_hashrate(last_difficulty)
    ratio = BLOCK_TIME / average_per_block
    if last_id >= 180_000:
        ratio = min(ratio, 2)
    hashrate *= ratio
    new_difficulty = hashrate_to_difficulty(hashrate)
    if new_difficulty < START_DIFFICULTY and last_id >= 590600:
        return START_DIFFICULTY
    return new_difficulty


def difficulty_schedule(chain: List[Tuple[int, Decimal]], timestamps: List[int]) -> List[Decimal]:
    """The difficulty the chain will require of each of the next blocks, given the (timestamp, difficulty)
    of every block so far (``chain``, block ids 1..n) and the planned timestamps of the next ones: what
    calculate_difficulty answers at each of those heights (benches mine headers ahead with it)."""
    ts = [t for t, _ in chain]
    ds = [Decimal(d) for _, d in chain]
    out = []
    for t in timestamps:
        last_id = len(ts)
        if last_id < BLOCKS_COUNT:
            d = START_DIFFICULTY
        elif last_id % BLOCKS_COUNT == 0:
            d = retarget(last_id, ds[-1], ts[-1], ts[last_id - int(BLOCKS_COUNT)])
        else:
            d = ds[-1]
        out.append(d)
        ts.append(int(t))
        ds.append(Decimal(d))
    return out


async def get_difficulty() -> Tuple[Decimal, dict]:
    if Manager.difficulty is None:
        Manager.difficulty = await calculate_difficulty()
    return Manager.difficulty


async def check_block_is_valid(block_content: str, mining_info: tuple = None) -> bool:
    """manager.py:130-151."""
    if mining_info is None:
        mining_info = await get_difficulty()
    difficulty, last_block = mining_info
    if 'hash' not in last_block:
        return True
    return check_pow(block_content, last_block['hash'], difficulty)


# ---------------------------------------------------------------------------------------------- emission
HALVING_BLOCKS = HALVING_INTERVAL  # one halving era: three years of 60 s blocks (1,576,800)
LAST_REWARD_BLOCK = NINE_HALVING_INTERVAL  # 14,191,200: no block reward after the ninth halving


def _era(block_no: int) -> int:
    """Halvings before ``block_no``: the last block of an era still pays the era's reward."""
    return (int(block_no) - 1) // HALVING_BLOCKS


def get_block_reward(block_no) -> Decimal:
    """Block subsidy (reference manager.py:154-168): 6 coins, halved every era, nothing past the ninth
    halving. The reference divides in binary floating point (``6 / 2 ** n``) and converts; every value of that
    sequence is exact in binary, and it is kept as written."""
    assert block_no > 0
    if block_no > LAST_REWARD_BLOCK:
        return Decimal(0)
    return Decimal(6 / (1 << _era(block_no)))


def get_inode_rewards(reward, inode_address_details, block_no=1):
    """Miner / inode split of a block reward (reference manager.py:171-212), as the same Decimal operation
    sequence: half to the miner; the other half over the inodes by emission share, rounded up (8 decimals,
    9 significant digits and the newer rounding after block 39,000). The shares of inodes under 1 % are pooled
    and, inside the per-inode pass as in the reference, the pool so far is re-spread over every inode at or
    above 1 % each time it is non-empty — so an early pool is paid more than once, and a >= 1 % inode listed
    after a < 1 % one is not in the result yet when the pool is spread (a KeyError, as in the reference).
    ``tests/test_consensus.py`` pins the results (including those errors) against golden outputs."""
    total = sum(d['emission'] for d in inode_address_details)
    if not inode_address_details or total <= 0:
        return reward, {}
    miner_reward = reward * Decimal(0.5)
    inode_half = reward * Decimal(0.5)
    newer = block_no > 39000
    round_up = round_up_decimal_new if newer else round_up_decimal
    big = [d['wallet'] for d in inode_address_details if d['emission'] >= 1]  # in list order, repeats kept
    shares = {}
    pooled = Decimal(0)
    with decimal.localcontext() as ctx:
        if newer:
            ctx.prec = 9
        for d in inode_address_details:
            exact = inode_half * Decimal(d['emission']) / Decimal(total)
            if d['emission'] >= 1:
                shares[d['wallet']] = round_up(exact)
            else:
                pooled += exact
            if pooled > 0:
                bonus = round_up(pooled / len(big))
                for w in big:
                    shares[w] += bonus
    return miner_reward, shares


def get_circulating_supply(block_no):
    """Coins minted up to ``block_no`` (reference manager.py:215-234): every completed era at its per-block
    reward plus the current era's blocks so far, summed era by era in binary floating point as the reference
    does (the result type and rounding are the reference's); the maximum supply past the ninth halving."""
    if block_no > LAST_REWARD_BLOCK:
        return Decimal(MAX_SUPPLY)
    done, into = divmod(block_no, HALVING_BLOCKS)
    blocks_per_era = [HALVING_BLOCKS] * done + ([into] if into else [])
    minted = 0
    for era, blocks in enumerate(blocks_per_era):
        minted += (6 / 2 ** era) * blocks
    return minted


# ---------------------------------------------------------------------------------------------- mempool GC
async def clear_pending_transactions(transactions=None):
    """manager.py:253-330. The reference restarts from scratch after every removal (O(n^2));
    here a conflict removes the tx and the scan continues with the remaining ones (same result set)."""
    database: Database = Database.instance
    await database.clear_duplicate_pending_transactions()
    while True:
        restart = False
        txs = transactions or await database.get_pending_transactions_limit(hex_only=True)
        transactions = None
        used_inputs = set()
        buckets = {k: [] for k in ('inode', 'vpower', 'dpower', 'iballot', 'vballot', 'regular')}
        for transaction in txs:
            if isinstance(transaction, str):
                tx_hash = sha256(transaction)
                transaction = await Transaction.from_hex(transaction, check_signatures=False)
            else:
                tx_hash = sha256(transaction.hex())
            tx_inputs = [(i.tx_hash, i.index) for i in transaction.inputs]
            if any(u in used_inputs for u in tx_inputs):
                await database.remove_pending_spent_outputs_by_tuple(tx_inputs)
                await database.remove_pending_transaction(tx_hash)
                logger.info(f'clear_pending_transactions: removed {tx_hash}')
                restart = True
                break
            used_inputs.update(tx_inputs)
            t = transaction.transaction_type
            key = {TransactionType.INODE_DE_REGISTRATION: 'inode', TransactionType.VOTE_AS_VALIDATOR: 'vpower',
                   TransactionType.VOTE_AS_DELEGATE: 'dpower', TransactionType.REVOKE_AS_VALIDATOR: 'iballot',
                   TransactionType.REVOKE_AS_DELEGATE: 'vballot'}.get(t, 'regular')
            buckets[key].extend(tx_inputs)
        if restart:
            continue
        lookups = (('regular', database.get_unspent_outputs), ('inode', database.get_inode_outputs),
                   ('vpower', database.get_validator_voting_power_outputs),
                   ('dpower', database.get_delegates_voting_power_outputs),
                   ('iballot', database.get_inodes_ballot_outputs), ('vballot', database.get_validators_ballot_outputs))
        for key, fn in lookups:
            if buckets[key]:
                await verify_outputs(buckets[key], await fn(buckets[key]))
        return None


async def verify_outputs(used_inputs, outputs):
    """manager.py:333-349."""
    database: Database = Database.instance
    double_spend_inputs = set(used_inputs) - set(outputs)
    if double_spend_inputs == set(used_inputs):
        await database.remove_pending_transactions()
    elif double_spend_inputs:
        await database.remove_pending_spent_outputs_by_tuple(list(double_spend_inputs))
        await database.remove_pending_transactions_by_contains(
            [tx_input[0] + bytes([tx_input[1]]).hex() for tx_input in double_spend_inputs])
        logger.info(f'clear_pending_transactions verify_outputs: removed {double_spend_inputs}')


def get_transactions_size(transactions: List[Transaction]) -> int:
    return sum(len(t.hex()) for t in transactions)


# ---------------------------------------------------------------------------------------------- blocks
_GOV_SPEND = (TransactionType.INODE_DE_REGISTRATION, TransactionType.VOTE_AS_VALIDATOR,
              TransactionType.VOTE_AS_DELEGATE, TransactionType.REVOKE_AS_VALIDATOR,
              TransactionType.REVOKE_AS_DELEGATE)


async def check_block_header(block_content: str, mining_info: tuple, error_list: list):
    """Header checks of manager.py:430-462 (PoW, previous hash, timestamp window).
    Returns (block_no, merkle_tree) or None after recording the error."""
    if mining_info is None:
        mining_info = await calculate_difficulty()
    difficulty, last_block = mining_info
    block_no = last_block['id'] + 1 if last_block != {} else 1
    previous_hash, address, merkle_tree, content_time, content_difficulty, random = split_block_content(block_content)
    if not await check_block_is_valid(block_content, mining_info):
        error_list.append('block not valid')
        logger.error('block not valid')
        return None
    content_time = int(content_time)
    if last_block != {} and previous_hash != last_block['hash']:
        error_list.append(error := 'Previous hash is not matched')
        logger.error(error)
        return None
    last_ts = last_block['timestamp'] if 'timestamp' in last_block else 0
    if last_ts > content_time or last_ts == content_time:
        error_list.append(error := 'timestamp younger than previous block')
        logger.error(error)
        return None
    current_timestamp = timestamp()
    if content_time > current_timestamp:
        error_list.append(error := f'timestamp in the future content_time: {content_time}, '
                                   f'current_timestamp {current_timestamp}')
        logger.error(error)
        return None
    return block_no, merkle_tree


async def check_block(block_content: str, transactions: List[Transaction], mining_info: tuple = None,
                      error_list=None) -> bool:
    """manager.py:422-647."""
    from .validate import verify_block_transactions
    if error_list is None:
        error_list = []
    t0 = perf_counter()
    hdr = await check_block_header(block_content, mining_info, error_list)
    if hdr is None:
        return False
    block_no, merkle_tree = hdr
    database: Database = Database.instance
    transactions = [tx for tx in transactions if isinstance(tx, Transaction)]
    if get_transactions_size(transactions) > MAX_BLOCK_SIZE_HEX:
        error_list.append(error := 'block is too big')
        logger.error(error)
        return False
    t_utxo = perf_counter()
    if transactions:
        def bucket(pred):
            return [(i.tx_hash, i.index) for tx in transactions if pred(tx.transaction_type) for i in tx.inputs]

        check_inputs = bucket(lambda t: t not in _GOV_SPEND)
        categories = [
            (check_inputs, await database.get_unspent_outputs(check_inputs), None),
            (bucket(lambda t: t == TransactionType.INODE_DE_REGISTRATION), None,
             'double spend in inode transaction in block'),
            (bucket(lambda t: t == TransactionType.VOTE_AS_VALIDATOR), None,
             'double spend in validator power transaction in block'),
            (bucket(lambda t: t == TransactionType.VOTE_AS_DELEGATE), None,
             'double spend in delegate power transaction in block'),
            (bucket(lambda t: t == TransactionType.REVOKE_AS_VALIDATOR), None,
             'double spend in inode_ballot revoke transaction in block'),
            (bucket(lambda t: t == TransactionType.REVOKE_AS_DELEGATE), None,
             'double spend in validators_ballot revoke transaction in block'),
        ]
        fns = [None, database.get_inode_outputs, database.get_validator_voting_power_outputs,
               database.get_delegates_voting_power_outputs, database.get_inodes_ballot_outputs,
               database.get_validators_ballot_outputs]
        for k in range(1, 6):
            inputs, _, msg = categories[k]
            categories[k] = (inputs, await fns[k](inputs), msg)
        unspent = categories[0][1]
        if len(set(check_inputs)) != len(check_inputs) or set(check_inputs) - set(unspent) != set():
            spent_outputs = set(check_inputs) - set(unspent)
            allowed = double_spend_dict.get(block_no)
            if allowed is None or spent_outputs - set(allowed) != set():
                error_list.append(error := f'double spend in block: {block_no}, utxo: {spent_outputs}')
                logger.error(error)
                return False
        for inputs, found, msg in categories[1:]:
            if len(set(inputs)) != len(inputs) or set(inputs) - set(found) != set():
                error_list.append(msg)
                logger.error(msg)
                return False
        input_txs = await database.get_transactions_info([i.tx_hash for tx in transactions for i in tx.inputs])
        for tx in transactions:
            await tx._fill_transaction_inputs(input_txs)
    t_verify = perf_counter()
    bad = await verify_block_transactions(transactions)
    if bad is not None:
        error_list.append(error := f'transaction {bad.hash()} has been not verified')
        logger.error(error)
        return False
    t_merkle = perf_counter()
    transactions_merkle_tree = get_transactions_merkle_tree(transactions)
    last_block_timings.update({'utxo_s': t_verify - t_utxo, 'verify_s': t_merkle - t_verify,
                               'merkle_s': perf_counter() - t_merkle, 'total_s': perf_counter() - t0,
                               'txs': len(transactions)})
    if merkle_tree != transactions_merkle_tree:
        if block_no == 340510 and merkle_tree == '54e7e3fbfe5c3c7b2a74d14efd22a61c231d157b2c5c2476fca67736736b9ac8':
            return True
        error_list.append(error := 'merkle tree does not match')
        logger.error(error)
        return False
    return True


async def _apply_block(block_no, block_hash, block_content, address, random, difficulty, block_reward, fees,
                       content_time, coinbase_transaction, transactions) -> bool:
    """DB writes of manager.py:706-730 (shared by create_block and the sync path), applied as ONE
    SQLite transaction: a failure at any stage leaves the ledger and the UTXO index untouched (the
    reference deletes the half-written block instead, manager.py:718-723)."""
    database: Database = Database.instance
    if database.writer is not None and block_no not in double_spend_dict:
        # through the ledger journal like the native path (commit point + background materialisers);
        # blocks of the double-spend exception table keep the synchronous path below, whose partial
        # deletes and uniqueness errors are decided by SQL
        from .database import numeric
        if isinstance(content_time, datetime):
            content_time = int(content_time.timestamp())
        row = {'id': block_no, 'hash': block_hash, 'content': block_content, 'address': address, 'random': int(random),
               'difficulty': numeric(difficulty, 1), 'reward': numeric(block_reward + fees, 6),
               'timestamp': int(content_time)}
        submitted = database._submitted
        try:
            await database.apply_object_block(row, coinbase_transaction, transactions)
        except Exception as e:
            if database._submitted != submitted:
                raise  # committed to the journal: a failure after the commit point is not a rejection
            logger.error(f'Transaction of {block_no} has not been added in block {e}')
            Manager.difficulty = None
            return False
        return True
    from .database import _commit_point
    _commit_point()  # a cluster node: every replica ready to write this block (no-op on a single node)
    try:
        with database.transaction():
            await database.add_block(block_no, block_hash, block_content, address, random, difficulty,
                                     block_reward + fees, content_time)
            database.checkpoint('block')
            await database.add_transaction(coinbase_transaction, block_hash)
            await database.add_transactions(transactions, block_hash)
            database.checkpoint('transactions')
            await database.add_transaction_outputs(transactions + [coinbase_transaction])
            database.checkpoint('outputs')
            if transactions:
                await database.remove_pending_transactions_by_hash([t.hash() for t in transactions])
                await database.remove_outputs(transactions)
                await database.remove_pending_spent_outputs(transactions)
            database.checkpoint('spent')
    except Exception as e:
        logger.error(f'Transaction of {block_no} has not been added in block {e}')
        database._rebuild_utxo_index()
        Manager.difficulty = None
        return False
    return True


_ledger_locks: 'weakref.WeakKeyDictionary' = weakref.WeakKeyDictionary()


_LOCK_OWNER: 'contextvars.ContextVar' = contextvars.ContextVar('upow_ledger_lock_owner', default=None)


class _LedgerLock:
    """``async with`` form of the loop's ledger lock, re-entrant for the task that holds it (a lean cluster
    follower materialising its op log from inside a block's critical section, ledger/lean.py). Another task
    — a child task included, which inherits the context — still waits for the lock."""
    __slots__ = ('lk', 'token')

    def __init__(self, lk: asyncio.Lock):
        self.lk, self.token = lk, None

    async def __aenter__(self):
        me = asyncio.current_task()
        if _LOCK_OWNER.get() is me and self.lk.locked():
            return self
        await self.lk.acquire()
        self.token = _LOCK_OWNER.set(me)
        return self

    async def __aexit__(self, *exc):
        if self.token is not None:
            _LOCK_OWNER.reset(self.token)
            self.token = None
            self.lk.release()

    def locked(self) -> bool:
        return self.lk.locked()


def ledger_lock() -> _LedgerLock:
    """One lock per event loop serialising every ledger mutation (block apply, rollback).

    The reference guards nothing: two concurrent ``/push_block`` calls can both pass ``check_block``
    on the same parent (race detection). Here check+apply is one critical section,
    so the second block at a height is checked against the first one's result."""
    loop = asyncio.get_running_loop()
    lk = _ledger_locks.get(loop)
    if lk is None:
        lk = _ledger_locks[loop] = asyncio.Lock()
    return _LedgerLock(lk)


async def create_block(block_content: str, transactions: List[Transaction], last_block: dict = None,
                       error_list=None) -> bool:
    """manager.py:650-757 (serialised by :func:`ledger_lock`)."""
    async with ledger_lock():
        t0 = perf_counter()
        ok = await _create_block(block_content, transactions, last_block, error_list)
        _record_block_metrics(ok, perf_counter() - t0, len(transactions), 'push')
        return ok


_TRACE_PATH = os.environ.get('UPOW_TRACE_FILE')  # JSON-lines block trace (one record per block)


def _trace_block(ok: bool, seconds: float, n_txs: int, path: str):
    """Append one record per validated block: verdict, path, tip, and the per-stage wall times the
    native path / batched validator recorded (decode, HBM UTXO pass, decompression, ECDSA, ledger
    writes, commit). Off unless ``UPOW_TRACE_FILE`` is set."""
    if not _TRACE_PATH:
        return
    import json
    import time as _time
    from . import fastpath, validate
    stages = {k: round(v * 1000, 3) for k, v in {**last_block_timings, **validate.timings, **fastpath.timings}.items()
              if k.endswith('_s') and isinstance(v, float)}
    rec = {'t': round(_time.time(), 3), 'ok': ok, 'path': path, 'txs': n_txs, 'ms': round(seconds * 1000, 3),
           'height': Database.instance._tip_id() if Database.instance else None, 'stages_ms': stages}
    try:
        with open(_TRACE_PATH, 'a') as f:
            f.write(json.dumps(rec) + '\n')
    except OSError as e:
        logger.error(f'block trace write failed: {e}')


def _record_block_metrics(ok: bool, seconds: float, n_txs: int, path: str):
    _trace_block(ok, seconds, n_txs, path)
    if ok:
        metrics.inc('upow_blocks_applied_total', labels={'path': path}, help='blocks validated and applied')
        metrics.inc('upow_transactions_applied_total', n_txs, help='non-coinbase transactions applied')
        metrics.observe('upow_block_apply_seconds', seconds, labels={'path': path},
                        help='check_block + ledger apply wall time')
        metrics.set_gauge('upow_chain_height', (Database.instance._tip_id() if Database.instance else 0),
                          help='id of the last applied block')
    else:
        metrics.inc('upow_blocks_rejected_total', labels={'path': path}, help='blocks rejected by validation')


async def _create_block(block_content: str, transactions: List[Transaction], last_block: dict = None,
                        error_list=None) -> bool:
    if error_list is None:
        error_list = []
    create_start_time = perf_counter()
    Manager.difficulty = None
    if last_block is None or last_block['id'] % BLOCKS_COUNT == 0:
        difficulty, last_block = await calculate_difficulty()
    else:
        difficulty, last_block = await get_difficulty()
    block_no = last_block['id'] + 1 if last_block != {} else 1
    logger.info(f'Creating block no. {block_no}')
    if not await check_block(block_content, transactions, (difficulty, last_block), error_list=error_list):
        return False
    fees = sum(t.fees for t in transactions)

    async def apply(block_hash, address, random, block_reward, content_time, coinbase_transaction):
        return await _apply_block(block_no, block_hash, block_content, address, random, difficulty, block_reward, fees,
                                  content_time, coinbase_transaction, transactions)
    return await _finalize_block(block_no, block_content, fees, len(transactions), apply, error_list,
                                 create_start_time)


async def _finalize_block(block_no: int, block_content: str, fees, n_txs: int, apply, error_list: list,
                          create_start_time: float) -> bool:
    """The part of manager.py:650-757 after ``check_block``: inode rewards, genesis-key rule, coinbase,
    ledger writes (``apply``), logs, UTXO snapshot cadence and the emission-details record. Shared by
    the object path (:func:`_create_block`) and the native block path (ledger/fastpath.py)."""
    database: Database = Database.instance
    roctx.push('finalize:rewards')
    block_hash = sha256(block_content)
    previous_hash, address, merkle_tree, content_time, content_difficulty, random = split_block_content(block_content)
    ta = perf_counter()
    active_inodes = await database.get_active_inodes()
    last_block_timings['active_inodes_s'] = perf_counter() - ta
    await update_active_inodes_cache_with_data(active_inodes)
    block_reward = get_block_reward(block_no)
    miner_reward, inode_rewards = get_inode_rewards(block_reward, active_inodes, block_no=block_no)
    genesis_block_content = await database.get_genesis_block()
    if genesis_block_content is not None:
        _, genesis_address, _, _, _, _ = split_block_content(genesis_block_content)
        if not ((address == genesis_address and block_no <= LAST_BLOCK_FOR_GENESIS_KEY) or inode_rewards):
            error_list.append(error := 'Emission detail is not formed. Hence you cannot mine currently.')
            logger.error(error)
            return False
    coinbase_transaction = CoinbaseTransaction(block_hash, address, miner_reward + fees)
    if inode_rewards:
        coinbase_transaction.outputs.extend([TransactionOutput(a, r) for a, r in inode_rewards.items()])
    if not all(o.verify() for o in coinbase_transaction.outputs):
        roctx.pop()
        return False
    roctx.pop()
    if not _commit_gate():
        return False
    if not await apply(block_hash, address, random, block_reward, content_time, coinbase_transaction):
        return False
    roctx.push('finalize:post')
    logger.info(f'Added {n_txs} transactions in block {block_no}. Reward: {block_reward}, Fees: {fees} '
                f'in {perf_counter() - create_start_time:.3f} seconds')
    if block_no % 10 == 0 and not database.lean:  # a lean follower leaves the K12 line to the leader
        await _log_utxo_hash(database, block_no)
    _maybe_snapshot(database, block_no)
    Manager.difficulty = None
    try:
        details = [{'power': str(i['power']), 'emission': str(i['emission']), 'wallet': i['wallet'],
                    'inode_reward': str(inode_rewards.get(i['wallet'], ''))} for i in active_inodes]
        database.emission_details.set(str(block_no), details)
    except Exception as e:
        logger.error(f'Error in creating block: {block_no} {str(e)}')
    roctx.pop()
    return True


def _commit_gate() -> bool:
    """On a multi-GPU cluster node: every replica agrees to commit this block before any of them writes it
    (parallel/cluster.py ``commit_gate``: the block is marked ready here; the vote is cast at the ledger's
    commit point, right before the journal write, after everything that can fail without writing); always
    True on a single node."""
    from ..parallel import cluster
    return cluster.commit_gate()


_K12_POOL = None


async def _log_utxo_hash(database, block_no: int):
    """The K12 log line every 10 blocks (reference manager.py:740-741, 833-834). Computed only when the line
    is emitted. The block path only takes a snapshot of the UTXO set at this block (one compaction launch);
    the sort, the message gather and the sequential SHA-256 over it (165 MB at 5 M UTXOs) run on a worker
    thread and the GPU's aux stream, so the next block waits for none of it."""
    global _K12_POOL
    import logging
    if not logger.isEnabledFor(logging.INFO):
        return
    if os.environ.get('UPOW_UTXO_HASH_SQL', '0') == '1':
        logger.info(f'unspent_outputs_hash on block no. {block_no}: {await database.get_unspent_outputs_hash()}')
        return
    from concurrent.futures import ThreadPoolExecutor
    from .utxo import TAG_BY_TABLE
    digest = database.utxo.k12_snapshot(TAG_BY_TABLE['unspent_outputs'])
    if _K12_POOL is None:
        _K12_POOL = ThreadPoolExecutor(max_workers=1, thread_name_prefix='upow-k12')
    _K12_POOL.submit(lambda: logger.info(f'unspent_outputs_hash on block no. {block_no}: {digest()}'))


SNAPSHOT_EVERY = int(os.environ.get('UPOW_SNAPSHOT_EVERY', '1000'))
# UPOW_SNAPSHOT_ASYNC=0: the periodic snapshot sorts, hashes and writes on the block path (A/B)
SNAPSHOT_ASYNC = os.environ.get('UPOW_SNAPSHOT_ASYNC', '1') != '0'


def _maybe_snapshot(database, block_no: int):
    """Periodic UTXO-index checkpoint (ledger/snapshot.py); never fails the block."""
    if SNAPSHOT_EVERY <= 0 or block_no % SNAPSHOT_EVERY or database.path == ':memory:' or database.lean:
        # a lean follower's index is ahead of its SQL tables: a snapshot is taken of a materialised state only
        return
    try:
        from . import snapshot
        res = snapshot.save(database, background=SNAPSHOT_ASYNC)
        if res is not None and SNAPSHOT_ASYNC:  # a failure of the background write is logged when it happens
            res.add_done_callback(lambda f: f.exception() and logger.error(
                f'UTXO snapshot at block {block_no} failed: {f.exception()}'))
    except Exception as e:
        logger.error(f'UTXO snapshot at block {block_no} failed: {e}')


async def create_block_in_syncing_old(block_content: str, transactions: List[Transaction],
                                      cb_transaction: CoinbaseTransaction, last_block: dict = None,
                                      error_list=None) -> bool:
    async with ledger_lock():
        t0 = perf_counter()
        ok = await _create_block_in_syncing_old(block_content, transactions, cb_transaction, last_block, error_list)
        _record_block_metrics(ok, perf_counter() - t0, len(transactions), 'sync')
        return ok


async def _create_block_in_syncing_old(block_content: str, transactions: List[Transaction],
                                       cb_transaction: CoinbaseTransaction, last_block: dict = None,
                                       error_list=None) -> bool:
    """manager.py:760-835: sync path, trusts the supplied coinbase."""
    if error_list is None:
        error_list = []
    create_start_time = perf_counter()
    Manager.difficulty = None
    if last_block is None or last_block['id'] % BLOCKS_COUNT == 0:
        difficulty, last_block = await calculate_difficulty()
    else:
        difficulty, last_block = await get_difficulty()
    block_no = last_block['id'] + 1 if last_block != {} else 1
    logger.info(f'Syncing block no. {block_no}')
    if not await check_block(block_content, transactions, (difficulty, last_block), error_list=error_list):
        return False
    fees = sum(t.fees for t in transactions)

    async def apply(block_hash, address, random, block_reward, content_time, coinbase_transaction):
        return await _apply_block(block_no, block_hash, block_content, address, random, difficulty, block_reward, fees,
                                  content_time, coinbase_transaction, transactions)
    return await _finalize_sync_block(block_no, block_content, fees, len(transactions), apply, cb_transaction,
                                      create_start_time)


async def _finalize_sync_block(block_no: int, block_content: str, fees, n_txs: int, apply,
                               cb_transaction: Optional[CoinbaseTransaction], create_start_time: float) -> bool:
    """Tail of manager.py:760-835 (trusted coinbase), shared with the native block path."""
    block_hash = sha256(block_content)
    previous_hash, address, merkle_tree, content_time, content_difficulty, random = split_block_content(block_content)
    block_reward = get_block_reward(block_no)
    if cb_transaction is None or not all(o.verify() for o in cb_transaction.outputs):
        return False
    if not _commit_gate():
        return False
    if not await apply(block_hash, address, random, block_reward, content_time, cb_transaction):
        return False
    logger.info(f'Added {n_txs} transactions in block {block_no}. Reward: {block_reward}, Fees: {fees} '
                f'in {perf_counter() - create_start_time:.3f} seconds')
    if block_no % 10 == 0 and not Database.instance.lean:
        await _log_utxo_hash(Database.instance, block_no)
    _maybe_snapshot(Database.instance, block_no)
    Manager.difficulty = None
    return True


double_spend_dict = {
    286523: [
        ('16c519171bfa7ee7d42af0d84fe731433048a1aedfd5df692b8beaa755ef6eb9', 0),
        ('747d753fcfecdce5d3a080666ff139ca9123d72d2eb529386f2c3f9f4a55f983', 1),
        ('856b36ecd55a3a427cc988550457435ee9dd7580a423bc3177c1d173b50ff101', 1),
        ('af33808f839698734d801e907f1eb1c24c3547d4cdd984ed0f2e41c58c6d1d9a', 1),
        ('db843078e1fd5f1bbf1c2f550f87548df6fe714ccd12a0ba4a1e25e10fea3ae0', 1),
        ('eb10fd11319aeee7a21766b85c89580f6c3f509a6afaf743df717ca91d33e0da', 1),
    ],
    347027: [
        ('4fd22d5ca99eaa044288de9f850385cbf758efdc4967a92623138e986ce4316e', 2),
        ('b88e9beef7559d48d99ea82e71f7c0601981d6972021feb929c04bc7b52368c2', 1),
        ('ed0f9e07d97ab8a5dc7b8e68ad631a5e78f3cfb6ee6f2aa013854caa64a7b1ae', 1),
    ],
    347034: [('047f5c343dcd15a16c44b3f05fe98bc467002405490ecfb517652207e5425858', 2)],
    349122: [
        ('691695269d8baa441b8e1638a17b3b8497295ec8322c750e8b5312768d4b9ce5', 1),
        ('f7894d0cab92445bd1bb7681106d8fb18d9b4af2465db8a73efbdb97431f855f', 1),
    ],
    395735: [
        ('461c359b956773ff97af6d2189ae84bcc52740e077224efc80b8b5826b51cb92', 1),
        ('ef573f3543ef22b087387fd81493cc7bc977adcc1ff4198483a98a67a6d10e6b', 1),
        ('9efcb290e4c24843bab40dc50591680ac897e52a28db62c7594e4a2b07702291', 1),
    ],
    395736: [
        ('d8421370cef17939c4a2b17c21c7674059c0c24766e80d6129c666f11e886e08', 1),
        ('af2422540ef2f4570b998b262c242b37f7f0e44fbadabcb0f52684dd0ce1ace5', 1),
    ],
}


# ---------------------------------------------------------------------------------------------- inode cache
async def update_cache() -> None:
    global cache_updating
    if cache_updating:
        return
    cache_updating = True
    try:
        cache['inodes'] = await Database.instance.get_active_inodes()
        cache['timestamp'] = datetime.utcnow()
    finally:
        cache_updating = False


async def update_active_inodes_cache_with_data(active_inodes) -> None:
    cache['inodes'] = active_inodes
    cache['timestamp'] = datetime.utcnow()


async def get_inodes_from_cache() -> list:
    """manager.py:886-900 (5 min cache, refreshed in the background)."""
    now = datetime.utcnow()
    if 'inodes' in cache and (now - cache['timestamp']) < cache_expiration:
        return cache['inodes']
    if not cache:
        await update_cache()
    else:
        asyncio.create_task(update_cache())
    return cache.get('inodes', [])


__all__ = ['Manager', 'calculate_difficulty', 'get_difficulty', 'check_block_is_valid', 'get_block_reward',
           'get_inode_rewards', 'get_circulating_supply', 'clear_pending_transactions', 'check_block',
           'create_block', 'create_block_in_syncing_old', 'get_transactions_merkle_tree', 'block_to_bytes',
           'split_block_content', 'get_inodes_from_cache', 'double_spend_dict', 'get_transactions_merkle_tree_ordered']
