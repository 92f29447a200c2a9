"""Ledger + consensus on an in-memory devnet (host backends): blocks, transfers, staking, UTXO hash."""
import asyncio
import hashlib
from decimal import Decimal

import pytest

from upow_amd import devnet
from upow_amd.ledger import manager
from upow_amd.ledger.database import Database
from upow_amd.models.transaction import Transaction
from upow_amd.ops import p256 as op
from upow_amd.utils.codec import point_to_string
from upow_amd.wallet import builders


def run(coro):
    return asyncio.get_event_loop().run_until_complete(coro) if False else asyncio.run(coro)


@pytest.fixture
def chain(monkeypatch):
    monkeypatch.setattr(manager, 'START_DIFFICULTY', Decimal('1.5'))
    manager.Manager.difficulty = None
    manager.cache.clear()

    async def setup():
        db = await Database.create(utxo_backend='host')
        return db
    db = asyncio.run(setup())
    yield db
    db.close()


KEY_A = 0x1111111111111111111111111111111111111111111111111111111111111111
KEY_B = 0x2222222222222222222222222222222222222222222222222222222222222222


def test_mine_transfer_and_balances(chain):
    async def go():
        a = builders.address_of(KEY_A)
        b = builders.address_of(KEY_B)
        base = 1_700_000_000
        await devnet.mine_block(a, ts=base + 1)
        await devnet.mine_block(a, ts=base + 2)
        assert await chain.get_next_block_id() == 3
        bal = await chain.get_address_balance(a)
        assert bal == Decimal(12)
        tx = await builders.create_transaction(KEY_A, b, '2.5')
        assert await chain.add_pending_transaction(tx)
        # the same input cannot be spent twice in the mempool
        tx2 = await builders.create_transaction(KEY_A, b, '1')
        assert tx2.inputs[0].tx_hash != tx.inputs[0].tx_hash or tx2.inputs[0].index != tx.inputs[0].index
        pend = await chain.get_pending_transactions_limit()
        assert [t.hash() for t in pend] == [tx.hash()]
        await devnet.mine_block(a, pend, ts=base + 3)
        assert await chain.get_address_balance(b) == Decimal('2.5')
        assert await chain.get_address_balance(a) == Decimal(18) - Decimal('2.5')
        assert await chain.get_pending_transactions_limit() == []
        # UTXO-set hash matches a recomputation from the full replay
        outs = await chain.get_unspent_outputs_from_all_transactions()
        h = hashlib.sha256(b''.join(bytes.fromhex(t) + bytes([i]) for t, i in sorted(outs))).hexdigest()
        assert await chain.get_unspent_outputs_hash() == h
        # parse round trip of every stored tx
        for blk in await chain.get_blocks(1, 10):
            for hx in blk['transactions']:
                t = await Transaction.from_hex(hx)
                assert t.hex() == hx
        nice = await chain.get_nice_transaction(tx.hash(), address=b)
        assert nice['delta'] == Decimal('2.5') and nice['is_confirm'] is True
    asyncio.run(go())


def test_double_spend_and_bad_signature_rejected(chain):
    async def go():
        a = builders.address_of(KEY_A)
        b = builders.address_of(KEY_B)
        base = 1_700_000_000
        await devnet.mine_block(a, ts=base + 1)
        await devnet.mine_block(a, ts=base + 2)
        tx = await builders.create_transaction(KEY_A, b, '1')
        # tamper the signature -> block rejected
        bad = await Transaction.from_hex(tx.hex())
        r, s = bad.inputs[0].signed
        for i in bad.inputs:
            i.signed = (r, (s + 1) % op.oracle.N)
        bad.tx_hash = None
        with pytest.raises(RuntimeError, match='has been not verified'):
            await devnet.mine_block(a, [bad], ts=base + 3)
        # the same tx twice in one block -> double spend
        with pytest.raises(RuntimeError, match='double spend'):
            await devnet.mine_block(a, [tx, await Transaction.from_hex(tx.hex())], ts=base + 3)
        await devnet.mine_block(a, [tx], ts=base + 3)
        with pytest.raises(RuntimeError, match='double spend'):
            await devnet.mine_block(a, [await Transaction.from_hex(tx.hex())], ts=base + 4)
    asyncio.run(go())


def test_stake_and_validator_flow(chain):
    async def go():
        a = builders.address_of(KEY_A)
        base = 1_700_000_000
        for k in range(1, 25):
            await devnet.mine_block(a, ts=base + k)
        stake = await builders.create_stake_transaction(KEY_A, '10')
        assert await chain.add_pending_transaction(stake)
        await devnet.mine_block(a, await chain.get_pending_transactions_limit(), ts=base + 30)
        assert await chain.get_address_stake(a) == Decimal(10)
        assert len(await chain.get_delegates_voting_power(a)) == 1
        val = await builders.create_validator_registration_transaction(KEY_A)
        assert await chain.add_pending_transaction(val)
        await devnet.mine_block(a, await chain.get_pending_transactions_limit(), ts=base + 31)
        assert await chain.is_validator_registered(a)
        assert len(await chain.get_validators_voting_power(a)) == 1
        with pytest.raises(Exception, match='Already staked'):
            await builders.create_stake_transaction(KEY_A, '5')
    asyncio.run(go())


@pytest.mark.parametrize('stage', ['block', 'transactions', 'outputs', 'spent'])
def test_block_apply_is_atomic_under_injected_failure(chain, stage):
    async def go():
        a = builders.address_of(KEY_A)
        b = builders.address_of(KEY_B)
        base = 1_700_000_000
        await devnet.mine_block(a, ts=base + 1)
        await devnet.mine_block(a, ts=base + 2)
        tx = await builders.create_transaction(KEY_A, b, '1')
        assert await chain.add_pending_transaction(tx)
        before = (await chain.get_next_block_id(), await chain.get_unspent_outputs_hash(), len(chain.utxo),
                  await chain.get_pending_transactions_limit(hex_only=True))
        chain.fail_after_stage = stage
        with pytest.raises(RuntimeError, match='block rejected'):
            await devnet.mine_block(a, [tx], ts=base + 3)
        after = (await chain.get_next_block_id(), await chain.get_unspent_outputs_hash(), len(chain.utxo),
                 await chain.get_pending_transactions_limit(hex_only=True))
        assert after == before
        chain.fail_after_stage = None
        await devnet.mine_block(a, [tx], ts=base + 3)
        assert await chain.get_address_balance(b) == 1
    asyncio.run(go())


def test_address_utxos_tool(chain, tmp_path, capsys):
    """``python -m upow_amd.tools address-utxos``: the index's view of an address equals the SQL view —
    spendable outputs and balance (get_address_balance, is_stake excluded), staked outputs, governance
    tables — with outputs sent to both string forms of the same key."""
    from upow_amd import tools
    from upow_amd.utils.codec import AddressFormat, string_to_point

    async def go():
        a = builders.address_of(KEY_A)
        b = builders.address_of(KEY_B)
        b_full = point_to_string(string_to_point(b), AddressFormat.FULL_HEX)
        base = 1_700_000_000
        for k in range(4):
            await devnet.mine_block(a, ts=base + 1 + k)
        tx = await builders.create_transaction(KEY_A, b, '2.5')
        assert await chain.add_pending_transaction(tx)
        a_full = point_to_string(string_to_point(a), AddressFormat.FULL_HEX)
        # a version-1 tx: every output in the full-hex (64-byte) form
        tx2 = await builders.create_transaction(KEY_A, b_full, '1.25', send_back_address=a_full)
        assert tx2.version == 1
        assert await chain.add_pending_transaction(tx2)
        await devnet.mine_block(a, [tx, tx2], ts=base + 10)
        stx = await builders.create_stake_transaction(KEY_B, '1')  # a staked output + delegate voting power
        assert await chain.add_pending_transaction(stx)
        await devnet.mine_block(a, [stx], ts=base + 11)
        for addr in (a, b, b_full, a_full):
            res = await tools.address_utxos(addr, db=chain)
            assert Decimal(res['spendable']) == await chain.get_address_balance(addr)
            assert Decimal(res['stake']) == await chain.get_address_stake(addr)
            sql = sorted((i.tx_hash, i.index) for i in await chain.get_spendable_outputs(addr))
            sql += sorted((i.tx_hash, i.index) for i in await chain.get_stake_outputs(addr))
            sql += sorted((i.tx_hash, i.index) for i in await chain.get_delegates_voting_power(addr))
            assert sorted((o['tx_hash'], o['index']) for o in res['outputs']) == sorted(sql)
        res = await tools.address_utxos(b, db=chain)
        assert sorted(o['amount'] for o in res['outputs'] if not o['is_stake'] and o['table'] == 'unspent_outputs') \
            == ['1.25', '2.5'] or Decimal(res['spendable']) == Decimal('3.75') - 1
        assert Decimal(res['stake']) == 1 and Decimal(res['tables']['delegates_voting_power']) == 10
    asyncio.run(go())
    with pytest.raises(SystemExit):
        tools.main(['address-utxos'])
    capsys.readouterr()


@pytest.mark.parametrize('backend', ['host', pytest.param('gpu', marks=pytest.mark.gpu)])
def test_rollback_restores_utxo_index(monkeypatch, backend, request):
    """remove_blocks (reference database.py:146-169) on either index backend: the index after rolling
    back block 4 (which spends block-3 outputs) equals the index at height 3 — keys, tags and payloads —
    and the UTXO-set hash and balances follow; re-mining the block afterwards applies cleanly."""
    if backend == 'gpu':
        request.getfixturevalue('gpu')
    monkeypatch.setattr(manager, 'START_DIFFICULTY', Decimal('1.5'))
    manager.Manager.difficulty = None
    manager.cache.clear()

    async def go():
        db = await Database.create(utxo_backend=backend)
        try:
            a = builders.address_of(KEY_A)
            b = builders.address_of(KEY_B)
            base = 1_700_000_000
            await devnet.mine_block(a, ts=base + 1)
            await devnet.mine_block(a, ts=base + 2)
            tx = await builders.create_transaction(KEY_A, b, '2.5')
            assert await db.add_pending_transaction(tx)
            await devnet.mine_block(a, [tx], ts=base + 3)
            recs3, pay3 = db.utxo.records_payload()
            hash3, bal3 = await db.get_unspent_outputs_hash(), await db.get_address_balance(b)
            tx2 = await builders.create_transaction(KEY_B, a, '1')
            assert await db.add_pending_transaction(tx2)
            await devnet.mine_block(a, [tx2], ts=base + 4)
            assert await db.get_address_balance(b) == Decimal('1.5')
            await db.remove_blocks(4)
            manager.Manager.difficulty = None
            assert await db.get_next_block_id() == 4
            recs, pay = db.utxo.records_payload()
            assert recs.tobytes() == recs3.tobytes() and pay.tobytes() == pay3.tobytes()
            assert await db.get_unspent_outputs_hash() == hash3
            assert await db.get_address_balance(b) == bal3 == Decimal('2.5')
            tx3 = await builders.create_transaction(KEY_B, a, '0.5')
            assert await db.add_pending_transaction(tx3)
            await devnet.mine_block(a, [tx3], ts=base + 5)
            assert await db.get_address_balance(b) == Decimal(2)
        finally:
            db.close()
    asyncio.run(go())
