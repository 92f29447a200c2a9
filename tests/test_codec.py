"""Byte-exact wire codecs and helper semantics (reference upow/helpers.py)."""
import asyncio
import hashlib
import random
from decimal import Decimal

import pytest
from hypothesis import given, settings, strategies as st

from upow_amd.models.transaction import CoinbaseTransaction, Transaction, TransactionInput, TransactionOutput
from upow_amd.ops import p256 as op
from upow_amd.utils import codec
from upow_amd.utils import p256 as o
from upow_amd.utils.codec import (AddressFormat, OutputType, TransactionType, b58decode, b58encode, bytes_to_string,
                                  get_transaction_type_from_message, point_to_bytes, point_to_string,
                                  round_up_decimal, round_up_decimal_new, string_to_bytes, string_to_point)


@given(st.binary(max_size=80))
@settings(max_examples=200, deadline=None)
def test_base58_roundtrip(b):
    assert b58decode(b58encode(b)) == b
    assert codec._b58decode_py(codec._b58encode_py(b)) == b
    assert b58encode(b) == codec._b58encode_py(b)


def test_address_forms_roundtrip():
    rng = random.Random(0)
    for _ in range(20):
        q = o.get_public_key(rng.randrange(1, o.N))
        comp = point_to_string(q)
        full = point_to_string(q, AddressFormat.FULL_HEX)
        assert string_to_point(comp) == q == string_to_point(full)
        assert len(string_to_bytes(comp)) == 33 and string_to_bytes(comp)[0] == (42 if q.y % 2 == 0 else 43)
        assert bytes.fromhex(full) == q.x.to_bytes(32, 'little') + q.y.to_bytes(32, 'little')
        assert bytes_to_string(point_to_bytes(q, AddressFormat.COMPRESSED)) == comp
        assert codec.address_forms(comp) == [full, comp]
    # an unknown specifier is normalised to 42 (the reference re-derives it from y's parity)
    q = o.get_public_key(7)
    raw = bytes([44]) + q.x.to_bytes(32, 'little')
    assert string_to_bytes(bytes_to_string(raw))[0] == 42


def test_tx_type_from_message():
    assert get_transaction_type_from_message(None) == TransactionType.REGULAR
    assert get_transaction_type_from_message(b'6') == TransactionType.VOTE_AS_VALIDATOR
    assert get_transaction_type_from_message(b'9') == TransactionType.REVOKE_AS_DELEGATE
    assert get_transaction_type_from_message(b'3') == TransactionType.REGULAR  # not a tx type
    assert get_transaction_type_from_message(b'\xff\xfe') == TransactionType.REGULAR
    assert get_transaction_type_from_message(b'hello') == TransactionType.REGULAR


def test_decimal_rounding():
    assert round_up_decimal(Decimal('1.123456789')) == Decimal('1.12345679')
    assert str(round_up_decimal(Decimal('1.5'))) == '1.5'  # untouched when already 8-decimal exact
    assert str(round_up_decimal_new(Decimal('1.5'))) == '1.50000000'
    # quantisation only happens when the value has more than 8 decimals (helpers.py:147-151)
    assert round_up_decimal(Decimal('33.333333'), '0.01') == Decimal('33.333333')
    assert round_up_decimal(Decimal(100) / 3, '0.01') == Decimal('33.33')


K1, K2, K3 = 0xabc, 0xdef, 0x123


def _signed_tx(n_inputs=2, keys=(K1,), message=None, version=None, outputs_fmt=AddressFormat.COMPRESSED):
    ins = []
    for k in range(n_inputs):
        key = keys[k % len(keys)]
        i = TransactionInput(hashlib.sha256(bytes([k])).hexdigest(), k, amount=Decimal(5),
                             public_key=op.public_key(key))
        ins.append(i)
    outs = [TransactionOutput(point_to_string(o.get_public_key(99), outputs_fmt), Decimal('1.23456789')),
            TransactionOutput(point_to_string(o.get_public_key(98), outputs_fmt), Decimal(3), OutputType.STAKE)]
    tx = Transaction(ins, outs, message, version)
    tx.sign(list(keys))
    return tx


def test_transaction_wire_layout():
    tx = _signed_tx()
    raw = bytes.fromhex(tx.hex())
    assert raw[0] == 3 and raw[1] == 2  # version 3 (33-byte outputs), 2 inputs
    assert raw[2:34] == bytes.fromhex(tx.inputs[0].tx_hash) and raw[34] == 0 and raw[35] == 0
    # output: addr 33 | amount length | amount LE (satoshi) | type
    o0 = 2 + 2 * 34 + 1
    assert raw[o0 - 1] == 2
    amt = 123456789
    assert raw[o0 + 33] == 4 and int.from_bytes(raw[o0 + 34:o0 + 38], 'little') == amt and raw[o0 + 38] == 0
    # no message -> specifier 0, then ONE de-duplicated signature (same key signed both inputs)
    end_out = o0 + 39 + 33 + 1 + 4 + 1
    assert raw[end_out] == 0 and len(raw) == end_out + 1 + 64
    assert tx.hash() == hashlib.sha256(raw).hexdigest()
    # the signed message excludes the specifier byte for no-message txs
    assert tx.hex(False) == raw[:end_out].hex()


@pytest.mark.parametrize('message', [None, b'hello', b'x' * 300])
@pytest.mark.parametrize('keys', [(K1,), (K1, K2), (K1, K2, K3)])
def test_transaction_parse_roundtrip(message, keys):
    n_in = 4 if len(keys) == 2 else len(keys) if len(keys) == 3 else 2
    tx = _signed_tx(n_in, keys, message)
    if len(keys) == 2 and n_in == 4:
        # 2 signatures for 4 inputs: the parser groups inputs by owner (needs the ledger) ->
        # with check_signatures=False no assignment happens
        p = asyncio.run(Transaction.from_hex(tx.hex(), check_signatures=False))
        assert p.inputs[0].signed is None
        return
    p = asyncio.run(Transaction.from_hex(tx.hex()))
    assert p.hex() == tx.hex() and p.hash() == tx.hash()
    assert [i.signed for i in p.inputs] == [i.signed for i in tx.inputs]
    assert p.message == message
    if message is not None:
        # v3 messages carry a u16 length and are part of the signed message
        raw = bytes.fromhex(tx.hex(False))
        assert raw.endswith(bytes([1]) + len(message).to_bytes(2, 'little') + message)


def test_v1_full_address_tx_and_coinbase():
    tx = _signed_tx(1, (K1,), b'hi', outputs_fmt=AddressFormat.FULL_HEX)
    assert tx.version == 1
    raw = bytes.fromhex(tx.hex())
    assert raw[0] == 1
    p = asyncio.run(Transaction.from_hex(tx.hex()))
    assert p.hex() == tx.hex()
    # v1/v2 message: u8 length, and hex(False) stops before the message for version <= 2
    assert tx.hex(False) == tx.hex()[:len(tx.hex(False))]
    cb = CoinbaseTransaction('ab' * 32, point_to_string(o.get_public_key(5)), Decimal('6.5'))
    cb.outputs.append(TransactionOutput(point_to_string(o.get_public_key(6)), Decimal('0.25')))
    raw = bytes.fromhex(cb.hex())
    assert raw[0] == 2 and raw[1] == 1 and raw[2:34] == bytes.fromhex('ab' * 32) and raw[34] == 0 and raw[35] == 0
    assert raw[-1] == 36
    pcb = asyncio.run(Transaction.from_hex(cb.hex()))
    assert isinstance(pcb, CoinbaseTransaction) and pcb.hex() == cb.hex() and pcb.block_hash == 'ab' * 32


def test_tx_limits():
    with pytest.raises(Exception, match='max 255 inputs'):
        Transaction([TransactionInput('00' * 32, 0)] * 256, [])
    with pytest.raises(AssertionError):
        TransactionOutput(point_to_string(o.get_public_key(5)), Decimal('0.000000001'))


def test_tx_hex_memo_tracks_in_place_edits():
    """Transaction.hex() is memoised; editing an output or input in place (same counts) must change
    the serialisation and therefore the signed message and the txid."""
    from decimal import Decimal

    from upow_amd.models.transaction import Transaction, TransactionInput, TransactionOutput
    from upow_amd.wallet.builders import address_of
    tx = Transaction([TransactionInput('ab' * 32, 0)], [TransactionOutput(address_of(5), Decimal('1'))])
    tx.inputs[0].signed = (7, 8)
    msg1, full1 = tx.hex(False), tx.hex()
    tx.outputs[0] = TransactionOutput(address_of(5), Decimal('2'))
    assert tx.hex(False) != msg1 and tx.hex() != full1
    msg2 = tx.hex(False)
    tx.outputs[0].amount = Decimal('3')
    assert tx.hex(False) != msg2
    msg3 = tx.hex(False)
    tx.inputs[0].index = 1
    assert tx.hex(False) != msg3
    tx.inputs[0].signed = (1, 2)
    assert tx.hex(False) == tx.hex(False) and tx.hex().endswith(
        (1).to_bytes(32, 'little').hex() + (2).to_bytes(32, 'little').hex())
