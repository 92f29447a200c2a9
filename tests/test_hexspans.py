"""Bodies parsed with their tx arrays left in place (csrc/jsonspan.cpp, upow_amd/utils/hexspans.py) and the
codec reading txs from them (csrc/txcodec.cpp decode_block_spans / pack_tx_spans).

The parse must equal json.loads on every body it takes (hypothesis over JSON documents with the span keys
at any depth, several layouts), raise like json.loads on bodies it does not, and the span decode must
produce the list decode's columns byte for byte."""
import json
import math
import random

import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings, strategies as st

from upow_amd.utils import hexspans
from upow_amd.utils.hexspans import HexSpans

from test_txcodec import _check_fast, _tx


def _plain(v):
    """A parse result with every HexSpans turned into the list it stands for."""
    if isinstance(v, HexSpans):
        return list(v)
    if isinstance(v, dict):
        return {k: _plain(x) for k, x in v.items()}
    if isinstance(v, list):
        return [_plain(x) for x in v]
    return v


def _same(a, b):
    if isinstance(a, float) and isinstance(b, float):
        return (math.isnan(a) and math.isnan(b)) or (a == b and math.copysign(1, a) == math.copysign(1, b))
    if type(a) is not type(b):
        return False
    if isinstance(a, dict):
        return list(a) == list(b) and all(_same(a[k], b[k]) for k in a)
    if isinstance(a, list):
        return len(a) == len(b) and all(_same(x, y) for x, y in zip(a, b))
    return a == b


_keys = st.one_of(st.sampled_from(['txs', 'transactions', 'block', 'id', 'block_content']), st.text(max_size=6))
_hex = st.text(alphabet='0123456789abcdefABCDEF', max_size=40)
_scalars = st.one_of(st.none(), st.booleans(), st.integers(min_value=-2**80, max_value=2**80),
                     st.floats(allow_nan=False, allow_infinity=False), st.text(max_size=12), _hex)
_json = st.recursive(_scalars, lambda inner: st.one_of(st.lists(inner, max_size=5), st.lists(_hex, max_size=6),
                                                       st.dictionaries(_keys, inner, max_size=5)), max_leaves=30)


@settings(max_examples=300, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(doc=_json, layout=st.sampled_from([None, 0, 2, 'compact']), ascii_only=st.booleans())
def test_parse_equals_json_loads(native, doc, layout, ascii_only):
    kw = {'separators': (',', ':')} if layout == 'compact' else {'indent': layout}
    body = json.dumps(doc, ensure_ascii=ascii_only, **kw).encode()
    ref = json.loads(body)
    got = hexspans.native_loads(body)  # the native parser itself, no fallback
    assert _same(_plain(got), ref)


def test_tx_arrays_become_spans(native):
    txs = ['ab' * 40, 'cd' * 64, 'ef' * 10]
    body = json.dumps({'block_content': 'x', 'txs': txs, 'other': txs, 'block_no': 7}).encode()
    d = hexspans.native_loads(body)
    assert isinstance(d['txs'], HexSpans) and d['txs'] == txs
    assert isinstance(d['other'], list) and d['block_no'] == 7
    page = json.dumps([{'block': {'id': 3, 'difficulty': 6.5}, 'transactions': txs}]).encode()
    rows = hexspans.native_loads(page)
    assert isinstance(rows[0]['transactions'], HexSpans) and rows[0]['transactions'] == txs
    assert rows[0]['block'] == {'id': 3, 'difficulty': 6.5}
    # an array the span form cannot hold stays a list: escapes, non-ASCII, non-strings
    for arr in (['a\\b'], ['é'], ['a', 1], [['a']], ['a"b']):
        d = hexspans.native_loads(json.dumps({'txs': arr}, ensure_ascii=False).encode())
        assert isinstance(d['txs'], list) and d['txs'] == arr


@pytest.mark.parametrize('body', [b'', b'{', b'{"a": NaN}', b'{"a": Infinity}', b'{"a": -Infinity}', b'[1,]',
                                  b'{"a":1} x', b'\xef\xbb\xbf{"a": 1}', b'{"a": "\x01"}', b'{"txs": ["\xff"]}',
                                  b'{"a": 01}', b'{"a": 1.}', b'{"a": .5}', b'{"a" 1}', b'"\\ud800"', b'{"a": tru}',
                                  '{"a": 1}'.encode('utf-16'), b'[' * 300 + b']' * 300])
def test_outside_the_subset_is_json_loads(native, body):
    try:
        ref = ('ok', json.loads(body))
    except Exception as e:  # noqa: BLE001
        ref = ('err', type(e))
    try:
        got = ('ok', _plain(hexspans.loads(body)))
    except Exception as e:  # noqa: BLE001
        got = ('err', type(e))
    assert got[0] == ref[0]
    if got[0] == 'ok':
        assert _same(got[1], ref[1])
    else:
        assert got[1] is ref[1]


def test_hexspans_sequence_behaviour():
    items = ['aa', 'bbbb', 'cc', 'dddddd', '24ee24']
    h = HexSpans.from_list(items)
    assert len(h) == 5 and list(h) == items and h[-1] == items[-1] and h[1:4] == items[1:4]
    assert h[::-2] == items[::-2] and h.take([4, 0]) == ['24ee24', 'aa']
    assert h[:2] + h[3:] == items[:2] + items[3:] and (h[:2] + h[3:]).buf is h.buf
    assert h + ['x'] == items + ['x'] and h.without(2) == items[:2] + items[3:]
    assert list(h.lengths) == [2, 4, 2, 6, 6] and h.tail2() == [b'aa', b'bb', b'cc', b'dd', b'24']
    mixed = h[:2] + ['zz'] + h[2:]  # spans after str items keep their order
    assert mixed == items[:2] + ['zz'] + items[2:]
    assert mixed.take([3, 2, 0]) == [items[2], 'zz', items[0]]
    assert json.dumps({'t': h}, default=hexspans.to_json) == json.dumps({'t': items})
    with pytest.raises(IndexError):
        h[5]


def test_span_decode_matches_list_decode(native):
    rng = random.Random(11)
    txs = [_tx(rng) for _ in range(50)] + [_tx(rng, version=1) for _ in range(3)] + [_tx(rng, msg=b'hi')]
    hexes = [t.hex() for t in txs]
    hexes[3] = hexes[3].upper()  # not canonical: comes back in hex_fix
    body = json.dumps({'txs': hexes, 'block_content': 'ab'}).encode()
    h = hexspans.native_loads(body)['txs']
    ref = native.decode_block_txs(hexes, 4)
    for extra in (0, 5):
        src = h if not extra else h[:-extra] + hexes[-extra:]
        d = native.decode_block_spans(src.buf, np.ascontiguousarray(src.spans).tobytes(), list(src.extra), 4)
        assert [k for k, _ in d['hex_fix']] == [3]
        for k, v in ref.items():
            if k not in ('hex', 'merkle_job'):
                assert d[k] == v, k
        assert d['merkle_job'].result() == ref['merkle_job'].result()
    from upow_amd.ledger import fastpath
    d = fastpath.decode(h, threads=4)
    assert d['hex'] == ref['hex'] and d['hex'][3] != hexes[3]
    _check_fast(d, hexes)
    with pytest.raises(ValueError):
        native.decode_block_spans(h.buf, np.array([[len(h.buf) - 2, 10]], np.int64).tobytes(), [], 1)


def test_pack_spans_matches_pack_list(native):
    rng = random.Random(3)
    hexes = [rng.randbytes(rng.randrange(0, 90)).hex() for _ in range(40)]
    h = HexSpans.from_list(hexes)
    assert native.pack_tx_spans(h.buf, h.spans.tobytes(), ['abcd'], 3) == native.pack_tx_hexes(hexes + ['abcd'], 3)
    from upow_amd.parallel.cluster import pack_groups, unpack_txs
    groups = [h[:10], h[10:25], h[25:]]
    assert unpack_txs(pack_groups(groups)) == hexes
    assert unpack_txs(pack_groups([hexes[:3], h[3:]])) == hexes
