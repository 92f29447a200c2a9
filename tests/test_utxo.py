"""UTXO index: the host C++ table (csrc/utxo_host.cpp), the Python dict and the HBM hash-table kernels (probe /
insert / erase / grow) against one another."""
import random

import numpy as np
import pytest

from upow_amd.ledger.utxo import MISSING, UtxoIndex, make_payload, pack_records


def _keys(n, seed):
    rng = random.Random(seed)
    return [(rng.randbytes(32).hex(), rng.randrange(0, 256)) for _ in range(n)]


def _exercise(backend):
    idx = UtxoIndex(backend=backend)
    keys = _keys(5000, 1)
    tags = [k % 7 for k in range(5000)]
    idx.reset(keys[:1000], tags[:1000])
    idx.insert(keys[1000:3000], 0)
    idx.insert(keys[3000:], tags[3000:])
    got = idx.probe(keys)
    want = np.array(tags[:1000] + [0] * 2000 + tags[3000:], dtype=np.uint8)
    assert (got == want).all()
    assert (idx.probe(_keys(100, 2)) == MISSING).all()
    # erase with tag filter + duplicate keys in one batch: each outpoint erased once
    er = idx.erase(keys[:10] + keys[:10], tag=None)
    assert ((er[:10] + er[10:]) == 1).all()  # exactly one copy wins (on the GPU either lane may)
    assert (idx.probe(keys[:10]) == MISSING).all()
    # tag-filtered erase leaves other tables alone
    k7 = [k for k, t in zip(keys[3000:3100], tags[3000:3100]) if t == 3]
    kn = [k for k, t in zip(keys[3000:3100], tags[3000:3100]) if t != 3]
    assert idx.erase(k7 + kn, tag=3)[:len(k7)].all()
    assert (idx.probe(kn) != MISSING).all()
    # filter() keeps first-seen order and uniqueness
    f = idx.filter([keys[2000], keys[2000], keys[1500], keys[0]], 0)
    assert f == [keys[2000], keys[1500]]
    # re-insert after tombstones
    idx.insert(keys[:10], 5)
    assert (idx.probe(keys[:10]) == 5).all()
    # payloads: (amount, address bytes) come back with the tag; absent -> len 0
    rng = random.Random(4)
    pk = _keys(300, 3)
    amounts = [rng.randrange(1 << 63) for _ in pk]
    addrs = [bytes([42]) + rng.randbytes(32) if k % 3 else rng.randbytes(64) for k in range(300)]
    idx.insert(pk, 0, make_payload(amounts, addrs))
    tags, pay = idx.lookup(pk + _keys(5, 77))
    assert (tags[:300] == 0).all() and (tags[300:] == MISSING).all()
    assert [int(a) for a in pay['amount'][:300]] == amounts and (pay['len'][300:] == 0).all()
    assert all(bytes(pay['addr'][k][:pay['len'][k]]) == addrs[k] for k in range(300))
    t2, p2 = idx.lookup_records(pack_records(pk[:50]))
    assert (t2 == 0).all() and [int(a) for a in p2['amount']] == amounts[:50]
    recs, allpay = idx.records_payload()
    assert len(recs) == len(idx) and len(allpay) == len(idx)
    return idx


HOSTS = ['host', 'host-py']


@pytest.mark.parametrize('backend', HOSTS)
def test_host_backend(backend):
    idx = _exercise(backend)
    assert len(idx) == 5000 + 300 - len([1 for t in range(3000, 3100) if t % 7 == 3])


@pytest.mark.gpu
def test_gpu_backend_matches_host(gpu):
    _exercise('gpu')
    # growth past 50% load triggers a rehash on device
    idx = UtxoIndex(backend='gpu')
    keys = _keys(1 << 19 | 12345, 9)
    amounts = list(range(len(keys)))
    idx.insert(keys, 1, make_payload(amounts, [bytes([43]) + bytes(32)] * len(keys)))
    assert len(idx) == len(keys)
    assert (idx.probe(keys[::97]) == 1).all()
    t, p = idx.lookup(keys[::97])  # payloads survive the device rehash
    assert (t == 1).all() and [int(a) for a in p['amount']] == amounts[::97]


def _block_inputs_case(idx, seed):
    rng = random.Random(seed)
    keys = _keys(4000, seed)
    amounts = [rng.randrange(1, 1 << 40) for _ in keys]
    addrs = [bytes([42]) + rng.randbytes(32) for _ in keys]
    idx.insert(keys[:3000], 0, make_payload(amounts[:3000], addrs[:3000]))
    idx.insert(keys[3000:3500], 3, make_payload(amounts[3000:3500], addrs[3000:3500]))
    # a block: 700 txs of 1-3 inputs drawn from live, wrong-table and unknown outpoints, plus duplicates
    spend = keys[:1500] + keys[3000:3010] + keys[3600:3610] + keys[5:9]
    rng.shuffle(spend)
    in_start = [0]
    while in_start[-1] < len(spend):
        in_start.append(min(len(spend), in_start[-1] + rng.randint(1, 3)))
    n_tx = len(in_start) - 1
    out_start = [0]
    for _ in range(n_tx):
        out_start.append(out_start[-1] + rng.randint(1, 2))
    out_amount = np.array([rng.randrange(1, 1 << 38) for _ in range(out_start[-1])], dtype=np.uint64)
    return pack_records(spend), np.array(in_start, np.int32), out_amount, np.array(out_start, np.int32)


@pytest.mark.parametrize('backend', HOSTS)
def test_block_inputs_host(backend):
    idx = UtxoIndex(backend=backend)
    recs, ins, outs, ost = _block_inputs_case(idx, 11)
    tags, pay, dup_of, fee, missing, n_dup = idx.block_inputs(recs, ins, outs, ost, 0)
    assert n_dup == 4 and int((dup_of > 0).sum()) == 4
    assert int(missing.sum()) == 20 + 4 * 0  # 10 wrong-table + 10 unknown (duplicates of live keys are found)
    amt = pay['amount'].astype(np.int64)
    for t in range(len(ins) - 1):
        assert fee[t] == amt[ins[t]:ins[t + 1]].sum() - outs[ost[t]:ost[t + 1]].astype(np.int64).sum()


@pytest.mark.gpu
def test_block_inputs_and_set_hash_gpu_match_host(gpu):
    h, g = UtxoIndex(backend='host'), UtxoIndex(backend='gpu')
    ch = _block_inputs_case(h, 13)
    cg = _block_inputs_case(g, 13)
    rh, rg = h.block_inputs(*ch, 0), g.block_inputs(*cg, 0)
    for k in (0, 1, 3, 4):  # tags, payloads, fees, missing: identical
        assert np.array_equal(np.asarray(rh[k]).view(np.uint8), np.asarray(rg[k]).view(np.uint8)), k
    # duplicates: which copy is flagged depends on lane order on the GPU; the count does not
    assert rh[5] == rg[5] == int((rg[2] > 0).sum()) == 4
    for tag in (0, 3, 5):
        assert h.set_hash(tag) == g.set_hash(tag)


@pytest.mark.parametrize('backend', [*HOSTS, pytest.param('gpu', marks=pytest.mark.gpu)])
def test_block_inputs_without_inputs(backend, request):
    """Txs with no inputs at all (n_in = 0, the arenas' input regions empty): fees are minus the outputs."""
    if backend == 'gpu':
        request.getfixturevalue('gpu')
    idx = UtxoIndex(backend=backend)
    idx.insert(_keys(10, 3), 0, make_payload([5] * 10, [bytes([42]) + bytes(32)] * 10))
    ins = np.zeros(4, np.int32)
    ost = np.array([0, 1, 3, 3], np.int32)
    outs = np.array([7, 11, 13], np.uint64)
    tags, pay, dup_of, fee, missing, n_dup = idx.block_inputs(np.zeros((0, 40), np.uint8), ins, outs, ost, 0)
    assert len(tags) == len(pay) == len(dup_of) == 0 and n_dup == 0
    assert list(fee) == [-7, -24, 0] and list(missing) == [0, 0, 0]


def _address_case(idx, seed):
    """3000 outputs over 40 owners (33-byte and 64-byte addresses) in three tables, some spent."""
    rng = random.Random(seed)
    owners = [bytes([42 + (k & 1)]) + rng.randbytes(32) if k % 4 else rng.randbytes(64) for k in range(40)]
    keys = _keys(3000, seed)
    own = [rng.randrange(40) for _ in keys]
    amounts = [rng.randrange(1, 1 << 44) for _ in keys]
    tags = [rng.choice((0, 0, 0, 3, 5)) for _ in keys]
    for t in (0, 3, 5):
        sel = [k for k in range(3000) if tags[k] == t]
        idx.insert([keys[k] for k in sel], t, make_payload([amounts[k] for k in sel], [owners[own[k]] for k in sel]))
    idx.erase(keys[:300])
    live = set(range(300, 3000))

    def want(o, tagset):
        ks = sorted((keys[k][0], keys[k][1]) for k in live if own[k] == o and tags[k] in tagset)
        amt = {keys[k]: amounts[k] for k in live}
        return ks, sum(amt[k] for k in ks)
    return owners, want


def _check_address_outputs(idx, owners, want):
    for o in (0, 1, 2, 3, 17):
        for tagset in ((0,), (0, 3, 5), (5,)):
            recs, pay, total = idx.address_outputs(owners[o], tagset)
            ks, amt = want(o, tagset)
            got = [(bytes(r[:32]).hex(), int(r[32:36].copy().view(np.uint32)[0])) for r in recs]
            assert got == ks and total == amt
            assert all(bytes(p['addr'][:p['len']]) == owners[o] for p in pay)
    # a 33-byte query never matches a 64-byte address that starts with the same bytes, and vice versa
    assert len(idx.address_outputs(owners[0][:33], (0, 3, 5))[0]) == 0
    assert idx.address_outputs(b'\x42' + bytes(32))[2] == 0


@pytest.mark.parametrize('backend', HOSTS)
def test_address_outputs_host(backend):
    idx = UtxoIndex(backend=backend)
    _check_address_outputs(idx, *_address_case(idx, 21))


@pytest.mark.gpu
def test_address_outputs_gpu_scan(gpu):
    """K14 utxo_address_scan kernel vs a plain host filter; the device amount sum matches too, and a
    result larger than the first-pass output buffer (4096) takes the resize pass."""
    idx = UtxoIndex(backend='gpu')
    owners, want = _address_case(idx, 21)
    _check_address_outputs(idx, owners, want)
    many = _keys(5000, 99)
    a = bytes([43]) + bytes(range(32))
    idx.insert(many, 0, make_payload([7] * len(many), [a] * len(many)))
    raw, pay, total = gpu.utxo_address_scan(idx.be.h, a, 1)
    assert len(raw) == 40 * 5000 and total == 7 * 5000
    recs, _, tot = idx.address_outputs(a)
    assert len(recs) == 5000 and tot == 35000


@pytest.mark.parametrize('backend', HOSTS + [pytest.param('gpu', marks=pytest.mark.gpu)])
def test_duplicate_insert_is_skipped(backend, request):
    """Inserting an outpoint that is already live leaves the entry (tag, payload) as it was and is
    counted, on both index backends (csrc/utxo_table.hip utxo_insert_kernel walks the probe chain)."""
    if backend == 'gpu':
        request.getfixturevalue('gpu')
    idx = UtxoIndex(backend=backend)
    keys = _keys(300, 5)
    addr = bytes([42]) + bytes(range(32))
    idx.insert(keys, 0, make_payload([5] * 300, [addr] * 300))
    before = idx.records_payload()
    idx.insert(keys[:10] + _keys(3, 77), 3, make_payload([9] * 13, [addr] * 13))
    assert idx.duplicates == 10 and len(idx) == 303
    recs, pay = idx.records_payload()
    tags, p = idx.lookup(keys[:10])
    assert (tags == 0).all() and (p['amount'] == 5).all()


@pytest.mark.gpu
def test_scan_fingerprint_after_rehash_and_tombstone_reuse(gpu):
    """The owner fingerprint lives in the key slot: it must be rewritten when the table grows (dump +
    re-insert) and when an insert reuses a tombstoned slot; stake flags follow the payload."""
    from upow_amd.ledger.utxo import STAKE_EXCLUDE, STAKE_ONLY, _GpuBackend
    g = UtxoIndex(backend='gpu')
    g.be = _GpuBackend(log2_cap=8)  # 128 entries before the first rehash
    h = UtxoIndex(backend='host')
    owners = [bytes([42 + (o & 1)]) + bytes([o] * 32) for o in range(4)]
    rng = np.random.default_rng(3)
    for round_ in range(6):
        keys = _keys(200, 1000 + round_)
        own = rng.integers(0, 4, len(keys))
        stake = (rng.random(len(keys)) < 0.3).tolist()
        pay = make_payload([int(a) for a in rng.integers(1, 10**6, len(keys))], [owners[o] for o in own], stake)
        for idx in (g, h):
            idx.insert(keys, 0, pay)
        gone = keys[::3]
        for idx in (g, h):
            idx.erase(gone)
            idx.insert(gone[:20], 0, make_payload([11] * 20, [owners[1]] * 20))  # lands in tombstones
    assert g.be.log2 > 8
    for o in owners:
        for sel in (0, STAKE_EXCLUDE, STAKE_ONLY):
            rg, pg, tg = g.address_outputs(o, (0,), sel)
            rh, ph, th = h.address_outputs(o, (0,), sel)
            assert rg.tobytes() == rh.tobytes() and pg.tobytes() == ph.tobytes() and tg == th


def _apply_blocks(backend):
    """Chained blocks through UtxoIndex.apply_block (the block path's post-commit update; on the GPU an
    async insert + erase queued on the node stream): spends of earlier blocks' outputs, a spend of an output
    created in the same block, lookups between blocks, a duplicate insert, then a rehash while an apply
    is pending."""
    rng = random.Random(21)
    idx = UtxoIndex(backend=backend)
    live = []
    for b in range(12):
        new = _keys(900, 100 + b)
        pay = make_payload([rng.randrange(1, 1 << 40) for _ in new], [bytes([42]) + rng.randbytes(32) for _ in new])
        spend = [live.pop(rng.randrange(len(live))) for _ in range(min(len(live), 600))] + new[:3]
        idx.apply_block([(pack_records(new[:700], 0), pay[:700]), (pack_records(new[700:], 0), pay[700:])],
                        pack_records(spend, 0))
        live += new[3:]
        # the next block's lookup sees this block's writes
        t, p = idx.lookup(live[-50:] + spend[:20])
        assert (t[:50] == 0).all() and (t[50:] == MISSING).all()
    before = idx.duplicates
    idx.apply_block([(pack_records(live[:5], 0), None)], np.zeros((0, 40), np.uint8))  # already live
    assert len(idx) == len(live)
    assert idx.duplicates == before + 5
    # a rehash (growth) right after an apply that is still pending
    big = _keys(700000, 999)
    idx.apply_block([(pack_records(big, 1), None)], pack_records(live[:100], 0))
    idx.insert(_keys(10, 1000), 2)
    assert len(idx) == len(live) - 100 + len(big) + 10
    assert (idx.probe(live[100:200]) == 0).all() and (idx.probe(live[:100]) == MISSING).all()
    assert (idx.probe(big[::1000]) == 1).all()
    return idx


@pytest.mark.parametrize('backend', HOSTS)
def test_apply_block_host(backend):
    _apply_blocks(backend)


def test_host_tables_agree_under_random_operations():
    """The C++ host table against the dict over random batches of inserts (with payloads, stake flags and
    re-inserts of live outpoints), tag-filtered erases, lookups and K14 scans; both key on the index byte."""
    from upow_amd.ledger.utxo import STAKE_EXCLUDE, STAKE_ONLY, _HostBackend, _NativeHostBackend
    n, d = UtxoIndex(backend='host'), UtxoIndex(backend='host-py')
    assert isinstance(n.be, _NativeHostBackend) and isinstance(d.be, _HostBackend)
    rng = random.Random(77)
    owners = [bytes([42]) + rng.randbytes(32) for _ in range(6)] + [rng.randbytes(64) for _ in range(2)]
    pool = _keys(3000, 78)
    for step in range(40):
        op = rng.random()
        ks = rng.sample(pool, rng.randint(1, 200))
        if op < 0.45:
            tag = rng.choice((0, 0, 1, 3, 6))
            pay = make_payload([rng.randrange(1, 1 << 50) for _ in ks], [rng.choice(owners) for _ in ks],
                               [rng.random() < 0.3 for _ in ks])
            for i in (n, d):
                i.insert(ks, tag, pay)
        elif op < 0.75:
            tag = rng.choice((None, 0, 3))
            assert (n.erase(ks, tag) == d.erase(ks, tag)).all()
        else:
            tn, pn = n.lookup(ks)
            td, pd = d.lookup(ks)
            assert (tn == td).all() and pn.tobytes() == pd.tobytes()
        assert len(n) == len(d) and n.duplicates == d.duplicates
    for o in owners:
        for sel in (0, STAKE_EXCLUDE, STAKE_ONLY):
            rn, pn, tn = n.address_outputs(o, (0, 1, 3), sel)
            rd, pd, td = d.address_outputs(o, (0, 1, 3), sel)
            assert rn.tobytes() == rd.tobytes() and pn.tobytes() == pd.tobytes() and tn == td
    rn, pn = n.records_payload()
    rd, pd = d.records_payload()
    assert rn.tobytes() == rd.tobytes() and pn.tobytes() == pd.tobytes()
    for tag in (0, 1, 3, 6):
        assert n.set_hash(tag) == d.set_hash(tag)
    # index bytes: the tables key on (txid, index & 0xff), as the HBM table does
    h = pool[0][0]
    n.erase([(h, i) for i in range(256)])
    n.insert([(h, 7)], 0)
    assert n.probe([(h, 7 + 256)])[0] == 0


@pytest.mark.gpu
def test_apply_block_gpu_async_matches_host(gpu):
    g, h = _apply_blocks('gpu'), _apply_blocks('host')
    rg, pg = g.records_payload()
    rh, ph = h.records_payload()
    og = np.lexsort(rg.T[::-1])
    oh = np.lexsort(rh.T[::-1])
    assert (rg[og] == rh[oh]).all() and (pg[og].view(np.uint8) == ph[oh].view(np.uint8)).all()
