"""Peer registry (upow_amd/node/peers.py) against the reference's peer-table behaviour
(upow/node/nodes_manager.py:24-26, 96-171): recent window, never-heard-from peers, gossip fan-out,
pruning after 90 days of silence, the 100-peer cap, persistence, legacy import and multi-process merge."""
import json
import random

import pytest

from upow_amd.node import peers as P

DAY = 86_400


def _book(tmp_path, seed=''):
    return P.PeerBook(str(tmp_path / 'peers.json'), seed)


def test_policies():
    now = 10_000_000
    rs = [P.Peer('a', 0, now - 10), P.Peer('b', 0, now - 8 * DAY), P.Peer('c', 0, 0), P.Peer('d', 0, now - 1),
          P.Peer('e', 0, now - 91 * DAY)]
    assert [p.url for p in P.recent(rs, now)] == ['d', 'a']
    assert [p.url for p in P.never_heard(rs)] == ['c']
    assert sorted(p.url for p in P.stale(rs, now)) == ['c', 'e']
    many = [P.Peer(f'r{k}', 0, now - k) for k in range(30)] + [P.Peer(f'z{k}', 0, 0) for k in range(30)]
    t = P.gossip_targets(many, now, random.Random(1))
    assert len(t) == 20 and sum(u.startswith('r') for u in t) == 10 and len(set(t)) == 20
    assert P.gossip_targets(rs, now) == ['d', 'a', 'c']


def test_seed_add_seen_persist(tmp_path, monkeypatch):
    b = _book(tmp_path, 'https://seed.example/')
    assert b.urls() == ['https://seed.example'] and b.recent_urls() == ['https://seed.example']
    assert b.add('http://p1/') and not b.add('http://p1')
    assert b.last_seen('http://p1') == 0 and 'http://p1' not in b.recent_urls()
    b.seen('http://p1')
    assert b.recent_urls()[0] in ('http://p1', 'https://seed.example')
    b.seen('http://p2')  # heard from an unknown peer: learned
    b.flush()
    raw = json.loads((tmp_path / 'peers.json').read_text())
    assert {r['url'] for r in raw['peers']} == {'https://seed.example', 'http://p1', 'http://p2'}
    b2 = _book(tmp_path, 'https://other-seed')
    assert set(b2.urls()) == {'https://seed.example', 'http://p1', 'http://p2'}  # the file wins over the seed


def test_prune_after_90_days_and_cap(tmp_path, monkeypatch):
    t = [1_800_000_000]
    monkeypatch.setattr(P, '_now', lambda: t[0])
    b = _book(tmp_path)
    for k in range(95):  # heard from long ago
        b.seen(f'http://old{k}')
    t[0] += 91 * DAY
    for k in range(6):
        b.seen(f'http://fresh{k}')
    assert len(b.urls()) == 101
    assert b.add('http://new')  # > 100 peers: the 95 silent for 91 days go, the new one is accepted
    assert sorted(b.urls()) == sorted([f'http://fresh{k}' for k in range(6)] + ['http://new'])
    # a full table of live peers refuses a new one
    for k in range(100):
        b.seen(f'http://live{k}')
    with pytest.raises(Exception, match='Too many nodes'):
        b.add('http://one-too-many')
    # never-heard-from peers beyond 10 trigger a prune of themselves (silent forever)
    b2 = P.PeerBook(str(tmp_path / 'b2.json'))
    for k in range(11):
        b2.add(f'http://z{k}')
    assert b2.add('http://z11') and b2.urls() == ['http://z11']


def test_legacy_nodes_json_import_and_merge(tmp_path):
    (tmp_path / 'nodes.json').write_text(json.dumps({'nodes': ['http://a/', 'http://b'],
                                                     'last_messages': {'http://a': 123, 'http://c': 456}}))
    b = _book(tmp_path)
    assert set(b.urls()) == {'http://a', 'http://b', 'http://c'} and b.last_seen('http://c') == 456
    b.flush()
    other = _book(tmp_path)  # a second process sharing the file
    other.seen('http://b')
    other.add('http://d')
    other.flush()
    b._stat_at = 0
    assert set(b.urls()) == {'http://a', 'http://b', 'http://c', 'http://d'} and b.last_seen('http://b') > 0


def test_flush_merges_other_process_additions_and_keeps_prunes(tmp_path, monkeypatch):
    """two books on one peers.json (two node processes). A flush re-reads the file under the lock
    and merges before writing, so the other book's additions survive; a peer this book pruned is not
    resurrected by the merge."""
    import json
    from upow_amd.node import peers as pm
    path = str(tmp_path / 'peers.json')
    a, b = pm.PeerBook(path), pm.PeerBook(path)
    a.add('http://a.example:3006')
    a.flush()
    b.add('http://b.example:3006')  # b has not looked at the file since a wrote it
    b.flush()
    a.add('http://c.example:3006')
    a.flush()
    urls = {r['url'] for r in json.load(open(path))['peers']}
    assert {'http://a.example:3006', 'http://b.example:3006', 'http://c.example:3006'} <= urls, urls
    # a prunes a long-silent peer that b still lists: the next merge of b's file must not bring it back
    now = pm._now()
    with a.lock:
        a._peers['http://old.example:3006'] = pm.Peer('http://old.example:3006', 1, now - pm.PRUNE_AFTER - 10)
        a._dirty = True
    a.flush()
    b._stat_at = 0.0
    b.records()  # b picks the old peer up from the file
    with a.lock:
        old = a._peers.pop('http://old.example:3006')
        a._pruned[old.url] = old.last_seen
        a._dirty = True
    b._dirty = True
    b.flush()  # b's table still has it
    a.flush()
    assert 'http://old.example:3006' not in {r['url'] for r in json.load(open(path))['peers']}
