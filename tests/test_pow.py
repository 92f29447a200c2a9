"""K1 PoW search: host C++ and gfx950 kernel vs the pure-Python reference predicate."""
import hashlib
import random

import pytest

from upow_amd.models.block import PowTarget, check_pow, header_prefix
from upow_amd.ops.pow import PowJob, search
from upow_amd.utils import p256
from upow_amd.utils.codec import AddressFormat, point_to_string


def _job(difficulty='2.5', v1=False, seed=1):
    rng = random.Random(seed)
    prev = hashlib.sha256(rng.randbytes(8)).hexdigest()
    key = p256.get_public_key(rng.randrange(1, p256.N))
    addr = point_to_string(key, AddressFormat.FULL_HEX if v1 else AddressFormat.COMPRESSED)
    pre = header_prefix(prev, addr, hashlib.sha256(rng.randbytes(8)).hexdigest(), 1_700_000_000 + seed, difficulty)
    return prev, PowJob.create(pre, PowTarget.from_difficulty(prev, difficulty))


def _brute(job, n):
    return sorted(job.word_to_nonce(w) for w in range(n) if job.exact_check(job.word_to_nonce(w)))


@pytest.mark.parametrize('difficulty', ['1', '2.5', '2.9', '3.0', '0.5'])
@pytest.mark.parametrize('v1', [False, True])
def test_target_matches_reference_predicate(difficulty, v1):
    prev, job = _job(difficulty, v1)
    for w in range(3000):
        n = job.word_to_nonce(w)
        hdr = job.header_with_nonce(n)
        digest = hashlib.sha256(hdr).hexdigest()
        # literal re-statement of upow/manager.py:142-151
        from decimal import Decimal
        from math import ceil, floor
        d = Decimal(difficulty)
        dec, di = d % 1, floor(d)
        if dec > 0:
            ref = digest.startswith(prev[-di:]) and digest[di] in '0123456789abcdef'[:ceil(16 * (1 - dec))]
        else:
            ref = digest.startswith(prev[-di:])
        assert job.exact_check(n) == ref == check_pow(hdr, prev, difficulty)


@pytest.mark.parametrize('v1', [False, True])
def test_host_search_matches_bruteforce(native, v1):
    _, job = _job('2.5', v1, seed=7)
    r = search(job, 0, 60000, device='cpu', threads=4)
    assert r.searched == 60000
    assert sorted(r.nonces) == _brute(job, 60000)


def test_nonce_word_bijection():
    _, job = _job()
    for n in (0, 1, 0x01020304, 0xffffffff, 0x80000000):
        assert job.word_to_nonce(job.nonce_to_word(n)) == n


@pytest.mark.gpu
@pytest.mark.parametrize('v1', [False, True])
@pytest.mark.parametrize('difficulty', ['2.5', '3.0', '4.3'])
def test_gpu_search_matches_host(gpu, v1, difficulty):
    _, job = _job(difficulty, v1, seed=11)
    n = 1 << 22
    g = search(job, 12345, n, device='gpu', chunk_iters=4)
    h = search(job, 12345, n, device='cpu', threads=8)
    assert g.searched == n and sorted(g.nonces) == sorted(h.nonces)
    assert g.candidates == len(g.nonces)  # H0 filter is exact for difficulty < 8


@pytest.mark.gpu
def test_gpu_search_ragged_and_variant(gpu):
    _, job = _job('2.0', False, seed=3)
    for count in (1, 255, 257, 65536 + 17):
        g = search(job, 99, count, device='gpu')
        h = search(job, 99, count, device='cpu', threads=2)
        assert g.searched == count and sorted(g.nonces) == sorted(h.nonces)
    a = search(job, 0, 1 << 21, device='gpu', variant=0)
    b = search(job, 0, 1 << 21, device='gpu', variant=1)
    c = search(job, 0, 1 << 21, device='gpu', variant=2)  # LDS-staged message schedule
    assert sorted(a.nonces) == sorted(b.nonces) == sorted(c.nonces)


@pytest.mark.gpu
def test_gpu_full_sweep_d63(gpu):
    """One full 2^32 sweep at the bench difficulty: every reported header passes the node check."""
    prev, job = _job('6.3', False, seed=5)
    r = search(job, 0, 1 << 32, device='gpu')
    assert r.searched == 1 << 32
    assert 100 < len(r.nonces) < 320  # expectation 2^32 / 22.37M = 192
    for n in r.nonces[:20]:
        assert check_pow(job.header_with_nonce(n), prev, '6.3')


def test_miner_tip_watcher_stops_stale_jobs():
    """The miner drops a job once the node's tip moves (upow_amd/miner.py TipWatcher)."""
    import time as _t

    from upow_amd.miner import TipWatcher
    tips = ['aa' * 32]
    w = TipWatcher('http://node/', 0.01, fetch=lambda url: {'last_block': {'hash': tips[-1]}})
    try:
        deadline = _t.time() + 5
        while w.tip is None and _t.time() < deadline:
            _t.sleep(0.01)
        assert not w.moved('aa' * 32)
        tips.append('bb' * 32)
        while not w.moved('aa' * 32) and _t.time() < deadline:
            _t.sleep(0.01)
        assert w.moved('aa' * 32) and not w.moved('bb' * 32)
    finally:
        w.close()


def test_miner_job_planner_never_resweeps_a_space():
    """After a job sweeps its whole space without a block, the next job of the same template only sweeps the
    timestamps added since; once the tip is trim_after_s old it drops one more trailing transaction (a fresh
    merkle root and a fresh window), and with nothing left to drop only new timestamps again
    (upow_amd/miner.py JobPlanner)."""
    from upow_amd.miner import JobPlanner
    job = lambda hs: {'last_block': {'hash': 'aa' * 32, 'timestamp': 100}, 'pending_transactions_hashes': list(hs)}
    p = JobPlanner(trim_after_s=8)
    assert p.plan(job('xyz'), 101) == (list('xyz'), 101)
    p.finished(True, 101)
    assert p.plan(job('xyz'), 101) == (list('xyz'), 102)  # young tip: wait for a new timestamp
    p.finished(True, 103)
    assert p.plan(job('xyz'), 104) == (list('xyz'), 104)
    p.finished(False, 104)  # stopped (tip moved / refresh): the same window again
    assert p.plan(job('xyz'), 105) == (list('xyz'), 104)
    p.finished(True, 108)
    assert p.plan(job('xyzw'), 108) == (list('xyzw'), 101)  # a new template: the full window
    p.finished(True, 108)
    assert p.plan(job('xyzw'), 108) == (list('xyz'), 101)  # tip 8 s old: new merkle root, full window
    p.finished(True, 108)
    assert p.plan(job('xyzw'), 109) == (list('xy'), 101)
    p.finished(True, 109)
    assert p.plan(job('xyzw'), 109) == (list('xy'), 110)  # half held back: only timestamps not yet swept
    p.finished(True, 110)
    assert p.plan(job('xyzw'), 111) == (list('xy'), 111)
    one = JobPlanner(trim_after_s=8)  # a one-transaction template is never mined empty
    assert one.plan(job('x'), 120) == (['x'], 101)
    one.finished(True, 120)
    assert one.plan(job('x'), 120) == (['x'], 121)
    # a changed template (or tip) starts over with every transaction
    assert p.plan(job('xyzwv'), 111) == (list('xyzwv'), 101)
    p.finished(True, 111)
    nxt = {'last_block': {'hash': 'bb' * 32, 'timestamp': 111}, 'pending_transactions_hashes': list('xyzw')}
    assert p.plan(nxt, 112) == (list('xyzw'), 112)


def test_cluster_miner_reports_stop_vs_exhausted():
    from upow_amd.parallel.dist import init_from_env
    from upow_amd.parallel.miner_dp import ClusterMiner
    ctx = init_from_env(want_gpu=False)

    class _Miss:  # a search that finds nothing
        nonces = []
    none = lambda job, pos, n, **kw: _Miss()
    m = ClusterMiner(ctx, 'aa' * 32, 'Dn7ufYB2yFEYdkJ1GAqLKnXSB2ytGTB5f4YfBk5eHGx6X', 'cc' * 32, 6, ts_max=101, ts_min=100,
                     chunk=1 << 31, search_fn=none)
    assert m.mine() is None and not m.stopped  # swept both timestamps
    assert m.mine(should_stop=lambda: True) is None and m.stopped
