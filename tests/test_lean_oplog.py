"""The lean follower's op log (upow_amd/ledger/lean.py ``OpLog``): what a restart replays, and what it drops.

A follower logs every tip-moving op as it arrived, then the tip it reached. Replay (``ops``) yields the ops that
moved the tip and the op still being applied (no marker yet), skips an op whose marker repeats the previous tip
(a rejected block), and a torn or corrupted tail is cut off when the log is opened."""
import os

from upow_amd.ledger import lean


def _frame(i: int, size: int = 100) -> bytes:
    return bytes([i % 256]) * size


def test_replay_skips_rejected_ops_and_yields_the_unmarked_one(tmp_path):
    log = lean.OpLog(str(tmp_path / 'l.oplog'))
    log.op(_frame(1))
    log.tip(1, 'aa' * 32)
    log.op(_frame(2))
    log.tip(1, 'aa' * 32)          # rejected: the tip did not move
    log.op(_frame(3, 10_000))      # larger than the CRC edges
    log.tip(2, 'bb' * 32)
    log.op(_frame(4))              # being applied when the follower stopped: no marker
    assert [o[:1] for o in log.ops(0)] == [b'\x01', b'\x03', b'\x04']
    assert log.last_tip() == (2, 'bb' * 32)
    log.close()
    again = lean.OpLog(str(tmp_path / 'l.oplog'))  # reopened: the same records
    assert len(again) == 7 and [len(o) for o in again.ops(0)] == [100, 10_000, 100]
    again.close()


def test_a_torn_or_corrupted_tail_is_dropped_on_open(tmp_path):
    p = str(tmp_path / 'l.oplog')
    log = lean.OpLog(p)
    log.op(_frame(1, 20_000))
    log.tip(1, 'aa' * 32)
    good = log.size
    log.op(_frame(2, 20_000))
    log.close()
    full = os.path.getsize(p)
    with open(p, 'r+b') as f:      # the last record's tail never reached the disk
        f.truncate(full - 500)
    log = lean.OpLog(p)
    assert len(log) == 2 and log.size == good == os.path.getsize(p)
    log.op(_frame(2, 20_000))
    log.close()
    with open(p, 'r+b') as f:      # a zero-filled block inside the last record's final 4 KB
        f.seek(os.path.getsize(p) - 1000)
        f.write(bytes(100))
    log = lean.OpLog(p)
    assert len(log) == 2 and log.last_tip() == (1, 'aa' * 32)
    log.clear()
    assert len(log) == 0 and os.path.getsize(p) == 0 and list(log.ops(0)) == []
    log.close()
