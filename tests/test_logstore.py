"""Append-only emission-details store (utils/logstore.py) — reference: the pickledb file rewritten whole
on every per-block ``set`` (upow/database.py:22, manager.py:741-756)."""
import json
import os
import time

from upow_amd.utils.logstore import LogStore


def test_set_cost_is_constant_with_100k_entries(tmp_path):
    path = str(tmp_path / 'emission_details.jsonl')
    st = LogStore(path)
    detail = [{'power': '12.5', 'emission': '50.00', 'wallet': 'D' * 45, 'inode_reward': '1.5'}] * 4

    def batch(start):
        t0 = time.perf_counter()
        for k in range(start, start + 2000):
            st.set(str(k), detail)
        return time.perf_counter() - t0

    first = batch(0)
    for k in range(2000, 98_000):
        st.set(str(k), detail)
    last = batch(98_000)
    assert len(st.keys()) == 100_000
    assert last < 3 * first + 0.05, (first, last)  # no O(n) rewrite per set
    st.set('7', [{'power': '1'}])  # a later line supersedes
    assert st.get('7') == [{'power': '1'}] and st.get('99999') == detail and st.get('nope') is None
    st.close()
    again = LogStore(path)
    assert len(again.keys()) == 100_000 and again.get('7') == [{'power': '1'}]
    again.close()


def test_torn_tail_legacy_migration_and_compaction(tmp_path):
    legacy = tmp_path / 'emission_details.json'
    legacy.write_text(json.dumps({'1': [{'wallet': 'a'}], '2': []}))
    path = str(tmp_path / 'emission_details.jsonl')
    st = LogStore(path, legacy_json=str(legacy))
    assert st.get('1') == [{'wallet': 'a'}] and st.get('2') == []
    assert not legacy.exists() and (tmp_path / 'emission_details.json.migrated').exists()
    st.set('3', ['x'])
    st.close()
    with open(path, 'ab') as f:
        f.write(b'{"k":"4","v":[1')  # crash mid-append
    st = LogStore(path, legacy_json=str(legacy))
    assert sorted(st.keys()) == ['1', '2', '3'] and st.get('4') is None
    for k in range(3000):
        st.set('3', [k])  # many superseded lines -> automatic compaction
    assert st.lines < 2 * len(st.keys()) + 1025
    assert st.get('3') == [2999]
    st.close()
    assert sum(1 for _ in open(path)) <= 1030


def test_file_log_goes_through_listener_thread(tmp_path):
    """Node/miner entry points turn file logging on (reference: logs/app.log always); records are
    written by a listener thread into <data dir>/logs/app.log."""
    import subprocess
    import sys
    code = "from upow_amd.utils.logger import get_logger; get_logger().info('hello from the node')"
    env = dict(os.environ, UPOW_FILE_LOG='1', UPOW_DATA_DIR=str(tmp_path), UPOW_LOG_DIR='')
    subprocess.run([sys.executable, '-c', code], env=env, check=True, cwd=os.path.dirname(os.path.dirname(__file__)))
    assert 'hello from the node' in (tmp_path / 'logs' / 'app.log').read_text()
