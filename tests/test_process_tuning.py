"""Process-level tuning the node applies at startup (upow_amd/utils/cpus.py): the pre-sized file-descriptor
table (no kernel table growth, and its RCU wait, in the middle of a run) and the stall probe that found it
(csrc/stall_probe.cpp). Each case runs in a child process so the test runner's own limits are untouched."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(code: str, **env):
    r = subprocess.run([sys.executable, '-c', code], cwd=ROOT, capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, PYTHONPATH=ROOT, **env))
    assert r.returncode == 0, r.stderr[-2000:]
    return r.stdout.strip().splitlines()[-1]


def test_presize_fd_table_grows_the_table_once():
    out = _run('import json, os, threading\n'
               'from upow_amd.utils.cpus import presize_fd_table\n'
               'def fdsize():\n'
               '    return int([l for l in open("/proc/self/status") if l.startswith("FDSize:")][0].split()[1])\n'
               'before = fdsize()\n'
               'got = presize_fd_table(4096)\n'
               'fds = [os.open(os.devnull, os.O_RDONLY) for _ in range(1000)]\n'
               'after = fdsize()\n'
               'for fd in fds: os.close(fd)\n'
               'print(json.dumps([before, got, after, max(fds)]))')
    before, got, after, top = json.loads(out)
    assert got >= 4096 and after == got  # a thousand more descriptors fit without another growth
    assert top < 4096


def test_presize_fd_table_can_be_disabled():
    out = _run('from upow_amd.utils.cpus import presize_fd_table\nprint(presize_fd_table(4096))',
               UPOW_FD_PRESIZE='0')
    assert out == '0'


def test_stall_probe_samples_another_process(tmp_path):
    path = tmp_path / 'ext.jsonl'
    out = _run('import subprocess, sys, time\n'
               'from upow_amd.ops.native import lib\n'
               'L = lib()\n'  # loads the extension (and torch) before the child's clock starts
               'child = subprocess.Popen([sys.executable, "-c", "import time; time.sleep(5)"])\n'
               'time.sleep(0.3)\n'
               f'p = L.StallProbe({str(path)!r}, None, child.pid, 10.0, 2000, child.pid)\n'
               'time.sleep(0.2)\n'
               'p.stop(); n = p.samples(); child.kill(); child.wait()\n'
               'print(n, child.pid)')
    n, pid = map(int, out.split())
    lines = [json.loads(x) for x in path.read_text().splitlines()]
    assert n == len(lines) and n >= 20  # every 2 ms while unconditioned (no heartbeat)
    loop = [t for r in lines for t in r['threads'] if t[0] == pid]
    assert loop and all(t[2] == 'S' for t in loop)  # the child's main thread, asleep


def test_stall_probe_heartbeat_gates_sampling(tmp_path):
    path = tmp_path / 'self.jsonl'
    out = _run('import threading, time\n'
               'import numpy as np\n'
               'from upow_amd.ops.native import lib\n'
               'hb = np.array([time.perf_counter()])\n'
               f'p = lib().StallProbe({str(path)!r}, hb, threading.get_native_id(), 20.0, 1000)\n'
               'end = time.perf_counter() + 0.2\n'
               'while time.perf_counter() < end:\n'
               '    hb[0] = time.perf_counter(); time.sleep(0.001)\n'
               'fresh = p.samples()\n'
               'time.sleep(0.15)\n'  # a 150 ms "stall": no heartbeat
               'p.stop()\n'
               'print(fresh, p.samples())')
    fresh, total = map(int, out.split())
    assert fresh == 0 and total >= 20
    lines = [json.loads(x) for x in path.read_text().splitlines()]
    assert len(lines) == total and all(r['late_ms'] > 20.0 for r in lines)


def test_cpu_budget_splits_a_cluster_node_by_role(monkeypatch):
    """utils/cpus.py: ranks sharing one affinity set split it, local rank 0 (a cluster node's leader, the rank
    that materialises SQL and serves HTTP) taking half and the lean followers the rest; UPOW_CPU_ROLE_SPLIT=0
    restores the equal split."""
    import builtins
    from upow_amd.utils import cpus
    monkeypatch.setattr(os, 'sched_getaffinity', lambda pid: set(range(64)))
    monkeypatch.setattr(os, 'cpu_count', lambda: 64)
    real_open = builtins.open
    monkeypatch.setattr(builtins, 'open', lambda p, *a, **k: (_ for _ in ()).throw(OSError())
                        if p == '/sys/fs/cgroup/cpu.max' else real_open(p, *a, **k))
    monkeypatch.setenv('LOCAL_WORLD_SIZE', '8')
    got = []
    for r in range(8):
        monkeypatch.setenv('LOCAL_RANK', str(r))
        got.append(cpus.cpu_budget())
    assert got == [32] + [4] * 7
    monkeypatch.setenv('UPOW_CPU_ROLE_SPLIT', '0')
    assert cpus.cpu_budget() == 8
    monkeypatch.setenv('LOCAL_WORLD_SIZE', '1')
    assert cpus.cpu_budget() == 64
