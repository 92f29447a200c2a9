"""scripts/gov_ab.py (the interleaved plain/governance block A/B): a tiny run on the CPU, so the script that
backs docs/ROUND4.md §8 keeps working; both chains must stay on the native path and report every stage."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_gov_ab_small_run(tmp_path):
    out = tmp_path / 'gov_ab.json'
    env = dict(os.environ, TMPDIR=str(tmp_path), UPOW_DISABLE_GPU='1')
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'scripts', 'gov_ab.py'), '--blocks', '2', '--warmup', '1',
                        '--txs', '200', '--out', str(out)], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads(out.read_text())
    assert d['device'] == 'cpu' and d['blocks_per_side'] == 2
    assert len(d['plain_ms']) == len(d['gov_ms']) == 2
    assert d['gov_stage_ms_median']['rules_s'] > 0 and 'decode_s' in d['plain_stage_ms_median']
    assert 0 < d['plain_over_gov_time'] < 10
