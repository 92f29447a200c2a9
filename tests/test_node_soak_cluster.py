"""BASELINE config 5 launcher (scripts/node_soak.py --cluster N): the multi-GPU node and the DP miner
started under torchrun as children of the soak script, here with 2 gloo ranks on CPU. Checks every pushed
tx is confirmed, both miner ranks report a hashrate, and every replica agrees (height, tip, K12 index hash
and SQL table hash via /cluster_info?deep=true)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.slow
def test_node_soak_cluster_launcher_gloo_world2(tmp_path):
    out = tmp_path / 'soak.json'
    env = dict(os.environ, UPOW_DISABLE_GPU='1', OMP_NUM_THREADS='1')
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'scripts', 'node_soak.py'), '--cluster', '2', '--rate', '20',
                        '--seconds', '6', '--difficulty', '3', '--fanout1', '4', '--fanout2', '40', '--out', str(out)],
                       cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    rep = json.loads(out.read_text())
    assert rep['pushed'] > 0 and rep['confirmed'] == rep['pushed'] and rep['push_errors'] == 0
    c = rep['cluster']
    assert c['gpus'] == 2 and c['world'] == 2 and c['backend'] == 'gloo' and c['agree'] is True
    assert len(c['replicas']) == 2 and all(x['sql_utxo_hash'] == x['utxo_hash'] for x in c['replicas'])
    assert c['miner_per_rank_mhs_median'] and len(c['miner_per_rank_mhs_median']) == 2
