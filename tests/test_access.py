"""Access policy (ip_config.json) semantics (reference upow/node/ip_manager.py:8-56)."""
import json

from upow_amd.node.access import AccessControl, AccessPolicy


def test_default_file_and_reload_after_ttl(tmp_path):
    t = [0.0]
    path = tmp_path / 'ip_config.json'
    ac = AccessControl(str(path), clock=lambda: t[0])
    assert json.loads(path.read_text()) == {'whitelist': [], 'blocklist': [], 'block_endpoints': [],
                                            'cache_duration': 300}
    assert ac.policy().admits('1.2.3.4') and not ac.policy().path_blocked('/push_tx')
    path.write_text(json.dumps({'blocklist': ['1.2.3.4'], 'block_endpoints': ['/push_tx'], 'cache_duration': 10}))
    assert ac.policy().admits('1.2.3.4')          # cached copy still fresh
    t[0] += 301
    p = ac.policy()
    assert not p.admits('1.2.3.4') and p.admits('5.6.7.8') and p.path_blocked('/push_tx')
    path.write_text('{broken')
    t[0] += 11
    assert not ac.policy().admits('1.2.3.4')      # malformed file keeps the previous policy


def test_allowlist_semantics_and_networks():
    p = AccessPolicy.from_json({'whitelist': ['10.0.0.0/8', '192.168.1.5'], 'blocklist': ['10.0.0.1']})
    assert p.admits('10.0.0.1')                   # allow-list wins over the block list
    assert p.admits('192.168.1.5') and not p.admits('192.168.1.6') and not p.admits(None)
    assert p.allowlisted('10.9.9.9') and not p.allowlisted('11.0.0.1')
    q = AccessPolicy.from_json({'blocklist': ['fd00::/8', 'not-an-ip']})
    assert not q.admits('fd00::1') and q.admits('::1') and not q.admits('not-an-ip') and q.admits(None)
