"""Node/miner configuration (reference: config.py:1 CORE_URL, env UPOW_DATABASE_*).

Everything is overridable by environment variables so tests and devnets never reach mainnet:
``UPOW_CORE_URL`` (bootstrap peer; empty disables), ``UPOW_DATA_DIR`` (ledger, nodes.json,
ip_config.json, emission_details.json), ``UPOW_DATABASE_PATH`` (SQLite file).
"""
import os

CORE_URL = os.environ.get('UPOW_CORE_URL', 'https://api.upow.ai/')
DATA_DIR = os.environ.get('UPOW_DATA_DIR', os.path.join(os.getcwd(), 'upow_data'))


def data_path(*parts: str) -> str:
    d = os.environ.get('UPOW_DATA_DIR', DATA_DIR)
    os.makedirs(d, exist_ok=True)
    return os.path.join(d, *parts)
