"""``python -m upow_amd.node [--host H] [--port P] [--data DIR] [--db PATH]`` (reference: run_node.py,
upow/node/run.py — uvicorn on port 3006)."""
import argparse
import os


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument('--host', default='0.0.0.0')
    ap.add_argument('--port', type=int, default=3006)
    ap.add_argument('--data', default=None, help='data directory (ledger, nodes.json, ip_config.json)')
    ap.add_argument('--db', default=None, help='SQLite ledger path')
    ap.add_argument('--core-url', default=None, help='bootstrap peer (empty string disables)')
    ap.add_argument('--log-level', default='info')
    a = ap.parse_args(argv)
    if a.data:
        os.environ['UPOW_DATA_DIR'] = a.data
    if a.db:
        os.environ['UPOW_DATABASE_PATH'] = a.db
    if a.core_url is not None:
        os.environ['UPOW_CORE_URL'] = a.core_url
    import uvicorn
    uvicorn.run('upow_amd.node.main:app', host=a.host, port=a.port, log_level=a.log_level)


if __name__ == '__main__':
    main()
