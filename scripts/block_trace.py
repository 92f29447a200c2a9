"""One timeline of a block: host stages (roctx ranges, UPOW_ROCTX=1) and GPU kernels (rocprofv3 kernel
trace), from one ``rocprofv3 --kernel-trace --marker-trace --output-format csv`` run.

    python scripts/block_trace.py TRACE_DIR [--out summary.json]

For every block (a ``block:decode`` range starts one) it reports each host stage's wall time and the
kernels that ran inside it (count, busy time), then the per-stage mean over the blocks, so the host share of
the block path and the device share sit on one clock.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def _rows(pattern: str):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f, newline='') as fh:
            out.extend(csv.DictReader(fh))
    return out


def _name(row: dict) -> str:
    for k in ('Message', 'Function', 'Name', 'Marker_Message'):
        v = row.get(k)
        if v and v.startswith(('block:', 'apply:', 'finalize:')):
            return v
    return ''


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('trace_dir')
    ap.add_argument('--out', default=None)
    a = ap.parse_args()
    markers = _rows(os.path.join(a.trace_dir, '**', '*marker_api_trace.csv'))
    kernels = _rows(os.path.join(a.trace_dir, '**', '*kernel_trace.csv'))
    ranges = sorted(((int(r['Start_Timestamp']), int(r['End_Timestamp']), _name(r)) for r in markers if _name(r)))
    ks = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'].split('(')[0]) for r in kernels)
    blocks, cur = [], None
    for t0, t1, name in ranges:
        if name == 'block:decode':
            cur = {'start': t0, 'stages': []}
            blocks.append(cur)
        if cur is not None:
            cur['stages'].append((name, t0, t1))
    per_stage = defaultdict(list)
    per_kernel = defaultdict(list)
    detail = []
    for b in blocks:
        end = max(t1 for _, _, t1 in b['stages'])
        row = {'wall_ms': (end - b['start']) / 1e6, 'stages': {}}
        for name, t0, t1 in b['stages']:
            inside = [(k0, k1, kn) for k0, k1, kn in ks if k0 >= t0 and k1 <= t1]
            busy = sum(k1 - k0 for k0, k1, _ in inside) / 1e6
            row['stages'][name] = {'host_ms': round((t1 - t0) / 1e6, 3), 'kernels': len(inside),
                                   'gpu_busy_ms': round(busy, 3)}
            per_stage[name].append(((t1 - t0) / 1e6, busy, len(inside)))
            if name.startswith('block:'):
                for k0, k1, kn in inside:
                    per_kernel[(name, kn)].append((k1 - k0) / 1e6)
        detail.append(row)
    mean = {name: {'host_ms': round(sum(v[0] for v in vals) / len(vals), 3),
                   'gpu_busy_ms': round(sum(v[1] for v in vals) / len(vals), 3),
                   'kernels': round(sum(v[2] for v in vals) / len(vals), 1)}
            for name, vals in per_stage.items()}
    kern = {f'{st} / {kn}': {'n_per_block': round(len(v) / max(1, len(blocks)), 2),
                             'mean_ms': round(sum(v) / len(v), 4)} for (st, kn), v in per_kernel.items()}
    gpu_total = sum(m['gpu_busy_ms'] for n, m in mean.items() if n.startswith('block:'))
    host_total = sum(m['host_ms'] for n, m in mean.items() if n.startswith('block:'))
    summary = {'blocks': len(blocks), 'block_wall_ms_mean': round(sum(d['wall_ms'] for d in detail) / max(1, len(detail)), 3),
               'stage_mean': mean, 'block_stage_host_ms_sum': round(host_total, 3),
               'block_stage_gpu_busy_ms_sum': round(gpu_total, 3), 'kernels_by_stage': kern, 'per_block': detail,
               'marker_rows': len(markers), 'kernel_rows': len(kernels)}
    text = json.dumps(summary, indent=1)
    if a.out:
        with open(a.out, 'w') as f:
            f.write(text)
    print(json.dumps({k: summary[k] for k in ('blocks', 'block_wall_ms_mean', 'block_stage_host_ms_sum',
                                                 'block_stage_gpu_busy_ms_sum', 'stage_mean')}, indent=1))


if __name__ == '__main__':
    main()
