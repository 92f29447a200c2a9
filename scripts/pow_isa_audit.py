#!/usr/bin/env python3
"""Instruction audit of the PoW search loop (csrc/pow_search.hip, K1; reference hot loop miner.py:83-98).

Compiles the kernel TU for gfx950 to assembly (the build's flags, device side only), cuts out the loop body
of each ``pow_search_kernel`` instantiation (from the loop-header label to the hit branch) and classifies its
instructions: rotates (v_alignbit), 3-input logic (v_bitop3: XOR3 of the Sigma functions, Maj, Ch), 3-input
and 2-input adds, shifts (the schedule's >>3 / >>10), compares, and scalar instructions. Then compares the
count with a hand-derived floor of the same formulation (one nonce per lane, rounds 10..63 of the tail block,
schedule words W16..W63 with every nonce-independent term folded):

    per compression round   S1: 3 rotates + XOR3    S0: 3 rotates + XOR3    Ch + Maj: 2 bitop3
                            t1 = add3(h, S1, Ch) + add3(t1, K+W)   e = d + t1   a = add3(t1, S0, Maj)
    per schedule word        s0, s1: 2 rotates + shift + XOR3 each; W = add3 + add

Usage: python scripts/pow_isa_audit.py [--out profiles/r6/pow_isa_r6.txt]
"""
import argparse
import collections
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLASSES = [('rotate (v_alignbit_b32)', r'^v_alignbit_b32'), ('bitop3 (XOR3 / Maj / Ch)', r'^v_bitop3_b32'),
           ('add3 (v_add3_u32)', r'^v_add3_u32'), ('add (v_add_u32)', r'^v_add_u32|^v_add_co_u32|^v_add_nc_u32'),
           ('shift (v_lshrrev_b32)', r'^v_lshrrev_b32|^v_lshlrev_b32'), ('bfi / cndmask', r'^v_bfi_b32|^v_cndmask'),
           ('compare', r'^v_cmp'), ('other VALU', r'^v_'), ('LDS', r'^ds_'), ('memory', r'^(global|buffer|flat)_'),
           ('SALU / branch', r'^s_')]


def compile_asm() -> str:
    out = os.path.join(tempfile.mkdtemp(prefix='pow_isa_'), 'pow.s')
    subprocess.run(['/opt/rocm/bin/hipcc', '--offload-arch=gfx950', '-O3', '-std=c++17', f'-I{ROOT}/csrc',
                    '--cuda-device-only', '-S', os.path.join(ROOT, 'csrc', 'pow_search.hip'), '-o', out], check=True,
                   stderr=subprocess.DEVNULL)
    return open(out).read()


def loop_bodies(asm: str) -> dict:
    """{kernel symbol: (loop-body instruction mnemonics, NumVgprs, Occupancy)} for every search kernel."""
    out = {}
    for m in re.finditer(r'^(_ZN4upow\w*pow_search\w*):', asm, re.M):
        name = m.group(1)
        end = asm.find('.Lfunc_end', m.end())
        body = asm[m.end():end]
        tail = asm[end:asm.find('.end_amdhsa_kernel', end) if '.end_amdhsa_kernel' in asm[end:] else end + 4000]
        stats = asm[end:end + 6000]
        vg = re.search(r'; NumVgprs: (\d+)', stats)
        occ = re.search(r'; Occupancy: (\d+)', stats)
        hdr = re.search(r'^(\.LBB\w+):\s*; =>This Inner Loop Header', body, re.M)
        if not hdr:
            continue
        loop = body[hdr.end():]
        stop = re.search(r's_cbranch_execz', loop)  # the hit test: everything before it runs once per nonce
        loop = loop[:stop.start()] if stop else loop
        ins = [ln.split()[0] for ln in loop.splitlines() if re.match(r'^\s+[a-z]', ln) and not ln.strip().startswith(';')]
        out[name] = (ins, int(vg.group(1)) if vg else None, int(occ.group(1)) if occ else None)
        del tail
    return out


def classify(ins):
    c = collections.OrderedDict((k, 0) for k, _ in CLASSES)
    for i in ins:
        for k, pat in CLASSES:
            if re.match(pat, i):
                c[k] += 1
                break
    return c


def floor_v2() -> dict:
    """The hand-derived VALU floor of the v2 search (see the module docstring)."""
    rounds = (63 - 11 + 1) * 14 - 1 + 2  # rounds 11..63 at 14 ops (e of round 63 unused), round 10: two adds
    # schedule: W16, W18, W20, W22 fold to constants; W17 and W24 are const + one nonce-dependent term
    sched = {17: 1, 19: 5, 21: 5, 23: 5, 24: 1, 25: 10, 26: 6, 27: 5, 28: 5, 29: 5, 30: 5, 31: 5}
    sched.update({i: 10 for i in range(32, 64)})
    return {'rounds': rounds, 'schedule': sum(sched.values()), 'total': rounds + sum(sched.values())}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--out', default=None)
    a = ap.parse_args()
    asm = compile_asm()
    lines = ['# PoW search loop: instructions per nonce (one loop iteration = one nonce per lane)',
             f'# source csrc/pow_search.hip, hipcc --offload-arch=gfx950 -O3 (scripts/pow_isa_audit.py)', '']
    for name, (ins, vgpr, occ) in loop_bodies(asm).items():
        c = classify(ins)
        valu = sum(v for k, v in c.items() if k not in ('LDS', 'memory', 'SALU / branch'))
        lines.append(f'{name}  (VGPRs {vgpr}, occupancy {occ} waves/SIMD)')
        for k, v in c.items():
            if v:
                lines.append(f'    {k:28s} {v:5d}')
        lines.append(f'    {"VALU per nonce":28s} {valu:5d}')
        lines.append('')
    f = floor_v2()
    lines.append(f'hand-derived floor of the v2 formulation: {f["total"]} VALU per nonce '
                 f'({f["rounds"]} round ops + {f["schedule"]} schedule ops)')
    text = '\n'.join(lines) + '\n'
    if a.out:
        os.makedirs(os.path.dirname(a.out), exist_ok=True)
        with open(a.out, 'w') as fh:
            fh.write(text)
    sys.stdout.write(text)


if __name__ == '__main__':
    main()
