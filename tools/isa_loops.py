"""Instruction census of a kernel's loops from the gfx950 assembly (the sweep consumer's tile loop).

usage: python tools/isa_loops.py [--kernel REGEX] [--min-stores N] [file.hip]

Compiles the file (default admm_kernels.hip) for gfx950 to assembly (device only, the library's flags),
takes each kernel whose mangled name matches REGEX (default: the C3 persistent sweep,
k_sweep_rows<8, 1, true, 32, 1>), finds its loops (a label followed later by a branch back to it)
that hold at least N vector stores (default 15: the consumer's per-tile plane stores), at least M
loads (default 10: its operand loads) and no MFMA, and prints each such loop's instruction count (the
largest is the whole tile loop; others are back edges inside it) with a histogram of the instruction
classes that matter for
the consumer's issue budget: VALU, transcendental, SGPR-spill lane moves (v_readlane / v_writelane),
s_nop, 64-bit moves, memory and LDS operations (tools/res.sh gives the registers and spills).
"""
import argparse
import collections
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, 'admm-lstm_amd', 'admm_amd', 'csrc')

CLASSES = [
    ('v_readlane/v_writelane (SGPR spill moves)', re.compile(r'^v_(readlane|writelane)_b32')),
    ('s_nop', re.compile(r'^s_nop')),
    ('v_mov_b64 / v_pk_mov', re.compile(r'^v_(mov_b64|pk_mov_b32)')),
    ('transcendental (exp/rcp/log/sqrt)', re.compile(r'^v_(exp|rcp|rsq|log|sqrt)_')),
    ('packed f32 (v_pk_*_f32)', re.compile(r'^v_pk_(fma|mul|add)_f32')),
    ('VALU (all v_ except memory)', re.compile(r'^v_')),
    ('buffer/global loads', re.compile(r'^(buffer|global)_load')),
    ('buffer/global stores', re.compile(r'^(buffer|global)_store')),
    ('LDS (ds_)', re.compile(r'^ds_')),
    ('scratch (VGPR spill loads/stores)', re.compile(r'^(scratch|buffer)_(load|store).*(scratch|off, s\[0:3\])|^scratch_')),
    ('MFMA', re.compile(r'^v_mfma')),
    ('SALU (s_ except waits/branches)', re.compile(r'^s_(?!waitcnt|cbranch|branch|barrier|nop)')),
    ('s_waitcnt', re.compile(r'^s_waitcnt')),
    ('s_barrier', re.compile(r'^s_barrier')),
]


def compile_asm(src):
    out = tempfile.mktemp(suffix='.s')
    cmd = ['/opt/rocm/bin/hipcc', '-O3', '-std=c++17', '--offload-arch=gfx950', '--cuda-device-only', '-S',
           '-I' + os.path.join(ROOT, 'include'), src, '-o', out]
    subprocess.run(cmd, check=True, cwd=CSRC)
    return open(out).read().splitlines()


def functions(lines):
    cur, body = None, []
    for ln in lines:
        m = re.match(r'^(\S+):\s*(;.*)?$', ln)
        if m and not m.group(1).startswith('.'):
            if cur:
                yield cur, body
            cur, body = m.group(1), []
            continue
        if cur:
            body.append(ln)
            if ln.strip().startswith('.Lfunc_end'):
                yield cur, body
                cur, body = None, []


def insts(body):
    """(index, label or None, mnemonic or None, text) per line."""
    for i, ln in enumerate(body):
        s = ln.strip()
        m = re.match(r'^(\.LBB\w+):', s)
        if m:
            yield i, m.group(1), None, s
            continue
        if not s or s.startswith(('.', ';', '//')):
            continue
        yield i, None, s.split()[0], s


def loops(body):
    seq = list(insts(body))
    pos = {lab: k for k, (_, lab, _, _) in enumerate(seq) if lab}
    for k, (_, _, mn, s) in enumerate(seq):
        if mn and mn.startswith('s_cbranch') or mn == 's_branch':
            tgt = s.split()[-1]
            if tgt in pos and pos[tgt] < k:
                yield [x for x in seq[pos[tgt]:k + 1] if x[2]]


def census(loop):
    h = collections.OrderedDict((name, 0) for name, _ in CLASSES)
    for _, _, mn, _ in loop:
        for name, rx in CLASSES:
            if rx.match(mn):
                h[name] += 1
    return h


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--kernel', default=r'k_sweep_rowsILi8ELi1ELb1ELi32ELi1E')
    ap.add_argument('--min-stores', type=int, default=15)
    ap.add_argument('--min-loads', type=int, default=10)
    ap.add_argument('--ops', type=int, default=0, help='also print the N most frequent mnemonics of the largest loop')
    ap.add_argument('--asm', help='read this assembly file instead of compiling')
    ap.add_argument('src', nargs='?', default='admm_kernels.hip')
    a = ap.parse_args()
    lines = open(a.asm).read().splitlines() if a.asm else compile_asm(a.src)
    rx = re.compile(a.kernel)
    found = False
    for name, body in functions(lines):
        if not rx.search(name):
            continue
        found = True
        def n(lp, pat):
            return sum(1 for x in lp if re.match(pat, x[2]))
        # the consumer's tile loop: its plane stores and operand loads, no MFMA (the producer's loops
        # have MFMAs; the epilogue's slab-write loops have no loads)
        cand = [lp for lp in loops(body) if n(lp, r'^(buffer|global)_store') >= a.min_stores
                and n(lp, r'^(buffer|global)_load') >= a.min_loads and n(lp, r'^v_mfma') == 0
                and n(lp, r'^s_endpgm') == 0]
        print(f'kernel {name}')
        if not cand:
            print('  no loop with that many stores')
            continue
        for lp in sorted(cand, key=len, reverse=True):
            print(f'  loop {lp[0][3][:40]!r} .. {lp[-1][3][:40]!r}: {len(lp)} instructions')
            for k, v in census(lp).items():
                print(f'    {k:45s} {v:5d}')
        if a.ops:
            ops = collections.Counter(x[2] for x in max(cand, key=len))
            print('  most frequent mnemonics of the largest loop:')
            for mn, c in ops.most_common(a.ops):
                print(f'    {mn:45s} {c:5d}')
    if not found:
        sys.exit(f'no kernel matches {a.kernel}')


if __name__ == '__main__':
    main()
