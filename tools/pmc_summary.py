"""Aggregate rocprofv3 --pmc CSV output per kernel (sum over dispatches / per dispatch).

usage: python tools/pmc_summary.py gpurun_out/pmc/<run dir> [...]
"""
import collections
import re
import csv
import glob
import os
import sys


def load(d):
    files = glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True) + glob.glob(os.path.join(d, '*counter_collection.csv'))
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for f in files:
        for r in csv.DictReader(open(f)):
            m = re.search(r'(k_[a-z_0-9]+)(<[^>]*>)?', r['Kernel_Name'])
            k = (m.group(1) + (m.group(2) or '')) if m else r['Kernel_Name'][:40]
            per[k][r['Counter_Name']] += float(r['Counter_Value'])
            disp[k].add(r['Dispatch_Id'])
    return per, disp


if __name__ == '__main__':
    for d in sys.argv[1:]:
        per, disp = load(d)
        print('==', d)
        for k in sorted(per, key=lambda k: -max(per[k].values())):
            n = len(disp[k])
            vals = ' '.join(f'{c}={v / n:.4g}' for c, v in sorted(per[k].items()))
            print(f'{k:40s} n={n:4d} {vals}')
