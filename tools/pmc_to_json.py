"""Per-kernel HBM traffic from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) -> JSON.

usage: python tools/pmc_to_json.py <fetch run dir> <write run dir> <out.json> [note]

Counters are KiB per dispatch.  Correction (MI355X_MICROARCH.md, HBM section): on gfx950
FETCH_SIZE reports half the bytes of wide coalesced streaming reads, so read bytes =
2 x FETCH_SIZE; WRITE_SIZE is exact.  traffic = 2*FETCH + WRITE bytes, per dispatch
(median over the dispatches of that kernel; the max is kept too, since line-search
passes after the first return early when every gate has chosen its step).
"""
import collections
import csv
import glob
import json
import os
import re
import statistics
import sys


def _load(d):
    out = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
        for r in csv.DictReader(open(f)):
            m = re.search(r'(k_[a-z_0-9]+)(<[^>]*>)?', r['Kernel_Name'])
            if not m:
                continue
            out[m.group(1) + (m.group(2) or '')].append(float(r['Counter_Value']) * 1024.0)
    return out


def main(fetch_dir, write_dir, out_path, note=''):
    fetch, write = _load(fetch_dir), _load(write_dir)
    res = {'note': note, 'units': 'bytes per dispatch', 'correction': 'read = 2 x FETCH_SIZE (gfx950)',
           'kernels': {}}
    for k in sorted(fetch):
        f, w = fetch[k], write.get(k, [0.0])
        res['kernels'][k] = {
            'dispatches': len(f),
            'read_bytes_median': 2 * statistics.median(f), 'write_bytes_median': statistics.median(w),
            'traffic_bytes_median': 2 * statistics.median(f) + statistics.median(w),
            'traffic_bytes_max': 2 * max(f) + max(w),
        }
    with open(out_path, 'w') as fh:
        json.dump(res, fh, indent=1)


if __name__ == '__main__':
    main(*sys.argv[1:])
