"""Per-kernel counters from rocprofv3 PMC passes -> JSON.

usage: python tools/pmc_to_json.py <fetch run dir> <write run dir> <out.json> [note]
       python tools/pmc_to_json.py --sq <run dir> <out.json> [note]

Traffic mode: counters are KiB per dispatch.  Correction (MI355X_MICROARCH.md, HBM section): on
gfx950 FETCH_SIZE reports half the bytes of wide coalesced streaming reads, so read bytes =
2 x FETCH_SIZE; WRITE_SIZE is exact.  traffic = 2*FETCH + WRITE bytes, per dispatch
(median over the dispatches of that kernel; the max is kept too, since line-search
passes after the first return early when every gate has chosen its step).

--sq mode: every counter of the pass (SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES, GRBM_GUI_ACTIVE ...)
per dispatch, median and max over the dispatches of each kernel (summed over the XCD/SE instances
rocprofv3 reports for one dispatch).
"""
import collections
import csv
import glob
import json
import os
import re
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def lib_stamp():
    """Source stamp of the library the profiled bench loaded (ADMM_LSTM_LIB or the in-tree build):
    bench.py takes counters only from summaries whose stamp equals its own library's."""
    import ctypes
    path = os.environ.get('ADMM_LSTM_LIB') or os.path.join(ROOT, 'admm-lstm_amd', 'admm_amd', 'libadmmlstm.so')
    try:
        fn = ctypes.CDLL(path).admm_build_info
        fn.restype = ctypes.c_char_p
        info = fn().decode()
    except (OSError, AttributeError):
        return 'unknown'
    return info.rsplit(' src ', 1)[1] if ' src ' in info else 'unstamped'


def _rows(d):
    for f in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
        for r in csv.DictReader(open(f)):
            m = re.search(r'(k_[a-z_0-9]+)(<[^>]*>)?', r['Kernel_Name'])
            if m:
                yield m.group(1) + (m.group(2) or ''), r


def _load(d):
    out = collections.defaultdict(list)
    for k, r in _rows(d):
        out[k].append(float(r['Counter_Value']) * 1024.0)
    return out


def main(fetch_dir, write_dir, out_path, note=''):
    fetch, write = _load(fetch_dir), _load(write_dir)
    res = {'note': note, 'units': 'bytes per dispatch', 'correction': 'read = 2 x FETCH_SIZE (gfx950)',
           'lib_stamp': lib_stamp(), 'kernels': {}}
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


def main_sq(run_dir, out_path, note=''):
    # (kernel, dispatch, counter) -> summed value (rocprofv3 may list one row per instance)
    acc = collections.defaultdict(float)
    for k, r in _rows(run_dir):
        acc[(k, r['Dispatch_Id'], r['Counter_Name'])] += float(r['Counter_Value'])
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for (k, _disp, c), v in acc.items():
        per[k][c].append(v)
    res = {'note': note, 'units': 'counter value per dispatch (SQ cycles as rocprofv3 reports them)',
           'lib_stamp': lib_stamp(), 'kernels': {}}
    for k in sorted(per):
        ent = {'dispatches': max(len(v) for v in per[k].values())}
        for c, vals in sorted(per[k].items()):
            ent[c + '_median'] = statistics.median(vals)
            ent[c + '_max'] = max(vals)
        res['kernels'][k] = ent
    with open(out_path, 'w') as fh:
        json.dump(res, fh, indent=1)


if __name__ == '__main__':
    if sys.argv[1] == '--sq':
        main_sq(*sys.argv[2:])
    else:
        main(*sys.argv[1:])
