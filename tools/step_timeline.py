"""One steady-state step's launches from a rocprofv3 --kernel-trace CSV (tools/gpu.sh trace:<cfg>).

usage: python tools/step_timeline.py <run dir or kernel_trace.csv> [step index from the end, default 2]

A step is taken to start at a k_sweep_rows launch that follows a k_sweep_wt / k_select launch
(the sweep closes the step: admm.py:72-76), i.e. from one sweep's end to the next sweep's end;
printed: start offset from the step's first launch, duration, grid and kernel (us), the sum of
durations and the span, so the gaps between launches are visible.
"""
import csv
import glob
import os
import re
import sys


def load(path):
    if os.path.isdir(path):
        files = glob.glob(os.path.join(path, '**', '*kernel_trace.csv'), recursive=True)
        path = files[0]
    rows = list(csv.DictReader(open(path)))
    rows = [r for r in rows if r.get('Kind', 'KERNEL_DISPATCH') == 'KERNEL_DISPATCH']
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    return rows


def short(name):
    m = re.search(r'(k_[a-z_0-9]+)(<[^>]*>)?', name)
    return (m.group(1) + (m.group(2) or '')) if m else name[:48]


def main(path, back=2):
    rows = load(path)
    names = [short(r['Kernel_Name']) for r in rows]
    # step boundaries: the first launch after each column-split / row-block sweep group
    ends = [i for i, n in enumerate(names) if n.startswith('k_sweep_rows') and
            (i + 1 >= len(names) or not names[i + 1].startswith('k_sweep_rows'))]
    if len(ends) < back + 1:
        sys.exit('not enough steps in the trace')
    a, b = ends[-back - 1] + 1, ends[-back] + 1
    t0 = int(rows[a]['Start_Timestamp'])
    tot = 0.0
    print('# start_us duration_us grid kernel')
    for r, n in zip(rows[a:b], names[a:b]):
        st, en = int(r['Start_Timestamp']), int(r['End_Timestamp'])
        d = (en - st) / 1e3
        tot += d
        grid = f"{int(r['Grid_Size_X']) // int(r['Workgroup_Size_X'])}x{r['Grid_Size_Y']}x{r['Grid_Size_Z']}"
        print(f'{(st - t0) / 1e3:9.2f} {d:8.2f} {grid:>10s} {n}')
    span = (int(rows[b - 1]['End_Timestamp']) - t0) / 1e3
    print(f'# {b - a} launches, sum of durations {tot:.1f} us, span {span:.1f} us')


if __name__ == '__main__':
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 2)
