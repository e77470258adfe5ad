"""Extract the two GoogleStock columns the reference reads (dataset.py:401-405) from
/root/reference/datasets/GoogleStock/GOOG.xls into tests/golden/goog_cols45.npz, with the
package's own BIFF8 reader (admm-lstm_amd/xls_biff.py).  The fixture lets the GPU box and
the tests use the real C1 data without the reference tree.

usage: python tools/extract_goog.py [path/to/GOOG.xls]
"""
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'admm-lstm_amd'))

import dataset  # noqa: E402

src = sys.argv[1] if len(sys.argv) > 1 else '/root/reference/datasets/GoogleStock/GOOG.xls'
col_x, col_y = dataset.google_stock_columns(src)
meta = {'source': 'datasets/GoogleStock/GOOG.xls of Frederick2309/ADMM-LSTM',
        'sha256': hashlib.sha256(open(src, 'rb').read()).hexdigest(),
        'rows': '1..4705 of sheet 0', 'x': 'column 5 (Adj Close)', 'y': 'column 4 (Close)',
        'reader': 'admm-lstm_amd/xls_biff.py', 'generator': 'tools/extract_goog.py'}
out = os.path.join(ROOT, 'tests', 'golden', 'goog_cols45.npz')
np.savez_compressed(out, col_x=np.array(col_x, dtype=np.float64), col_y=np.array(col_y, dtype=np.float64),
                    meta_json=np.array(json.dumps(meta)))
print(f'wrote {out}: {len(col_x)} rows, x max {max(col_x)}, y max {max(col_y)}')
