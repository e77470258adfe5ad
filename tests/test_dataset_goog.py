"""C1 input path: GOOG.xls without xlrd.

* the package's BIFF8 reader against the committed column fixture (extracted by
  tools/extract_goog.py; re-checked here against the workbook when the reference tree is
  present in this container);
* the restated windowing (dataset.py:406-440): shapes, dtype, normalisation, window layout;
* RK number decoding (BIFF8 compressed numbers).
"""
import os

import numpy as np
import pytest
import torch

from golden_io import GOLDEN, Golden

XLS = '/root/reference/datasets/GoogleStock/GOOG.xls'


def _cols():
    f = np.load(os.path.join(GOLDEN, 'goog_cols45.npz'), allow_pickle=False)
    return f['col_x'], f['col_y']


@pytest.mark.skipif(not os.path.exists(XLS), reason='reference workbook not present (GPU box)')
def test_biff_reader_matches_fixture():
    import dataset
    import xls_biff
    x, y = dataset.google_stock_columns(XLS)
    fx, fy = _cols()
    assert np.array_equal(np.array(x), fx) and np.array_equal(np.array(y), fy)
    cells = xls_biff.read_sheet(XLS, 0)
    assert [xls_biff.cell_value(cells, 0, c) for c in range(7)] == \
        ['Date', 'Open', 'High', 'Low', 'Close', 'Adj Close', 'Volume']
    assert len(cells) == 4706 * 7 and xls_biff.cell_value(cells, 4706, 0) == ''


def test_windows_follow_reference_layout():
    import dataset
    fx, fy = _cols()
    tx, ty, vx, vy = dataset.google_stock_windows(fx.tolist(), fy.tolist())
    assert tuple(tx.shape) == (4224, 10, 1) and tuple(ty.shape) == (4224, 1)
    assert tuple(vx.shape) == (461, 10, 1) and tuple(vy.shape) == (461, 1)
    assert all(t.dtype == torch.float32 for t in (tx, ty, vx, vy))
    xs = torch.tensor(fx, dtype=torch.float32)
    ys = torch.tensor(fy, dtype=torch.float32)
    xn, yn = xs / xs.max(), ys / ys.max()
    assert torch.equal(tx[0, :, 0], xn[0:10]) and torch.equal(ty[0, 0], yn[10])
    assert torch.equal(tx[-1, :, 0], xn[4223:4233]) and torch.equal(ty[-1, 0], yn[4233])
    assert torch.equal(vx[0, :, 0], xn[4234:4244]) and torch.equal(vy[-1, 0], yn[4704])
    assert float(tx.max()) <= 1.0 and float(tx.min()) > 0.0


def test_c1_golden_uses_these_windows():
    import dataset
    fx, fy = _cols()
    tx, ty, vx, vy = dataset.google_stock_windows(fx.tolist(), fy.tolist())
    g = Golden('c1_goog')
    assert torch.equal(g.x, tx) and torch.equal(g.y, ty)
    assert torch.equal(g.t('val_x'), vx) and torch.equal(g.t('val_y'), vy)


def test_rk_decoding():
    import struct

    import xls_biff
    assert xls_biff._rk((1234 << 2) | 2) == 1234.0             # integer
    assert xls_biff._rk((1234 << 2) | 3) == 12.34              # integer / 100
    assert xls_biff._rk(((-7) & 0x3FFFFFFF) << 2 | 2) == -7.0  # signed 30-bit integer
    hi = struct.unpack('<Q', struct.pack('<d', 2.5))[0] >> 32
    assert xls_biff._rk(hi) == 2.5                              # top 30 bits of a double
    assert xls_biff._rk(hi | 1) == 0.025
