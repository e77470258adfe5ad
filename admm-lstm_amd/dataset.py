"""GoogleStock input path of the reference (``dataset.py:386-443``) without ``xlrd``.

Only the dataset ``demo.py`` uses by default (``demo.py:39, 137-148``) is provided; the
reference's other loaders need OpenCV, torchvision, yfinance or downloads and are outside
this package's scope.

``GoogleStockDataset().data()`` returns ``(train_x [4224,10,1], train_y [4224,1],
test_x [461,10,1], test_y [461,1])`` float32 tensors on ``_global.device``, built exactly as
the reference builds them: column 5 ("Adj Close") as input and column 4 ("Close") as
target of rows 1..4705 of sheet 0 (``dataset.py:401-405``), each divided by its float32 max
(``dataset.py:406-417``), windows of 10 inputs predicting the next target, train rows
10..4233 and validation rows 4244..4704 (``dataset.py:418-437``).  The workbook is read with
``xls_biff`` (OLE2 + BIFF8, standard library only).
"""
from __future__ import annotations

import os
from typing import Sequence, Tuple

import torch

from _global import device

supported_datasets = ['GoogleStock']

__all__ = ['supported_datasets', 'GoogleStockDataset', 'google_stock_columns', 'google_stock_windows']

_SEARCH = ('datasets/GoogleStock/GOOG.xls', '../datasets/GoogleStock/GOOG.xls')   # dataset.py:392-399
N_ROWS, WINDOW, TRAIN_END, VAL_BEGIN = 4705, 10, 4234, 4244


def google_stock_columns(path: str | None = None) -> Tuple[Sequence[float], Sequence[float]]:
    """(input column 5, target column 4) of rows 1..4705 of GOOG.xls (dataset.py:401-405)."""
    import xls_biff
    paths = [path] if path else [p for p in _SEARCH]
    for p in paths:
        if os.path.exists(p):
            cells = xls_biff.read_sheet(p, 0)
            x = [xls_biff.cell_value(cells, i, 5) for i in range(1, N_ROWS + 1)]
            y = [xls_biff.cell_value(cells, i, 4) for i in range(1, N_ROWS + 1)]
            return x, y
    raise FileNotFoundError(f'GOOG.xls not found (tried {paths})')


def google_stock_windows(col_x: Sequence[float], col_y: Sequence[float]):
    """The reference's normalisation and windowing (dataset.py:406-440), on CPU."""
    input_x = torch.zeros((N_ROWS,))
    output_y = torch.zeros((N_ROWS,))
    for i in range(N_ROWS):                      # float64 cell values -> float32 tensor elements
        output_y[i] = col_y[i]
        input_x[i] = col_x[i]
    x = input_x / input_x.max()                  # elementwise float32 division by the float32 max
    y = output_y / output_y.max()
    train_x = torch.stack([x[i - WINDOW:i] for i in range(WINDOW, TRAIN_END)])
    train_y = torch.stack([y[i] for i in range(WINDOW, TRAIN_END)]).reshape(TRAIN_END - WINDOW, 1)
    test_x = torch.stack([x[i - WINDOW:i] for i in range(VAL_BEGIN, N_ROWS)])
    test_y = torch.stack([y[i] for i in range(VAL_BEGIN, N_ROWS)]).reshape(N_ROWS - VAL_BEGIN, 1)
    return train_x.unsqueeze(2), train_y, test_x.unsqueeze(2), test_y


class GoogleStockDataset:
    """dataset.GoogleStockDataset of the reference (dataset.py:386-443)."""

    def __init__(self, path: str | None = None) -> None:
        col_x, col_y = google_stock_columns(path)
        tx, ty, vx, vy = google_stock_windows(col_x, col_y)
        self.train_x, self.train_y, self.test_x, self.test_y = (t.to(device) for t in (tx, ty, vx, vy))

    def data(self) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]:
        return self.train_x, self.train_y, self.test_x, self.test_y
