"""C1 of BASELINE.json: ``demo.py -d GoogleStock -e 30 --hidden 10`` (demo.py:311-376,
383-408) on the MI355X step, without the reference's plotting / CLI plumbing.

    python admm-lstm_amd/c1_demo.py [--epochs 30] [--hidden 10] [--xls path/to/GOOG.xls]

Reads GOOG.xls with the package's BIFF8 reader (dataset.py); without the workbook it uses
the extracted columns in tests/golden/goog_cols45.npz.  Prints the training and validation
loss before training and after each epoch, and the time of each step (the timer of
demo.py:350-352 wraps step() only).
"""
import argparse
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import torch  # noqa: E402

import admm  # noqa: E402
import dataset  # noqa: E402
from blocks.lstm import LSTM  # noqa: E402
from parameters import example_parameter_dictionary  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--epochs', type=int, default=30)
    ap.add_argument('--hidden', type=int, default=10)
    ap.add_argument('--xls', default=None)
    args = ap.parse_args()
    torch.manual_seed(0)                                   # demo.py:281-284
    try:
        tx, ty, vx, vy = dataset.GoogleStockDataset(args.xls).data()
    except FileNotFoundError:
        import numpy as np
        f = np.load(os.path.join(os.path.dirname(HERE), 'tests', 'golden', 'goog_cols45.npz'))
        tx, ty, vx, vy = (t.to(dataset.device) for t in dataset.google_stock_windows(f['col_x'].tolist(),
                                                                                       f['col_y'].tolist()))
    model = LSTM(tx.size(2), args.hidden, ty.size(1)).to(tx.device)
    opt = admm.ADMMBasedOptimizer(model, (tx, ty), example_parameter_dictionary['GoogleStock'], verbose=False)
    mse = torch.nn.MSELoss()

    def losses():
        with torch.no_grad():
            return float(mse(model(tx), ty)), float(mse(model(vx), vy))

    tr, va = losses()
    print(f'epoch 0: train {tr:.8f} val {va:.8f}')
    total = 0.0
    for e in range(1, args.epochs + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        opt.step()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        total += dt
        tr, va = losses()
        print(f'epoch {e}: train {tr:.8f} val {va:.8f} ({dt * 1e3:.2f} ms)')
    print(f'{args.epochs} steps in {total:.3f} s ({args.epochs / total:.1f} it/s)')


if __name__ == '__main__':
    main()
