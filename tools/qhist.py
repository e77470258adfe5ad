"""Distribution of the line-search trial directions |q| (analysis tool, GPU box).

Runs K steps of the C3 bench problem through the library, then recomputes in torch (fp32)
the x-stage and h-stage trial directions of the next step's first search of each gate
(q = A G, G = rho sum A^T R; admm.py:302-312) and prints a histogram of log2 |q| per gate,
i.e. how many elements need per-candidate evaluation at a given Taylor threshold.
usage: python tools/qhist.py [steps]
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'admm-lstm_amd'), ROOT]
import bench  # noqa: E402


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    dev = torch.device('cuda:0')
    import admm
    from blocks.lstm import LSTM
    from parameters import example_parameter_dictionary
    B, T, D, H = 8192, 32, 16, 256
    x, y = bench.make_data('uniform', B, T, D)
    x, y = x.to(dev), y.to(dev)
    torch.manual_seed(0)
    m = LSTM(D, H, 1).to(dev)
    opt = admm.ADMMBasedOptimizer(m, (x, y), example_parameter_dictionary['GoogleStock'], verbose=False)
    for _ in range(K):
        opt.step()
    torch.cuda.synchronize()
    S, L = opt.gates, opt.duals
    Hp = S['h'][:, :T, :].reshape(B * T, H)
    X = x.reshape(B * T, D)
    edges = list(range(-16, 5))
    for qi, q in enumerate('ifgo'):
        Wx, Wh = getattr(m, f'x2{q}').detach(), getattr(m, f'h2{q}').detach()
        rho = float(opt.rhos[q])
        z = X @ Wx + Hp @ Wh
        tgt = (L[q][:, 1:, :] / rho + S[q][:, 1:, :]).reshape(B * T, H)
        phi = torch.tanh(z) if q == 'g' else torch.sigmoid(z)
        dphi = 1 - phi * phi if q == 'g' else phi * (1 - phi)
        R = (phi - tgt) * dphi
        for side, A in (('x', X), ('h', Hp)):
            G = rho * (A.t() @ R)
            Q = (A @ G).abs().flatten()
            lg = torch.log2(Q.clamp_min(2.0 ** -40))
            n = Q.numel()
            cnt = [(lg <= e).sum().item() / n for e in edges]
            print(f'{side}2{q}: |G|max {G.abs().max().item():.3e}  frac(|q| <= 2^e) ' +
                  ' '.join(f'{e}:{c:.3f}' for e, c in zip(edges, cnt)), flush=True)


if __name__ == '__main__':
    main()
