"""GPU debug: one step with and without ADMM_TGT_SWEEP from the same start; the states after the
step must be bit-identical (the x and h stages of step 1 do not read the sweep's tgt)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'admm-lstm_amd'))
import torch
import admm
from admm_amd import _native as N
from blocks.lstm import LSTM
from parameters import example_parameter_dictionary

dev = torch.device('cuda:0')
B, T, D, H = (int(v) for v in (sys.argv[1:5] if len(sys.argv) > 4 else (2048, 16, 16, 64)))
g = torch.Generator().manual_seed(1234)
x = torch.rand(B, T, D, generator=g)
y = 0.8 * x.mean((1, 2)).unsqueeze(1) + 0.1 * torch.rand(B, 1, generator=g)
x, y = x.to(dev), y.to(dev)
admm.with_dual_y = False
runs = []
for mode in ('0', '1'):
    os.environ['ADMM_TGT_SWEEP'] = mode
    torch.manual_seed(0)
    m = LSTM(D, H, 1).to(dev)
    opt = admm.ADMMBasedOptimizer(m, (x, y), example_parameter_dictionary['GoogleStock'], verbose=False)
    opt.step()
    torch.cuda.synchronize()
    zc = torch.empty(4, B * T, H, device=dev)
    N.load().admm_debug_workspace(opt._ctx, 0, N.ptr(zc), zc.numel() * 4, N.stream_handle(dev))
    torch.cuda.synchronize()
    runs.append(({k: v.clone() for k, v in opt.gates.items()}, {k: v.clone() for k, v in opt.duals.items()},
                 {n: p.detach().clone() for n, p in m.named_parameters()}, zc))
    del opt
(ga, da, wa, za), (gb, db, wb, zb) = runs
for n in wa:
    print('weight', n, float((wa[n] - wb[n]).abs().max()))
for k in ga:
    d = (ga[k] - gb[k]).abs()
    bad = (d > 0).nonzero()
    print('gate', k, float(d.max()), int(bad.shape[0]), bad[:4].tolist())
for k in da:
    d = (da[k] - db[k]).abs()
    bad = (d > 0).nonzero()
    print('dual', k, float(d.max()), int(bad.shape[0]), bad[:4].tolist())
for q in range(4):
    d = (za[q] - zb[q]).abs()
    print('zc', q, float(d.max()), int((d > 0).sum()))
