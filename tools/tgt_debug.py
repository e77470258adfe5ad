"""GPU debug: with ADMM_TGT_SWEEP=1, compare the sweep-written tgt workspace with lam/rho + S
of the state after each step (C2-like shape), and report where the trajectory turns non-finite."""
import os
import sys
os.environ['ADMM_TGT_SWEEP'] = sys.argv[1] if len(sys.argv) > 1 else '1'
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'admm-lstm_amd'))
import torch
import admm
from admm_amd import _native as N
from blocks.lstm import LSTM
from parameters import example_parameter_dictionary

dev = torch.device('cuda:0')
B, T, D, H = 2048, 16, 16, 64
g = torch.Generator().manual_seed(1234)
x = torch.rand(B, T, D, generator=g)
y = 0.8 * x.mean((1, 2)).unsqueeze(1) + 0.1 * torch.rand(B, 1, generator=g)
x, y = x.to(dev), y.to(dev)
torch.manual_seed(0)
m = LSTM(D, H, 1).to(dev)
admm.with_dual_y = False
opt = admm.ADMMBasedOptimizer(m, (x, y), example_parameter_dictionary['GoogleStock'], verbose=False)
lib = N.load()
buf = torch.empty(4, B * T, H, device=dev)
for s in range(int(sys.argv[2]) if len(sys.argv) > 2 else 4):
    opt.step()
    torch.cuda.synchronize()
    valid = lib.admm_debug_workspace(opt._ctx, 1, N.ptr(buf), buf.numel() * 4, N.stream_handle(dev))
    torch.cuda.synchronize()
    w_ok = all(torch.isfinite(p).all().item() for p in m.parameters())
    print(f'step {s + 1}: tgt valid {valid}, weights finite {w_ok}, loss {float(torch.nn.functional.mse_loss(m(x), y)):.6g}')
    for qi, q in enumerate('ifgo'):
        rho = float(opt.rhos[q])
        ref = (opt.duals[q][:, 1:, :] / rho + opt.gates[q][:, 1:, :]).reshape(B * T, H)
        d = (buf[qi] - ref).abs()
        print(f'  {q}: max|tgt - ref| {float(d.max()):.3e}  nonfinite tgt {int((~torch.isfinite(buf[qi])).sum())}'
              f'  nonfinite ref {int((~torch.isfinite(ref)).sum())}  argmax row {int(d.max(1).values.argmax())}')
        bad = (~torch.isfinite(buf[qi])).nonzero()
        if 0 < bad.shape[0] <= 64:
            for r, c in bad.tolist():
                b, t = divmod(r, T)
                print(f'    row {r} (b {b}, t {t + 1}) col {c}: tgt {float(buf[qi][r, c])} ref {float(ref[r, c])}'
                      f' S {float(opt.gates[q][b, t + 1, c])} L {float(opt.duals[q][b, t + 1, c])}')
    for k in ('i', 'f', 'g', 'o', 'c', 'h'):
        nf = int((~torch.isfinite(opt.gates[k])).sum()), int((~torch.isfinite(opt.duals[k])).sum())
        if nf != (0, 0):
            print('  nonfinite state', k, nf)
