"""Cross-build bit-identity check: run a few C3-shaped ADMM steps with the library named by
ADMM_LSTM_LIB (default: the in-tree build) and save every weight, gate and dual plane plus the
line-search exponents.  Run once per build, then compare:

  ADMM_LSTM_LIB=ablib/lib_old.so python3 tools/libcmp.py run gpurun_out/old.pt
  python3 tools/libcmp.py run gpurun_out/new.pt
  python3 tools/libcmp.py cmp gpurun_out/old.pt gpurun_out/new.pt
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'admm-lstm_amd'), ROOT]


def run(path, B=2048, T=8, D=16, H=256, steps=4):
    import torch
    import admm
    from blocks.lstm import LSTM
    from parameters import example_parameter_dictionary
    dev = torch.device('cuda:0')
    g = torch.Generator().manual_seed(21)
    x = torch.rand(B, T, D, generator=g).to(dev)
    y = torch.rand(B, 1, generator=g).to(dev)
    torch.manual_seed(0)
    m = LSTM(D, H, 1).to(dev)
    opt = admm.ADMMBasedOptimizer(m, (x, y), example_parameter_dictionary['GoogleStock'], verbose=False)
    ks = []
    for _ in range(steps):
        opt.step()
        st = opt.last_step_stats()
        ks.append(list(st['k'].values()) + [st['theta_h']] + list(st['grad_sq'].values()))
    torch.cuda.synchronize()
    out = {'W': torch.cat([p.detach().flatten() for p in m.parameters()]).cpu(),
           'S': torch.cat([v.flatten() for v in opt.gates.values()]).cpu(),
           'L': torch.cat([v.flatten() for v in opt.duals.values()]).cpu(), 'k': ks}
    torch.save(out, path)
    print('saved', path, 'k', ks[-1] if ks else None)


def cmp(a, b):
    import torch
    A, Bv = torch.load(a, weights_only=True), torch.load(b, weights_only=True)
    ok = True
    for key in ('W', 'S', 'L'):
        same = torch.equal(A[key], Bv[key])
        ok &= same
        print(key, 'bit-identical' if same else f'differs (max {float((A[key] - Bv[key]).abs().max()):.3e})')
    print('k', 'equal' if A['k'] == Bv['k'] else f'differ {A["k"]} {Bv["k"]}')
    sys.exit(0 if ok and A['k'] == Bv['k'] else 1)


if __name__ == '__main__':
    if sys.argv[1] == 'run':
        run(sys.argv[2])
    else:
        cmp(sys.argv[2], sys.argv[3])
