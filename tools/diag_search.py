"""Diagnostic (GPU box): one step of a golden trajectory, then the x- and h-side searches of that
step re-evaluated three ways from the library's own inputs (z cache, targets, traced G):
fp64 in torch, the library's trial arithmetic (admm_debug_trial, fp32 elements / fp64 sums),
and the library's own decision.  Also compares the traced G with rho X^T R recomputed in fp64.

usage: python tools/diag_search.py GOLDEN STEP"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'admm-lstm_amd'), os.path.join(ROOT, 'tests')]

from golden_io import Golden  # noqa: E402
from test_gpu_fullsize import _load_mods  # noqa: E402
from test_gpu_parity import _optimizer  # noqa: E402
from admm_amd import _native as N  # noqa: E402


def main(name, step):
    dev = torch.device('cuda:0')
    g = Golden(name)
    model, opt = _optimizer(g, _load_mods(), dev)
    B, T, D, H = g.B, g.T, g.D, g.H
    lib = opt._lib
    gx = torch.zeros(4, D, H, device=dev)
    gh = torch.zeros(4, H, H, device=dev)
    N.check(lib.admm_debug_trace(opt._ctx, N.ptr(gx), N.ptr(gh)), 'trace')
    for s in range(1, step):
        opt.step()
    opt._sync_bindings()
    zc = torch.empty(4, B * T, H, device=dev)
    print('z valid', lib.admm_debug_workspace(opt._ctx, 0, N.ptr(zc), zc.numel() * 4, N.stream_handle(dev)))
    tg = torch.empty(4, B * T, H, device=dev)
    print('tgt valid', lib.admm_debug_workspace(opt._ctx, 1, N.ptr(tg), tg.numel() * 4, N.stream_handle(dev)))
    W0 = {k: p.detach().clone() for k, p in model.named_parameters()}
    S = {k: v.clone() for k, v in opt.gates.items()}
    L = {k: v.clone() for k, v in opt.duals.items()}
    opt.step()
    st = opt.last_step_stats()
    ks = list(st['k'].values())
    print('step', step, 'k', ks, 'gsq', [f'{v:.4g}' for v in st['grad_sq'].values()])
    X = g.x.to(dev).reshape(B * T, D)
    Hp = S['h'][:, :T, :].reshape(B * T, H)
    for qi, q in enumerate('ifgo'):
        act = torch.tanh if q == 'g' else torch.sigmoid
        rho = float(opt.rhos[q])
        tgt = (L[q][:, 1:, :] / opt.rhos[q] + S[q][:, 1:, :]).reshape(B * T, H)
        print(f'gate {q}: |tgt(state) - tgt(lib)| max {float((tgt - tg[qi]).abs().max()):.3g}')
        for side, (z, A, G) in enumerate([(zc[qi], X, gx[qi]),
                                          (zc[qi].double() + X.double() @ (getattr(model, f'x2{q}').detach().double()
                                                                           - W0[f'x2{q}'].double()), Hp, gh[qi])]):
            z64, t64, A64, G64 = z.double(), tgt.double(), A.double(), G.double()
            p0 = act(z64)
            dphi = 1 - p0 * p0 if q == 'g' else p0 * (1 - p0)
            Gref = rho * A64.T @ ((p0 - t64) * dphi)
            rel = float((G64 - Gref).norm() / Gref.norm())
            qd = A64 @ G64
            c = (1 + T / 2) * float((G64 * G64).sum())
            out = (ctypes.c_double * 16)()
            zf, tf, qf = z.float().contiguous(), tgt.contiguous(), qd.float().contiguous()
            N.check(lib.admm_debug_trial(N.ptr(zf), N.ptr(tf), N.ptr(qf), zf.numel(), int(q == 'g') | 2, 0, out,
                                         N.stream_handle(dev)), 'debug_trial')
            d0 = p0 - t64
            print(f'  side {side}: k_lib {ks[2 * qi + side]}  |G - rho A^T R(fp64)| / |G| = {rel:.3g}   '
                  f'|G|^2 lib {float((G64 * G64).sum()):.6g}')
            for k in range(0, 16):
                sk = 2.0 ** -k
                Dk = act(z64 + qd * sk) - p0
                inc64 = 0.5 * rho * float((Dk * (2 * d0 + Dk)).sum())
                inclib = 0.5 * rho * out[k]
                flag = '>' if inc64 > c * sk else '<='
                print(f'    k={k:2d} inc64 {inc64: .8e} inc_lib(trial arith) {inclib: .8e} est {c * sk: .8e} '
                      f'fp64 {flag}')
    torch.cuda.synchronize()


if __name__ == '__main__':
    main(sys.argv[1], int(sys.argv[2]))
