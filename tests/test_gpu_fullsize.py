"""Reference-anchored parity at the BASELINE configs' full size, and the line-search claim.

* ``c3``: the headline config C3 (uniform, B=8192, T=32, D=16, H=256), 5 steps;
* ``c5_1gpu``: C5's per-GPU shape (no_dual_y, random-walk windows, B=4096, T=64, D=1, H=512), 3 steps.

Both goldens were captured from the reference itself (``tests/golden/make_golden.py``: weights,
training loss and every line-search comparison per step; inputs as their SURVEY.md 8(d)
generator + sha256).  Checks per step, through the C ABI:

* training loss within 1e-5 relative of the reference's (north_star's bar);
* all nine weights within 1e-5 of the reference's, relative to each weight's largest entry;
* every line-search exponent that differs from the reference's must be the fp64 oracle's
  decision from the GPU's own pre-step state (``oracle.admm_oracle.fp64_decisions``, run in fp64
  on the GPU), exactly where that decision has a margin above 1e-3, else within one doubling;
* ``test_line_search_follows_fp64`` (t2_c2 and c3): EVERY GPU exponent equals the fp64 one from
  the same pre-step state wherever the fp64 margin exceeds 1 % -- whether or not the reference
  agrees -- except searches whose gradient is exactly zero on the GPU (step 1's x side: the stored
  gates are phi(z) bit for bit, so k = 0 as in the reference, while fp64 sees the fp32 rounding of
  the state as a gradient);
* C3 only: ADMM_Q_PIECES=3 (f32-accurate trial direction) gives a bitwise-identical run.

The fixture also holds the fp64 oracle's exponents from the REFERENCE's own state before every
step: the test records (and DESIGN.md section 2 cites) how often the reference's fp32 decision
departs from them.  Set ``ADMM_PARITY_OUT=<dir>`` to write a JSON summary per case.
"""
import json
import os

import pytest
import torch

from golden_io import COMPACT, Golden
from oracle import admm_oracle as O
from test_gpu_parity import LOSS_RTOL, _loss, _optimizer

pytestmark = pytest.mark.gpu

W_RTOL = 1e-5


@pytest.fixture(scope='module')
def dev():
    return torch.device('cuda:0')


def _load_mods():
    import importlib.util
    import admm
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location('admm_no_dual_y', os.path.join(root, 'admm-lstm_amd',
                                                                                 'admm.no_dual_y.py'))
    nd = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(nd)
    return admm, nd


def _fp64(g, model, opt, dev):
    W = {k: p.detach() for k, p in model.named_parameters()}
    hp = O.Hyper.from_dict(g.params, g.variant, g.with_dual_y)
    dec = O.fp64_decisions(g.x, g.y, W, opt.gates, opt.duals, hp, global_batch=g.B, device=dev)
    return [(k, m) for _, k, m in dec['weights']], dec['theta_h']


def _run(g, mods, dev, arbitrate_all):
    """Steps the GPU along the golden; returns per-step records."""
    model, opt = _optimizer(g, mods, dev)
    x, y = g.x.to(dev), g.y.to(dev)
    names = list(opt.last_step_stats()['k'].keys())
    recs = []
    assert _loss(model, x, y) == pytest.approx(g.losses[0], rel=LOSS_RTOL)
    for s in range(1, g.steps + 1):
        fp64 = theta64 = None
        if arbitrate_all:
            fp64, theta64 = _fp64(g, model, opt, dev)
            pre = None
        else:   # keep the pre-step state for a lazy arbitration
            pre = ({k: p.detach().clone() for k, p in model.named_parameters()},
                   {k: v.clone() for k, v in opt.gates.items()}, {k: v.clone() for k, v in opt.duals.items()})
        opt.step()
        st = opt.last_step_stats()
        assert st['unresolved'] == 0 and st['nonfinite'] == 0, (s, st)
        ks = [st['k'][n] for n in names]
        ref = g.ks(s)
        if fp64 is None and ks != ref:
            W, S, L = pre
            hp = O.Hyper.from_dict(g.params, g.variant, g.with_dual_y)
            dec = O.fp64_decisions(g.x, g.y, W, S, L, hp, global_batch=g.B, device=dev)
            fp64, theta64 = [(k, m) for _, k, m in dec['weights']], dec['theta_h']
        del pre
        loss = _loss(model, x, y)
        wdiff = {}
        for n, p in model.named_parameters():
            got, want = p.detach().cpu(), g.t(f'w{s}_{n}')
            if not g.full_weights(s) and n.startswith('h2'):
                got = got.reshape(-1)[::g.compact['wstride']]
            wdiff[n] = float((got - want).abs().max()) / max(float(want.abs().max()), 1e-30)
        recs.append({'step': s, 'loss': loss, 'ref_loss': g.losses[s], 'k': ks, 'ref_k': ref,
                     'grad_sq': list(st['grad_sq'].values()), 'theta_h': st['theta_h'],
                     'fp64': fp64, 'theta64': theta64, 'wdiff': wdiff,
                     'weights': {n: p.detach().clone() for n, p in model.named_parameters()}})
    del opt
    torch.cuda.empty_cache()
    return recs


def _write(name, recs, g):
    out = os.environ.get('ADMM_PARITY_OUT')
    if not out:
        return
    os.makedirs(out, exist_ok=True)
    summ = []
    for r in recs:
        d = {k: v for k, v in r.items() if k != 'weights'}
        if g.meta.get('fp64'):
            d['fp64_at_ref_state'] = g.fp64_ks(r['step'])
        summ.append(d)
    with open(os.path.join(out, f'parity_{name}.json'), 'w') as f:
        json.dump(summ, f, indent=1)


@pytest.mark.parametrize('name', COMPACT)
def test_fullsize_matches_reference(name, dev, monkeypatch):
    g = Golden(name)
    mods = _load_mods()
    recs = _run(g, mods, dev, arbitrate_all=(name == 'c3'))
    _write(name, recs, g)
    for r in recs:
        s = r['step']
        assert r['loss'] == pytest.approx(r['ref_loss'], rel=LOSS_RTOL), (s, r['loss'], r['ref_loss'])
        for n, d in r['wdiff'].items():
            assert d <= W_RTOL, (s, n, d)
        for i, (a, b) in enumerate(zip(r['k'], r['ref_k'])):
            if a == b:
                continue
            k64, margin = r['fp64'][i]
            assert a == k64 or (margin < 1e-3 and abs(a - k64) <= 1), (s, i, r['k'], r['ref_k'], r['fp64'])
    if name == 'c3':
        _check_follows_fp64(recs)
    if name == 'c3':   # the trial direction on f32-accurate split3 products: the same run bit for bit
        monkeypatch.setenv('ADMM_Q_PIECES', '3')
        model, opt = _optimizer(g, mods, dev)
        for r in recs:
            opt.step()
            assert list(opt.last_step_stats()['k'].values()) == r['k'], r['step']
            for n, p in model.named_parameters():
                assert torch.equal(p.detach(), r['weights'][n]), (r['step'], n)


def _check_follows_fp64(recs):
    """Every GPU exponent equals the fp64 oracle's from the same pre-step state wherever the fp64
    margin exceeds 1 %, whether or not the reference's agrees."""
    checked = 0
    for r in recs:
        for i, (a, (k64, margin)) in enumerate(zip(r['k'], r['fp64'])):
            if r['grad_sq'][i] == 0.0:      # exact zero gradient: k = 0 (reference and GPU)
                assert a == 0 and r['ref_k'][i] == 0, (r['step'], i)
                continue
            if margin > 0.01:
                checked += 1
                assert a == k64, (r['step'], i, r['k'], r['fp64'])
            else:
                assert abs(a - k64) <= 1, (r['step'], i, r['k'], r['fp64'])
    assert checked >= 4 * len(recs), checked


def test_line_search_follows_fp64_c2(dev):
    """The same claim along the C2 golden (t2_c2, 6 steps); c3 checks it inside
    test_fullsize_matches_reference."""
    g = Golden('t2_c2')
    recs = _run(g, _load_mods(), dev, arbitrate_all=True)
    _write('t2_c2_fp64', recs, g)
    _check_follows_fp64(recs)
