"""Generate golden fixtures by running the *reference* ADMM-LSTM optimizer on CPU.

This script is the ONLY place that imports the reference implementation
(``/root/reference``, read-only).  It runs in this build container only; the
reference never travels to the GPU box.  What it writes are small ``.npz``
fixtures of inputs and outputs (data, not source):

* inputs: ``x`` [B,T,D], ``y`` [B,O], initial weights (seeded LSTM init,
  ``blocks/lstm.py:23-29``), the rho/beta dictionary used;
* per step ``s`` (after ``ADMMBasedOptimizer.step()``, ``admm.py:62-78``):
  all nine weights, the training loss ``MSE(model(x), y)`` (as ``demo.py:341``),
  and every line-search comparison the reference evaluated, as the pair of
  operands of ``>`` (``f(beta)``, ``estimate``) for the eight weight searches
  (``admm.py:334``) and the ``h_T`` search (``admm.py:475``), so the chosen
  exponents *and* their margins are pinned;
* for the small cases, the full primal/dual state (``gates``/``duals``/``a``/
  dual ``y``) after every step, which doubles as teacher-forced step pairs.

Line-search comparisons are captured by wrapping ``torch.Tensor.__gt__`` in this
process and reading the calling frame's function name -- the reference files
are not modified.

Usage:  python tests/golden/make_golden.py [case ...]
"""
from __future__ import annotations

import importlib.util
import json
import os
import sys
import time

import numpy as np
import torch

REF = '/root/reference'
OUT = os.path.dirname(os.path.abspath(__file__))
GATES = ('i', 'f', 'g', 'o', 'c', 'h')
WNAMES = ('x2i', 'h2i', 'x2f', 'h2f', 'x2g', 'h2g', 'x2o', 'h2o', 'out')

# name -> (variant, with_dual_y, gen, B, T, D, H, steps, full_state, param_set)
CASES = {
    # tiny, full state every step (teacher-forced pairs), D=1 random walk
    't0_admm':      ('admm', False, 'rw', 64, 8, 1, 10, 5, True, 'GoogleStock'),
    't0_nodualy':   ('no_dual_y', False, 'rw', 64, 8, 1, 10, 5, True, 'GoogleStock'),
    't0_dualy':     ('admm', True, 'rw', 64, 8, 1, 10, 5, True, 'GoogleStock'),
    # tiny with D>1 (x-side K>1), uniform inputs, other rho/beta sets
    't0_uniform':   ('admm', False, 'uniform', 48, 5, 3, 8, 4, True, 'GoogleStock'),
    't0_yahoo':     ('admm', False, 'uniform', 40, 6, 2, 12, 4, True, 'YahooFinance'),
    # mid-size teacher-forced pairs, D=16
    't3_tf':        ('admm', False, 'uniform', 64, 6, 16, 32, 3, True, 'GoogleStock'),
    # GoogleStock-shaped random walk (C1-like), 30 epochs, weights + losses + searches
    't1_gstock':    ('admm', False, 'rw', 4224, 10, 1, 10, 30, False, 'GoogleStock'),
    't1_gstock_nd': ('no_dual_y', False, 'rw', 4224, 10, 1, 10, 30, False, 'GoogleStock'),
    # C2 shapes
    't2_c2':        ('admm', False, 'uniform', 2048, 16, 16, 64, 6, False, 'GoogleStock'),
    't2_c2_nd_rw':  ('no_dual_y', False, 'rw', 1024, 16, 1, 64, 6, False, 'GoogleStock'),
    # C1: the real GoogleStock windows (demo.py defaults: hidden 10, 30 epochs), train + val losses
    'c1_goog':      ('admm', False, 'goog', 4224, 10, 1, 10, 30, False, 'GoogleStock'),
    # BASELINE configs at full size (compact: inputs as generator recipe + sha256, no state)
    'c3':           ('admm', False, 'uniform', 8192, 32, 16, 256, 5, False, 'GoogleStock'),
    'c5_1gpu':      ('no_dual_y', False, 'rw', 4096, 64, 1, 512, 3, False, 'GoogleStock'),
    # the bench's own trajectory (bench.py default: 5 warm-up + 20 timed steps = steps 1..25 of C3), and the
    # same capture on 4 threads (a different reduction order) as the reference's own noise floor
    'c3_25':        ('admm', False, 'uniform', 8192, 32, 16, 256, 25, False, 'GoogleStock'),
    'c3_25_t4':     ('admm', False, 'uniform', 8192, 32, 16, 256, 25, False, 'GoogleStock'),
    # C5's per-GPU shape over 10 steps (the second BASELINE config's arithmetic over a longer horizon)
    'c5_10':        ('no_dual_y', False, 'rw', 4096, 64, 1, 512, 10, False, 'GoogleStock'),
    # C4's global problem (65536 samples; the 8-GPU run shards exactly this) on one device
    'c4g':          ('admm', False, 'uniform', 65536, 32, 16, 256, 3, False, 'GoogleStock'),
    # perturbed starting state (golden_io.perturb_state: 1e-2 noise on gates and duals), so that the
    # eight weight updates move the weights far above fp32 resolution at H >= 256 (the sizes where
    # the library runs its split-bf16 h-stage GEMMs and row-pair trials); full weights every step
    't4_pert_h256': ('admm', False, 'uniform', 1024, 8, 16, 256, 3, False, 'GoogleStock'),
    't4_pert_h512': ('no_dual_y', False, 'rw', 512, 8, 1, 512, 3, False, 'GoogleStock'),
    # ... and at C3's own T = 32 (both line-search forms asserted at the headline's T)
    't32_pert_h256': ('admm', False, 'uniform', 1024, 32, 16, 256, 3, False, 'GoogleStock'),
}

# compact cases: which steps keep their full weights (the others keep x2q/out in full and
# every WSTRIDE-th entry of h2q), and whether each pre-step reference state is also stepped
# once by the fp64 oracle (oracle.admm_oracle.fp64_decisions) to record how the reference's
# fp32 line-search decisions compare with fp64 ones from the same state
COMPACT = {'c3': {'full_w': (1, 2, 3, 4, 5), 'fp64': True},
           'c3_25': {'full_w': (5, 10, 15, 20, 25), 'fp64': False},
           'c3_25_t4': {'full_w': (25,), 'fp64': False},
           'c5_10': {'full_w': (5, 10), 'fp64': False},
           'c5_1gpu': {'full_w': (3,), 'fp64': False},
           'c4g': {'full_w': (3,), 'fp64': False},
           't4_pert_h256': {'full_w': (1, 2, 3), 'fp64': True},
           't4_pert_h512': {'full_w': (1, 2, 3), 'fp64': True},
           't32_pert_h256': {'full_w': (1, 2, 3), 'fp64': True}}
# perturbed cases: golden_io.perturb_state(seed, scale) right after the optimizer is constructed
PERTURB = {'t4_pert_h256': {'seed': 11, 'scale': 1e-2}, 't4_pert_h512': {'seed': 11, 'scale': 1e-2},
           't32_pert_h256': {'seed': 11, 'scale': 1e-2}}
WSTRIDE = 16
# torch CPU threads per case (default: whatever torch picks, 8 in this container)
THREADS = {'c3_25': 8, 'c3_25_t4': 4, 'c5_10': 8}


def goog_windows():
    """C1 inputs: GOOG.xls columns (tests/golden/goog_cols45.npz, extracted by
    tools/extract_goog.py) through the package's restatement of dataset.py:406-440."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(OUT)), 'admm-lstm_amd'))
    import dataset as ds  # the package's dataset module (GoogleStock only)
    f = np.load(os.path.join(OUT, 'goog_cols45.npz'))
    tx, ty, vx, vy = ds.google_stock_windows(f['col_x'].tolist(), f['col_y'].tolist())
    sys.path.pop(0)
    sys.modules.pop('dataset', None)
    return tx.contiguous(), ty.contiguous(), vx.contiguous(), vy.contiguous()


def make_inputs(gen: str, B: int, T: int, D: int):
    """Synthetic inputs of SURVEY.md section 8(d)."""
    if gen == 'goog':
        tx, ty, _, _ = goog_windows()
        assert tuple(tx.shape) == (B, T, D)
        return tx, ty
    if gen == 'uniform':
        g = torch.Generator().manual_seed(1234)
        x = torch.rand(B, T, D, generator=g)
        y = 0.8 * x.mean((1, 2)).unsqueeze(1) + 0.1 * torch.rand(B, 1, generator=g)
        return x.contiguous(), y.contiguous()
    if gen == 'rw':
        assert D == 1
        g = torch.Generator().manual_seed(7)
        s = torch.cumsum(torch.randn(B + T + 1, generator=g), 0)
        s = (s - s.min()) / (s.max() - s.min())
        x = torch.stack([s[b:b + T] for b in range(B)]).unsqueeze(2)
        y = torch.stack([s[b + T] for b in range(B)]).unsqueeze(1)
        return x.contiguous(), y.contiguous()
    raise ValueError(gen)


class GtRecorder:
    """Wraps torch.Tensor.__gt__ and records operands by calling function."""

    def __init__(self):
        self.orig = torch.Tensor.__gt__
        self.log = []

    def __enter__(self):
        rec = self

        def gt(a, b):
            r = rec.orig(a, b)
            fn = sys._getframe(1).f_code.co_name
            try:
                rec.log.append((fn, float(a), float(b), bool(r)))
            except (TypeError, ValueError, RuntimeError):
                pass
            return r

        torch.Tensor.__gt__ = gt
        return self

    def __exit__(self, *exc):
        torch.Tensor.__gt__ = self.orig


def split_searches(log, fn_name):
    """Group consecutive comparisons of one function into searches (end at first False)."""
    out, cur = [], []
    for fn, a, b, r in log:
        if fn != fn_name:
            continue
        cur.append((a, b, r))
        if not r:
            out.append(cur)
            cur = []
    if cur:
        out.append(cur)
    return out


def run_case(name):
    variant, dual_y, gen, B, T, D, H, steps, full, pset = CASES[name]
    os.chdir('/tmp')
    if name in THREADS:
        torch.set_num_threads(THREADS[name])
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import admm as ref_admm
    from blocks.lstm import LSTM
    from parameters import example_parameter_dictionary
    if variant == 'admm':
        mod = ref_admm
        mod.with_dual_y = dual_y
    else:
        spec = importlib.util.spec_from_file_location('admm_no_dual_y', os.path.join(REF, 'admm.no_dual_y.py'))
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
    pdict = example_parameter_dictionary[pset]
    x, y = make_inputs(gen, B, T, D)
    torch.manual_seed(0)
    model = LSTM(D, H, 1)
    compact = COMPACT.get(name)
    arrays = {} if compact else {'x': x.numpy(), 'y': y.numpy()}
    if not compact:
        for w in WNAMES:
            arrays[f'w0_{w}'] = getattr(model, w).detach().numpy().copy()
    fp64_recs = []
    if compact and compact['fp64']:
        sys.path.insert(0, os.path.dirname(os.path.dirname(OUT)))
        from oracle import admm_oracle as O
        hyper = O.Hyper.from_dict(pdict, variant, dual_y)
    loss_fn = torch.nn.MSELoss()

    def loss():
        with torch.no_grad():
            return float(loss_fn(model(x), y))

    vx = vy = None
    if gen == 'goog':
        _, _, vx, vy = goog_windows()
        arrays['val_x'], arrays['val_y'] = vx.numpy(), vy.numpy()

    def val_loss():
        with torch.no_grad():
            return float(loss_fn(model(vx), vy)) if vx is not None else None

    opt = mod.ADMMBasedOptimizer(model, (x, y), pdict, verbose=False)
    pert = PERTURB.get(name)
    if pert:
        sys.path.insert(0, os.path.dirname(OUT))
        from golden_io import perturb_state
        sys.path.pop(0)
        perturb_state(opt.gates, opt.duals, B, T, H, pert['seed'], pert['scale'])

    def snap_state(prefix):
        for q in GATES:
            arrays[f'{prefix}_S_{q}'] = opt.gates[q].detach().numpy().copy()
            arrays[f'{prefix}_L_{q}'] = opt.duals[q].detach().numpy().copy()
        arrays[f'{prefix}_a'] = opt.gates['a'].detach().numpy().copy()
        arrays[f'{prefix}_Ly'] = opt.duals['y'].detach().numpy().copy()

    if full:
        snap_state('s0')
    losses = [loss()]
    val_losses = [val_loss()]
    searches, step_times = [], []
    for s in range(1, steps + 1):
        if compact and compact['fp64']:
            t0 = time.time()
            W = {w: getattr(model, w).detach() for w in WNAMES}
            dec = O.fp64_decisions(x, y, W, opt.gates, opt.duals, hyper)
            fp64_recs.append({'k': [k for _, k, _ in dec['weights']], 'margin': [m for _, _, m in dec['weights']],
                              'theta_h': dec['theta_h']})
            print(f'{name}: fp64 decisions before step {s}: {fp64_recs[-1]["k"]} ({time.time() - t0:.1f}s)', flush=True)
        with GtRecorder() as rec:
            t0 = time.time()
            opt.step()
            step_times.append(time.time() - t0)
        w_s = split_searches(rec.log, '__update_weights')
        h_s = split_searches(rec.log, '__update_primal_h')
        wy_s = split_searches(rec.log, '__update_wy')
        c_s = split_searches(rec.log, '__update_primal_c')
        assert len(w_s) == 8, (name, s, len(w_s))
        searches.append({
            'weights': [[[a, b, r] for a, b, r in srch] for srch in w_s],
            'hT': [[a, b, r] for srch in h_s for a, b, r in srch],
            'wy_true': sum(r for srch in wy_s for _, _, r in srch),
            'c_true': sum(r for srch in c_s for _, _, r in srch),
            'c_count': sum(len(srch) for srch in c_s),
        })
        for w in WNAMES:
            v = getattr(model, w).detach().numpy().copy()
            if compact and s not in compact['full_w'] and w.startswith('h2'):
                v = v.reshape(-1)[::WSTRIDE].copy()
            arrays[f'w{s}_{w}'] = v
        if full:
            snap_state(f's{s}')
        losses.append(loss())
        val_losses.append(val_loss())
        print(f'{name}: step {s} loss {losses[-1]:.8f} k={[len(v) - 1 for v in searches[-1]["weights"]]} '
              f'hT={len(searches[-1]["hT"])} ({step_times[-1]:.2f}s)', flush=True)
    meta = {
        'name': name, 'variant': variant, 'with_dual_y': dual_y, 'gen': gen,
        'B': B, 'T': T, 'D': D, 'H': H, 'O': 1, 'steps': steps, 'full_state': full,
        'param_set': pset, 'params': pdict, 'losses': losses, 'val_losses': val_losses, 'searches': searches,
        'torch': torch.__version__, 'threads': torch.get_num_threads(), 'step_times': step_times,
        'generator': 'tests/golden/make_golden.py',
    }
    if compact:
        import hashlib
        meta['compact'] = {'full_w': list(compact['full_w']), 'wstride': WSTRIDE,
                           'x_sha256': hashlib.sha256(x.numpy().tobytes()).hexdigest(),
                           'y_sha256': hashlib.sha256(y.numpy().tobytes()).hexdigest(),
                           'inputs': f'make_inputs({gen!r}, {B}, {T}, {D}) (SURVEY.md 8(d) generator)'}
        meta['fp64'] = fp64_recs
    if pert:
        meta['perturb'] = pert
    arrays['meta_json'] = np.array(json.dumps(meta))
    path = os.path.join(OUT, f'{name}.npz')
    np.savez_compressed(path, **arrays)
    print(f'wrote {path} ({os.path.getsize(path) / 1e6:.2f} MB)')


if __name__ == '__main__':
    names = sys.argv[1:] or list(CASES)
    for n in names:
        run_case(n)
