"""Generate tests/golden/c5g.npz: C5's GLOBAL problem (no_dual_y, random-walk windows, B=32768, T=64,
D=1, H=512, GoogleStock rho/beta), 3 steps.

The reference cannot run it where the other goldens were made: its state alone is 12 x [32768, 65, 512]
fp32 = 52 GB, and its per-call clones push it past the build container's 64 GB.  This script runs the
CPU oracle's restatement (oracle/admm_oracle.py: the reference's op structure, bit-exact with the
reference on every other golden in this repo) on the GPU box's device in fp32 instead -- test
infrastructure generating a fixture, not the product -- and writes the compact golden format of
tests/golden/make_golden.py (weights per step, h2q strided except at the last step, losses, every
line-search comparison; inputs as generator + sha256).  Its fp32 line-search decisions are its own
rounding noise where the reference's would be: the parity test accepts a
differing exponent only where it is the fp64 search's from the library's own inputs.

usage (GPU box): python tools/make_c5g.py OUT.npz
"""
import hashlib
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))
sys.path.insert(0, os.path.join(ROOT, 'admm-lstm_amd'))

from golden_io import make_inputs            # noqa: E402
from oracle import admm_oracle as O          # noqa: E402
from parameters import example_parameter_dictionary   # noqa: E402

NAME, VARIANT, GEN, B, T, D, H, STEPS = 'c5g', 'no_dual_y', 'rw', 32768, 64, 1, 512, 3
WSTRIDE = 16
WNAMES = ('x2i', 'h2i', 'x2f', 'h2f', 'x2g', 'h2g', 'x2o', 'h2o', 'out')


def main(out):
    dev = torch.device('cuda:0')
    pdict = example_parameter_dictionary['GoogleStock']
    x, y = make_inputs(GEN, B, T, D)
    torch.manual_seed(0)
    W = O.init_weights(D, H, 1)
    st = O.init_state(x.to(dev), y.to(dev), {k: v.to(dev) for k, v in W.items()})
    hyper = O.Hyper.from_dict(pdict, VARIANT)
    hyper = O.Hyper({k: v.to(dev) for k, v in hyper.rho.items()}, {k: v.to(dev) for k, v in hyper.beta.items()},
                    hyper.variant, hyper.with_dual_y)
    stp = O.Stepper(hyper)
    arrays, searches, losses, times = {}, [], [O.mse(st.x, st.y, st.W)], []
    for s in range(1, STEPS + 1):
        t0 = time.time()
        rec = stp.step(st)
        torch.cuda.synchronize()
        times.append(time.time() - t0)
        searches.append({'weights': [[[a, b, r] for a, b, r in w['tests']] for w in rec['weights']],
                         'hT': [[a, b, r] for a, b, r in rec['hT']['tests']], 'wy_true': 0, 'c_true': 0, 'c_count': T})
        for w in WNAMES:
            v = st.W[w].detach().cpu().numpy().copy()
            if s != STEPS and w.startswith('h2'):
                v = v.reshape(-1)[::WSTRIDE].copy()
            arrays[f'w{s}_{w}'] = v
        losses.append(O.mse(st.x, st.y, st.W))
        print(f'{NAME}: step {s} loss {losses[-1]:.8f} k={[w["k"] for w in rec["weights"]]} ({times[-1]:.1f} s)',
              flush=True)
    meta = {
        'name': NAME, 'variant': VARIANT, 'with_dual_y': False, 'gen': GEN, 'B': B, 'T': T, 'D': D, 'H': H, 'O': 1,
        'steps': STEPS, 'full_state': False, 'param_set': 'GoogleStock', 'params': pdict, 'losses': losses,
        'val_losses': [None] * (STEPS + 1), 'searches': searches, 'torch': torch.__version__,
        'threads': torch.get_num_threads(), 'step_times': times,
        'source': 'oracle',   # an oracle fixture (tests/golden_io.py Golden.source), not a reference one
        'generator': 'tools/make_c5g.py: oracle/admm_oracle.py (the reference op structure) in fp32 on the GPU box '
                     '(the reference itself needs > 64 GB for this batch)',
        'device': torch.cuda.get_device_name(0),
        'compact': {'full_w': [STEPS], 'wstride': WSTRIDE,
                    'x_sha256': hashlib.sha256(x.numpy().tobytes()).hexdigest(),
                    'y_sha256': hashlib.sha256(y.numpy().tobytes()).hexdigest(),
                    'inputs': f'make_inputs({GEN!r}, {B}, {T}, {D}) (SURVEY.md 8(d) generator)'},
        'fp64': [],
    }
    arrays['meta_json'] = np.array(json.dumps(meta))
    np.savez_compressed(out, **arrays)
    print(f'wrote {out} ({os.path.getsize(out) / 1e6:.2f} MB)')


if __name__ == '__main__':
    main(sys.argv[1] if len(sys.argv) > 1 else 'c5g.npz')
