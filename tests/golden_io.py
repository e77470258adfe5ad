"""Loading helpers for the golden fixtures in tests/golden/ (data only, no pickles).

Compact fixtures (the BASELINE configs at full size: ``c3``, ``c5_1gpu``) hold no input
arrays: their inputs are regenerated from SURVEY.md 8(d)'s seeded generators and checked
against the sha256 recorded when the reference ran on them."""
import hashlib
import json
import os

import numpy as np
import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')
WEIGHT_NAMES = ('x2i', 'h2i', 'x2f', 'h2f', 'x2g', 'h2g', 'x2o', 'h2o', 'out')
GATES6 = ('i', 'f', 'g', 'o', 'c', 'h')


class Golden:
    def __init__(self, name):
        self.name = name
        self.z = np.load(os.path.join(GOLDEN, f'{name}.npz'), allow_pickle=False)
        self.meta = json.loads(str(self.z['meta_json']))

    def __getattr__(self, k):
        meta = self.__dict__['meta']
        if k in meta:
            return meta[k]
        raise AttributeError(k)

    def t(self, key):
        return torch.from_numpy(self.z[key].copy())

    @property
    def compact(self):
        return self.meta.get('compact')

    @property
    def source(self):
        """'reference' (made by importing /root/reference: tests/golden/make_golden.py) or 'oracle'
        (made by this repo's CPU restatement where the reference cannot run: tools/make_c5g.py, C5's
        global batch needs > 64 GB in the reference).  An oracle fixture pins the library to the oracle
        (oracle consistency), not to the reference."""
        src = self.meta.get('source')
        if src is None:   # fixtures written before the key existed: the generator says which
            src = 'oracle' if 'oracle/admm_oracle.py' in self.meta.get('generator', '') else 'reference'
        return src

    def _inputs(self):
        if 'xy' not in self.__dict__:
            if self.compact:
                x, y = make_inputs(self.gen, self.B, self.T, self.D)
                for v, key in ((x, 'x_sha256'), (y, 'y_sha256')):
                    assert hashlib.sha256(v.numpy().tobytes()).hexdigest() == self.compact[key], (self.name, key)
            else:
                x, y = self.t('x'), self.t('y')
            self.__dict__['xy'] = (x, y)
        return self.__dict__['xy']

    @property
    def x(self):
        return self._inputs()[0]

    @property
    def y(self):
        return self._inputs()[1]

    def weights(self, step):
        return {k: self.t(f'w{step}_{k}') for k in WEIGHT_NAMES}

    def full_weights(self, step) -> bool:
        return not self.compact or step in self.compact['full_w']

    def fp64_ks(self, step):
        """Compact fixtures with fp64 records: the fp64 oracle's exponents from the reference's
        own state before ``step`` (1-based)."""
        return self.meta['fp64'][step - 1]['k']

    def state(self, step):
        S = {q: self.t(f's{step}_S_{q}') for q in GATES6}
        S['a'] = self.t(f's{step}_a')
        L = {q: self.t(f's{step}_L_{q}') for q in GATES6}
        L['y'] = self.t(f's{step}_Ly')
        return S, L

    def ks(self, step):
        """Chosen line-search exponents of the 8 weight updates at ``step`` (1-based)."""
        return [len(v) - 1 for v in self.searches[step - 1]['weights']]


def perturb_state(gates, duals, B: int, T: int, H: int, seed: int = 11, scale: float = 1e-2):
    """The perturbed starting state of the ``t4_pert_*`` fixtures (and of the GPU line-search
    test ``test_line_search_matches_fp64_oracle``): seeded ``scale``-sized noise on every gate at
    t >= 1 and on the i, f, g, o, c duals, so that the weight gradients are far above the fp32
    rounding of the residual and the eight weight updates move the weights visibly
    (``admm.py:282-343``).  The dual of h stays zero (the reference ascends it only at T).
    ``gates`` / ``duals`` are the optimizer's dicts of [B, T+1, H] tensors, edited in place."""
    gen = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for q in GATES6:
            noise = scale * torch.randn(B, T + 1, H, generator=gen)
            noise[:, 0] = 0
            gates[q].add_(noise.to(gates[q].device))
            if q != 'h':
                duals[q].copy_(scale * torch.randn(B, T + 1, H, generator=gen))
    return gates, duals


def make_inputs(gen: str, B: int, T: int, D: int):
    """SURVEY.md 8(d) synthetic inputs (the generators tests/golden/make_golden.py ran the
    reference on): uniform (seed 1234) and random-walk windows (seed 7)."""
    if gen == 'uniform':
        g = torch.Generator().manual_seed(1234)
        x = torch.rand(B, T, D, generator=g)
        y = 0.8 * x.mean((1, 2)).unsqueeze(1) + 0.1 * torch.rand(B, 1, generator=g)
        return x.contiguous(), y.contiguous()
    assert gen == 'rw' and D == 1, gen
    g = torch.Generator().manual_seed(7)
    s = torch.cumsum(torch.randn(B + T + 1, generator=g), 0)
    s = (s - s.min()) / (s.max() - s.min())
    idx = torch.arange(B).unsqueeze(1) + torch.arange(T).unsqueeze(0)
    return s[idx].unsqueeze(2).contiguous(), s[torch.arange(B) + T].unsqueeze(1).contiguous()


# step fixtures (goog_cols45.npz holds the C1 input columns, not a step trajectory); the compact
# full-size ones are run by their own tests
_NAMES = sorted(f[:-4] for f in os.listdir(GOLDEN) if f.endswith('.npz') and not f.startswith('goog_'))
# perturbed-state fixtures start from perturb_state(), not from the optimizer's own initial state:
# tests/test_gpu_weight_phase.py runs them
PERTURBED = [n for n in _NAMES if Golden(n).meta.get('perturb')]
COMPACT = [n for n in _NAMES if Golden(n).compact and n not in PERTURBED]
# long full-size trajectories (the bench's own 25 steps of C3, captured at two thread counts, and 10 steps
# of C5's per-GPU shape): tests/test_gpu_trajectory.py runs them
LONG = [n for n in COMPACT if Golden(n).meta['steps'] >= 10]
# full-size fixtures the reference itself produced, and those the oracle produced (c5g)
COMPACT_REF = [n for n in COMPACT if Golden(n).source == 'reference' and n not in LONG]
COMPACT_ORACLE = [n for n in COMPACT if Golden(n).source == 'oracle' and n not in LONG]
ALL = [n for n in _NAMES if n not in COMPACT and n not in PERTURBED]
FULL = [n for n in ALL if Golden(n).full_state]
