"""Loading helpers for the golden fixtures in tests/golden/ (data only, no pickles)."""
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
    def x(self):
        return self.t('x')

    @property
    def y(self):
        return self.t('y')

    def weights(self, step):
        return {k: self.t(f'w{step}_{k}') for k in WEIGHT_NAMES}

    def state(self, step):
        S = {q: self.t(f's{step}_S_{q}') for q in GATES6}
        S['a'] = self.t(f's{step}_a')
        L = {q: self.t(f's{step}_L_{q}') for q in GATES6}
        L['y'] = self.t(f's{step}_Ly')
        return S, L

    def ks(self, step):
        """Chosen line-search exponents of the 8 weight updates at ``step`` (1-based)."""
        return [len(v) - 1 for v in self.searches[step - 1]['weights']]


# step fixtures (goog_cols45.npz holds the C1 input columns, not a step trajectory)
ALL = sorted(f[:-4] for f in os.listdir(GOLDEN) if f.endswith('.npz') and not f.startswith('goog_'))
FULL = [n for n in ALL if Golden(n).full_state]
