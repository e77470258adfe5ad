"""rho / beta dictionaries of the ADMM-LSTM optimizer, per dataset.

Drop-in for ``parameters.py`` of Frederick2309/ADMM-LSTM (``parameters.py:9-91``):
``example_parameter_dictionary[name] = {'rho': {i,f,g,o,c,h,y}, 'beta': {wi,vi,...,wy}}``
and ``default_epoch``.  The values (including which are ints and which are floats)
are the reference's; the table below is only a more compact spelling of it.
"""
from typing import Dict

__all__ = ['example_parameter_dictionary', 'default_epoch']

default_epoch = 100

_RHO_KEYS = ('i', 'f', 'g', 'o', 'c', 'h', 'y')
_BETA_KEYS = ('wi', 'vi', 'wf', 'vf', 'wg', 'vg', 'wo', 'vo', 'wy')

# dataset -> (rho values in _RHO_KEYS order, beta for w*/v* , beta for wy)
_TABLE = {
    'GoogleStock': ((1., 1., 1., 1., 0.008, 0.00045, 0.0000562), 8e-7, 8e-7),
    'GEFCOM2012': ((1, 1, 1, 1, 0.1, 0.01, 0.01), 8e-7, 8e-7),
    'YahooFinance': ((1, 1, 1, 1, 0.1, 0.02, 0.01), 1e-8, 1e-8),
    'MNISTDataset': ((1, 1, 1, 1, 0.012, 0.0012, 0.00005), 1, 10),   # deprecated upstream
    'UCF101': ((.1, .1, .1, .1, 0.008, 0.0001, 0.000001), 1e-9, 1e-9),  # deprecated upstream
    'HAR': ((1.5, 1.5, 1.5, 1.5, 0.005, 8e-04, 4e-04), 8e-7, 8e-7),
    'PTB': ((.8, .8, .8, .8, 5e-4, 5e-4, 1e-5), 8e-7, 8e-7),
    'DNA1': ((1., 1., 1., 1., 0.001, 0.03, 0.002), 8e-9, 8e-9),
    'SMSSpam': ((1.0, 1.0, 1.0, 1.0, 0.01, 0.001, 4e-05), 8e-9, 8e-9),
}


def _entry(rhos, beta_w, beta_y) -> Dict[str, Dict[str, float]]:
    beta = {k: (beta_y if k == 'wy' else beta_w) for k in _BETA_KEYS}
    return {'rho': dict(zip(_RHO_KEYS, rhos)), 'beta': beta}


example_parameter_dictionary: Dict[str, Dict[str, Dict[str, float]]] = {
    name: _entry(*row) for name, row in _TABLE.items()
}
