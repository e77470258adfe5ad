"""Drop-in for ``admm.no_dual_y.py`` of Frederick2309/ADMM-LSTM (the "Fast ADMM"
variant without a dual for y), running on MI355X.

Same class name and surface as ``admm.py``; differences from it follow the reference
(``admm.no_dual_y.py:226-249`` wy update with theta 0.005 and 2*beta_y,
``:414-449`` h_T search with trial point g/theta and gradient scaled by rho_h,
``:451-456`` a update).  Like the reference this file has a dot in its name and is
loaded with ``importlib.util.spec_from_file_location``.
"""
import torch  # noqa: F401

from admm_amd import _native
from admm_amd.optimizer import make_optimizer_class
from blocks.lstm import LSTM  # noqa: F401
from parameters import example_parameter_dictionary  # noqa: F401

ADMMBasedOptimizer = make_optimizer_class(
    _native.VARIANT_NO_DUAL_Y, None,
    """ADMM-based optimizer, no-dual-y variant (admm.no_dual_y.py:12-66).""")
