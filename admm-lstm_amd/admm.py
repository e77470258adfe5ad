"""Drop-in for ``admm.py`` of Frederick2309/ADMM-LSTM, running on MI355X.

``from admm import ADMMBasedOptimizer, example_parameter_dictionary`` works as in
``demo.py:23``.  ``ADMMBasedOptimizer(model, (train_x, train_y), parameter_dictionary,
verbose)`` and ``.step()`` keep the reference's signature, attributes and error
behaviour (``admm.py:22-78``); the step itself -- wy update, eight backtracking
proximal-linearised weight updates, the sequential gate/cell/hidden sweep, the ``a``
update and dual ascent -- runs in libadmmlstm.so (hand-written gfx950 HIP kernels).

``with_dual_y`` is the reference's module flag (``admm.py:12``), read at every step.
"""
import sys

import torch  # noqa: F401

from admm_amd import _native
from admm_amd.optimizer import make_optimizer_class
from blocks.lstm import LSTM  # noqa: F401  (re-exported like the reference module)
from parameters import example_parameter_dictionary  # noqa: F401

with_dual_y = False

ADMMBasedOptimizer = make_optimizer_class(
    _native.VARIANT_ADMM, sys.modules[__name__],
    """ADMM-based optimizer for the LSTM-Linear model of blocks/lstm.py (admm.py:22-78).

    One step: update Wy, then Wi, Vi, Wf, Vf, Wg, Vg, Wo, Vo; then for t = 1..T update
    i, f, g, o, c, h and the dual variables at t.""")
