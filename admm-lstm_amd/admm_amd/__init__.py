"""Native (gfx950 HIP) implementation behind the admm-lstm_amd drop-in modules.

Layout of the drop-in directory (put ``admm-lstm_amd/`` on ``sys.path``, as the
reference's own directory is when ``demo.py`` runs):

* ``admm.py`` / ``admm.no_dual_y.py`` -- ``ADMMBasedOptimizer`` (both variants)
* ``blocks/lstm.py`` -- ``LSTM`` model container
* ``parameters.py`` -- rho/beta dictionaries
* ``_global.py`` -- device and message/exit conventions
* ``admm_amd/`` -- ctypes binding (``_native``), host logic (``optimizer``), HIP sources
  (``csrc/``) and the built ``libadmmlstm.so``
"""
from . import _native  # noqa: F401

__all__ = ['_native']
