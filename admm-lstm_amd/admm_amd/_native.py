"""ctypes binding of libadmmlstm.so (the C ABI declared in include/admm_lstm.h).

The library is built in-tree (``admm_amd/csrc/Makefile`` -> ``admm_amd/libadmmlstm.so``)
and is the only compute path of this package: there is no CPU fallback.  Loading fails
loudly (``NativeUnavailable``) when the library is missing, and every compute entry
point requires a visible HIP device.

``torch`` is imported before the library is loaded so that libadmmlstm.so binds to the
HIP runtime / RCCL that PyTorch already loaded (same SONAMEs), i.e. one HIP runtime per
process, and raw ``tensor.data_ptr()`` / ``torch.cuda.current_stream().cuda_stream``
values can be handed across the boundary.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, Structure, c_char_p, c_double, c_float, c_int, c_int32, c_int64, c_void_p

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

LIB_PATH = os.environ.get('ADMM_LSTM_LIB') or os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                          'libadmmlstm.so')

ABI_VERSION = 3

# the sources whose sha256 the Makefile embeds in admm_build_info() (csrc/Makefile SRC_STAMP: SRC then HDR)
_CSRC = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'csrc')
_STAMP_FILES = ('admm_kernels.hip', 'admm_split3.hip', 'admm_host.hip', 'admm_dev.hpp', 'admm_kernels.hpp',
                'admm_split3.hpp', os.path.join('..', '..', '..', 'include', 'admm_lstm.h'))


def tree_stamp() -> str:
    """The source stamp of the library sources in this tree (what a fresh build would embed)."""
    import hashlib
    h = hashlib.sha256()
    for f in _STAMP_FILES:
        with open(os.path.join(_CSRC, f), 'rb') as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def lib_stamp(lib=None) -> str:
    """The source stamp the loaded library was built from (admm_build_info: '... src <stamp>')."""
    info = (lib or load()).admm_build_info().decode()
    return info.rsplit(' src ', 1)[1] if ' src ' in info else 'unstamped'
VARIANT_ADMM, VARIANT_NO_DUAL_Y = 0, 1
NCCL_UNIQUE_ID_BYTES = 128

# kernel classes of admm_profile (include/admm_lstm.h)
PROF_CLASSES = ('sweep', 'trial', 'trial_extra', 'atr_x', 'atr_h', 'qgemm_x', 'qgemm_h', 'resid', 'small',
                'zgemm', 'comm', 'trial_h')


class NativeUnavailable(RuntimeError):
    """libadmmlstm.so could not be loaded (not built, or not an MI355X environment)."""


class AdmmError(RuntimeError):
    """A libadmmlstm.so call returned an error code."""

    def __init__(self, msg: str, code: int = 0):
        super().__init__(msg)
        self.code = code


EFAULT = -6   # ADMM_EFAULT: the bound state is invalid (a column-split hand-off timed out)


class AdmmDims(Structure):
    _fields_ = [('batch', c_int64), ('global_batch', c_int64), ('seq_len', c_int32),
                ('input_size', c_int32), ('hidden_size', c_int32), ('output_size', c_int32)]


class AdmmParams(Structure):
    _fields_ = [('rho', c_float * 7), ('beta_x', c_float * 4), ('beta_h', c_float * 4), ('beta_y', c_float),
                ('variant', c_int32), ('with_dual_y', c_int32)]


class AdmmBuffers(Structure):
    _fields_ = [('x', c_void_p), ('y', c_void_p), ('wx', c_void_p * 4), ('wh', c_void_p * 4), ('wy', c_void_p),
                ('gates', c_void_p * 6), ('duals', c_void_p * 6), ('a', c_void_p), ('dual_y', c_void_p)]


class AdmmStats(Structure):
    _fields_ = [('steps', c_int32), ('k', c_int32 * 8), ('passes', c_int32 * 2), ('f_w', c_double * 8),
                ('grad_sq', c_double * 8), ('theta_h', c_float), ('unresolved', c_int32), ('nonfinite', c_int32),
                ('direct_frac', c_double * 8), ('handoff_fail', c_int32), ('sweep_fallbacks', c_int32),
                ('graph_captures', c_int32), ('graph_disabled', c_int32), ('graph_replays', c_int64),
                ('sweep_split_off', c_int32)]


# name -> (restype, argtypes)
_SIGNATURES = {
    'admm_abi_version': (c_int32, []),
    'admm_build_info': (c_char_p, []),
    'admm_last_error': (c_char_p, []),
    'admm_create': (c_int, [POINTER(AdmmDims), POINTER(AdmmParams), c_int, POINTER(c_void_p)]),
    'admm_destroy': (c_int, [c_void_p]),
    'admm_bind': (c_int, [c_void_p, POINTER(AdmmBuffers)]),
    'admm_init_state': (c_int, [c_void_p, c_void_p]),
    'admm_step': (c_int, [c_void_p, c_void_p]),
    'admm_set_with_dual_y': (c_int, [c_void_p, c_int32]),
    'admm_invalidate_cache': (c_int, [c_void_p]),
    'admm_ack_fault': (c_int, [c_void_p]),
    'admm_comm_unique_id': (c_int, [c_void_p, c_int64]),
    'admm_set_comm': (c_int, [c_void_p, c_void_p, c_int64, c_int, c_int]),
    'admm_set_comm_host': (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int]),
    'admm_get_stats': (c_int, [c_void_p, POINTER(AdmmStats)]),
    'admm_poll_status': (c_int, [c_void_p, POINTER(c_int32), POINTER(c_int32)]),
    'admm_poll_faults': (c_int, [c_void_p, POINTER(c_int32), POINTER(c_int32)]),
    'admm_debug_fault': (c_int, [c_void_p, c_int32]),
    'admm_profile': (c_int, [c_void_p, ctypes.c_uint32]),
    'admm_profile_read': (c_int, [c_void_p, POINTER(c_double), POINTER(c_int32)]),
    'admm_debug_workspace': (c_int, [c_void_p, c_int32, c_void_p, c_int64, c_void_p]),
    'admm_debug_trace': (c_int, [c_void_p, c_void_p, c_void_p]),
    'admm_debug_trace_resid': (c_int, [c_void_p, c_void_p, c_void_p]),
    'admm_debug_force': (c_int, [c_void_p, c_void_p, c_int32]),
    'admm_debug_own': (c_int, [c_void_p, c_void_p, POINTER(c_float)]),
    'admm_debug_trial': (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int32, c_int32, POINTER(c_double),
                                 c_void_p]),
    'admm_forward': (c_int, [c_void_p, c_int64, c_int32, c_int32, c_int32, c_int32, c_void_p * 4, c_void_p * 4,
                             c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
}
EXPORTS = tuple(_SIGNATURES)

# int (*admm_host_allreduce_fn)(void* host_buf, int64_t count, int32_t dtype, void* user)
HOST_ALLREDUCE_FN = ctypes.CFUNCTYPE(c_int, c_void_p, c_int64, c_int32, c_void_p)

_lib = None


def load() -> ctypes.CDLL:
    """Load (once) and return the library, with argtypes/restype declared."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeUnavailable(
            f'{LIB_PATH} not found: build it with `make -C admm-lstm_amd/admm_amd/csrc` '
            f'(or __graft_entry__.build()). There is no CPU fallback.')
    try:
        lib = ctypes.CDLL(LIB_PATH)
    except OSError as e:  # pragma: no cover - environment dependent
        raise NativeUnavailable(f'cannot load {LIB_PATH}: {e}') from e
    for name, (res, args) in _SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype, fn.argtypes = res, args
    if lib.admm_abi_version() != ABI_VERSION:
        raise NativeUnavailable(f'{LIB_PATH}: ABI {lib.admm_abi_version()} != expected {ABI_VERSION}')
    _lib = lib
    return lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = _lib.admm_last_error().decode(errors='replace') if _lib is not None else ''
        raise AdmmError(f'{what} failed (code {rc}): {msg}', rc)


def require_device(t: torch.Tensor, name: str) -> None:
    if not t.is_cuda:
        raise RuntimeError(f'{name} must be a HIP device tensor (got {t.device}); '
                           'admm-lstm_amd has no CPU execution path')


def ptr(t: torch.Tensor) -> c_void_p:
    return c_void_p(t.data_ptr())


def stream_handle(device: torch.device | None = None) -> c_void_p:
    return c_void_p(torch.cuda.current_stream(device).cuda_stream)
