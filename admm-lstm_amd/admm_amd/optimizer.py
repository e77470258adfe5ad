"""Host side of the drop-in ``ADMMBasedOptimizer`` (both ``admm.py`` and ``admm.no_dual_y.py``).

Mirrors the reference class surface (``admm.py:22-78``; ``admm.no_dual_y.py:12-66``):
constructor arguments and validation (``log_assert``/``error`` -> ``SystemExit``), the
public attributes ``model, train_x, train_y, batch_size, seq_len, input_size,
output_size, hidden_size, verbose, betas, rhos, gates, duals, summary`` and ``step()``.
All arithmetic runs in libadmmlstm.so on the HIP device; this module only owns the
tensors (PyTorch allocations in the reference's [B, T+1, H] layout), validates them and
hands raw pointers across the C ABI.

Extension beyond the reference (keyword-only, default off): ``distributed=True`` makes
each rank of an initialised ``torch.distributed`` job own a shard of the sample batch;
the batch sums of the step are all-reduced with RCCL inside the library and the
``a``-update uses the global batch size (``admm.py:496-502``).
"""
from __future__ import annotations

import ctypes
from typing import Dict, Optional, Tuple

import torch

import _global
from _global import error, log_assert, warning
from parameters import example_parameter_dictionary

from . import _native as N

GATES6 = ('i', 'f', 'g', 'o', 'c', 'h')
GATES4 = ('i', 'f', 'g', 'o')
WEIGHT_ORDER = ('x,i', 'h,i', 'x,f', 'h,f', 'x,g', 'h,g', 'x,o', 'h,o')


class AdmmOptimizerBase(object):
    """Shared implementation; subclasses set ``_variant`` and ``_flag_module``."""

    _variant = N.VARIANT_ADMM
    _flag_module = None  # module whose ``with_dual_y`` global is read at every step

    def __init__(self, model, training_samples: Tuple[torch.Tensor, torch.Tensor],
                 parameter_dictionary: Dict[str, Dict[str, float]] = None, verbose: bool = True, *,
                 distributed: bool = False) -> None:
        device = _global.device
        self.model = model.to(device)
        self.train_x, self.train_y = training_samples
        (self.batch_size, self.seq_len, self.input_size, self.output_size,
         self.hidden_size) = self._training_constants(training_samples)
        self.verbose = verbose
        self.betas, self.rhos = dict(), dict()
        self.summary = None
        self._read_normalization_factors(parameter_dictionary, device)
        self._read_penalties(parameter_dictionary, device)

        self._ctx = None
        self._lib = N.load()
        self._device = device
        self._world, self._rank = 1, 0
        self._global_batch = self.batch_size
        self._distributed = bool(distributed)
        if distributed:
            self._join_process_group()
        self._x = self._device_tensor(self.train_x, 'train_x')
        self._y = self._device_tensor(self.train_y, 'train_y')
        self._create_context()

        kw = dict(dtype=torch.float32, device=device)
        B, T, H, O = self.batch_size, self.seq_len, self.hidden_size, self.output_size
        self.gates = {q: torch.empty(B, T + 1, H, **kw) for q in GATES6}
        self.gates['a'] = torch.empty(B, O, **kw)
        self.duals = {q: torch.empty(B, T + 1, H, **kw) for q in GATES6}
        self.duals['y'] = torch.empty(B, O, **kw)
        self._bound = None
        self._sync_bindings()
        # admm.py:164-173: gates from the LSTM forward, zero duals
        N.check(self._lib.admm_init_state(self._ctx, N.stream_handle(device)), 'admm_init_state')
        self._snapshot()

    # ------------------------------------------------------------------ validation (admm.py:92-162)
    def _training_constants(self, training_samples):
        train_x, train_y = training_samples
        train_batch, train_seq, train_feat = train_x.size()
        train_label_batch, train_label_feat = train_y.size()
        log_assert(train_batch == train_label_batch,
                   f'Batch size of samples mismatch (Got train_x: {train_batch}, train_y: {train_label_batch}).')
        log_assert(train_feat == self.model.input_size and train_label_feat == self.model.output_size,
                   f'Input and output size of samples must match that of the model '
                   f'(Got train_x: {train_feat}, train_y: {train_label_feat}, '
                   f'model: {self.model.input_size} -> {self.model.output_size}).')
        return train_batch, train_seq, train_feat, train_label_feat, self.model.hidden_size

    def _note(self, msg: str) -> None:
        # the reference keeps only the first summary fragment (admm.py:80-90)
        if not self.summary:
            self.summary = msg

    def _read_normalization_factors(self, param_dict, device) -> None:
        if not param_dict:
            example = example_parameter_dictionary['GoogleStock']
            warning(f'Parameter dictionary is empty, a default one will be applied: '
                    f'{{\n    \'beta\': {example["beta"]},\n    \'rho\': {example["rho"]}\n}})')
            # upstream keys these by the dictionary's own names (admm.py:116-118)
            self.betas, self.rhos = [{k: torch.tensor(v) for k, v in example[part].items()}
                                     for part in ('beta', 'rho')]
            return
        try:
            beta_dict = param_dict['beta']
        except KeyError:
            error('Normalization factors missing in parameter dictionary.')
        self._note('Parameters:\n  {\n    \'beta\': {')

        def checked(key):
            try:
                value = beta_dict[key]
            except KeyError:
                error(f'Key {key} missing in normalization factors.')
            log_assert(isinstance(value, (float, int)), f'Beta {key} must be a float or integer.')
            log_assert(value >= 0, f'Beta {key} must be non-negative.')
            return value

        self.betas['wy'] = torch.tensor(checked('wy'), dtype=torch.float, device=device)
        for kind, side in (('w', 'x'), ('v', 'h')):
            for q in GATES4:
                self.betas[f'{side}2{q}'] = torch.tensor(checked(kind + q), dtype=torch.float, device=device)

    def _read_penalties(self, param_dict, device) -> None:
        if not param_dict:
            return
        log_assert('rho' in param_dict.keys(), 'Penalties missing in parameter dictionary.')
        rho_dict = param_dict['rho']
        for gate in ('i', 'f', 'g', 'o', 'c', 'h', 'y'):
            log_assert(gate in rho_dict.keys(), 'Penalties missing in parameter dictionary.')
            log_assert(isinstance(rho_dict[gate], (float, int)), 'Penalties must be a float or integer.')
            self.rhos[gate] = torch.tensor(rho_dict[gate], dtype=torch.float, device=device)
        if self.verbose:
            self.summary = None

    # ------------------------------------------------------------------ native context
    def _native_params(self) -> N.AdmmParams:
        p = N.AdmmParams()
        # float(...) of the 0-dim fp32 tensors gives exactly the fp32 values the reference uses
        vals = {k: float(v) for k, v in self.rhos.items()}
        for i, k in enumerate(('i', 'f', 'g', 'o', 'c', 'h', 'y')):
            p.rho[i] = vals.get(k, 0.0)
        for i, q in enumerate(GATES4):
            p.beta_x[i] = float(self.betas.get(f'x2{q}', self.betas.get('w' + q, 0.0)))
            p.beta_h[i] = float(self.betas.get(f'h2{q}', self.betas.get('v' + q, 0.0)))
        p.beta_y = float(self.betas.get('wy', 0.0))
        p.variant = self._variant
        p.with_dual_y = int(self._dual_y_flag())
        return p

    def _dual_y_flag(self) -> bool:
        if self._variant != N.VARIANT_ADMM or self._flag_module is None:
            return False
        return bool(getattr(self._flag_module, 'with_dual_y', False))

    def _device_tensor(self, t: torch.Tensor, name: str) -> torch.Tensor:
        if self._device.type != 'cuda':
            raise RuntimeError('admm-lstm_amd needs a HIP device (MI355X); none is visible. '
                               'There is no CPU execution path.')
        return t.to(device=self._device, dtype=torch.float32).contiguous()

    def _create_context(self) -> None:
        d = N.AdmmDims(self.batch_size, self._global_batch, self.seq_len, self.input_size, self.hidden_size,
                       self.output_size)
        ctx = ctypes.c_void_p()
        dev_index = self._device.index if self._device.index is not None else torch.cuda.current_device()
        N.check(self._lib.admm_create(ctypes.byref(d), ctypes.byref(self._native_params()), dev_index,
                                      ctypes.byref(ctx)), 'admm_create')
        self._ctx = ctx
        self._dual_y_sent = self._dual_y_flag()
        if self._distributed:
            self._connect_comm()

    def _join_process_group(self) -> None:
        import torch.distributed as dist
        if not (dist.is_available() and dist.is_initialized()):
            raise RuntimeError('distributed=True needs an initialised torch.distributed process group')
        self._world, self._rank = dist.get_world_size(), dist.get_rank()
        n = torch.tensor([self.batch_size], dtype=torch.int64)
        if self._rccl_group():
            n = n.to(self._device)
        dist.all_reduce(n)
        self._global_batch = int(n.item())

    @staticmethod
    def _rccl_group() -> bool:
        """True when the default group reaches the GPU through RCCL: backend 'nccl', or a
        combined per-device backend string such as 'cpu:gloo,cuda:nccl'."""
        import torch.distributed as dist
        return 'nccl' in str(dist.get_backend()).lower()

    def _connect_comm(self) -> None:
        import torch.distributed as dist
        if not self._rccl_group():
            warning(f'process group backend {dist.get_backend()!r} has no RCCL: every all-reduce of step() '
                    'is staged through host memory (slow; meant for tests)', use_logger=False)
            self._connect_host_comm()
            return
        uid = ctypes.create_string_buffer(N.NCCL_UNIQUE_ID_BYTES)
        if self._rank == 0:
            N.check(self._lib.admm_comm_unique_id(uid, N.NCCL_UNIQUE_ID_BYTES), 'admm_comm_unique_id')
        box = [bytes(uid.raw)]
        dist.broadcast_object_list(box, src=0)
        raw = ctypes.create_string_buffer(box[0], N.NCCL_UNIQUE_ID_BYTES)
        N.check(self._lib.admm_set_comm(self._ctx, raw, N.NCCL_UNIQUE_ID_BYTES, self._rank, self._world),
                'admm_set_comm')

    def _connect_host_comm(self) -> None:
        """Non-RCCL process groups (gloo): the library stages each all-reduce through host
        memory and calls back here (``admm_set_comm_host``).  This is how the sharded step is
        tested with several processes on one GPU; RCCL (``nccl`` backend) is the product path."""
        import numpy as np
        import torch.distributed as dist

        def allreduce(buf, count, dtype, _user):
            try:
                ct = ctypes.c_float if dtype == 0 else ctypes.c_double
                arr = np.ctypeslib.as_array(ctypes.cast(buf, ctypes.POINTER(ct)), shape=(int(count),))
                t = torch.from_numpy(arr)   # shares the library's staging buffer
                dist.all_reduce(t)
                return 0
            except Exception as exc:  # pragma: no cover - re-raised by step() after the library fails
                self._host_ar_error = exc
                return 1

        self._host_ar = N.HOST_ALLREDUCE_FN(allreduce)   # keep the thunk alive with the context
        N.check(self._lib.admm_set_comm_host(self._ctx, self._host_ar, None, self._rank, self._world),
                'admm_set_comm_host')

    # ------------------------------------------------------------------ bindings
    def _tensors(self):
        m = self.model
        return ([self._x, self._y] + [getattr(m, f'x2{q}') for q in GATES4] + [getattr(m, f'h2{q}') for q in GATES4]
                + [m.out] + [self.gates[q] for q in GATES6] + [self.duals[q] for q in GATES6]
                + [self.gates['a'], self.duals['y']])

    def _check_tensor(self, t: torch.Tensor, name: str, shape) -> None:
        N.require_device(t, name)
        if t.dtype != torch.float32 or not t.is_contiguous() or tuple(t.shape) != tuple(shape) \
                or t.device != self._x.device:
            raise ValueError(f'{name} must be a contiguous float32 tensor of shape {tuple(shape)} on '
                             f'{self._x.device} (got {tuple(t.shape)} {t.dtype} on {t.device})')

    def _sync_bindings(self) -> None:
        ts = self._tensors()
        ptrs = tuple(t.data_ptr() for t in ts)
        if self._bound != ptrs:
            B, T, D, H, O = self.batch_size, self.seq_len, self.input_size, self.hidden_size, self.output_size
            shapes = [(B, T, D), (B, O)] + [(D, H)] * 4 + [(H, H)] * 4 + [(H, O)] + [(B, T + 1, H)] * 12 \
                + [(B, O), (B, O)]
            names = ['train_x', 'train_y'] + [f'model.x2{q}' for q in GATES4] + [f'model.h2{q}' for q in GATES4] \
                + ['model.out'] + [f"gates['{q}']" for q in GATES6] + [f"duals['{q}']" for q in GATES6] \
                + ["gates['a']", "duals['y']"]
            for t, n, s in zip(ts, names, shapes):
                self._check_tensor(t, n, s)
            b = N.AdmmBuffers()
            b.x, b.y = ptrs[0], ptrs[1]
            for q in range(4):
                b.wx[q], b.wh[q] = ptrs[2 + q], ptrs[6 + q]
            b.wy = ptrs[10]
            for q in range(6):
                b.gates[q], b.duals[q] = ptrs[11 + q], ptrs[17 + q]
            b.a, b.dual_y = ptrs[23], ptrs[24]
            N.check(self._lib.admm_bind(self._ctx, ctypes.byref(b)), 'admm_bind')
            self._bound = ptrs
            self._versions = None
        versions = self._cache_versions()
        if self._versions is not None and versions != self._versions:
            # weights / h / x were modified in place outside step(): recompute the z cache
            N.check(self._lib.admm_invalidate_cache(self._ctx), 'admm_invalidate_cache')

    def _cache_versions(self):
        """In-place versions of every tensor the library's caches are derived from: the z
        cache (x, the eight gate weights, h) and the x stage's targets tgt = dual/rho + gate
        (the i, f, g, o gate and dual planes), plus c and the remaining duals, which the
        library treats as known (dual h is zero before T unless the caller writes it), and the
        next wy stage's residual rho_y (h_T wy - a - dual_y / rho_y) (model.out, a, dual y)."""
        m = self.model
        ts = ([self._x] + [getattr(m, f'{s}2{q}') for s in 'xh' for q in GATES4] + [m.out]
              + [self.gates[q] for q in GATES6] + [self.duals[q] for q in GATES6]
              + [self.gates['a'], self.duals['y']])
        return tuple(t._version for t in ts)

    def _snapshot(self) -> None:
        self._versions = self._cache_versions()

    # ------------------------------------------------------------------ the step (admm.py:62-78)
    def step(self) -> None:
        for q in GATES4:  # upstream raises KeyError here with a defaulted (empty) dictionary
            self.betas[f'x2{q}'], self.betas[f'h2{q}']
        flag = self._dual_y_flag()
        if flag != self._dual_y_sent:
            N.check(self._lib.admm_set_with_dual_y(self._ctx, int(flag)), 'admm_set_with_dual_y')
            self._dual_y_sent = flag
        self._sync_bindings()
        self._host_ar_error = None
        rc = self._lib.admm_step(self._ctx, N.stream_handle(self._device))
        if rc != 0 and self._host_ar_error is not None:   # the host-staged all-reduce's own error
            raise N.AdmmError(f'admm_step failed (code {rc}): the host-staged all-reduce raised '
                              f'{self._host_ar_error!r}') from self._host_ar_error
        N.check(rc, 'admm_step')
        self._snapshot()
        self._poll_status()

    def _poll_status(self) -> None:
        """Warn (without a device sync) when a line search ran out of its exponent window, saw
        non-finite objective values, or the column-split sweep fell back to the row-block sweep
        (its grid was not resident); raise ``AdmmError`` when a column-split hand-off timed out
        (the state is invalid).  The counts lag by the steps still in flight."""
        unres, nonfin = ctypes.c_int32(), ctypes.c_int32()
        hf, fb = ctypes.c_int32(), ctypes.c_int32()
        N.check(self._lib.admm_poll_faults(self._ctx, ctypes.byref(hf), ctypes.byref(fb)), 'admm_poll_faults')
        N.check(self._lib.admm_poll_status(self._ctx, ctypes.byref(unres), ctypes.byref(nonfin)), 'admm_poll_status')
        seen = getattr(self, '_status_seen', (0, 0, 0))
        if unres.value > seen[0]:
            warning(f'{unres.value - seen[0]} weight line search(es) found no accepted exponent below 2^64 '
                    f'(admm.py:334-336 would keep doubling); theta = 2^63 was applied (last_step_stats()).')
        if nonfin.value > seen[1]:
            warning(f'{nonfin.value - seen[1]} non-finite line-search objective value(s) seen.')
        if fb.value > seen[2]:
            warning(f'{fb.value - seen[2]} column-split sweep launch(es) could not have their whole grid resident '
                    f'(another kernel or process on the GPU?): the row-block sweep ran instead (slower, same result); '
                    f'from the third one on this optimizer runs the row-block sweep directly.')
        self._status_seen = (unres.value, nonfin.value, fb.value)

    # ------------------------------------------------------------------ extras
    def last_step_stats(self) -> dict:
        """Line-search outcomes of the last step (synchronises the device)."""
        s = N.AdmmStats()
        N.check(self._lib.admm_get_stats(self._ctx, ctypes.byref(s)), 'admm_get_stats')
        return {
            'steps': s.steps,
            'k': {name: s.k[i] for i, name in enumerate(WEIGHT_ORDER)},
            'passes': list(s.passes),
            'f_w': {name: s.f_w[i] for i, name in enumerate(WEIGHT_ORDER)},
            'grad_sq': {name: s.grad_sq[i] for i, name in enumerate(WEIGHT_ORDER)},
            'theta_h': s.theta_h,
            'unresolved': s.unresolved,
            'nonfinite': s.nonfinite,
            'direct_frac': {name: s.direct_frac[i] for i, name in enumerate(WEIGHT_ORDER)},
            'handoff_fail': s.handoff_fail,
            'sweep_fallbacks': s.sweep_fallbacks,
            'graph_captures': s.graph_captures,
            'graph_disabled': bool(s.graph_disabled),
            'graph_replays': s.graph_replays,
            'sweep_split_off': bool(s.sweep_split_off),
        }

    # ------------------------------------------------------------------ checkpoint
    def state_dict(self) -> dict:
        """The primal/dual state (``gates``, ``duals`` incl. ``a`` and dual ``y``) as CPU
        tensors plus the shape; ``torch.save`` of it loads back with ``weights_only=True``.
        With the model's own ``state_dict`` this is everything a later step depends on (the
        z cache is rebuilt from them)."""
        return {
            'format': 'admm-lstm-mi355x/optimizer-state/1',
            'shape': [self.batch_size, self.seq_len, self.input_size, self.hidden_size, self.output_size],
            'gates': {k: v.detach().cpu().clone() for k, v in self.gates.items()},
            'duals': {k: v.detach().cpu().clone() for k, v in self.duals.items()},
        }

    def load_state_dict(self, state: dict) -> None:
        """Copy a ``state_dict()`` into this optimizer's (bound) device tensors.  This is a
        restore: it also acknowledges a column-split hand-off fault (``AdmmError`` code -6) that
        left the previous state invalid (``acknowledge_fault``); restore the model's weights first."""
        shape = [self.batch_size, self.seq_len, self.input_size, self.hidden_size, self.output_size]
        if list(state.get('shape', [])) != shape:
            raise ValueError(f'checkpoint is for shape {state.get("shape")}, this optimizer has {shape}')
        with torch.no_grad():
            for part, dst in (('gates', self.gates), ('duals', self.duals)):
                src = state[part]
                if set(src) != set(dst):
                    raise ValueError(f'checkpoint {part} keys {sorted(src)} != {sorted(dst)}')
                for k, t in dst.items():
                    if tuple(src[k].shape) != tuple(t.shape):
                        raise ValueError(f'checkpoint {part}[{k!r}] has shape {tuple(src[k].shape)}')
                    t.copy_(src[k].to(t.device, torch.float32))
        # gates['h'] changed version: the next step() rebuilds the z cache
        self.acknowledge_fault()

    def acknowledge_fault(self) -> None:
        """Declare the bound state restored after a column-split hand-off fault (``admm_ack_fault``).
        Until this (or ``load_state_dict``) is called, every ``step()`` raises ``AdmmError`` (code -6):
        an in-place edit of the invalid state does not clear the fault."""
        N.check(self._lib.admm_ack_fault(self._ctx), 'admm_ack_fault')

    def profile(self, classes=()) -> None:
        """Enable live hipEvent timing of the named kernel classes (``_native.PROF_CLASSES``)."""
        mask = 0
        for name in classes:
            mask |= 1 << N.PROF_CLASSES.index(name)
        N.check(self._lib.admm_profile(self._ctx, mask), 'admm_profile')

    def profile_read(self) -> dict:
        """{class: (total_ms, launches)} of the events recorded since the last read (synchronises)."""
        n = len(N.PROF_CLASSES)
        ms, cnt = (ctypes.c_double * n)(), (ctypes.c_int32 * n)()
        N.check(self._lib.admm_profile_read(self._ctx, ms, cnt), 'admm_profile_read')
        return {name: (ms[i], cnt[i]) for i, name in enumerate(N.PROF_CLASSES) if cnt[i]}

    def __del__(self):
        ctx = getattr(self, '_ctx', None)
        lib = getattr(self, '_lib', None)
        if ctx is not None and lib is not None:
            try:
                lib.admm_destroy(ctx)
            except Exception:  # pragma: no cover - interpreter shutdown
                pass
            self._ctx = None


def make_optimizer_class(variant: int, flag_module: Optional[object], doc: str):
    cls = type('ADMMBasedOptimizer', (AdmmOptimizerBase,), {'_variant': variant, '_flag_module': flag_module,
                                                            '__doc__': doc})
    return cls
