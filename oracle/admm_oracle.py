"""CPU oracle for the ADMM-LSTM update step -- TEST INFRASTRUCTURE, NOT PRODUCT CODE.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module, and only as the *checker* / the timed CPU
baseline.  The product path (``admm-lstm_amd/``) never imports it and fails
loudly when its HIP library is missing.

What it is: a from-scratch restatement, in PyTorch fp32 on the CPU, of
``ADMMBasedOptimizer.step()`` of Frederick2309/ADMM-LSTM (``admm.py:62-78``)
and of its variant ``admm.no_dual_y.py:52-66``.  It deliberately keeps the
reference's *operation structure* -- per-timestep GEMMs, ``f(W)`` recomputed
inside every line-search estimate, autograd gradients where the reference uses
them, per-call clones -- so that

* in a single process it produces bit-identical results to the reference
  (same torch ops, same operand layouts, same evaluation order), and
* timed on the GPU box's host cores it is a faithful stand-in for the
  reference's CPU cost (``cpu_baseline.kind == "port"`` in ``bench.py``).

Pinning: ``tests/test_oracle_golden.py`` checks it against the golden fixtures
in ``tests/golden/`` that ``tests/golden/make_golden.py`` captured from the
reference itself (weights, losses, every line-search comparison and, for the
small cases, the full primal/dual state after every step).

Sharded mode: every sum over the sample batch goes through ``comm.allreduce``
(identity by default), and the ``a`` update uses the *global* batch size
(``admm.py:496-502``).  ``tests/test_sharded_oracle.py`` runs it on 2 gloo ranks
and compares with the 1-rank result -- the decomposition the HIP path's RCCL
all-reduces implement.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional

import torch

GATES4 = ('i', 'f', 'g', 'o')
GATES6 = ('i', 'f', 'g', 'o', 'c', 'h')
WEIGHT_NAMES = ('x2i', 'h2i', 'x2f', 'h2f', 'x2g', 'h2g', 'x2o', 'h2o', 'out')


class _LocalComm:
    """Single-process communicator: the all-reduce is the identity."""
    world_size = 1

    def allreduce(self, t: torch.Tensor) -> torch.Tensor:
        return t


@dataclass
class Hyper:
    """rho/beta as 0-dim fp32 tensors, keyed like the reference (``admm.py:110-162``)."""
    rho: Dict[str, torch.Tensor]
    beta: Dict[str, torch.Tensor]          # keys x2i..h2o, wy
    variant: str = 'admm'                  # 'admm' | 'no_dual_y'
    with_dual_y: bool = False              # module flag ``admm.with_dual_y`` (admm.py:12)

    @staticmethod
    def from_dict(pdict, variant='admm', with_dual_y=False) -> 'Hyper':
        f32 = lambda v: torch.tensor(v, dtype=torch.float)  # noqa: E731
        beta = {'wy': f32(pdict['beta']['wy'])}
        for kind, side in (('w', 'x'), ('v', 'h')):
            for q in GATES4:
                beta[f'{side}2{q}'] = f32(pdict['beta'][kind + q])
        rho = {k: f32(pdict['rho'][k]) for k in ('i', 'f', 'g', 'o', 'c', 'h', 'y')}
        return Hyper(rho, beta, variant, with_dual_y)

    def cast(self, dtype: torch.dtype) -> 'Hyper':
        c = lambda d: {k: v.to(dtype) for k, v in d.items()}  # noqa: E731
        return Hyper(c(self.rho), c(self.beta), self.variant, self.with_dual_y)


@dataclass
class State:
    """Optimizer state in the reference's layout: gates/duals are [B, T+1, H]."""
    x: torch.Tensor                  # [B, T, D]
    y: torch.Tensor                  # [B, O]
    W: Dict[str, torch.Tensor]       # x2q [D,H], h2q [H,H], out [H,O]
    S: Dict[str, torch.Tensor]       # primal gates i f g o c h (+ 'a' [B,O])
    L: Dict[str, torch.Tensor]       # duals i f g o c h (+ 'y' [B,O])
    global_batch: int = 0
    trace: List[dict] = field(default_factory=list)

    @property
    def T(self) -> int:
        return self.x.shape[1]

    def clone(self) -> 'State':
        c = lambda d: {k: v.clone() for k, v in d.items()}  # noqa: E731
        return State(self.x, self.y, c(self.W), c(self.S), c(self.L), self.global_batch)


# ----------------------------------------------------------------------------- model side

def init_weights(D: int, H: int, O: int) -> Dict[str, torch.Tensor]:
    """Seeded init in the reference's order (``blocks/lstm.py:23-29``): randn for
    x2q [D,H] and h2q [H,H] per gate i,f,g,o, then out [H,O]; then xavier_normal_
    over the parameters in registration order."""
    shapes = {}
    for q in GATES4:
        shapes[f'x2{q}'] = (D, H)
        shapes[f'h2{q}'] = (H, H)
    shapes['out'] = (H, O)
    W = {name: torch.randn(*shp) for name, shp in shapes.items()}
    for name in W:                      # same order as nn.Module.parameters()
        torch.nn.init.xavier_normal_(W[name])
    return W


def lstm_gates(x: torch.Tensor, W: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    """Initial primal state = LSTM forward (``blocks/lstm.py:65-88``)."""
    B, T, _ = x.shape
    H = W['h2i'].shape[0]
    out = {q: torch.zeros(B, T + 1, H, dtype=x.dtype, device=x.device) for q in GATES6}
    for t in range(1, T + 1):
        xt, hp = x[:, t - 1, :], out['h'][:, t - 1, :]
        out['i'][:, t, :] = torch.sigmoid(xt @ W['x2i'] + hp @ W['h2i'])
        out['f'][:, t, :] = torch.sigmoid(xt @ W['x2f'] + hp @ W['h2f'])
        out['g'][:, t, :] = torch.tanh(xt @ W['x2g'] + hp @ W['h2g'])
        out['o'][:, t, :] = torch.sigmoid(xt @ W['x2o'] + hp @ W['h2o'])
        out['c'][:, t, :] = out['f'][:, t, :] * out['c'][:, t - 1, :] + out['i'][:, t, :] * out['g'][:, t, :]
        out['h'][:, t, :] = out['o'][:, t, :] * torch.tanh(out['c'][:, t, :])
    out['a'] = out['h'][:, T, :] @ W['out']
    return out


def predict(x: torch.Tensor, W: Dict[str, torch.Tensor]) -> torch.Tensor:
    """``LSTM.forward`` with ``with_grad=False`` (``blocks/lstm.py:43-46``)."""
    return lstm_gates(x, W)['a']


def mse(x, y, W) -> float:
    return float(torch.nn.functional.mse_loss(predict(x, W), y))


def init_state(x, y, W, global_batch: Optional[int] = None) -> State:
    """Optimizer construction (``admm.py:164-173``): gates from the forward pass,
    zero duals of shape [B, T+1, H] and dual y [B, O]."""
    B, T, _ = x.shape
    H = W['h2i'].shape[0]
    S = lstm_gates(x, W)
    L = {q: torch.zeros(B, T + 1, H, dtype=x.dtype, device=x.device) for q in GATES6}
    L['y'] = torch.zeros(B, y.shape[1], dtype=x.dtype, device=x.device)
    return State(x, y, {k: v.clone() for k, v in W.items()}, S, L, global_batch or B)


# ----------------------------------------------------------------------------- helpers

def _autograd(fn: Callable[[torch.Tensor], torch.Tensor], at: torch.Tensor) -> torch.Tensor:
    """Gradient of a scalar objective by autograd (``admm.py:15-19``).  The reference casts to
    fp32; an fp64 state (the arbitration oracle of the GPU tests) stays fp64."""
    v = at.clone().detach().to(_wide(at)).requires_grad_(True)
    fn(v).backward()
    return v.grad


def _wide(t: torch.Tensor) -> torch.dtype:
    """The reference's hard-coded ``dtype=torch.float`` (admm.py:16, 302, 316), widened to fp64
    when the state is fp64 -- identical for the reference's own fp32 state."""
    return torch.float64 if t.dtype == torch.float64 else torch.float


def _sq(v: torch.Tensor) -> torch.Tensor:
    return torch.sum(v * v)


def _act(q: str):
    return torch.tanh if q == 'g' else torch.sigmoid


def _dact(q: str):
    if q == 'g':
        return lambda z: 1 - torch.tanh(z) ** 2
    return lambda z: torch.sigmoid(z) * (1 - torch.sigmoid(z))


# ----------------------------------------------------------------------------- the step

class Stepper:
    """Runs ``step()`` on a ``State`` (admm.py:62-78 / admm.no_dual_y.py:52-66)."""

    def __init__(self, hyper: Hyper, comm=None, trace_fw: bool = False):
        self.hp = hyper
        self.comm = comm or _LocalComm()
        self.trace_fw = trace_fw  # also record f(W) per search (one extra objective pass; off when timing)
        # (k8, ht_fails) or None: replay given line-search outcomes instead of searching -- the eight
        # exponents in step order (x2i, h2i, x2f, ...) and the number of failing h_T tests, i.e. the
        # theta the reference's loops end with (admm.py:331-343, 474-482); the library's twin is
        # admm_debug_force.  Set before each step() (tests/test_gpu_trajectory.py)
        self.force = None

    # -- accessors that copy, like the reference's getters (admm.py:187-222)
    def _slice(self, store, q, t):
        return store[q][:, t, :].clone().detach()

    def _r(self, k):
        return self.hp.rho[k].clone().detach()

    def step(self, st: State) -> dict:
        rec = {'weights': [], 'hT': None}
        self._wy(st)
        for q in GATES4:                           # admm.py:69-71, Gauss-Seidel x then h
            for side in ('x', 'h'):
                rec['weights'].append(self._weight(st, side, q))
        T = st.T
        for t in range(1, T + 1):                  # admm.py:72-76
            for q in GATES4:
                self._gate(st, q, t)
            self._cell(st, t)
            hT = self._hidden(st, t)
            if hT is not None:
                rec['hT'] = hT
            if t == T:
                self._a(st)
            self._duals(st, t)
        if self.hp.variant == 'admm' and self.hp.with_dual_y:
            self._dual_y(st)                       # admm.py:541-546
        st.trace.append(rec)
        return rec

    # -- output weight (admm.py:246-280; admm.no_dual_y.py:226-249)
    def _wy(self, st: State):
        T = st.T
        h = self._slice(st.S, 'h', T)
        a = st.S['a'].clone().detach()
        wy = st.W['out'].clone().detach()
        ry = self._r('y')
        shift = st.L['y'].clone().detach() / ry if self.hp.with_dual_y else 0

        def f(b):
            return 0.5 * ry * _sq(h @ b - a - shift)

        if self.hp.variant == 'admm':
            grad = self.comm.allreduce(_autograd(f, wy))
            theta = 1
        else:
            grad = self.comm.allreduce(ry * (h.T @ (h @ wy - a)))
            theta = 0.01
        trial = wy + grad / theta
        fb = self.comm.allreduce(f(trial))
        est = fb + torch.sum(grad * (trial - wy)) + 0.5 * theta * _sq(trial - wy)
        assert not bool(fb > est)                  # the search is dead (estimate contains f itself)
        theta /= 2
        by = self.hp.beta['wy'].clone().detach()
        if self.hp.variant == 'admm':
            st.W['out'] = (theta * wy - grad) / (theta + by)
        else:
            st.W['out'] = (theta * wy - grad) / (theta + 2 * by)

    # -- one backtracking proximal-linearised weight update (admm.py:282-343)
    def _weight(self, st: State, side: str, q: str) -> dict:
        T = st.T
        name = f'{side}2{q}'
        w = st.W[name].clone().detach()
        rq = self._r(q)
        act, dact = _act(q), _dact(q)
        if side == 'x':
            A, A2 = st.x, st.S['h'].clone().detach()
            w2 = st.W[f'h2{q}'].clone().detach()
        else:
            A, A2 = st.S['h'].clone().detach(), st.x
            w2 = st.W[f'x2{q}'].clone().detach()

        grad = torch.zeros_like(w, dtype=_wide(w))
        for t in range(1, T + 1):
            at, ot = A[:, t - 1, :], A2[:, t - 1, :]
            z = at @ w + ot @ w2
            resid = (act(z) - self._slice(st.L, q, t) / rq - self._slice(st.S, q, t)) * dact(z)
            grad += at.T @ resid
        grad = self.comm.allreduce(grad) if self.comm.world_size > 1 else grad
        grad = grad * rq

        def f(b):
            acc = torch.zeros((), dtype=_wide(w), device=w.device)
            for t in range(1, T + 1):
                at, ot = A[:, t - 1, :], A2[:, t - 1, :]
                acc += 0.5 * self._r(q) * _sq(
                    act(at @ b + ot @ w2) - self._slice(st.L, q, t) / rq - self._slice(st.S, q, t))
            return self.comm.allreduce(acc)

        def est(b, th):
            return f(w) + torch.sum(grad * (b - w)) + T * 0.5 * th * _sq(b - w)

        theta = 1
        trial = w + grad / theta
        tests = []
        while self.force is None:
            fb, e = f(trial), est(trial, theta)
            worse = bool(fb > e)
            tests.append((float(fb), float(e), worse))
            if not worse:
                break
            theta *= 2
            trial = w + grad / theta
        k = len(tests) - 1
        if self.force is not None:   # the loop above would have ended at theta = 2^k
            k = self.force[0][2 * GATES4.index(q) + (side == 'h')]
            theta = 2 ** k
        theta /= 2
        bq = self.hp.beta[name].clone().detach()
        st.W[name] = (0.5 * rq * T * theta * w - grad) / (bq + 0.5 * rq * theta * T)
        rec = {'name': name, 'k': k, 'tests': tests}
        if self.trace_fw:
            rec['f_w'] = float(f(w))
            rec['grad'] = grad
        return rec

    # -- i, f, g, o closed forms (admm.py:353-386)
    def _gate(self, st: State, q: str, t: int):
        z = st.x[:, t - 1, :] @ st.W[f'x2{q}'].clone().detach() + \
            self._slice(st.S, 'h', t - 1) @ st.W[f'h2{q}'].clone().detach()
        r1 = self._r(q)
        lam = self._slice(st.L, q, t)
        g_ = lambda k, s: self._slice(st.S, k, s)  # noqa: E731
        if q == 'i':
            p1, p2, p3 = g_('g', t), g_('f', t), g_('c', t - 1)
        elif q == 'f':
            p1, p2, p3 = g_('c', t - 1), g_('g', t), g_('i', t)
        elif q == 'g':
            p1, p2, p3 = g_('i', t), g_('f', t), g_('c', t - 1)
        else:
            p1, p2, p3 = torch.tanh(g_('c', t)), 0., 0.
        if q == 'o':
            v2, r2, l2 = g_('h', t), self._r('h'), self._slice(st.L, 'h', t)
        else:
            v2, r2, l2 = g_('c', t), self._r('c'), self._slice(st.L, 'c', t)
        new = - (lam - r1 * _act(q)(z) + (r2 * (p2 * p3 - v2) - l2) * p1) / (r1 + r2 * p1 * p1)
        st.S[q][:, t, :] = new.clone().detach()

    # -- cell state (admm.py:388-436); its search is dead, theta* = 0.5
    def _cell(self, st: State, t: int):
        g_ = lambda k, s: self._slice(st.S, k, s)  # noqa: E731
        c, o, h = g_('c', t), g_('o', t), g_('h', t)
        div_h = self._slice(st.L, 'h', t) / self._r('h')
        div_c = self._slice(st.L, 'c', t) / self._r('c')
        rc = self._r('c')
        target = h + div_h

        def f(v):
            return .5 * _sq(torch.tanh(v) * o - target)

        grad = _autograd(f, c)
        base = f(c)
        off = div_c - g_('f', t) * g_('c', t - 1) - g_('i', t) * g_('g', t)
        upd = lambda th: (th * c - grad - rc * off) / (rc + th)  # noqa: E731
        theta = 1
        cur = c.detach().clone()
        assert not bool(f(cur) > base + torch.sum(grad * (cur - c)) + .5 * theta * _sq(cur - c))
        theta /= 2
        st.S['c'][:, t, :] = upd(theta).clone().detach()

    # -- hidden state (admm.py:439-487; admm.no_dual_y.py:414-449)
    def _hidden(self, st: State, t: int):
        T = st.T
        g_ = lambda k, s: self._slice(st.S, k, s)  # noqa: E731
        h = g_('h', t)
        wy = st.W['out'].clone().detach()
        rh = self._r('h')
        lam = self._slice(st.L, 'h', t)
        a = st.S['a'].clone().detach()
        o = g_('o', t)
        tc = torch.tanh(g_('c', t))
        nd = self.hp.variant == 'no_dual_y'
        if nd:
            grad = rh * ((h @ wy - a) @ wy.T)
        if t < T:
            st.S['h'][:, t, :] = ((rh * o * tc - lam) / rh).clone().detach()
            return None
        ry = self._r('y')
        shift = st.L['y'].clone().detach() / ry if (self.hp.with_dual_y and not nd) else 0

        def f(b):
            return self.comm.allreduce(0.5 * self._r('y') * _sq(b @ wy - a - shift))

        if not nd:
            grad = _autograd(lambda b: 0.5 * self._r('y') * _sq(b @ wy - a - shift), h)
        f_h = f(h)

        def est(b, th):
            return f_h + self.comm.allreduce(torch.sum(grad * (b - h))) + \
                0.5 * th * self.comm.allreduce(_sq(b - h))

        point = (lambda th: grad / th) if nd else \
            (lambda th: (th * h + rh * o * tc - lam - grad) / (th + rh))
        theta, cap = 0.1, 1
        trial = point(theta)
        tests = []
        if self.force is not None:   # the loop below doubles theta once per failing test
            theta = 0.1 * 2 ** self.force[1]
        while self.force is None:
            fb, e = f(trial), est(trial, theta)
            worse = bool(fb > e)
            tests.append((float(fb), float(e), worse))
            if not worse:
                break
            theta *= 2
            trial = point(theta)
            if theta >= cap:
                break
        theta /= 2
        st.S['h'][:, t, :] = ((theta * h + rh * o * tc - lam - grad) / (theta + rh)).clone().detach()
        return {'theta': theta, 'tests': tests}

    # -- a (admm.py:489-502; admm.no_dual_y.py:451-456): uses the GLOBAL batch size
    def _a(self, st: State):
        T = st.T
        ry = self._r('y')
        Bg = st.global_batch
        hw = self._slice(st.S, 'h', T) @ st.W['out'].clone().detach()
        if self.hp.variant == 'admm':
            corr = Bg * st.L['y'].clone().detach() if self.hp.with_dual_y else 0
            st.S['a'] = ((2 * st.y + Bg * ry * hw - corr) / (2 + Bg * ry)).clone().detach()
        else:
            st.S['a'] = ((Bg * ry * hw + 2 * st.y) / (2 + Bg * ry)).clone().detach()

    # -- dual ascent (admm.py:504-539)
    def _duals(self, st: State, t: int):
        T = st.T
        g_ = lambda k, s: self._slice(st.S, k, s)  # noqa: E731
        for q in GATES4:
            z = st.x[:, t - 1, :] @ st.W[f'x2{q}'].clone().detach() + \
                g_('h', t - 1) @ st.W[f'h2{q}'].clone().detach()
            upd = self._slice(st.L, q, t) + self._r(q) * (g_(q, t) - _act(q)(z))
            st.L[q][:, t, :] = upd.clone().detach()
        upd = self._slice(st.L, 'c', t) + self._r('c') * (
            g_('c', t) - (g_('f', t) * g_('c', t - 1) + g_('i', t) * g_('g', t)))
        st.L['c'][:, t, :] = upd.clone().detach()
        if t == T:
            upd = self._slice(st.L, 'h', t) + self._r('h') * (g_('h', t) - g_('o', t) * torch.tanh(g_('c', t)))
            st.L['h'][:, t, :] = upd.clone().detach()

    def _dual_y(self, st: State):
        T = st.T
        hw = self._slice(st.S, 'h', T) @ st.W['out'].clone().detach()
        st.L['y'] = (st.L['y'].clone().detach() + self._r('y') * (st.S['a'].clone().detach() - hw)).clone().detach()


# ----------------------------------------------------------------------------- fp64 arbitration

def fp64_decisions(x, y, W, S, L, hyper: Hyper, global_batch: Optional[int] = None,
                   device: Optional[torch.device] = None) -> dict:
    """ONE step of the restatement above in fp64 from the given (fp32) state, for its
    line-search decisions only: the arbiter of the GPU parity tests and of the golden
    fixtures' ``fp64`` records.

    The reference decides ``f(W + G/2^k) > est`` in fp32 (admm.py:331-336), where both sides
    are sums of ~1e3 that differ in the 7th-8th digit at the exponents taken at C3-like sizes:
    its k there is rounding noise.  In fp64 the same comparisons have ~9 more digits.  Returns
    ``{'weights': [(name, k, margin)], 'theta_h': theta}`` in step order, where margin = the
    smallest |f(beta) - est| / |est - f(W)| of the deciding comparisons (the last failing
    one and the passing one): decisions with margin below ~1e-6 are ties even in fp64."""
    dev = device or x.device
    d = lambda m: {k: v.detach().to(dev, torch.float64) for k, v in m.items()}  # noqa: E731
    st = State(x.to(dev, torch.float64), y.to(dev, torch.float64), d(W), d(S), d(L),
               global_batch or x.shape[0])
    rec = Stepper(hyper.cast(torch.float64), trace_fw=True).step(st)
    out = []
    for r in rec['weights']:
        ms = [abs(a - b) / abs(b - r['f_w']) for a, b, _ in r['tests'][-2:] if b != r['f_w']]
        out.append((r['name'], r['k'], min(ms) if ms else float('inf')))
    return {'weights': out, 'theta_h': rec['hT']['theta'] if rec['hT'] else None,
            'grads': [r['grad'] for r in rec['weights']]}


def fp64_search(q: str, z, tgt, A, G, rho: float, T: int, kmax: int = 64, orig: bool = False):
    """The backtracking search of ``admm.py:316-343`` for ONE gate weight, in fp64, from given
    inputs: z [R, H] the pre-activations at W, tgt [R, H] = dual/rho + gate, A [R, K] the rows
    of the side's input (X or H_prev), G [K, H] the (rho-scaled) gradient, i.e. the search
    direction.  With beta - W = G/theta = s G the test ``f(beta) > est(beta, theta)`` reads
    f(W + s G) - f(W) > (1 + T/2) |G|^2 s.  G is grad f(W) (admm.py:302-312), so
    f(W + s G) - f(W) = s |G|^2 + r(s) and the test is r(s) > (T/2) |G|^2 s with the remainder
    r(s) = 0.5 rho sum[D^2 + 2 d0 (D - s phi'(z) q)], D = phi(z + s q) - phi(z), q = A G,
    d0 = phi(z) - tgt -- the form the library evaluates (k_select).  In it d0 enters only at
    second order, so the decision does not depend on the rounding of phi(z) - tgt.

    Returns (k, margin, eps_g): margin = the smallest |r - (T/2)|G|^2 s| / ((T/2)|G|^2 s) of the
    deciding comparisons (the last failing one and the passing one); eps_g = |G - rho A^T R| / |G|
    with R = (phi(z) - tgt) phi'(z) in fp64 from the same z and tgt: how much of G itself is the
    fp32 rounding of the residual (phi(z) - tgt is a difference of O(1) numbers that agree to
    ~1e-7 when the ADMM residuals are that small) -- recorded, it is the same in the reference.

    orig=True also evaluates the reference's test in its ORIGINAL form with the same G,
    f(W + s G) - f(W) > (1 + T/2) |G|^2 s, f in fp64 from the same z and tgt
    (f(W + s G) - f(W) = 0.5 rho sum[D^2 + 2 d0 D]), and returns (k, margin, eps_g, k_orig,
    margin_orig).  The two forms differ by s (<grad f, G> - |G|^2): zero when G is the exact
    gradient of the fp64 objective, of relative size ~eps_g (2/T) against the threshold otherwise."""
    act = torch.tanh if q == 'g' else torch.sigmoid
    z, tgt, A, G = (v.to(torch.float64) for v in (z, tgt, A, G))
    p0 = act(z)
    d0 = p0 - tgt
    dphi = 1.0 - p0 * p0 if q == 'g' else p0 * (1.0 - p0)
    g_exact = rho * (A.T @ (d0 * dphi))
    gn = float(G.norm())
    # G == 0 exactly (step 1's x side: the stored gates are phi(z) bit for bit): k = 0 is exact
    eps_g = float((G - g_exact).norm()) / gn if gn > 0 else 0.0
    del g_exact
    qd = A @ G
    lin = dphi * qd
    c = 0.5 * T * float((G * G).sum())
    tests = []
    for k in range(kmax):
        s = 2.0 ** -k
        D = act(z + qd * s) - p0
        rem = 0.5 * rho * float((D * D + 2.0 * d0 * (D - s * lin)).sum())
        est = c * s
        tests.append((rem, est))
        if not rem > est:
            break
    ms = [abs(a - b) / b for a, b in tests[-2:] if b > 0]
    out = (len(tests) - 1, (min(ms) if ms else float('inf')), eps_g)
    if not orig:
        return out
    c1 = (1.0 + 0.5 * T) * float((G * G).sum())
    tests = []
    for k in range(kmax):
        s = 2.0 ** -k
        D = act(z + qd * s) - p0
        inc = 0.5 * rho * float((D * D + 2.0 * d0 * D).sum())
        tests.append((inc, c1 * s))
        if not inc > c1 * s:
            break
    ms = [abs(a - b) / b for a, b in tests[-2:] if b > 0]
    return out + (len(tests) - 1, (min(ms) if ms else float('inf')))
