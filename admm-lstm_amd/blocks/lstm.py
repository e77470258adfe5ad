"""LSTM-Linear model container for ADMM training (drop-in for ``blocks/lstm.py``).

Same constructor, parameter names, registration order and seeded initialisation as
the reference (``blocks/lstm.py:12-29``: randn for x2q [D,H] / h2q [H,H] per gate
i,f,g,o, then out [H,O]; then ``xavier_normal_`` over ``parameters()``), so
``torch.manual_seed(s); LSTM(D, H, O)`` yields the reference's weights bit for bit.

``init_gate_variables`` / ``forward`` (``blocks/lstm.py:43-46, 65-88``) run the
gfx950 time-step kernel of libadmmlstm.so (``admm_forward``); they require HIP
device tensors.  ``with_grad=True`` (``blocks/lstm.py:48-63``) is the autograd
path the reference uses for its gradient-descent baselines; it is plain PyTorch.
"""
from __future__ import annotations

import ctypes
from typing import Dict

import torch
from torch import nn
from torch.nn import init

GATES4 = ('i', 'f', 'g', 'o')


class LSTM(nn.Module):
    def __init__(self, input_size: int, hidden_size: int, output_size: int, with_grad: bool = False) -> None:
        super().__init__()
        self.input_size, self.hidden_size, self.output_size = input_size, hidden_size, output_size
        self.init_parameters()
        self.sigmoid, self.tanh = nn.Sigmoid(), nn.Tanh()
        self.with_grad = with_grad

    def init_parameters(self) -> None:
        D, H, O = self.input_size, self.hidden_size, self.output_size
        for q in GATES4:
            self.register_parameter(f'x2{q}', nn.Parameter(torch.randn(D, H)))
            self.register_parameter(f'h2{q}', nn.Parameter(torch.randn(H, H)))
        self.register_parameter('out', nn.Parameter(torch.randn(H, O)))
        for p in self.parameters():
            init.xavier_normal_(p)

    # -- accessors (blocks/lstm.py:31-41): getters return detached copies
    def get_weight(self, map_from: str, map_to: str) -> torch.Tensor:
        return getattr(self, f'{map_from}2{map_to}').clone().detach()

    def set_weight(self, map_from: str, map_to: str, value: torch.Tensor) -> None:
        setattr(self, f'{map_from}2{map_to}', nn.Parameter(value.clone().detach()))

    def get_wy(self) -> torch.Tensor:
        return self.out.clone().detach()

    def set_wy(self, value: torch.Tensor) -> None:
        self.out = nn.Parameter(value)

    # -- forward
    def forward(self, x: torch.Tensor, c: torch.Tensor = None, h: torch.Tensor = None) -> torch.Tensor:
        if self.with_grad:
            return self.grad_forward(x, c, h)
        if c is None and h is None:
            return _native_predict(self, x)
        return self.init_gate_variables(x, c, h)['a']

    def grad_forward(self, x: torch.Tensor, c: torch.Tensor = None, h: torch.Tensor = None) -> torch.Tensor:
        assert x.size(2) == self.input_size
        B, T, _ = x.shape
        c = torch.zeros(B, self.hidden_size, dtype=x.dtype, device=x.device) if c is None else c
        h = torch.zeros(B, self.hidden_size, dtype=x.dtype, device=x.device) if h is None else h
        for t in range(T):
            xt = x[:, t, :]
            pre = {q: xt @ getattr(self, f'x2{q}') + h @ getattr(self, f'h2{q}') for q in GATES4}
            c = self.sigmoid(pre['f']) * c + self.sigmoid(pre['i']) * self.tanh(pre['g'])
            h = self.sigmoid(pre['o']) * self.tanh(c)
        return h @ self.out

    @torch.no_grad()
    def init_gate_variables(self, x: torch.Tensor, c: torch.Tensor = None, h: torch.Tensor = None,
                            z_out: torch.Tensor = None) -> Dict[str, torch.Tensor]:
        """Gate trajectories i,f,g,o,c,h as [B,T+1,H] (index 0 = initial state) and
        a = h_T @ out.  Passed-in c/h [B,T+1,H] are used as the buffers, as upstream."""
        assert x.size(2) == self.input_size
        from admm_amd import _native as N
        lib = N.load()
        N.require_device(x, 'x')
        B, T, _ = x.shape
        H, O = self.hidden_size, self.output_size
        kw = dict(dtype=torch.float32, device=x.device)
        out = {q: torch.zeros(B, T + 1, H, **kw) for q in GATES4}
        out['c'] = c if c is not None else torch.zeros(B, T + 1, H, **kw)
        out['h'] = h if h is not None else torch.zeros(B, T + 1, H, **kw)
        for k in ('c', 'h'):
            # the library writes B rows with a row stride of (T+1)*H into these buffers
            if not (tuple(out[k].shape) == (B, T + 1, H) and out[k].is_contiguous()
                    and out[k].dtype == torch.float32 and out[k].device == x.device):
                raise ValueError(f'{k} must be a contiguous float32 tensor of shape {(B, T + 1, H)} on '
                                 f'{x.device} (got {tuple(out[k].shape)} {out[k].dtype} on {out[k].device})')
        a = torch.empty(B, O, **kw)
        xc = x.contiguous().float()
        wx, wh, wy = _weight_ptrs(self, x.device)
        gates = (ctypes.c_void_p * 6)(*[out[q].data_ptr() for q in ('i', 'f', 'g', 'o', 'c', 'h')])
        N.check(lib.admm_forward(N.ptr(xc), B, T, self.input_size, H, O, wx, wh, wy, gates, None, None,
                                 N.ptr(z_out) if z_out is not None else None, N.ptr(a), N.stream_handle(x.device)),
                'admm_forward')
        out['a'] = a
        return out


def _weight_ptrs(model: LSTM, dev: torch.device):
    from admm_amd import _native as N
    ps = []
    for name in [f'x2{q}' for q in GATES4] + [f'h2{q}' for q in GATES4] + ['out']:
        p = getattr(model, name)
        N.require_device(p, f'model.{name}')
        if p.device != dev or p.dtype != torch.float32 or not p.is_contiguous():
            raise ValueError(f'model.{name} must be a contiguous float32 tensor on {dev}')
        ps.append(p.data_ptr())
    return (ctypes.c_void_p * 4)(*ps[0:4]), (ctypes.c_void_p * 4)(*ps[4:8]), ctypes.c_void_p(ps[8])


@torch.no_grad()
def _native_predict(model: LSTM, x: torch.Tensor) -> torch.Tensor:
    """``forward`` without keeping the gate trajectories: ping-pong h/c scratch."""
    from admm_amd import _native as N
    lib = N.load()
    N.require_device(x, 'x')
    assert x.size(2) == model.input_size
    B, T, _ = x.shape
    kw = dict(dtype=torch.float32, device=x.device)
    hs = torch.empty(2, B, model.hidden_size, **kw)
    cs = torch.empty(2, B, model.hidden_size, **kw)
    a = torch.empty(B, model.output_size, **kw)
    xc = x.contiguous().float()
    wx, wh, wy = _weight_ptrs(model, x.device)
    N.check(lib.admm_forward(N.ptr(xc), B, T, model.input_size, model.hidden_size, model.output_size, wx, wh, wy,
                             None, N.ptr(hs), N.ptr(cs), None, N.ptr(a), N.stream_handle(x.device)), 'admm_forward')
    return a
