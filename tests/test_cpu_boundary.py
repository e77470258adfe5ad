"""CPU-side checks of the drop-in boundary (no GPU compute):
* libadmmlstm.so loads and exports every entry point include/admm_lstm.h declares;
* the Python surface mirrors the reference: seeded LSTM init, parameter dictionaries,
  constructor validation (SystemExit(1) via log_assert/error, admm.py:92-162),
  and a loud failure when no HIP device / no CPU path is available.
"""
import ctypes
import os
import re

import pytest
import torch

from golden_io import ALL, Golden

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_functions():
    src = open(os.path.join(ROOT, 'include', 'admm_lstm.h')).read()
    src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
    return sorted(set(re.findall(r'\b(admm_[a-z_0-9]+)\s*\(', src)))


def test_library_exports_every_declared_symbol():
    from admm_amd import _native as N
    lib = N.load()
    declared = _declared_functions()
    assert len(declared) >= 15
    for name in declared:
        assert hasattr(lib, name), name
        assert name in N.EXPORTS, f'{name} has no ctypes signature in _native.py'
    assert lib.admm_abi_version() == N.ABI_VERSION
    assert b'gfx950' in lib.admm_build_info()


def test_create_rejects_unsupported_output_width():
    """O is bounded only by the h_T kernels' LDS row (4 waves x O floats): O <= 4096.  Larger
    widths fail in admm_create's argument check, before any device call, with a message."""
    from admm_amd import _native as N
    lib = N.load()
    p = N.AdmmParams()
    for i in range(7):
        p.rho[i] = 1.0
    ctx = ctypes.c_void_p()
    d = N.AdmmDims(64, 64, 4, 3, 16, 5000)
    rc = lib.admm_create(ctypes.byref(d), ctypes.byref(p), 0, ctypes.byref(ctx))
    assert rc != 0 and not ctx.value
    assert b'output_size 5000 > 4096' in lib.admm_last_error()


def test_struct_layouts_match_header():
    from admm_amd import _native as N
    assert ctypes.sizeof(N.AdmmDims) == 32
    assert ctypes.sizeof(N.AdmmParams) == 4 * (7 + 4 + 4 + 1) + 8
    assert ctypes.sizeof(N.AdmmBuffers) == 8 * (2 + 4 + 4 + 1 + 6 + 6 + 2)


def test_c_abi_rejects_bad_arguments_without_gpu():
    from admm_amd import _native as N
    lib = N.load()
    ctx = ctypes.c_void_p()
    d = N.AdmmDims(0, 0, 4, 1, 8, 1)
    p = N.AdmmParams()
    assert lib.admm_create(ctypes.byref(d), ctypes.byref(p), 0, ctypes.byref(ctx)) == -1
    assert b'positive' in lib.admm_last_error()
    d = N.AdmmDims(8, 4, 4, 1, 8, 1)     # global batch < local batch
    assert lib.admm_create(ctypes.byref(d), ctypes.byref(p), 0, ctypes.byref(ctx)) == -1
    assert lib.admm_step(None, None) == -1


@pytest.mark.parametrize('name', ['t0_uniform', 't2_c2', 't0_yahoo'])
def test_seeded_lstm_init_matches_reference(name):
    from blocks.lstm import LSTM
    g = Golden(name)
    torch.manual_seed(0)
    m = LSTM(g.D, g.H, g.O)
    assert [n for n, _ in m.named_parameters()] == list(g.weights(0))
    for n, p in m.named_parameters():
        assert torch.equal(p.detach(), g.t(f'w0_{n}')), n


def test_parameter_dictionaries_match_fixtures():
    from parameters import default_epoch, example_parameter_dictionary
    assert default_epoch == 100
    for name in ALL:
        g = Golden(name)
        assert example_parameter_dictionary[g.param_set] == g.params


def _make(x_shape=(16, 4, 2), y_shape=(16, 1), D=2, H=8, O=1, params='GoogleStock', **kw):
    import admm
    from blocks.lstm import LSTM
    from parameters import example_parameter_dictionary as E
    torch.manual_seed(0)
    pd = E[params] if isinstance(params, str) else params
    return admm.ADMMBasedOptimizer(LSTM(D, H, O), (torch.rand(*x_shape), torch.rand(*y_shape)), pd, **kw)


@pytest.mark.parametrize('kwargs', [
    dict(y_shape=(15, 1)),                       # batch mismatch (admm.py:99-101)
    dict(x_shape=(16, 4, 3)),                    # feature mismatch (admm.py:103-106)
    dict(params={'rho': {}}),                    # beta dict missing (admm.py:120-123)
    dict(params={'beta': {'wi': 1e-7}}),         # key wy missing (admm.py:131-135)
    dict(params={'beta': {k: (-1.0 if k == 'vf' else 1e-7) for k in
                          ('wy', 'wi', 'wf', 'wg', 'wo', 'vi', 'vf', 'vg', 'vo')},
                 'rho': {k: 1.0 for k in 'ifgochy'}}),     # negative beta
    dict(params={'beta': {k: 1e-7 for k in ('wy', 'wi', 'wf', 'wg', 'wo', 'vi', 'vf', 'vg', 'vo')}}),  # no rho
    dict(params={'beta': {k: 1e-7 for k in ('wy', 'wi', 'wf', 'wg', 'wo', 'vi', 'vf', 'vg', 'vo')},
                 'rho': {k: 1.0 for k in 'ifgoch'}}),      # rho y missing
    dict(params={'beta': {k: 1e-7 for k in ('wy', 'wi', 'wf', 'wg', 'wo', 'vi', 'vf', 'vg', 'vo')},
                 'rho': {k: ('1' if k == 'c' else 1.0) for k in 'ifgochy'}}),  # non-numeric rho
])
def test_constructor_validation_exits(kwargs, tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    with pytest.raises(SystemExit) as e:
        _make(**kwargs)
    assert e.value.code == 1


def test_no_cpu_execution_path(tmp_path, monkeypatch):
    """Valid arguments on a machine without a HIP device: loud RuntimeError, no fallback."""
    monkeypatch.chdir(tmp_path)
    if torch.cuda.is_available():
        pytest.skip('GPU present')
    with pytest.raises(RuntimeError, match='HIP device'):
        _make()
    from blocks.lstm import LSTM
    with pytest.raises(RuntimeError, match='HIP device'):
        LSTM(2, 8, 1)(torch.rand(4, 3, 2))


def test_empty_dictionary_defaults_like_reference(tmp_path, monkeypatch, capsys):
    """admm.py:111-119: warning, GoogleStock values keyed by the dictionary's own names."""
    monkeypatch.chdir(tmp_path)
    if torch.cuda.is_available():
        pytest.skip('GPU present')
    with pytest.raises(RuntimeError):
        _make(params={})
    assert 'Parameter dictionary is empty' in capsys.readouterr().out


def test_grad_forward_is_plain_autograd():
    """with_grad=True (blocks/lstm.py:48-63) is the autograd path of the gradient baselines."""
    from blocks.lstm import LSTM
    from oracle import admm_oracle as O
    torch.manual_seed(0)
    m = LSTM(3, 6, 2, with_grad=True)
    x = torch.rand(5, 4, 3)
    out = m(x)
    out.sum().backward()
    W = {n: p.detach() for n, p in m.named_parameters()}
    assert torch.allclose(out.detach(), O.predict(x, W), atol=1e-6)
    assert m.x2i.grad is not None
