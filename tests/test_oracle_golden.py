"""Pin the CPU oracle (oracle/admm_oracle.py) to the reference's golden fixtures.

The fixtures were captured from the reference itself (tests/golden/make_golden.py).
The oracle keeps the reference's op structure, so in one process on the CPU it
must reproduce them BIT-EXACTLY: weights, losses, line-search decisions and their
operands, and the full primal/dual state.
"""
import pytest
import torch

from golden_io import (ALL, COMPACT_ORACLE, COMPACT_REF, FULL, GATES6, LONG, PERTURBED, WEIGHT_NAMES, Golden,
                       perturb_state)
from oracle import admm_oracle as O

FAST = [n for n in ALL if not n.startswith('t1_')] + ['t1_gstock']


def _run(g: Golden, steps=None):
    torch.manual_seed(0)
    W = O.init_weights(g.D, g.H, g.O)
    st = O.init_state(g.x, g.y, W)
    stp = O.Stepper(O.Hyper.from_dict(g.params, g.variant, g.with_dual_y))
    for s in range(1, (steps or g.steps) + 1):
        rec = stp.step(st)
        yield s, st, rec


@pytest.mark.parametrize('name', ALL)
def test_seeded_init_matches(name):
    g = Golden(name)
    torch.manual_seed(0)
    W = O.init_weights(g.D, g.H, g.O)
    for k in WEIGHT_NAMES:
        assert torch.equal(W[k], g.t(f'w0_{k}')), k
    assert O.mse(g.x, g.y, W) == g.losses[0]


@pytest.mark.parametrize('name', FULL)
def test_initial_state_matches(name):
    g = Golden(name)
    st = O.init_state(g.x, g.y, g.weights(0))
    S, L = g.state(0)
    for q in GATES6:
        assert torch.equal(st.S[q], S[q]), q
        assert torch.equal(st.L[q], L[q]), q
    assert torch.equal(st.S['a'], S['a'])


@pytest.mark.parametrize('name', FAST)
def test_trajectory_bit_exact(name):
    g = Golden(name)
    for s, st, rec in _run(g, steps=min(g.steps, 8)):
        assert [r['k'] for r in rec['weights']] == g.ks(s), f'step {s}'
        for r, ref in zip(rec['weights'], g.searches[s - 1]['weights']):
            assert [(a, b, w) for a, b, w in r['tests']] == [tuple(v) for v in ref]
        assert [tuple(v) for v in g.searches[s - 1]['hT']] == [tuple(v) for v in rec['hT']['tests']]
        for k in WEIGHT_NAMES:
            assert torch.equal(st.W[k], g.t(f'w{s}_{k}')), (s, k)
        assert O.mse(g.x, g.y, st.W) == g.losses[s]
        if g.full_state:
            S, L = g.state(s)
            for q in GATES6:
                assert torch.equal(st.S[q], S[q]), (s, q)
                assert torch.equal(st.L[q], L[q]), (s, q)
            assert torch.equal(st.S['a'], S['a'])
            assert torch.equal(st.L['y'], L['y'])


@pytest.mark.parametrize('name', PERTURBED)
def test_perturbed_trajectory_bit_exact(name):
    """The t4_pert_* fixtures: the reference stepped from a perturbed state (golden_io.perturb_state)
    at H = 256 and H = 512, the sizes of the library's fast weight-stage kernels.  The oracle from the
    same perturbed state reproduces every weight, search comparison and loss bit for bit."""
    g = Golden(name)
    torch.manual_seed(0)
    W = O.init_weights(g.D, g.H, g.O)
    st = O.init_state(g.x, g.y, W)
    perturb_state(st.S, st.L, g.B, g.T, g.H, g.perturb['seed'], g.perturb['scale'])
    stp = O.Stepper(O.Hyper.from_dict(g.params, g.variant, g.with_dual_y))
    for s in range(1, g.steps + 1):
        rec = stp.step(st)
        assert [r['k'] for r in rec['weights']] == g.ks(s), f'step {s}'
        for r, ref in zip(rec['weights'], g.searches[s - 1]['weights']):
            assert [(a, b, w) for a, b, w in r['tests']] == [tuple(v) for v in ref]
        for k in WEIGHT_NAMES:
            assert torch.equal(st.W[k], g.t(f'w{s}_{k}')), (s, k)
        assert O.mse(g.x, g.y, st.W) == g.losses[s]


@pytest.mark.parametrize('name', FULL)
def test_teacher_forced_step(name):
    """From the reference's state after step k, one oracle step gives its state after k+1."""
    g = Golden(name)
    stp = O.Stepper(O.Hyper.from_dict(g.params, g.variant, g.with_dual_y))
    for k in range(g.steps):
        S, L = g.state(k)
        st = O.State(g.x, g.y, g.weights(k), S, L, g.B)
        stp.step(st)
        S1, L1 = g.state(k + 1)
        for q in GATES6:
            assert torch.equal(st.S[q], S1[q]) and torch.equal(st.L[q], L1[q]), (k, q)
        for n in WEIGHT_NAMES:
            assert torch.equal(st.W[n], g.t(f'w{k + 1}_{n}')), (k, n)


def test_dead_searches_are_dead():
    """The wy and c searches never iterate in the reference: pinned by the capture."""
    for name in ALL:
        g = Golden(name)
        for rec in g.searches:
            assert rec['wy_true'] == 0 and rec['c_true'] == 0
            assert rec['c_count'] == g.T


def test_fixture_sources():
    """Every fixture says who made it: the reference (tests/golden/make_golden.py) for all
    but c5g, which the oracle made (tools/make_c5g.py) and which is therefore only an oracle-consistency
    case (test_gpu_fullsize.test_fullsize_matches_oracle_fixture)."""
    assert COMPACT_ORACLE == ['c5g']
    assert set(COMPACT_REF) == {'c3', 'c5_1gpu', 'c4g'}
    assert set(LONG) == {'c3_25', 'c3_25_t4', 'c5_10'}
    for n in ALL + PERTURBED + COMPACT_REF + LONG:
        g = Golden(n)
        assert g.source == 'reference', n
        assert g.meta.get('generator', 'tests/golden/make_golden.py').startswith('tests/golden/make_golden.py'), n


def test_long_capture_reproduces_c3():
    """The 25-step capture of the bench's trajectory (c3_25) repeats the 5-step c3 capture bit for bit over
    their common steps (both the reference on 8 threads in this container): same losses, exponents and
    weights.  c3_25_t4 (4 threads) is the reference's own spread, compared in tests/test_gpu_trajectory.py."""
    g25, g5 = Golden('c3_25'), Golden('c3')
    assert g25.threads == g5.threads == 8 and Golden('c3_25_t4').threads == 4
    assert g25.compact['x_sha256'] == g5.compact['x_sha256'] and g25.compact['y_sha256'] == g5.compact['y_sha256']
    assert g25.losses[:6] == g5.losses
    for s in range(1, 6):
        assert g25.ks(s) == g5.ks(s), s
        for k in WEIGHT_NAMES:
            a, b = g25.t(f'w{s}_{k}'), g5.t(f'w{s}_{k}')
            if a.shape == b.shape:
                assert torch.equal(a, b), (s, k)


@pytest.mark.parametrize('name', ['t0_admm', 't0_nodualy', 't2_c2'])
def test_forced_replay_bit_exact(name):
    """Stepper.force (replay given line-search outcomes instead of searching; the oracle's twin of the
    library's admm_debug_force) with the reference's own recorded outcomes reproduces the reference
    bit for bit: the searches only pick theta, and forcing sets the theta their loops ended with."""
    g = Golden(name)
    torch.manual_seed(0)
    W = O.init_weights(g.D, g.H, g.O)
    st = O.init_state(g.x, g.y, W)
    stp = O.Stepper(O.Hyper.from_dict(g.params, g.variant, g.with_dual_y))
    for s in range(1, min(g.steps, 4) + 1):
        stp.force = (g.ks(s), sum(1 for _, _, r in g.searches[s - 1]['hT'] if r))
        rec = stp.step(st)
        assert [r['k'] for r in rec['weights']] == g.ks(s) and all(not r['tests'] for r in rec['weights'])
        for k in WEIGHT_NAMES:
            assert torch.equal(st.W[k], g.t(f'w{s}_{k}')), (s, k)
        assert O.mse(g.x, g.y, st.W) == g.losses[s]
