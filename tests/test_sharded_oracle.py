"""The batch-sharded decomposition of the step on 2 gloo ranks.

Every cross-sample coupling of the step is a sum over the batch: the wy gradient, the
weight gradients G, the line-search objective values, the h_T search sums; plus the
global batch size in the a-update.  The oracle routes exactly those through an
all-reduce (``Stepper(comm=...)``).  Running it on 2 ranks that each hold half of the
rows must reproduce the 1-rank full-batch run -- the same decomposition the HIP path
implements with RCCL all-reduces (admm_host.hip).
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class _GlooComm:
    def __init__(self):
        self.world_size = dist.get_world_size()

    def allreduce(self, t):
        t = t.detach().clone()
        dist.all_reduce(t)
        return t


def _problem():
    g = torch.Generator().manual_seed(1234)
    B, T, D, H = 64, 5, 3, 12
    x = torch.rand(B, T, D, generator=g)
    y = 0.8 * x.mean((1, 2)).unsqueeze(1) + 0.1 * torch.rand(B, 1, generator=g)
    return x, y, D, H


def _run(rank, world, port, variant, steps, out):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, 'admm-lstm_amd'))
    from oracle import admm_oracle as O
    from parameters import example_parameter_dictionary
    torch.set_num_threads(1)
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    x, y, D, H = _problem()
    per = x.shape[0] // world
    xs, ys = x[rank * per:(rank + 1) * per], y[rank * per:(rank + 1) * per]
    torch.manual_seed(0)
    W = O.init_weights(D, H, 1)
    st = O.init_state(xs, ys, W, global_batch=x.shape[0])
    stp = O.Stepper(O.Hyper.from_dict(example_parameter_dictionary['GoogleStock'], variant), comm=_GlooComm())
    for _ in range(steps):
        stp.step(st)
    # numpy copies: tensors sent through a Queue need the sender alive (shared memory)
    if rank == 0:
        out['W'] = {k: v.numpy().copy() for k, v in st.W.items()}
    out[f'S{rank}'] = {k: v.numpy().copy() for k, v in st.S.items()}
    dist.destroy_process_group()


def _worker(rank, world, port, variant, steps, q):
    out = {}
    _run(rank, world, port, variant, steps, out)
    q.put((rank, out))


@pytest.mark.parametrize('variant', ['admm', 'no_dual_y'])
def test_two_gloo_ranks_equal_one(variant):
    from oracle import admm_oracle as O
    from parameters import example_parameter_dictionary
    steps = 3
    x, y, D, H = _problem()
    torch.manual_seed(0)
    W = O.init_weights(D, H, 1)
    st = O.init_state(x, y, W)
    stp = O.Stepper(O.Hyper.from_dict(example_parameter_dictionary['GoogleStock'], variant))
    for _ in range(steps):
        stp.step(st)
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    with socket.socket() as sk:   # a free port (parallel test workers must not collide)
        sk.bind(('127.0.0.1', 0))
        port = sk.getsockname()[1]
    procs = [ctx.Process(target=_worker, args=(r, 2, port, variant, steps, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res = {r: {k: {n: torch.from_numpy(a) for n, a in d.items()} for k, d in o.items()} for r, o in res.items()}
    for k, v in res[0]['W'].items():
        assert torch.allclose(v, st.W[k], rtol=1e-4, atol=1e-6), k
    per = x.shape[0] // 2
    for r in range(2):
        for q_ in ('i', 'f', 'g', 'o', 'c', 'h'):
            part = st.S[q_][r * per:(r + 1) * per]
            assert torch.allclose(res[r][f'S{r}'][q_], part, atol=1e-5), (r, q_)
        assert torch.allclose(res[r][f'S{r}']['a'], st.S['a'][r * per:(r + 1) * per], atol=1e-5)
    assert O.mse(x, y, res[0]['W']) == pytest.approx(O.mse(x, y, st.W), rel=1e-5)
