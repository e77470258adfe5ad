"""RCCL path of the sharded step on the GPU box: one torchrun rank
with distributed=True must reproduce the single-process step exactly (all-reduces over one
rank are identities), which exercises admm_comm_unique_id / admm_set_comm and every
collective of admm_step.  N > 1 ranks are the driver's (one GPU per rank)."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _launch(world, backend, shape, variant='admm', extra_env=None):
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={world}',
           '--master-addr=127.0.0.1', f'--master-port={_free_port()}',
           os.path.join(ROOT, 'tests', '_dist_worker.py')]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY='0', ADMM_DIST_BACKEND=backend, ADMM_DIST_SHAPE=shape,
               ADMM_DIST_VARIANT=variant, OMP_NUM_THREADS='4', **(extra_env or {}))
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0 and 'DIST OK' in out, out[-3000:]
    print([ln for ln in out.splitlines() if 'DIST' in ln])


def test_rccl_world1_matches_single_process():
    _launch(1, 'nccl', '256,8,4,32')


def test_rccl_world1_fast_path():
    _launch(1, 'nccl', '512,6,16,256')


def test_rccl_world1_step_graph():
    """ADMM_GRAPH=1 with RCCL: the steady-state step, its all-reduces included, captured into one HIP
    graph and replayed (the worker steps enough times to replay it)."""
    _launch(1, 'nccl', '512,6,16,256', extra_env={'ADMM_GRAPH': '1', 'ADMM_DIST_STEPS': '6'})


@pytest.mark.parametrize('shape,variant', [
    ('512,6,16,256', 'admm'),        # fast path: persistent sweep, split3, row-pair trials
    ('200,5,16,64', 'admm'),         # persistent sweep at H = 64, ragged row blocks
    ('96,4,3,40', 'no_dual_y'),      # generic kernels, the variant's h_T / wy forms
])
def test_host_comm_world2_matches_single_process(shape, variant):
    _launch(2, 'gloo', shape, variant)
