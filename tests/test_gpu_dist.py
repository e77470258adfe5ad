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


def test_rccl_world1_matches_single_process():
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node=1',
           '--master-addr=127.0.0.1', f'--master-port={_free_port()}',
           os.path.join(ROOT, 'tests', '_dist_worker.py')]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY='0')
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0 and 'DIST OK' in out, out[-3000:]
