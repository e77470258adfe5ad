"""Worker for tests/test_gpu_dist.py, launched with torch.distributed.run.

Backend (env ADMM_DIST_BACKEND): ``nccl`` = RCCL inside libadmmlstm.so, one GPU per rank;
``gloo`` = the library's host-staged all-reduce (admm_set_comm_host), which lets several
ranks share one GPU.  Shape (env ADMM_DIST_SHAPE = "B_per_rank,T,D,H", variant in
ADMM_DIST_VARIANT).

Each rank owns a contiguous shard of one global synthetic batch and steps an
ADMMBasedOptimizer(distributed=True).  Every rank also steps a single-process optimizer
over the whole global batch on its own GPU; the sharded run must reproduce it (exactly at
world 1, where the all-reduces are identities; to fp32 summation order otherwise).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, 'admm-lstm_amd'), ROOT):
    sys.path.insert(0, p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    rank, world = int(os.environ['RANK']), int(os.environ['WORLD_SIZE'])
    backend = os.environ.get('ADMM_DIST_BACKEND', 'nccl')
    dev = torch.device('cuda', int(os.environ.get('LOCAL_RANK', '0')) % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    if backend == 'nccl':
        dist.init_process_group('nccl', device_id=dev)
    else:
        dist.init_process_group('gloo')
    import importlib.util
    if os.environ.get('ADMM_DIST_VARIANT', 'admm') == 'no_dual_y':
        spec = importlib.util.spec_from_file_location('admm_nd', os.path.join(ROOT, 'admm-lstm_amd', 'admm.no_dual_y.py'))
        admm = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(admm)
    else:
        import admm
    from blocks.lstm import LSTM
    from parameters import example_parameter_dictionary
    pd = example_parameter_dictionary['GoogleStock']
    per, T, D, H = (int(v) for v in os.environ.get('ADMM_DIST_SHAPE', '256,8,4,32').split(','))
    Bg, steps = per * world, int(os.environ.get('ADMM_DIST_STEPS', '3'))
    g = torch.Generator().manual_seed(1234)
    x = torch.rand(Bg, T, D, generator=g)
    y = 0.8 * x.mean((1, 2)).unsqueeze(1) + 0.1 * torch.rand(Bg, 1, generator=g)
    xs, ys = x[rank * per:(rank + 1) * per], y[rank * per:(rank + 1) * per]

    torch.manual_seed(0)
    m_sh = LSTM(D, H, 1).to(dev)
    opt_sh = admm.ADMMBasedOptimizer(m_sh, (xs.to(dev), ys.to(dev)), pd, verbose=False, distributed=True)
    torch.manual_seed(0)
    m_1 = LSTM(D, H, 1).to(dev)
    opt_1 = admm.ADMMBasedOptimizer(m_1, (x.to(dev), y.to(dev)), pd, verbose=False)
    for _ in range(steps):
        opt_sh.step()
        opt_1.step()
    torch.cuda.synchronize()
    st_sh, st_1 = opt_sh.last_step_stats(), opt_1.last_step_stats()
    k_sh, k_1 = list(st_sh['k'].values()), list(st_1['k'].values())
    # the a update uses the global batch (admm.py:496-502)
    da = float((opt_sh.gates['a'] - opt_1.gates['a'][rank * per:(rank + 1) * per]).abs().max())
    dw = max(float((a - b).abs().max()) for a, b in zip(m_sh.parameters(), m_1.parameters()))
    ds = max(float((opt_sh.gates[q] - opt_1.gates[q][rank * per:(rank + 1) * per]).abs().max())
             for q in ('i', 'f', 'g', 'o', 'c', 'h'))
    exact = world == 1
    same_theta = st_sh['theta_h'] == st_1['theta_h']
    if exact:
        ok = dw == 0.0 and ds == 0.0 and da == 0.0 and k_sh == k_1 and same_theta
    else:   # sums in a different order: fp32 rounding only, same decisions
        ok = dw <= 1e-5 and ds <= 1e-5 and da <= 1e-5 and k_sh == k_1 and same_theta
    flag = torch.tensor([1 if ok else 0], device=dev if backend == 'nccl' else 'cpu')
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    if rank == 0:
        print(f'DIST {"OK" if int(flag.item()) else "FAIL"} world={world} max|dW|={dw:.3e} '
              f'max|dS|={ds:.3e} max|da|={da:.3e} backend={backend} k_sharded={k_sh} k_single={k_1}', flush=True)
    dist.destroy_process_group()
    sys.exit(0 if int(flag.item()) else 1)


if __name__ == '__main__':
    main()
