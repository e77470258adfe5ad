"""Worker for tests/test_gpu_dist.py, launched with torch.distributed.run (RCCL backend).

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
    dev = torch.device('cuda', int(os.environ.get('LOCAL_RANK', '0')))
    torch.cuda.set_device(dev)
    dist.init_process_group('nccl', device_id=dev)
    import admm
    from blocks.lstm import LSTM
    from parameters import example_parameter_dictionary
    pd = example_parameter_dictionary['GoogleStock']
    Bg, T, D, H, steps = 256 * world, 8, 4, 32, 3
    g = torch.Generator().manual_seed(1234)
    x = torch.rand(Bg, T, D, generator=g)
    y = 0.8 * x.mean((1, 2)).unsqueeze(1) + 0.1 * torch.rand(Bg, 1, generator=g)
    per = Bg // world
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
    k_sh = list(opt_sh.last_step_stats()['k'].values())
    k_1 = list(opt_1.last_step_stats()['k'].values())
    dw = max(float((a - b).abs().max()) for a, b in zip(m_sh.parameters(), m_1.parameters()))
    ds = max(float((opt_sh.gates[q] - opt_1.gates[q][rank * per:(rank + 1) * per]).abs().max())
             for q in ('i', 'f', 'g', 'o', 'c', 'h'))
    exact = world == 1
    ok = (dw == 0.0 and ds == 0.0 and k_sh == k_1) if exact else (dw <= 1e-5 and ds <= 1e-5)
    flag = torch.tensor([1 if ok else 0], device=dev)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    if rank == 0:
        print(f'DIST {"OK" if int(flag.item()) else "FAIL"} world={world} max|dW|={dw:.3e} '
              f'max|dS|={ds:.3e} k_sharded={k_sh} k_single={k_1}', flush=True)
    dist.destroy_process_group()
    sys.exit(0 if int(flag.item()) else 1)


if __name__ == '__main__':
    main()
