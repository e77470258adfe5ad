import sys, os
sys.path.insert(0, '/root/repo/admm-lstm_amd'); sys.path.insert(0, '/root/repo')
import torch
import admm
from blocks.lstm import LSTM
from parameters import example_parameter_dictionary
import bench
dev = torch.device('cuda:0')
for cfg in ('c3', 'c2'):
    B, T, D, H, variant, gen = bench.CONFIGS[cfg]
    x, y = bench.make_data(gen, B, T, D)
    torch.manual_seed(0)
    m = LSTM(D, H, 1)
    opt = admm.ADMMBasedOptimizer(m, (x.to(dev), y.to(dev)), example_parameter_dictionary['GoogleStock'], verbose=False)
    for s in range(40):
        opt.step()
        st = opt.last_step_stats()
        print(cfg, s, list(st['k'].values()), st['passes'], round(st['theta_h'], 3), flush=True)
