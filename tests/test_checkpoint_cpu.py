"""Checkpoint formats without a GPU.

* whole-module ``torch.save(model)`` as the reference's demo writes it (demo.py:302-308):
  our LSTM pickles under the same class path with the same attributes and loads back;
* ``save_checkpoint`` output is tensors only (``torch.load(weights_only=True)``).
"""
import os

import torch


def test_whole_model_roundtrip(tmp_path):
    from admm_amd.checkpoint import save_model
    from blocks.lstm import LSTM
    torch.manual_seed(0)
    m = LSTM(3, 5, 2, with_grad=True)
    path = save_model('unit', m, save_dir=str(tmp_path))
    assert os.path.basename(path) == 'unit.pt'
    m2 = torch.load(path, weights_only=False)          # a file this test wrote
    assert type(m2).__module__ == 'blocks.lstm' and type(m2).__name__ == 'LSTM'
    assert [n for n, _ in m2.named_parameters()] == [n for n, _ in m.named_parameters()] == \
        ['x2i', 'h2i', 'x2f', 'h2f', 'x2g', 'h2g', 'x2o', 'h2o', 'out']
    x = torch.rand(4, 6, 3)
    assert torch.equal(m2(x), m(x))                     # grad_forward path on CPU


class _FakeOpt:
    def __init__(self):
        self.s = {'format': 'admm-lstm-mi355x/optimizer-state/1', 'shape': [2, 3, 1, 4, 1],
                  'gates': {'i': torch.rand(2, 4, 4), 'a': torch.rand(2, 1)},
                  'duals': {'i': torch.rand(2, 4, 4), 'y': torch.rand(2, 1)}}
        self.loaded = None

    def state_dict(self):
        return self.s

    def load_state_dict(self, s):
        self.loaded = s


def test_checkpoint_is_weights_only(tmp_path):
    from admm_amd.checkpoint import load_checkpoint, save_checkpoint
    from blocks.lstm import LSTM
    torch.manual_seed(1)
    m = LSTM(1, 4, 1)
    opt = _FakeOpt()
    path = str(tmp_path / 'ck' / 'c.pt')
    save_checkpoint(path, m, opt)
    ck = torch.load(path, weights_only=True)
    assert ck['format'] == 'admm-lstm-mi355x/checkpoint/1'
    torch.manual_seed(2)
    m2 = LSTM(1, 4, 1)
    opt2 = _FakeOpt()
    load_checkpoint(path, m2, opt2)
    for (n, a), (_, b) in zip(m.named_parameters(), m2.named_parameters()):
        assert torch.equal(a, b), n
    assert torch.equal(opt2.loaded['gates']['i'], opt.s['gates']['i'])
