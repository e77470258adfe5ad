"""Training checkpoints.

The reference saves only the model, as a whole pickled module (``demo.py:302-308``:
``torch.save(model, 'SAVED_MODELS/<name>.pt')``, read back by
``comparison_experiment/visualization.py:47-54``).  ``blocks.lstm.LSTM`` here has the same
module path and attributes, so those files stay interchangeable.  To resume ADMM training the
optimizer's primal/dual state is needed as well: ``save_checkpoint`` writes the model's and
the optimizer's ``state_dict`` (tensors only, so ``torch.load(..., weights_only=True)``
reads it) and ``load_checkpoint`` restores both in place.
"""
from __future__ import annotations

import os

import torch

FORMAT = 'admm-lstm-mi355x/checkpoint/1'


def save_checkpoint(path: str, model: torch.nn.Module, optimizer) -> None:
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    torch.save({'format': FORMAT,
                'model': {k: v.detach().cpu() for k, v in model.state_dict().items()},
                'optimizer': optimizer.state_dict()}, path)


def load_checkpoint(path: str, model: torch.nn.Module, optimizer=None) -> None:
    ck = torch.load(path, map_location='cpu', weights_only=True)
    if ck.get('format') != FORMAT:
        raise ValueError(f'{path}: not an {FORMAT} file')
    with torch.no_grad():
        for k, p in model.named_parameters():
            p.copy_(ck['model'][k].to(p.device, p.dtype))   # in place: the optimizer keeps its bindings
    if optimizer is not None:
        optimizer.load_state_dict(ck['optimizer'])


def save_model(name: str, model: torch.nn.Module, save_dir: str = 'SAVED_MODELS') -> str:
    """demo.py:302-308: the whole module, as the reference writes it."""
    os.makedirs(save_dir, exist_ok=True)
    path = os.path.join(save_dir, f'{name}.pt')
    torch.save(model, path)
    return path
