"""Runtime conventions of the drop-in (device, messages, fatal errors).

Mirrors the behaviour the reference's hot path relies on (``_global.py`` of
Frederick2309/ADMM-LSTM): ``device`` is fixed at import (``_global.py:217``);
``info``/``warning`` print a timestamped line and append it to a log file;
``error`` prints, logs and terminates with ``SystemExit(code)``
(``_global.py:183-188``); ``log_assert`` calls ``error`` when its condition is
false (``_global.py:197-200``).  ``global_dict`` is the process-wide key/value
store ``demo.py`` imports (``demo.py:30, 286, 364``; reference ``_global.py:68-88``):
the file logger registers itself there under ``'loggers'`` and publishes the path it
writes to as ``'logger_filename'`` (``_global.py:113-142``).  The reference's colour
helpers, memory probes and decorators are not on the optimizer path and are not kept.
"""
from __future__ import annotations

import inspect
import logging
import os
import sys
from datetime import datetime
from typing import Any, Dict, Iterator, NoReturn

import torch

device = torch.device('cuda' if torch.cuda.is_available() else 'cpu')
PATH = os.path.abspath(os.getcwd())          # _global.py:92 (the run's working directory)


class GlobalDict:
    """Process-wide key/value store (``_global.py:68-88``): ``set``/``get``/``keys`` and item
    access; ``get`` of a missing key raises ``KeyError`` as the reference's does."""

    def __init__(self) -> None:
        self.contents: Dict[str, Any] = {}

    def set(self, key: str, value: Any) -> None:
        self.contents[key] = value

    def get(self, key: str) -> Any:
        return self.contents[key]

    def keys(self):
        return self.contents.keys()

    def __setitem__(self, key: str, value: Any) -> None:
        self.set(key, value)

    def __getitem__(self, key: str) -> Any:
        return self.get(key)

    def __contains__(self, key: object) -> bool:
        return key in self.contents

    def __iter__(self) -> Iterator[str]:
        return iter(self.contents)


global_dict = GlobalDict()
global_dict.set('loggers', {})

_DEFAULT_LOG = os.path.join('logs', 'ADMMRunningLogs.log')
_COLOURS = {'INFO': '\033[32m', 'WARNING': '\033[33m', 'ERROR': '\033[31m', 'ASSERTION FAILURE': '\033[31m'}


def _free_name(path: str) -> str:
    """``x.log`` if it does not exist yet, else the first free ``x_1.log``, ``x_2.log`` ...
    (one log file per run, _global.py:121-131)."""
    if not os.path.exists(path):
        return path
    stem = path[:-len('.log')] if path.endswith('.log') else path
    i = 1
    while os.path.exists(f'{stem}_{i}.log'):
        i += 1
    return f'{stem}_{i}.log'


def _logger_for(filename: str | None = None) -> logging.Logger:
    """The run's file logger, created on first use and registered in ``global_dict``."""
    loggers: Dict[str, logging.Logger] = global_dict['loggers']
    if filename is None:
        if loggers:
            filename = next(iter(loggers))
        else:
            os.makedirs(os.path.dirname(_DEFAULT_LOG), exist_ok=True)
            filename = _DEFAULT_LOG
    if filename not in loggers:
        filename = _free_name(filename)
        lg = logging.getLogger(filename)
        lg.setLevel(logging.DEBUG)
        handler = logging.FileHandler(filename)
        handler.setFormatter(logging.Formatter('%(asctime)s - %(name)s - %(levelname)s - %(message)s'))
        lg.addHandler(handler)
        loggers[filename] = lg
    global_dict.set('logger_filename', filename)
    return loggers[filename]


def _log(level: int, msg: str) -> None:
    _logger_for().log(level, msg)


def _emit(tag: str, msg: Any) -> None:
    print(f'[{datetime.now():%H:%M:%S}] {_COLOURS[tag]}{tag}\033[0m: {msg}')


def _where() -> str:
    frame = inspect.currentframe().f_back.f_back.f_back
    return f'\n  - reported from "{frame.f_code.co_name}" in {frame.f_code.co_filename}:{frame.f_lineno}'


def info(msg: Any = '', use_logger: bool = True) -> None:
    if use_logger:
        _log(logging.INFO, str(msg))
    _emit('INFO', msg)


def warning(msg: Any = '', warning_type: str | None = None, use_logger: bool = True, verbose: bool = True) -> None:
    if not verbose:
        return
    if use_logger:
        _log(logging.WARNING, str(msg))
    _emit('WARNING', msg)


def error(msg: Any = '', code: int = 1, use_logger: bool = True, assertion: bool = False) -> NoReturn:
    text = f'{msg}{_where()}'
    if use_logger:
        _log(logging.ERROR, text)
    _emit('ASSERTION FAILURE' if assertion else 'ERROR', text)
    sys.exit(code)


def log_assert(condition: bool, msg: Any = '', code: int = 1) -> None:
    if not condition:
        error(msg, code, assertion=True)
