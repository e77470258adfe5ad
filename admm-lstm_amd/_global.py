"""Runtime conventions of the drop-in (device, messages, fatal errors).

Mirrors the behaviour the reference's hot path relies on (``_global.py`` of
Frederick2309/ADMM-LSTM): ``device`` is fixed at import (``_global.py:217``);
``info``/``warning`` print a timestamped line and append it to a log file;
``error`` prints, logs and terminates with ``SystemExit(code)``
(``_global.py:183-188``); ``log_assert`` calls ``error`` when its condition is
false (``_global.py:197-200``).  The reference's colour helpers, GlobalDict,
memory probes and decorators are not on the optimizer path and are not kept.
"""
from __future__ import annotations

import inspect
import logging
import os
import sys
from datetime import datetime
from typing import Any, NoReturn

import torch

device = torch.device('cuda' if torch.cuda.is_available() else 'cpu')

_LOG_PATH = os.path.join('logs', 'ADMMRunningLogs.log')
_logger: logging.Logger | None = None
_COLOURS = {'INFO': '\033[32m', 'WARNING': '\033[33m', 'ERROR': '\033[31m', 'ASSERTION FAILURE': '\033[31m'}


def _log(level: int, msg: str) -> None:
    global _logger
    if _logger is None:
        os.makedirs(os.path.dirname(_LOG_PATH), exist_ok=True)
        _logger = logging.getLogger('admm_amd')
        _logger.setLevel(logging.DEBUG)
        handler = logging.FileHandler(_LOG_PATH)
        handler.setFormatter(logging.Formatter('%(asctime)s - %(levelname)s - %(message)s'))
        _logger.addHandler(handler)
    _logger.log(level, msg)


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
