"""Host AddressSanitizer run of the C ABI ("race detection / sanitizers").

``csrc/Makefile`` target ``asan`` builds ``libadmmlstm_asan.so`` -- the product kernels with the
host code of ``admm_host.hip`` (argument validation, create / bind / destroy, the step's launch
sequence, the communicator and debug hooks) instrumented by ``-Xarch_host -fsanitize=address`` --
and the driver ``tests/native/abi_asan.cpp``, which calls every entry point of
``include/admm_lstm.h``.  ASan aborts the driver on the first invalid host access or leak.

* CPU: argument and state validation of every entry point (no device is touched).
* GPU: five full contexts on device 0 (generic path, ragged persistent sweep, the C3 and C5 kernel
  families, a 300-wide output layer): create, invalid binds, bind, init_state, steps with
  profiling, cache invalidation, gradient tracing and forced decisions, stats, poll, workspace
  copies, the context-free forward, destroy.
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, 'admm-lstm_amd', 'admm_amd')
EXE = os.path.join(PKG, 'abi_asan')
# LeakSanitizer on, with the ROCm runtime's own process-lifetime allocations suppressed
# (tests/native/lsan.supp); leaks from the library's code still fail the run
ENV = dict(os.environ, ASAN_OPTIONS='detect_leaks=1:abort_on_error=0:halt_on_error=1',
           LSAN_OPTIONS='suppressions=' + os.path.join(ROOT, 'tests', 'native', 'lsan.supp') + ':print_suppressions=0')


def _exe():
    if not os.path.exists(EXE):   # CPU hosts: build it (the GPU box uses the prebuilt one)
        r = subprocess.run(['make', '-s', '-C', os.path.join(PKG, 'csrc'), 'asan'])
        if r.returncode != 0 or not os.path.exists(EXE):
            pytest.skip('the host-ASan driver does not build with this toolchain (make ... asan failed)')
    return EXE


def test_abi_argument_validation_under_asan():
    r = subprocess.run([_exe(), 'args'], env=ENV, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert 'abi_asan args: ok' in r.stdout
    assert 'AddressSanitizer' not in r.stderr and 'LeakSanitizer' not in r.stderr, r.stderr


@pytest.mark.gpu
def test_abi_full_contexts_under_asan():
    if not os.path.exists(EXE):   # __graft_entry__.build() makes it best-effort
        pytest.skip('host-ASan driver not built (make -C admm-lstm_amd/admm_amd/csrc asan)')
    # AddressSanitizer only: LeakSanitizer's stop-the-world check after the GPU contexts deadlocked
    # against the ROCm runtime's threads on 2 of 4 boxes (the contexts themselves had finished in under
    # a second); the CPU run above keeps the leak check
    env = dict(ENV, ASAN_OPTIONS='detect_leaks=0:abort_on_error=0:halt_on_error=1')
    r = subprocess.run([EXE, 'gpu'], env=env, capture_output=True, text=True, timeout=150)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert 'abi_asan gpu: ok' in r.stdout
    assert 'AddressSanitizer' not in r.stderr, r.stderr[-4000:]
