#!/usr/bin/env python
"""Headline benchmark: ADMM iterations/sec of ``ADMMBasedOptimizer.step()``.

BASELINE.json metric: "ADMM iters/sec at hidden=256, batch=8192, seq=32; 1/2/4/8-GPU
scaling".  One *step* = one ``step()`` (admm.py:62-78) over the synthetic uniform
regression problem of SURVEY.md 8(d) (config C3: B=8192, T=32, D=16, H=256, O=1,
GoogleStock rho/beta), fp32, inputs and state resident in HBM before timing.

Multi-GPU (``torchrun --nproc-per-node N``): one process per GPU, the step's batch sums
all-reduced with RCCL inside libadmmlstm.so.  ``value`` is STRONG scaling by default: the
global batch stays the config's (8192 at C3), each rank steps 8192/N rows, and ``value`` is the
it/s of that global problem.  A second, weak-scaling measurement (8192 rows per rank, the C4
shape at N = 8) is reported beside it under ``weak`` ({global_batch, it_s, value in batch-8192
units = it/s x global_batch / 8192}); ``--scaling weak`` makes that the headline instead.

Also reported (rank 0):
* ``roofline`` for the dominant kernel class of the timed region, timed live with
  hipEvents on the step's stream (admm_profile); algorithmic bytes/flops per launch
  are those of DESIGN.md "Roofline accounting";
* ``step_roofline``: the whole step against SURVEY.md 8(d)'s t_roof (GEMMs at the fp32 matrix
  peak) and against ``t_roof_built`` (the GEMMs priced at the bf16/fp16 matrix rate of the split
  products they run as), with ``step_frac`` / ``step_frac_built``;
* ``cpu_baseline``: the CPU oracle (a port of the reference op structure, see
  oracle/admm_oracle.py) timed on this host on a bounded sample (N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, 'admm-lstm_amd'))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

PEAK_FP32_MFMA = 157.3e12   # MI355X_MICROARCH.md: Peak FP32 (matrix) 157.3 TFLOPS
PEAK_HBM = 8.0e12           # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
PEAK_BF16_MFMA = 2.5e15     # MI355X_MICROARCH.md: BF16 ~2.5 PF dense
# f32-accurate products from three-way bf16 splits take 6 bf16 MFMAs (admm_dev.hpp split3):
# the matrix peak of the kernels that use them, in f32-equivalent flops
PEAK_SPLIT3_MFMA = PEAK_BF16_MFMA / 6
SPLIT3_CLASSES = ('sweep', 'atr_h', 'qgemm_h')
HEADLINE_B = 8192

CONFIGS = {
    # name: (B per rank, T, D, H, variant, input generator)
    'c2': (2048, 16, 16, 64, 'admm', 'uniform'),
    'c3': (8192, 32, 16, 256, 'admm', 'uniform'),
    'c5': (4096, 64, 1, 512, 'no_dual_y', 'rw'),
    # diagnostic: C4's global batch on one GPU (the line-search exponents of the 8-GPU run)
    'c4g': (65536, 32, 16, 256, 'admm', 'uniform'),
    # strong-scaling rank of C3 at N = 8: 1024 of the 8192 samples (the per-rank step of the 8-GPU run)
    'c3s': (1024, 32, 16, 256, 'admm', 'uniform'),
    # ... and at N = 2 and N = 4 (4096 and 2048 samples per rank)
    'c3h': (4096, 32, 16, 256, 'admm', 'uniform'),
    'c3q': (2048, 32, 16, 256, 'admm', 'uniform'),
}
CPU_BASELINE_OFF = {'c4g'}   # configs whose CPU baseline is skipped unless --cpu-baseline


def make_data(gen: str, B: int, T: int, D: int, seed_offset: int = 0):
    """SURVEY.md 8(d) generators (uniform: seed 1234; rw: seed 7)."""
    if gen == 'uniform':
        g = torch.Generator().manual_seed(1234 + seed_offset)
        x = torch.rand(B, T, D, generator=g)
        y = 0.8 * x.mean((1, 2)).unsqueeze(1) + 0.1 * torch.rand(B, 1, generator=g)
        return x, y
    g = torch.Generator().manual_seed(7 + seed_offset)
    s = torch.cumsum(torch.randn(B + T + 1, generator=g), 0)
    s = (s - s.min()) / (s.max() - s.min())
    idx = torch.arange(B).unsqueeze(1) + torch.arange(T).unsqueeze(0)
    return s[idx].unsqueeze(2).contiguous(), s[torch.arange(B) + T].unsqueeze(1).contiguous()


def persistent_sweep(H: int) -> bool:
    """k_sweep_rows: 32-row tiles for 64 <= H <= 256, 16-row tiles for 256 < H <= 512 (H % 64 == 0)."""
    r16 = 256 < H <= 512 and H % 64 == 0 and os.environ.get('ADMM_SWEEP_R16', '1') != '0'
    return os.environ.get('ADMM_SWEEP_ROWS', '1') != '0' and ((64 <= H <= 256 and H % 32 == 0) or r16)


def tgt_from_sweep(H: int) -> bool:
    """The persistent sweep writes the next x stage's targets unless disabled."""
    return persistent_sweep(H) and os.environ.get('ADMM_TGT_SWEEP', '1') != '0'


def survey_terms(B: int, T: int, D: int, H: int):
    """SURVEY.md 8(d)'s algorithmic work per step: (F_w, B_w) of the eight weight updates and
    (F_B, B_B) of the time sweep.  B_B = 4 B T (D + 25 H): per (b, t) read x_t, h_{t-1},
    c_{t-1}, 6 gates and 6 duals, write 6 gates and 5 duals."""
    F_w = T * 4.0 * (3 * 2.0 * B * H * H + 4 * 2.0 * B * D * H)
    B_w = 64.0 * B * T * (D + 3 * H)
    F_B = T * 2.0 * B * (D + H) * 4 * H
    B_B = 4.0 * B * T * (D + 25 * H)
    return (F_w, B_w), (F_B, B_B)


def step_roofline_s(B: int, T: int, D: int, H: int) -> float:
    """t_roof = sum over the two phases of max(F / fp32 MFMA peak, B / HBM peak) (SURVEY.md 8(d);
    3.77 ms at C3)."""
    return sum(max(f / PEAK_FP32_MFMA, b / PEAK_HBM) for f, b in survey_terms(B, T, D, H))


# The GEMMs as built (DESIGN.md sections 4 and 7): (flops of one f32 GEMM, bf16/fp16 products per
# f32 product, peak) per step at (B, T, D, H).  Sweep: split3 (6 bf16 products); h-side gradient:
# scaled fp16 two-way splits (3 products); h-side trial direction: two-piece Hprev x one-piece G
# (2 products); x side (G_x in the sweep, q = X G_x and X dWx in the trials): f32 MFMA.
def built_gemms(B: int, T: int, D: int, H: int):
    gh = 2.0 * B * T * H * 4 * H
    gx = 2.0 * B * T * D * 4 * H
    return {'sweep': [(T * 2.0 * B * (D + H) * 4 * H, 6, PEAK_BF16_MFMA)],
            'weights': [(gh, 3, PEAK_BF16_MFMA), (gh, 2, PEAK_BF16_MFMA), (3 * gx, 1, PEAK_FP32_MFMA)]}


def step_roofline_built_s(B: int, T: int, D: int, H: int) -> float:
    """t_roof with the GEMMs priced as they run: sum over the two phases of max(sum of product
    work / its matrix peak, SURVEY.md 8(d)'s algorithmic bytes / 8 TB/s) (2.49 ms at C3)."""
    (_, bw), (_, bb) = survey_terms(B, T, D, H)
    g = built_gemms(B, T, D, H)
    t = 0.0
    for phase, byts in (('weights', bw), ('sweep', bb)):
        t += max(sum(f * n / peak for f, n, peak in g[phase]), byts / PEAK_HBM)
    return t


def roofline_terms(cls: str, B: int, T: int, D: int, H: int):
    """(flops, bytes) of ONE launch of a kernel class as this design moves them:
    for the sweep these include the z-cache, target and G_x-partial writes that replace work
    of the next step's x stage (bench reports SURVEY.md 8(d)'s algorithmic bytes beside them)."""
    f4 = 4  # bytes per fp32
    tgt = tgt_from_sweep(H)
    if cls == 'sweep':            # whole sweep t = 1..T: per t [B, D+H] x [D+H, 4H] + fused gate/dual updates
        flops = T * 2.0 * B * (D + H) * 4 * H
        if not tgt:               # per-t sweep: 11 state/dual loads (incl. c_{t-1}), 15 stores (6 gates, 5 duals, 4 z)
            return flops, T * f4 * B * (D + 26 * H)
        # persistent sweep, per (b, t, j): 9 state/dual loads (f, g, c, h; duals of i, f, g, o, c),
        # 19 stores (6 gates, 5 duals, 4 z, 4 tgt).  c_{t-1} comes from registers after t = 1 and
        # the h dual is read only at T while it is zero before T (the reference's invariant):
        # one plane slice each, once.  With D <= 16 the sweep also forms the next x stage's
        # X^T R partials: x once more, and a [blocks][4][D][H] slab.
        lamh_all = os.environ.get('ADMM_LAMH_SKIP', '1') == '0'
        byts = T * f4 * B * (D + (29 if lamh_all else 28) * H) + f4 * B * (1 if lamh_all else 2) * H
        if D <= 16 and H <= 256 and os.environ.get('ADMM_GX_SWEEP', '1') != '0':
            byts += f4 * B * T * D + f4 * ((B + 31) // 32) * 4 * D * H
        return flops, byts
    n = float(B) * T * H          # elements of one [B*T, H] plane
    if cls == 'atr_h':            # G_q = Hprev^T R_q, 4 gates
        return 2.0 * B * T * H * 4 * H, f4 * (B * T * H + 4 * n)
    if cls == 'atr_x':
        return 2.0 * B * T * D * 4 * H, f4 * (B * T * D + 4 * n)
    if cls == 'qgemm_h':          # Q_q = Hprev G_q
        return 2.0 * B * T * H * 4 * H, f4 * (B * T * H + 4 * n)
    if cls == 'qgemm_x':
        return 2.0 * B * T * D * 4 * H, f4 * (B * T * D + 4 * n)
    if cls in ('trial', 'trial_h', 'trial_extra'):
        # three planes per gate either way: pass 0 of the x side reads z and tgt and (H % 256 == 0)
        # writes the h stage's residual R_h for the predicted exponent; the h side reads z, tgt and Q
        return 0.0, f4 * 3 * 4 * n
    if cls == 'resid':            # x-stage residual (read z and tgt, or z, lam, S and write tgt) + z += X dWx
        return 0.0, f4 * ((2 if tgt else 4) + 2) * 4 * n
    return None


# kernel symbols of each profile class (admm_kernels.hip), for the committed PMC traffic
CLASS_KERNELS = {'sweep': ('k_sweep_rows', 'k_sweep_t'), 'atr_h': ('k_atr3', 'k_atr_fused', 'k_atr<128'), 'qgemm_h': ('k_qgemm3', 'k_qgemm<true, 1>'),
                 'trial': ('k_trial_mx<true>', 'k_trial_rows<0', 'k_trial_fast<0', 'k_trial<'),
                 'trial_h': ('k_trial_rows<1', 'k_trial_fast<1', 'k_trial<'),
                 'resid': ('k_resid_gx', 'k_apply_dwx', 'k_resid<')}


def counter_file(kind: str, cfg_name: str):
    """(path, why) of the newest committed counter summary profiles/r*_<kind>_<cfg>.json (written by
    tools/pmc_to_json.py) that measured THIS library: its lib_stamp must equal the source stamp the
    loaded libadmmlstm.so was built from (admm_build_info).  path None: why says what is missing."""
    import glob
    import json
    from admm_amd import _native as N
    want = N.lib_stamp()
    files = sorted(glob.glob(os.path.join(ROOT, 'profiles', f'r*_{kind}_{cfg_name}.json')))
    for f in reversed(files):
        if json.load(open(f)).get('lib_stamp') == want:
            return f, None
    return None, (f'no profiles/r*_{kind}_{cfg_name}.json measured this library (src {want}); '
                  f'{len(files)} older summar{"y" if len(files) == 1 else "ies"} ignored')


def pmc_traffic(cls: str, cfg_name: str):
    """(HBM bytes per launch of a kernel class, source) from the newest committed PMC summary of this
    library (counter_file: rocprofv3 FETCH_SIZE / WRITE_SIZE passes of this same bench command), or
    (None, why)."""
    import json
    path, why = counter_file('pmc', cfg_name)
    if path is None:
        return None, why
    src = os.path.relpath(path, ROOT)
    if cls not in CLASS_KERNELS:
        return None, f'{src}: no kernel family for class {cls}'
    kern = json.load(open(path))['kernels']
    # trial passes after the first return early (gates already decided): use the full pass; the
    # column-split sweep is followed by its gated row-block launch, which exits at once: the max
    key = 'traffic_bytes_max' if cls in ('trial', 'trial_h', 'sweep') else 'traffic_bytes_median'
    for prefix in CLASS_KERNELS[cls]:     # the first kernel family present in the profile
        vals = [v[key] for k, v in kern.items() if k.startswith(prefix)]
        if vals:
            break
    if not vals:
        return None, f'{src}: no {cls} kernel in the summary'
    per = sum(vals) / len(vals)
    if cls == 'sweep' and prefix == 'k_sweep_t':   # per-t sweep: T time steps x 2 sample halves
        T = CONFIGS[cfg_name][1]
        per *= 2 * T
    return per, src


# kernel families whose MFMA-busy fraction bench.py reports (SQ pass of tools/gpu.sh mfma:<cfg>)
MFMA_KERNELS = {'sweep': ('k_sweep_rows',), 'atr_h': ('k_atr3w<2, true>', 'k_atr3w'), 'qgemm_h': ('k_qgemm_res', 'k_qgemm3'),
                'trial': ('k_trial_mx<true',)}


def pmc_mfma_busy(cfg_name: str):
    """Counted MFMA-busy fraction per kernel family from the newest committed SQ pass of this library
    (counter_file: profiles/r*_sq_<cfg>.json, tools/gpu.sh mfma:<cfg>, tools/pmc_to_json.py --sq):
    SQ_VALU_MFMA_BUSY_CYCLES (cycles the matrix pipe of a SIMD is busy, summed over SIMDs) over
    4 SIMDs x SQ_BUSY_CU_CYCLES (the dispatch's busy cycles summed over CUs), i.e. the share of the
    kernel's time the matrix cores are issuing, against gfx950's MFMA peak issue rate.  Per dispatch,
    the largest over the family's dispatches (the gated row-block sweep launch after a column split
    does no work).  {'source': None, 'why': ...} if no pass of this config measured this library."""
    import json
    path, why = counter_file('sq', cfg_name)
    if path is None:
        return {'source': None, 'why': why}
    kern = json.load(open(path))['kernels']
    out = {'source': os.path.relpath(path, ROOT)}
    for cls, prefixes in MFMA_KERNELS.items():
        for prefix in prefixes:
            vals = [v['SQ_VALU_MFMA_BUSY_CYCLES_max'] / (4.0 * v['SQ_BUSY_CU_CYCLES_max'])
                    for k, v in kern.items() if k.startswith(prefix)
                    and v.get('SQ_BUSY_CU_CYCLES_max') and 'SQ_VALU_MFMA_BUSY_CYCLES_max' in v]
            if vals:
                out[cls] = round(max(vals), 4)
                break
    return out


def reference_loss(cfg_name: str, step: int, loss: float):
    """The reference's training loss after ``step`` steps of this config's trajectory, where a committed
    golden holds it (tests/golden/c3_25.npz: the reference's 25 steps of C3 = the default 5 warm-up + 20
    timed steps, tests/golden/make_golden.py), beside this run's final loss: {step, loss, rel_diff}."""
    import json
    import numpy as np
    if cfg_name != 'c3':
        return None
    path = os.path.join(ROOT, 'tests', 'golden', 'c3_25.npz')
    if not os.path.exists(path):
        return None
    losses = json.loads(str(np.load(path, allow_pickle=False)['meta_json']))['losses']
    if step >= len(losses):
        return None
    ref = losses[step]
    return {'step': step, 'loss': ref, 'rel_diff': abs(loss - ref) / abs(ref), 'bar': 1e-5,
            'source': 'tests/golden/c3_25.npz (the reference itself, tests/golden/make_golden.py)'}


def host_cpu():
    """(model name, sockets, physical cores per socket) of this host from /proc/cpuinfo."""
    model, phys = 'unknown', {}
    try:
        cur = {}
        for line in open('/proc/cpuinfo').read().splitlines() + ['']:
            if not line.strip():
                if 'physical id' in cur and 'core id' in cur:
                    phys.setdefault(cur['physical id'], set()).add(cur['core id'])
                cur = {}
                continue
            k, _, v = line.partition(':')
            cur[k.strip()] = v.strip()
            if k.strip() == 'model name':
                model = v.strip()
    except OSError:  # pragma: no cover
        pass
    sockets = len(phys) or 1
    cores = max((len(v) for v in phys.values()), default=os.cpu_count() or 1)
    return model, sockets, cores


def _read(path):
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def _cpu_list(text):
    out = []
    for part in (text or '').split(','):
        if '-' in part:
            a, b = part.split('-')
            out.extend(range(int(a), int(b) + 1))
        elif part.strip():
            out.append(int(part))
    return out


def gpu_socket_cores(dev_index: int = 0):
    """BASELINE.md / SURVEY.md 8(d) CPU-baseline protocol: the physical cores (one hardware thread
    each) of the socket the GPU hangs off, among the CPUs this process may run on.  Returns
    (cpu ids, socket id, how the socket was found)."""
    allowed = set(os.sched_getaffinity(0)) if hasattr(os, 'sched_getaffinity') else set(range(os.cpu_count() or 1))
    pkg_of = {c: _read(f'/sys/devices/system/cpu/cpu{c}/topology/physical_package_id') for c in allowed}
    socket, how = None, 'socket of the lowest visible CPU (GPU NUMA node unknown)'
    try:   # the GPU's PCI device -> its NUMA node -> that node's package
        import torch as _t
        pr = _t.cuda.get_device_properties(dev_index)
        bdf = f'{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}.0'
        node = int(_read(f'/sys/bus/pci/devices/{bdf}/numa_node') or -1)
        if node >= 0:
            cpus = [c for c in _cpu_list(_read(f'/sys/devices/system/node/node{node}/cpulist')) if c in allowed]
            if cpus:
                socket = pkg_of.get(cpus[0])
                how = f'GPU {bdf} on NUMA node {node}, package {socket}'
    except Exception:  # pragma: no cover - older torch / no sysfs
        pass
    if socket is None:
        socket = pkg_of.get(min(allowed))
    cores, seen = [], set()
    for c in sorted(allowed):
        if pkg_of.get(c) != socket:
            continue
        sib = _cpu_list(_read(f'/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list') or str(c))
        key = min(sib) if sib else c
        if key in seen:
            continue
        seen.add(key)
        cores.append(c)
    return cores or sorted(allowed), socket, how


def cgroup_cpus():
    """The cgroup (v2) CPU quota in CPUs, or None if unlimited / unknown."""
    q = _read('/sys/fs/cgroup/cpu.max')
    if not q:
        return None
    a, _, b = q.partition(' ')
    return None if a == 'max' else round(int(a) / int(b), 2)


def port_vs_reference(cfg_name: str):
    """The CPU port's time against the reference's own, from the build container's alternated records
    (tools/cpu_port_vs_ref.py -> profiles/r06_cpu_port_vs_ref_*.json; the reference never travels to the
    GPU box, so the ratio is measured there and reported here beside the port's time): port / reference
    per record of this config (pooled medians, wall and, where recorded, process CPU time), with the
    per-round ratios.  Below 1 the port is faster than the reference, i.e. the GPU/CPU ratio is understated."""
    import glob
    out = []
    for f in sorted(glob.glob(os.path.join(ROOT, 'profiles', 'r06_cpu_port_vs_ref_*.json'))):
        try:
            with open(f) as fh:
                d = json.load(fh)
        except (OSError, ValueError):
            continue
        sm = d.get('summary', {}).get(cfg_name)
        if not sm or 'port_over_ref' not in sm:
            continue
        r = {'source': os.path.relpath(f, ROOT), 'threads': d.get('host', {}).get('threads'),
             'rounds': len(sm.get('port_s', [])), 'port_over_ref_wall': round(sm['port_over_ref'], 3)}
        if 'port_over_ref_cpu' in sm:
            r['port_over_ref_cpu_time'] = round(sm['port_over_ref_cpu'], 3)
        if 'port_over_ref_per_round' in sm:
            pr = sorted(sm['port_over_ref_per_round'])
            r['per_round_cpu_time'] = [round(v, 3) for v in sm['port_over_ref_per_round']]
            r['per_round_median'] = round(pr[len(pr) // 2], 3)   # robust to one disturbed round
        r['max_rel_loss_diff'] = sm.get('max_rel_loss_diff')
        out.append(r)
    return out or None


def cpu_baseline(cfg_name: str, timed_steps: int = 5, crosscheck_threads: int = 8):
    """SURVEY.md 8(d) CPU-baseline protocol on this host: the CPU oracle (a port of the reference's
    op structure, oracle/admm_oracle.py) on the FULL batch of the config, on all physical cores of the
    GPU-local socket, pinned in-process (os.sched_setaffinity, no re-exec), step 1 untimed (it is
    cheaper: zero x-side gradients), the median of steps 2..1+timed_steps (2..6), and one more step on
    ``crosscheck_threads`` of those cores to compare with the survey container's 8-thread 27.6 s/it
    at C3 (and with the reference itself run there: tools/cpu_port_vs_ref.py)."""
    from oracle import admm_oracle as O
    from parameters import example_parameter_dictionary
    B, T, D, H, variant, gen = CONFIGS[cfg_name]
    model, sockets, per_socket = host_cpu()
    cores, socket, how = gpu_socket_cores(0)
    quota = cgroup_cpus()
    # The protocol's "all physical cores of the GPU-local socket" is bounded by the CPU time this
    # process may use: under a cgroup quota of Q CPUs, more than Q threads only time-share them (on the
    # GPU box, 64 threads under a 16-CPU quota ran 64.9 s/it against 20 s on 16: profiles/
    # r05c_c3_bench_cpu64_throttled.json), so the threads are the socket's cores up to the quota
    if quota and quota >= 1 and int(quota) < len(cores):
        how += f'; {int(quota)} of its {len(cores)} cores (cgroup CPU quota {quota})'
        cores = cores[:int(quota)]
    old_aff = os.sched_getaffinity(0) if hasattr(os, 'sched_getaffinity') else None
    old_threads = torch.get_num_threads()
    threads = len(cores)
    try:
        if old_aff is not None:
            os.sched_setaffinity(0, cores)
        torch.set_num_threads(threads)
        x, y = make_data(gen, B, T, D)
        torch.manual_seed(0)
        W = O.init_weights(D, H, 1)
        st = O.init_state(x, y, W)
        stp = O.Stepper(O.Hyper.from_dict(example_parameter_dictionary['GoogleStock'], variant))
        times = []
        for s in range(1 + timed_steps):
            t0 = time.time()
            stp.step(st)
            times.append(time.time() - t0)
            print(f'cpu_baseline: step {s + 1} on {threads} threads: {times[-1]:.2f} s', file=sys.stderr, flush=True)
        med = sorted(times[1:])[len(times[1:]) // 2]
        cross = None
        if crosscheck_threads and crosscheck_threads < threads:
            if old_aff is not None:
                os.sched_setaffinity(0, cores[:crosscheck_threads])
            torch.set_num_threads(crosscheck_threads)
            t0 = time.time()
            stp.step(st)
            cross = time.time() - t0
            print(f'cpu_baseline: step {2 + timed_steps} on {crosscheck_threads} threads: {cross:.2f} s',
                  file=sys.stderr, flush=True)
    finally:
        torch.set_num_threads(old_threads)
        if old_aff is not None:
            os.sched_setaffinity(0, old_aff)
    return {
        'value': round(1.0 / med, 6), 'unit': 'it/s', 'cores': threads, 'kind': 'port',
        'sample': f'oracle/admm_oracle.py (reference op structure, fp32 torch CPU) on the full {cfg_name} batch '
                  f'B={B} T={T} D={D} H={H}: median of steps 2-{1 + timed_steps} = {med:.2f} s/it '
                  f'(steps: {", ".join(f"{t:.2f}" for t in times)} s) on {threads} threads pinned to the '
                  f'physical cores of the GPU-local socket ({how}); '
                  + (f'step {2 + timed_steps} on {crosscheck_threads} threads {cross:.2f} s '
                     f'(survey container, 8 threads, reference itself: 27.6 s/it at C3); ' if cross else '')
                  + f'host: {model}, {sockets} socket(s) x {per_socket} physical cores'
                  + (f', cgroup CPU quota {quota} CPUs' if quota else ''),
        'median_step_s': round(med, 3), 'step_s': [round(t, 3) for t in times],
        'crosscheck': {'threads': crosscheck_threads, 'step_s': round(cross, 3)} if cross else None,
        'host_cpu': {'model': model, 'sockets': sockets, 'physical_cores_per_socket': per_socket,
                     'socket': socket, 'pinned_cpus': cores, 'cgroup_cpu_quota': quota},
        'port_vs_reference': port_vs_reference(cfg_name),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=5)
    ap.add_argument('--config', default='c3', choices=sorted(CONFIGS))
    ap.add_argument('--scaling', default='strong', choices=['weak', 'strong'],
                    help='headline at N > 1: strong (the config global batch, default) or weak (its batch per rank)')
    ap.add_argument('--no-weak', action='store_true', help='N > 1: skip the extra weak-scaling measurement')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    # the CPU oracle runs the config's full batch: at C4g (65536 rows, 8x C3) four steps take ~15 min,
    # so it is off there unless asked for
    ap.add_argument('--cpu-baseline', action='store_true', help='time the CPU baseline even where it is off by default (c4g)')
    ap.add_argument('--cpu-steps', type=int, default=5, help='timed CPU-baseline steps after step 1 (median; 2..6)')
    ap.add_argument('--profile-classes', default='sweep,trial,trial_h,trial_extra,atr_x,atr_h,qgemm_x,qgemm_h,resid,small')
    # rehearsal of the N > 1 path on a one-GPU box: every rank on device 0, torch.distributed over
    # gloo, so the library stages its all-reduces through the host (not a performance number)
    ap.add_argument('--dist-backend', default='nccl', choices=['nccl', 'gloo'])
    ap.add_argument('--one-device', action='store_true', help='all ranks on cuda:0 (rehearsal only)')
    args = ap.parse_args()
    if args.one_device and args.dist_backend == 'nccl':   # RCCL refuses two ranks on one GPU
        print('--one-device runs every rank on cuda:0: using --dist-backend gloo (host-staged all-reduces)',
              file=sys.stderr)
        args.dist_backend = 'gloo'

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local_rank = int(os.environ.get('LOCAL_RANK', '0'))
    if world != args.gpus:
        print(f'warning: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE', file=sys.stderr)
    dev_index = 0 if args.one_device else local_rank
    torch.cuda.set_device(dev_index)
    dev = torch.device('cuda', dev_index)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if args.dist_backend == 'nccl':
            dist.init_process_group('nccl', device_id=dev)
        else:
            dist.init_process_group('gloo')

    import admm
    from blocks.lstm import LSTM
    from parameters import example_parameter_dictionary
    if CONFIGS[args.config][4] == 'no_dual_y':
        import importlib.util
        spec = importlib.util.spec_from_file_location('admm_no_dual_y',
                                                      os.path.join(ROOT, 'admm-lstm_amd', 'admm.no_dual_y.py'))
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
    else:
        mod = admm

    B, T, D, H, variant, gen = CONFIGS[args.config]

    def barrier():
        torch.cuda.synchronize(dev)
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize(dev)

    cdev = dev if args.dist_backend == 'nccl' else torch.device('cpu')

    def measure(Bg: int, with_profile: bool):
        """Warm up, (optionally) profile the kernel classes, then time exactly args.steps steps of the
        global problem of Bg samples, each rank stepping its contiguous row block of Bg / world."""
        per = Bg // world
        x_all, y_all = make_data(gen, Bg, T, D)
        x = x_all[rank * per:(rank + 1) * per].contiguous().to(dev)
        y = y_all[rank * per:(rank + 1) * per].contiguous().to(dev)
        del x_all, y_all

        def fresh():
            torch.manual_seed(0)
            m = LSTM(D, H, 1).to(dev)
            o = mod.ADMMBasedOptimizer(m, (x, y), example_parameter_dictionary['GoogleStock'], verbose=False,
                                       distributed=world > 1)
            for _ in range(args.warmup):
                o.step()
            barrier()
            return m, o

        prof = {}
        if with_profile:
            # kernel classes: hipEvent pairs around each class on the step's stream over the steps the
            # timed run below takes (same seed and data: the same trajectory); the event records cost
            # about 0.2 ms per step, so this run is not the timed one
            classes = [c for c in args.profile_classes.split(',') if c]
            model, opt = fresh()
            opt.profile(classes)
            for _ in range(args.steps):
                opt.step()
            barrier()
            opt.profile(())
            prof = opt.profile_read()
            del opt, model
            torch.cuda.empty_cache()
        # timed region: plain steps, no events between the launches
        model, opt = fresh()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            opt.step()
        barrier()
        elapsed = time.perf_counter() - t0
        if dist is not None:
            t = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
        stats = opt.last_step_stats()
        loss = float(torch.nn.functional.mse_loss(model(x), y))
        if dist is not None:
            lt = torch.tensor([loss * per], dtype=torch.float64, device=cdev)
            dist.all_reduce(lt)
            loss = float(lt.item()) / Bg
        del opt, model, x, y
        torch.cuda.empty_cache()
        return per, elapsed, prof, stats, loss

    Bg = B * world if args.scaling == 'weak' else B
    per, elapsed, prof, stats, loss = measure(Bg, True)
    weak = None
    if world > 1 and args.scaling == 'strong' and not args.no_weak:
        wper, wel, _, _, _ = measure(B * world, False)
        weak = {'global_batch': B * world, 'batch_per_gpu': wper, 'ms_per_step': round(wel / args.steps * 1e3, 4),
                'it_s': round(args.steps / wel, 4),
                'value': round(args.steps / wel * B * world / HEADLINE_B, 4),
                'unit': 'batch-8192 it/s (it/s x global_batch / 8192)'}

    it_s = args.steps / elapsed
    value = it_s * Bg / HEADLINE_B if args.scaling == 'weak' else it_s
    # roofline of the dominant kernel class
    roof = None
    ranked = sorted(((ms, c) for c, (ms, n) in prof.items() if roofline_terms(c, per, T, D, H)), reverse=True)
    if ranked:
        ms, cls = ranked[0]
        n = prof[cls][1]
        avg_s = ms / n / 1e3
        flops, nbytes = roofline_terms(cls, per, T, D, H)
        design_bytes = nbytes
        if cls == 'sweep':          # the sweep's algorithmic work is (F_B, B_B)
            flops, nbytes = survey_terms(per, T, D, H)[1]
        peak_mfma = PEAK_SPLIT3_MFMA if cls in SPLIT3_CLASSES else PEAK_FP32_MFMA
        t_mfma, t_hbm = flops / peak_mfma, nbytes / PEAK_HBM
        if t_mfma >= t_hbm:
            roof = {'bound': 'mfma', 'achieved': flops / avg_s / 1e12, 'peak': peak_mfma / 1e12,
                    'unit': 'TFLOP/s'}
        else:
            roof = {'bound': 'hbm', 'achieved': nbytes / avg_s / 1e9, 'peak': PEAK_HBM / 1e9, 'unit': 'GB/s'}
        roof['frac'] = roof['achieved'] / roof['peak']
        # traffic: measured HBM bytes per launch (PMC, DESIGN.md "Measurement"), next to the
        # algorithmic bytes per launch and the bytes this design moves
        roof['traffic'], roof['traffic_source'] = pmc_traffic(cls, args.config)
        roof['algorithmic_bytes'] = nbytes
        roof['design_bytes'] = design_bytes
        roof['algorithmic_flops'] = flops
        roof['mfma_frac_fp32'] = flops / avg_s / PEAK_FP32_MFMA    # SURVEY.md 8(d)'s MFMA fraction
        # the counted one (rocprofv3 SQ_VALU_MFMA_BUSY_CYCLES): matrix-pipe busy share of the kernel's time
        busy = pmc_mfma_busy(args.config)
        roof['mfma_busy_frac'] = busy.get(cls)
        roof['mfma_busy_source'] = busy['source'] or busy['why']
        roof['mfma_busy'] = busy
        roof['kernel'] = cls
        roof['avg_launch_us'] = avg_s * 1e6
        roof['launches'] = n
        roof = {k: (round(v, 4) if isinstance(v, float) else v) for k, v in roof.items()}
    t_roof = step_roofline_s(per, T, D, H)
    t_built = step_roofline_built_s(per, T, D, H)
    t_step = elapsed / args.steps
    step_roof = {'t_roof_ms': round(t_roof * 1e3, 4), 'step_frac': round(t_roof / t_step, 4),
                 'basis': 'SURVEY.md 8(d): sum over weight phase and sweep of max(F/157.3 TFLOP/s, B/8 TB/s)',
                 't_roof_built_ms': round(t_built * 1e3, 4), 'step_frac_built': round(t_built / t_step, 4),
                 'basis_built': 'GEMMs as built: sum over the two phases of max(sum of split-product work / '
                                'its matrix peak (bf16/fp16 2.5 PFLOP/s: sweep 6 products, G_h 3, Q_h 2; '
                                'x side fp32 157.3 TFLOP/s), SURVEY.md 8(d) bytes / 8 TB/s)'}
    kernel_ms = {c: {'ms_per_step': round(ms / args.steps, 4), 'launches_per_step': n / args.steps}
                 for c, (ms, n) in sorted(prof.items(), key=lambda kv: -kv[1][0])}

    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline and (args.cpu_baseline or args.config not in CPU_BASELINE_OFF):
            cpu = cpu_baseline(args.config, args.cpu_steps)
        out = {
            'metric': 'ADMM iters/sec at hidden=256, batch=8192, seq=32; 1/2/4/8-GPU scaling',
            'value': round(value, 4), 'unit': 'it/s', 'n_gpus': world, 'steps': args.steps, 'warmup': args.warmup,
            'ms_per_step': round(elapsed / args.steps * 1e3, 4), 'higher_is_better': True,
            'scaling': args.scaling, 'vs_baseline': None, 'dtype': 'f32', 'data': 'synthetic',
            **({'rehearsal': f'{world} ranks on one device over {args.dist_backend} (host-staged all-reduces): '
                             'not a performance number'} if args.one_device else {}),
            'config': {'workload': f'{args.config.upper()}: ADMMBasedOptimizer.step() ({variant}), '
                                   f'uniform synthetic regression' if gen == 'uniform' else
                                   f'{args.config.upper()}: ADMMBasedOptimizer.step() ({variant}), random-walk windows',
                       'global_batch': Bg, 'batch_per_gpu': per, 'seq_len': T, 'input_size': D, 'hidden': H,
                       'output_size': 1, 'params': 'GoogleStock', 'parallelism': f'dp{world}',
                       'global_it_per_s': round(it_s, 4),
                       # the arithmetic of the step's GEMMs (all f32-accurate or trial-direction only)
                       'gemm_arithmetic': {
                           'sweep z = [x|h] [Wx;Wh]': 'split3 bf16, 6 products (f32-accurate)',
                           'G_h = rho Hprev^T R': 'scaled fp16 two-way splits, 3 products (f32-accurate); '
                                                  'split3 at the first step after (re)binding',
                           'Q_h = Hprev G_h': 'two-piece bf16 Hprev x bf16 G, stored bf16 (line-search '
                                              'direction only)',
                           'x side (G_x, X G_x, X dWx)': 'fp32 MFMA',
                           'ADMM_ATR_F16': os.environ.get('ADMM_ATR_F16', '1')}},
            **({'weak': weak} if weak else {}),
            'roofline': roof,
            'step_roofline': step_roof,
            'cpu_baseline': cpu,
            'kernels': kernel_ms,
            'line_search_k': list(stats['k'].values()),
            'trial_passes': stats['passes'],
            'direct_frac': [round(v, 4) for v in stats['direct_frac'].values()],
            # column-split sweep health on rank 0: fallbacks to the row-block sweep and
            # whether the context has turned the split off; hand-off timeouts would have raised
            'sweep': {'fallbacks': stats['sweep_fallbacks'], 'split_off': stats['sweep_split_off'],
                      'handoff_fail': stats['handoff_fail']},
            'final_train_mse': loss,
            **({'reference_loss': ref} if (ref := reference_loss(args.config, args.warmup + args.steps, loss)) else {}),
        }
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
