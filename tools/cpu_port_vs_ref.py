"""Container record: the CPU port (oracle/admm_oracle.py, bench.py's cpu_baseline) against the reference
itself (/root/reference admm.py, imported read-only), same inputs, same thread count, alternated in
separate processes (the port must time within +-15 % of the
reference before it stands in for it on the GPU box, where the reference never travels).

usage: python tools/cpu_port_vs_ref.py [--threads 8] [--rounds 2] [--steps 6] [--configs c2,c3] [--out FILE]

Each (config, implementation) run is a fresh process: inputs per SURVEY.md 8(d) (bench.make_data),
torch.manual_seed(0) LSTM init, GoogleStock rho/beta, `steps` steps; the median of steps 2..steps is
the steady time.  The per-step training losses of the two implementations are compared too.
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = '/root/reference'


def child(impl, cfg, threads, steps):
    import torch
    torch.set_num_threads(threads)
    sys.path.insert(0, ROOT)
    import bench
    B, T, D, H, variant, gen = bench.CONFIGS[cfg]
    x, y = bench.make_data(gen, B, T, D)
    times, losses, cpu = [], [], []
    if impl == 'ref':
        os.chdir('/tmp')   # the reference's logger writes logs/ in the cwd
        # bench put this repo's drop-in package on the path: the reference's own modules instead
        sys.path[:] = [p for p in sys.path if 'admm-lstm_amd' not in p]
        for m in list(sys.modules):
            if m.split('.')[0] in ('blocks', 'parameters', 'admm', '_global', 'dataset', 'admm_amd'):
                del sys.modules[m]
        sys.path.insert(0, REF)
        import admm
        from blocks.lstm import LSTM
        from parameters import example_parameter_dictionary
        assert variant == 'admm'
        torch.manual_seed(0)
        model = LSTM(D, H, 1)
        opt = admm.ADMMBasedOptimizer(model, (x, y), example_parameter_dictionary['GoogleStock'], verbose=False)
        for _ in range(steps):
            t0, c0 = time.time(), time.process_time()
            opt.step()
            times.append(time.time() - t0)
            cpu.append(time.process_time() - c0)
            losses.append(float(torch.nn.functional.mse_loss(model(x), y)))
    else:
        sys.path.insert(0, os.path.join(ROOT, 'admm-lstm_amd'))
        from oracle import admm_oracle as O
        from parameters import example_parameter_dictionary
        torch.manual_seed(0)
        W = O.init_weights(D, H, 1)
        st = O.init_state(x, y, W)
        stp = O.Stepper(O.Hyper.from_dict(example_parameter_dictionary['GoogleStock'], variant))
        for _ in range(steps):
            t0, c0 = time.time(), time.process_time()
            stp.step(st)
            times.append(time.time() - t0)
            cpu.append(time.process_time() - c0)
            losses.append(O.mse(x, y, st.W))
    print(json.dumps({'impl': impl, 'config': cfg, 'threads': threads, 'step_s': times, 'cpu_s': cpu, 'loss': losses}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--threads', type=int, default=8)
    ap.add_argument('--rounds', type=int, default=2)
    ap.add_argument('--steps', type=int, default=6)
    ap.add_argument('--configs', default='c2,c3')
    ap.add_argument('--out', default=os.path.join(ROOT, 'profiles', 'r05_cpu_port_vs_ref.json'))
    ap.add_argument('--child', nargs=2)
    a = ap.parse_args()
    if a.child:
        child(a.child[0], a.child[1], a.threads, a.steps)
        return
    runs = []
    for cfg in a.configs.split(','):
        for r in range(a.rounds):
            for impl in ('port', 'ref') if r % 2 == 0 else ('ref', 'port'):
                out = subprocess.run([sys.executable, __file__, '--child', impl, cfg, '--threads', str(a.threads),
                                      '--steps', str(a.steps)], capture_output=True, text=True, check=True)
                rec = json.loads(out.stdout.strip().splitlines()[-1])
                st = sorted(rec['step_s'][1:])
                rec['median_2_on'] = st[len(st) // 2]
                sc = sorted(rec['cpu_s'][1:])
                rec['cpu_median_2_on'] = sc[len(sc) // 2]
                rec['round'] = r
                runs.append(rec)
                print(f"{cfg} round {r} {impl}: median of steps 2-{a.steps} {rec['median_2_on']:.3f} s "
                      f"(process CPU {rec['cpu_median_2_on']:.2f} s) "
                      f"(steps {', '.join(f'{t:.2f}' for t in rec['step_s'])})", flush=True)
    summary = {}
    for cfg in a.configs.split(','):
        med = {impl: sorted(r['median_2_on'] for r in runs if r['config'] == cfg and r['impl'] == impl)
               for impl in ('port', 'ref')}
        lp = [r['loss'] for r in runs if r['config'] == cfg and r['impl'] == 'port'][0]
        lr = [r['loss'] for r in runs if r['config'] == cfg and r['impl'] == 'ref'][0]
        cmed = {impl: sorted(r['cpu_median_2_on'] for r in runs if r['config'] == cfg and r['impl'] == impl)
                for impl in ('port', 'ref')}
        rounds = sorted(set(r['round'] for r in runs if r['config'] == cfg))
        per_round = [[r['median_2_on'] for r in runs if r['config'] == cfg and r['round'] == k and r['impl'] == 'port'][0]
                     / [r['median_2_on'] for r in runs if r['config'] == cfg and r['round'] == k and r['impl'] == 'ref'][0]
                     for k in rounds]
        summary[cfg] = {'port_cpu_s': cmed['port'], 'ref_cpu_s': cmed['ref'],
                        'port_over_ref_cpu': sum(cmed['port']) / sum(cmed['ref']),
                        'port_over_ref_per_round': per_round,
                        'port_s': med['port'], 'ref_s': med['ref'],
                        'port_over_ref': sum(med['port']) / sum(med['ref']),
                        'max_rel_loss_diff': max(abs(p - q) / abs(q) for p, q in zip(lp, lr))}
    doc = {'note': 'tools/cpu_port_vs_ref.py in the build container (no GPU): the CPU port against the reference '
                   'itself, alternated in separate processes, same inputs and threads; median of steps 2..N',
           'host': {'cpu': open('/proc/cpuinfo').read().split('model name')[1].split('\n')[0].strip(' :\t'),
                    'threads': a.threads, 'torch': __import__('torch').__version__},
           'summary': summary, 'runs': runs}
    with open(a.out, 'w') as f:
        json.dump(doc, f, indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == '__main__':
    main()
