#!/usr/bin/env python3
"""Diagnostic (GPU): the iteration count T of every amp_vamp_run variant on the reference-moved
golden points (tests/golden/g4_curves.json entries holding T_runs), beside the reference's runs.

  python tools/t_probe.py
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, '..', 'tests'), os.path.join(HERE, '..'),
                os.path.join(HERE, '..', 'amp-sparc-spatialmodulation_amd')]
import golden_io as gio  # noqa: E402
from test_gpu_vamp import VARIANTS, _config, _regen_inputs  # noqa: E402


def main():
    from vamp import VAMP
    curves = gio.g4_curves()
    for name, ent in curves.items():
        if ent.get('algo') != 'vamp':
            continue
        for key, ref in sorted(ent['points'].items()):
            if 'T_runs' not in ref:
                continue
            seed, ebn0 = int(key.split('/')[0]), float(key.split('/')[1])
            cfg = _config(ent['Nt'], ent['Na'], ent['Nr'], ent['B'], ent['alphabet'], iterations=ent['iterations'])
            inp = _regen_inputs(cfg, seed, ebn0)
            line = f'{name:16s} {key:6s} ref runs {[int(t) for t in ref["T_runs"]]}'
            for variant, (eng, gemm) in sorted(VARIANTS.items()):
                Ts = []
                for _ in range(3):
                    det = VAMP(cfg, engine=eng, gemm=gemm)
                    L = det(inp['U'], inp['s'], inp['Vh'], inp['y'], inp['SNR'], inp['x'], inp['sym'], inp['idx'])
                    Ts.append(int(L.loss['T']))
                line += f'  {variant} {Ts}'
            print(line, flush=True)


if __name__ == '__main__':
    main()
