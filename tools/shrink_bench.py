#!/usr/bin/env python3
"""Throughput of the Shrink kernels (csrc/amp_shrink.hip) against the HBM roofline.

Each kernel is timed with HIP events on the stream it runs on (median of 20 after 5 warmup
launches) at cfg4's r (4096 x 256 complex64, 1 M elements) and at a 64 M-element batch where
launch overhead no longer hides the memory time.  Algorithmic bytes per element:
  bayes     complex64 r in, complex64 out  (+4 B per-element cov)   = 16 (20) B
  shrinkOOK float32 Re r in, float32 out   (+4 B cov)               =  8 (12) B
  sw_ook    float32 Re r in, complex64 + float32 out (+4 B cov)     = 16 (20) B
(the host's r.real copy that feeds shrinkOOK / sw_ook is a separate torch copy, not counted).
Prints one JSON line per (kernel, size, cov kind)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'amp-sparc-spatialmodulation_amd'))

import torch  # noqa: E402

import amp_native as nat  # noqa: E402
from config import Config  # noqa: E402
from shrink import Shrink  # noqa: E402

PEAK_GBS = 8000.0


def timed(fn, reps=20, warm=5):
    st = torch.cuda.current_stream()
    for _ in range(warm):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record(st)
        fn()
        b.record(st)
    torch.cuda.synchronize()
    t = sorted(a.elapsed_time(b) for a, b in ev)
    return t[len(t) // 2]


def main():
    dev = torch.device('cuda:0')
    L = nat.lib()
    for B in (4096, 262144):
        Nt, Na = 256, 8
        cfg = Config(Nt, Na, 2 * Nt, 1, 1, batch=B, generator_mode='sparc', alphabet='16QAM', device='cuda',
                     channel_profile='uniform', channel_truncation='tail')
        n = B * Nt
        g = torch.Generator(device=dev).manual_seed(0)
        r = (torch.randn(B, Nt, 1, dtype=torch.complex64, device=dev, generator=g) * 0.6)
        re = r.real.contiguous()
        cov_v = torch.rand(B, Nt, 1, device=dev, generator=g) * 0.3 + 0.02
        out_c = torch.empty_like(r)
        out_f = torch.empty_like(re)
        var = torch.empty_like(re)
        dxdr = torch.empty((), device=dev)
        Sb = Shrink(cfg, 'bayes')
        So = Shrink(cfg, 'shrinkOOK')
        k = Sb._constellation()
        wsb = L.amp_shrink_ook_workspace_bytes(n)
        ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
        stp = nat.stream_ptr(dev)
        for cov_kind in ('scalar', 'vec'):
            cv = None if cov_kind == 'scalar' else cov_v.data_ptr()
            extra = 0 if cov_kind == 'scalar' else 4
            runs = {
                'bayes': (lambda: L.amp_shrink_bayes(k, n, 1, r.data_ptr(), 0.15, cv, float(Sb.P0), float(Sb.Ps),
                                                     out_c.data_ptr(), stp), 16 + extra),
                'shrinkOOK': (lambda: L.amp_shrink_ook(n, 0, re.data_ptr(), 0.15, cv, So._theta, out_f.data_ptr(),
                                                       dxdr.data_ptr(), ws.data_ptr(), wsb, stp), 8 + extra),
                'sw_shrinkOOK': (lambda: L.amp_shrink_sw_ook(B * Na, Nt // Na, 0, re.data_ptr(), 0.15, cv,
                                                             out_c.data_ptr(), var.data_ptr(), stp), 16 + extra),
            }
            for name, (fn, bpe) in runs.items():
                nat.check(fn(), name)
                ms = timed(fn)
                gbs = n * bpe / (ms * 1e-3) / 1e9
                print(json.dumps({'kernel': name, 'elements': n, 'cov': cov_kind, 'ms': round(ms, 5),
                                  'bytes_per_element': bpe, 'achieved_GBs': round(gbs, 1), 'peak_GBs': PEAK_GBS,
                                  'frac': round(gbs / PEAK_GBS, 3),
                                  'elements_per_s': n / (ms * 1e-3)}), flush=True)
    nat.unload()


if __name__ == '__main__':
    main()
