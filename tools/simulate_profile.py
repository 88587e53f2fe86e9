#!/usr/bin/env python3
"""cProfile of Model.simulate in throughput mode (rng='device') at cfg4: where the host time of
an epoch goes outside the detector.  python tools/simulate_profile.py"""
import cProfile
import os
import pstats
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'amp-sparc-spatialmodulation_amd'))
sys.path.insert(0, REPO)

import torch  # noqa: E402

from config import Config  # noqa: E402
from model import Model  # noqa: E402

cfg = Config(256, 8, 512, 1, 1, batch=4096, generator_mode='sparc', iterations=20, alphabet='16QAM',
             channel_profile='uniform', channel_truncation='tail', device='cuda')
with tempfile.TemporaryDirectory() as d:
    m = Model(cfg, 'vamp', path=d, seed=0, rng='device')
    m.simulate(2, start=8.0, final=8.0, res=20)
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    m.simulate(20, start=8.0, final=8.0, res=20)
    torch.cuda.synchronize()
    pr.disable()
pstats.Stats(pr).sort_stats('tottime').print_stats(18)
