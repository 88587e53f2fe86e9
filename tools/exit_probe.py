"""Bisect a process-exit crash under rocprofv3: run one bench-like VAMP forward with the chosen
engine (and optionally the HIP-event profile call), then exit normally.
  python3 tools/exit_probe.py launches|persistent [profile|x] [unload]
The launch path of the persistent engine is chosen by AMP_PERSIST_LAUNCH (coop = cooperative)."""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
sys.argv += [''] * 3
import bench  # noqa: E402
import ctypes as C  # noqa: E402
import torch  # noqa: E402
import amp_native as nat  # noqa: E402
from config import Config  # noqa: E402
from vamp import VAMP  # noqa: E402

eng = {'launches': nat.ENGINE_LAUNCHES, 'persistent': nat.ENGINE_PERSISTENT}[sys.argv[1]]
cfg = Config(256, 8, 512, 1, 1, batch=4096, generator_mode='sparc', iterations=20, alphabet='16QAM',
             channel_profile='uniform', channel_truncation='tail', device='cuda')
inp = bench.make_inputs(cfg, 0, 8.0, torch.device('cuda', 0))
det = VAMP(cfg, engine=eng)
for _ in range(3):
    L = det(inp['U'], inp['s'], inp['Vh'], inp['y'], inp['SNR'], inp['x'], inp['sym'], inp['idx'])
if sys.argv[2] == 'profile':
    Tr = det.detect(inp['U'], inp['s'], inp['Vh'], inp['y'], inp['SNR'])
    ms = (C.c_float * 4)()
    nat.check(nat.lib().amp_vamp_profile(C.byref(Tr.dims), C.byref(Tr.const), C.byref(Tr.args), ms, Tr.stream), 'p')
torch.cuda.synchronize()
print('probe ok', sys.argv[1:], os.environ.get('AMP_PERSIST_LAUNCH'), float(L.loss['ser']), int(L.loss['T']),
      flush=True)
if sys.argv[3] == 'unload':
    nat.unload()
