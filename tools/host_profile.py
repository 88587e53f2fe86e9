import sys, time, os
sys.path[:0] = ['amp-sparc-spatialmodulation_amd', '.']
import torch, numpy as np, ctypes as C
import bench, amp_native as nat
from config import Config
from vamp import VAMP, Tracker, read_result
cfg = Config(256, 8, 512, 1, 1, batch=4096, generator_mode='sparc', iterations=20, alphabet='16QAM',
             channel_profile='uniform', channel_truncation='tail', device='cuda')
inp = bench.make_inputs(cfg, 0, 8.0, torch.device('cuda', 0))
det = VAMP(cfg)
for _ in range(3):
    det(inp['U'], inp['s'], inp['Vh'], inp['y'], inp['SNR'], inp['x'], inp['sym'], inp['idx'])
torch.cuda.synchronize()
import cProfile, pstats
pr = cProfile.Profile()
pr.enable()
for _ in range(50):
    det(inp['U'], inp['s'], inp['Vh'], inp['y'], inp['SNR'], inp['x'], inp['sym'], inp['idx'])
pr.disable()
st = pstats.Stats(pr); st.sort_stats('tottime').print_stats(25)
