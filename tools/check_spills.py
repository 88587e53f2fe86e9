#!/usr/bin/env python3
"""Build-time check (run by the csrc Makefile after linking): no persistent-engine instantiation
that the host can dispatch may spill VGPRs to scratch, except the documented ones below.

Reads the gfx950 code object of each object file (the .hip_fatbin offload bundle), its
amdhsa.kernels metadata (.vgpr_spill_count, .private_segment_fixed_size), and fails when a
vamp_persist / scamp_persist kernel spills and is not listed in ALLOWED.  Why spills matter here:
scratch is per-lane memory traffic inside the persistent loop, and the round-3 review tied the
two-workgroups-per-CU corruption to the spilling instantiations (DESIGN.md §3.8 has the outcome
of that investigation).

  python tools/check_spills.py amp-sparc-spatialmodulation_amd/build/*.o [--list]
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = '/opt/rocm/lib/llvm/bin'

# Documented exceptions: (kernel-name regex, reason).  Each is an instantiation the host can
# dispatch whose spills are loop-invariant values reloaded a few times per iteration.
ALLOWED = [
    # vamp_persist<NT=2, KK=16, NWV=4, DU=2, X3, OCC=2, H2?>: the cfg2 two-per-CU build (256 VGPRs),
    # 12 / 25 spilled values = the per-lane s^2 / y~ registers kept across the loop
    (r'_ZN3amp12vamp_persistILi2ELi16ELi4ELi2ELb1ELi2ELb[01]E', 'cfg2 16-QAM two-per-CU build'),
    # the other two-per-CU alphabets (BPSK / QPSK / 8-PSK / 64-QAM at N = 64, side-by-side epochs;
    # the fp16x2 BPSK build keeps 2 values since the fused decision is force-inlined)
    (r'_ZN3amp12vamp_persistILi2ELi(1|2|4|8|64)ELi4ELi[124]ELb1ELi2ELb[01]E', 'N = 64 two-per-CU builds'),
    # 64-point alphabets at N = 256 (no BASELINE VAMP config): the wide denoiser's chunked table
    # beside the N = 256 GEMM registers, 12 values reloaded once per iteration
    (r'_ZN3amp12vamp_persistILi8ELi64ELi4ELi1ELb[01]ELi1ELb[01]E', '64-point alphabet at N = 256'),
    # the int8x4 engine at N = 256: loop-invariant values stored once in the prologue and reloaded
    # outside the GEMMs (none inside them)
    (r'_ZN3amp12vamp_persistILi(8|4)ELi(1|2|4|8|16|64)ELi(4|8)ELi[124]ELb1ELi1ELb0ELb1E', 'int8x4 at N = 256 (opt-in)'),
    # the eight-wave bf16x3 form (the N = 256 default): 256 registers per wave; loop-invariant
    # addresses and constants reloaded outside the GEMMs
    (r'_ZN3amp12vamp_persistILi4ELi(1|2|4|8|16|64)ELi8ELi[124]ELb1ELi1ELb0ELb0E', 'eight-wave bf16x3 at N = 256'),
    # the four-wave bf16x3 form at N = 256 (AMP_VAMP_X3_WAVES=4, A/B runs only): the per-epoch
    # channel pointers, the force-inlined decision and the in-kernel counter fold cost BPSK / QPSK
    # 12-24 loop-invariant values (8-point alphabets 12 since the prologue's y~ loads became
    # unconditional clamped loads)
    (r'_ZN3amp12vamp_persistILi8ELi(1|2|4|8)ELi4ELi[124]ELb1ELi1ELb0ELb0E', 'four-wave bf16x3 at N = 256 (A/B form)'),
    # the eight-wave bf16x3 SCAMP form (cfg3's shape), the same kind of loop invariants
    (r'_ZN3amp13scamp_persistILi4ELi16ELi2ELi32ELi(1|2|4|8|16|64)ELb1ELb0ELi8E', 'eight-wave bf16x3 SCAMP'),
]


def kernels(obj):
    """[(name, vgpr_spill, private_segment)] of the gfx950 code object inside `obj`."""
    with tempfile.TemporaryDirectory() as td:
        fb = os.path.join(td, 'fb.bin')
        dev = os.path.join(td, 'dev.o')
        subprocess.run([f'{LLVM}/llvm-objcopy', '--dump-section=.hip_fatbin=' + fb, obj, os.path.join(td, 'h.o')],
                       check=True, capture_output=True)
        subprocess.run([f'{LLVM}/clang-offload-bundler', '--type=o', '--unbundle', '--input=' + fb,
                        '--targets=hipv4-amdgcn-amd-amdhsa--gfx950', '--output=' + dev], check=True,
                       capture_output=True)
        notes = subprocess.run([f'{LLVM}/llvm-readelf', '--notes', dev], check=True, capture_output=True,
                               text=True).stdout
    out = []
    for blk in re.split(r'\n\s*- \.agpr_count:', notes)[1:]:
        name = re.search(r'\.name:\s+(\S+)', blk)
        spill = re.search(r'\.vgpr_spill_count:\s+(\d+)', blk)
        priv = re.search(r'\.private_segment_fixed_size:\s+(\d+)', blk)
        if name:
            out.append((name.group(1), int(spill.group(1)) if spill else 0, int(priv.group(1)) if priv else 0))
    return out


def main(argv):
    objs = [a for a in argv if not a.startswith('--')]
    listing = '--list' in argv
    bad = []
    for obj in objs:
        for name, spill, priv in kernels(obj):
            if not re.search(r'(vamp|scamp)_persist', name):
                continue
            allowed = [why for rx, why in ALLOWED if re.search(rx, name)]
            if listing or (spill and not allowed):
                print(f'{os.path.basename(obj):32s} spill {spill:4d} private {priv:5d}  {name}'
                      + (f'  [allowed: {allowed[0]}]' if spill and allowed else ''))
            if spill and not allowed:
                bad.append(name)
    if bad:
        print(f'check_spills: {len(bad)} persistent instantiation(s) spill VGPRs (tools/check_spills.py ALLOWED)',
              file=sys.stderr)
        return 1
    return 0


if __name__ == '__main__':
    sys.exit(main(sys.argv[1:]))
