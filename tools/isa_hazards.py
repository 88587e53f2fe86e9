#!/usr/bin/env python3
"""Scan the gfx950 code objects of a HIP shared library for two hardware hazards that LLVM's
gfx950 hazard model (ROCm 7.2) leaves unguarded, both measured on MI355X:

  store-data  a vector-memory store with more than 8 bytes of data (global_/buffer_/scratch_/
              flat_store_dwordx3 / x4, *_store_b96 / b128) whose data VGPRs an instruction
              writes fewer than 2 wait states after the store issued: the store can send the NEW
              value (tools/ubench/store_war.hip: stale at 0 wait states, and at 1 when the other
              wave of the SIMD runs; clean at 2; 4- and 8-byte stores and LDS writes are clean at 0);
  trans-pk    a transcendental result (v_exp_f32, v_rcp_f32, ...) read by a packed-f32 VALU
              instruction (v_pk_*) at distance 1 (tools/ubench/trans_pk.hip: stale at 0 fillers).

Every instruction counts one wait state, `s_nop N` counts N + 1.  The device code is read from
the library's .hip_fatbin section (every clang offload bundle in it: one per translation unit)
and disassembled with llvm-objdump.

  python tools/isa_hazards.py [lib.so] [--list]       # exit status 1 if any hazard is found
"""
import os
import re
import struct
import subprocess
import sys
import tempfile

LLVM = '/opt/rocm/lib/llvm/bin'
MAGIC = b'__CLANG_OFFLOAD_BUNDLE__'
TRANS = ('v_exp_f32', 'v_rcp_f32', 'v_log_f32', 'v_sqrt_f32', 'v_rsq_f32', 'v_rcp_iflag_f32', 'v_sin_f32',
         'v_cos_f32')
WIDE_STORE = re.compile(r'^(global|buffer|scratch|flat)_store_(dwordx3|dwordx4|b96|b128)\b')
STORE_WAIT = 2   # wait states a >8-byte store's data VGPRs must stay untouched


def fatbin(so):
    """The .hip_fatbin section of an ELF shared object (pure Python: no binutils needed)."""
    data = open(so, 'rb').read()
    if data[:4] != b'\x7fELF' or data[4] != 2:
        raise SystemExit(f'{so}: not a 64-bit ELF')
    shoff, = struct.unpack_from('<Q', data, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from('<HHH', data, 0x3A)
    sec = [struct.unpack_from('<IIQQQQIIQQ', data, shoff + i * shentsize) for i in range(shnum)]
    stroff = sec[shstrndx][4]
    for s in sec:
        name = data[stroff + s[0]:data.index(b'\0', stroff + s[0])].decode()
        if name == '.hip_fatbin':
            return data[s[4]:s[4] + s[5]]
    raise SystemExit(f'{so}: no .hip_fatbin section')


def code_objects(fb, arch='gfx950'):
    """Every `arch` code object of every offload bundle in a fatbin blob."""
    out = []
    pos = fb.find(MAGIC)
    while pos >= 0:
        n, = struct.unpack_from('<Q', fb, pos + len(MAGIC))
        p = pos + len(MAGIC) + 8
        for _ in range(n):
            off, size, tl = struct.unpack_from('<QQQ', fb, p)
            triple = fb[p + 24:p + 24 + tl].decode()
            p += 24 + tl
            if triple.endswith(arch):
                out.append(fb[pos + off:pos + off + size])
        pos = fb.find(MAGIC, pos + len(MAGIC))
    return out


def disassemble(co):
    with tempfile.NamedTemporaryFile(suffix='.co', delete=False) as f:
        f.write(co)
        path = f.name
    try:
        return subprocess.run([os.path.join(LLVM, 'llvm-objdump'), '-d', '--mcpu=gfx950', '--no-show-raw-insn',
                               '--no-leading-addr', path], capture_output=True, text=True, check=True).stdout
    finally:
        os.unlink(path)


def regs(text):
    out = set()
    for m in re.finditer(r'\bv\[(\d+):(\d+)\]', text):
        out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    for m in re.finditer(r'(?<![\w\[:])v(\d+)\b', text):
        out.add(int(m.group(1)))
    return out


def parse(listing):
    """(function, [instructions]) in listing order; an instruction is (mnemonic, operand text)."""
    funcs, cur, name = [], None, None
    for line in listing.splitlines():
        m = re.match(r'^\s*(?:[0-9a-f]+\s+)?<([^>]+)>:\s*$', line)
        if m:
            name = m.group(1)
            cur = []
            funcs.append((name, cur))
            continue
        s = line.split(';')[0].split('//')[0].strip()
        if cur is None or not s or s.endswith(':') or s.startswith('.') or s.startswith('Disassembly'):
            continue
        parts = s.split(None, 1)
        cur.append((parts[0], parts[1] if len(parts) > 1 else ''))
    return funcs


def dst_regs(mn, ops):
    """VGPRs a VALU instruction writes at issue (its first operand).  Loads and MFMAs write their
    destinations tens of cycles after issue, past any store's data read, so they do not count."""
    if mn.startswith('v_') and not mn.startswith(('v_mfma', 'v_smfmac')):
        return regs(ops.split(',')[0])
    return set()


def wait_states(mn, ops):
    if mn == 's_nop':
        try:
            return int(ops.split()[0], 0) + 1
        except ValueError:
            return 1
    return 1


def scan(funcs):
    found = []
    for name, ins in funcs:
        for i, (mn, ops) in enumerate(ins):
            if WIDE_STORE.match(mn):
                # data operand: the second for global/scratch/flat (vaddr, vdata), the first for buffer
                fields = [f.strip() for f in ops.split(',')]
                data = regs(fields[0] if mn.startswith('buffer') else (fields[1] if len(fields) > 1 else ''))
                ws = 0
                for j in range(i + 1, min(i + 4, len(ins))):
                    if ws >= STORE_WAIT:
                        break
                    m2, o2 = ins[j]
                    if m2 in ('s_endpgm', 's_branch', 's_setpc_b64'):   # the next listed instruction is not next in time
                        break
                    if dst_regs(m2, o2) & data:
                        found.append(('store-data', name, ws, [f'{a} {b}' for a, b in ins[i:j + 1]]))
                        break
                    ws += wait_states(m2, o2)
            elif mn.startswith(TRANS):
                dst = regs(ops.split(',')[0])
                if i + 1 < len(ins):
                    m2, o2 = ins[i + 1]
                    if m2.startswith('v_pk_') and regs(o2.split(',', 1)[1] if ',' in o2 else '') & dst:
                        found.append(('trans-pk', name, 0, [f'{a} {b}' for a, b in ins[i:i + 2]]))
    return found


def scan_library(so):
    found = []
    for co in code_objects(fatbin(so)):
        found += scan(parse(disassemble(co)))
    return found


def main():
    args = [a for a in sys.argv[1:] if not a.startswith('--')]
    so = args[0] if args else os.path.join(os.path.dirname(__file__), '..', 'amp-sparc-spatialmodulation_amd', 'lib',
                                           'libampsparc.so')
    found = scan_library(so)
    kinds = {}
    for k, fn, ws, seq in found:
        kinds.setdefault(k, set()).add(fn)
    print(f'{so}: {len(found)} hazard sites in {sum(len(v) for v in kinds.values())} functions')
    for k, fns in kinds.items():
        print(f'  {k}: {len(fns)} functions')
    if '--list' in sys.argv:
        for k, fn, ws, seq in found:
            print(f'{k} {fn} (wait states {ws}):\n    ' + '\n    '.join(seq))
    return 1 if found else 0


if __name__ == '__main__':
    sys.exit(main())
