#!/usr/bin/env python3
"""Scan a gfx950 assembly listing (hipcc -S --offload-device-only) for transcendental results
(v_exp_f32, v_rcp_f32, ...) read by a later VALU instruction within 5 instructions: prints
(consumer kind, distance, s_nop wait states) counts and examples of packed (v_pk_*) consumers
(tools/ubench/trans_pk.hip probes the pattern on the hardware).

  python tools/ubench/hazard_scan.py listing.s
"""
import re, sys, collections
lines=[l.rstrip('\n') for l in open(sys.argv[1])]
ins=[]
for l in lines:
    s=l.strip()
    if not s or s.startswith(';') or s.startswith('.') or s.endswith(':'): continue
    s=s.split(';')[0].strip()
    if not s: continue
    ins.append(s)
def regs(op):
    out=set()
    for m in re.finditer(r'v\[(\d+):(\d+)\]', op):
        out.update(range(int(m.group(1)), int(m.group(2))+1))
    for m in re.finditer(r'(?<![\w\[:])v(\d+)\b', op):
        out.add(int(m.group(1)))
    return out
TRANS=('v_exp_f32','v_rcp_f32','v_log_f32','v_sqrt_f32','v_rsq_f32','v_rcp_iflag_f32')
stats=collections.Counter(); examples=collections.defaultdict(list)
for i,s in enumerate(ins):
    op=s.split()[0]
    if not op.startswith(TRANS): continue
    parts=s.split(None,1)[1].split(',')
    dst=regs(parts[0])
    nops=0
    for d in range(1,6):
        if i+d>=len(ins): break
        t=ins[i+d]; top=t.split()[0]
        if top.startswith('s_nop'):
            nops+=int(t.split()[1])+1; continue
        if top.startswith('s_'): continue
        srcs=t.split(None,1)[1].split(',',1)
        src=regs(srcs[1]) if len(srcs)>1 else set()
        if dst & src:
            kind='pk' if top.startswith('v_pk_') else ('dpp' if '_dpp' in top or 'row_' in t or 'quad_perm' in t else 'valu')
            key=(kind, d, nops)
            stats[key]+=1
            if len(examples[key])<2: examples[key].append(ins[i:i+d+1])
            break
for k,v in sorted(stats.items()): print(k, v)
for k,ex in examples.items():
    if k[0]=='pk':
        print('== example', k)
        for e in ex: print('   ', ' | '.join(e))
