"""The shipped gfx950 code is free of the two hardware hazards measured on MI355X that LLVM's
gfx950 hazard model (ROCm 7.2) leaves unguarded (tools/isa_hazards.py):

* store-data: a vector-memory store of more than 8 bytes whose data VGPRs a VALU instruction
  rewrites fewer than 2 wait states after the store (tools/ubench/store_war.hip,
  profiles/r06_store_war.txt: the store then sends the new value);
* trans-pk: a transcendental result read by a packed-f32 instruction at distance 1
  (tools/ubench/trans_pk.hip, profiles/r05_trans_pk_probe.txt).

The scanner itself is checked on synthetic listings first, so a clean library scan means
"scanned and clean", not "scanner blind".  CPU only: the code objects are read from the
library's .hip_fatbin section and disassembled with llvm-objdump (no GPU calls).
"""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'tools'))
import isa_hazards as H  # noqa: E402

LIB = os.path.join(REPO, 'amp-sparc-spatialmodulation_amd', 'lib', 'libampsparc.so')


def _scan(text):
    return H.scan(H.parse('<k>:\n' + text))


def test_scanner_store_data():
    hit = _scan('global_store_dwordx4 v[0:1], v[4:7], off sc1\nv_mov_b32_e32 v5, 0\n')
    assert [(k, ws) for k, _, ws, _ in hit] == [('store-data', 0)]
    hit = _scan('buffer_store_dwordx4 v[12:15], v50, s[28:31], s4 offen sc1\n'
                'v_pk_mov_b32 v[12:13], v[22:23], v[24:25] op_sel:[1,0]\n')
    assert [k for k, *_ in hit] == ['store-data']
    # one wait state is not enough (the other wave of the SIMD running: stale in 2-3 % of lanes)
    hit = _scan('scratch_store_dwordx4 off, v[26:29], off\ns_nop 0\nv_add_f32_e32 v28, v1, v2\n')
    assert [(k, ws) for k, _, ws, _ in hit] == [('store-data', 1)]
    # clean: two wait states, an 8-byte store, an LDS write, a load or an MFMA overwriting the data
    for text in ('global_store_dwordx4 v[0:1], v[4:7], off\ns_nop 1\nv_mov_b32_e32 v5, 0\n',
                 'global_store_dwordx4 v[0:1], v[4:7], off\nv_add_u32_e32 v9, 1, v9\nv_add_u32_e32 v9, 1, v9\n'
                 'v_mov_b32_e32 v5, 0\n',
                 'global_store_dwordx2 v[0:1], v[4:5], off\nv_mov_b32_e32 v5, 0\n',
                 'ds_write_b128 v1, v[4:7]\nv_mov_b32_e32 v5, 0\n',
                 'scratch_store_dwordx4 off, v[26:29], off\nds_read_b128 v[26:29], v1 offset:144\n',
                 'global_store_dwordx4 v[0:1], v[4:7], off\nv_mfma_f32_16x16x32_bf16 v[4:7], v[8:11], v[12:15], v[4:7]\n',
                 'global_store_dwordx4 v2, v[0:3], s[86:87] offset:160 nt\ns_endpgm\nv_cndmask_b32_e32 v0, s0, v0, vcc\n'):
        assert _scan(text) == [], text


def test_scanner_trans_pk():
    hit = _scan('v_exp_f32_e32 v10, v2\nv_pk_add_f32 v[12:13], v[10:11], v[14:15]\n')
    assert [k for k, *_ in hit] == ['trans-pk']
    assert _scan('v_exp_f32_e32 v10, v2\nv_add_u32_e32 v9, 1, v9\nv_pk_add_f32 v[12:13], v[10:11], v[14:15]\n') == []


def test_bundles_parsed():
    """Every translation unit's gfx950 code object is found (one offload bundle each)."""
    if not os.path.exists(LIB):
        pytest.skip('libampsparc.so not built (build() / make -C amp-sparc-spatialmodulation_amd/csrc)')
    cos = H.code_objects(H.fatbin(LIB))
    assert len(cos) >= 10   # amp_weights, amp_vamp, the persistent instantiation units, ...


@pytest.mark.skipif(not os.path.exists(os.path.join(H.LLVM, 'llvm-objdump')), reason='llvm-objdump not installed')
def test_library_free_of_measured_hazards():
    if not os.path.exists(LIB):
        pytest.skip('libampsparc.so not built (build() / make -C amp-sparc-spatialmodulation_amd/csrc)')
    found = H.scan_library(LIB)
    assert found == [], [(k, fn, ws, seq) for k, fn, ws, seq in found[:5]]
