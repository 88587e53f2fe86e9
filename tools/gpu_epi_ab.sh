#!/usr/bin/env bash
# Same-box A/B of the persistent VAMP engine's epilogue parts (diagnostic builds whose results are
# wrong by construction: no output stores / no fused decision / no in-kernel fold), in-loop time.
# The libraries need guards in amp_vamp_persist_kernel.h's epilogue (#ifndef AMP_DIAG_NO_OUT around
# the r / xmmse / var stores, AMP_DIAG_NO_DECIDE around decide_epilogue, AMP_DIAG_NO_FOLD on the
# fold condition; profiles/r06_epilogue_cost.txt) and are built in the container, e.g.
#   make -C amp-sparc-spatialmodulation_amd/csrc SPILLCHECK=true OBJDIR=../build_nofold \
#     OUT=../lib_diag/libampsparc_nofold.so CXXFLAGS="<Makefile flags> -DAMP_DIAG_NO_FOLD=1" ../lib_diag/libampsparc_nofold.so
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-epi}; mkdir -p "$OUT"
for v in def nofold nodec noout def2 nofold2 nodec2 noout2; do
  L=""; case $v in def*) ;; *) L="AMP_LIB_PATH=amp-sparc-spatialmodulation_amd/lib_diag/libampsparc_${v%2}.so";; esac
  timeout -k 10 300 env $L python3 bench.py --no-cpu-baseline > "$OUT/$v.log" 2>&1 || { echo "$v failed"; tail -5 "$OUT/$v.log"; exit 1; }
  echo "$v $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$v.log") $(grep -o '"vamp_persist_in_loop": [0-9.]*' "$OUT/$v.log")"
done
