set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
OUT=gpurun_out/r6c34; mkdir -p $OUT
D=amp-sparc-spatialmodulation_amd/lib_diag/libampsparc_prev.so
PYT="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 1000 $PYT tests/test_gpu_bamp_scamp.py tests/test_gpu_cfg5.py tests/test_gpu_isi_model.py tests/test_gpu_published.py -m gpu > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for v in def prev def2 prev2; do
  L=""; case $v in prev*) L="AMP_LIB_PATH=$D";; esac
  timeout -k 10 300 env $L python3 tools/isi_bench.py 512 50 > $OUT/isi_$v.log 2>&1 || { echo "isi $v failed"; exit 1; }
  timeout -k 10 300 env $L python3 tools/cfg5_bench.py > $OUT/cfg5_$v.log 2>&1 || { echo "cfg5 $v failed"; exit 1; }
  echo "== $v"; grep -h '^{' $OUT/isi_$v.log $OUT/cfg5_$v.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l)
    print(d.get('algo', ''), d.get('workload', '')[:40], d.get('ms_per_iteration', d.get('detector_ms')), d.get('frac_fp32_peak', d.get('mfma_frac')), d.get('T'), d.get('fer'), d.get('ser'))"
done
