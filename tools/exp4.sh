set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/exp4
hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -shared -fPIC -o /tmp/libdu.so tools/ubench/denoise_ubench.hip 2>/dev/null || exit 1
rocprofv3 -L > gpurun_out/exp4/counters.txt 2>&1 || true
grep -o "SQ_[A-Z0-9_]*" gpurun_out/exp4/counters.txt | sort -u > gpurun_out/exp4/sq_names.txt || true
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS -d gpurun_out/exp4/p1 -o p1 --output-format csv -- python3 -c "import ctypes; ctypes.CDLL('/tmp/libdu.so').ubench_main()" > gpurun_out/exp4/p1.log 2>&1 || exit $?
python3 - <<'PY'
import csv,glob,collections
rows=list(csv.DictReader(open(glob.glob('gpurun_out/exp4/p1/*counter_collection.csv')[0])))
agg=collections.defaultdict(list)
for r in rows: agg[(r['Dispatch_Id'],r['Kernel_Name'][:40],r['Counter_Name'])].append(float(r['Counter_Value']))
for k,v in sorted(agg.items()): print(k, sum(v))
PY
