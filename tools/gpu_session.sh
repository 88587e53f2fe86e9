#!/usr/bin/env bash
# GPU session driver (run from the repo root on the box).  STEPS names the steps to run,
# in order, e.g. STEPS="bench bench_h2 trace tests_vamp".  Each GPU step has its own time limit;
# any non-zero exit ends the session (no retries).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05}
mkdir -p "$OUT"
run() {
    local name=$1 lim=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"; tail -4 "$OUT/$name.log"
    if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
run_nogate() {   # a step whose failures are data (e.g. the list of failing T checks): the session goes on
    local name=$1 lim=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"; tail -4 "$OUT/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name"; exit $rc; fi
}
PYT="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread"
for s in ${STEPS:-bench}; do
    case $s in
    bench) run bench 300 python3 bench.py ;;
    bench_nocpu) run bench_nocpu 300 python3 bench.py --no-cpu-baseline ;;
    bench_h2) run bench_h2 300 python3 bench.py --no-cpu-baseline --gemm h2 ;;
    bench_w8) run bench_w8 300 env AMP_VAMP_X3_WAVES=8 python3 bench.py --no-cpu-baseline ;;
    trace_w8) run trace_w8 300 env AMP_VAMP_X3_WAVES=8 python3 tools/trace_persist.py --config cfg4 ;;
    tests_w8) run tests_w8 900 env AMP_VAMP_X3_WAVES=8 $PYT tests/test_gpu_vamp.py -m gpu -k "persistent and not f32 and not h2 and not i8" ;;
    ab_w8) run ab_def 300 python3 bench.py --no-cpu-baseline &&
           run ab_pin 300 env AMP_LIB_PATH=amp-sparc-spatialmodulation_amd/lib_diag/libampsparc_w8pin.so python3 bench.py --no-cpu-baseline &&
           run ab_du1 300 env AMP_LIB_PATH=amp-sparc-spatialmodulation_amd/lib_diag/libampsparc_w8du1.so python3 bench.py --no-cpu-baseline &&
           run ab_def2 300 python3 bench.py --no-cpu-baseline ;;
    bench_i8) run bench_i8 300 python3 bench.py --no-cpu-baseline --gemm i8 ;;
    trace_i8) run trace_i8 300 python3 tools/trace_persist.py --config cfg4 --gemm i8 ;;
    tests_i8) run tests_i8 900 $PYT tests/test_gpu_vamp.py -m gpu -k "i8 or split_engines" ;;
    bench_f32) run bench_f32 300 python3 bench.py --no-cpu-baseline --gemm f32 ;;
    trace) run trace 300 python3 tools/trace_persist.py --config cfg4 ;;
    trace_h2) run trace_h2 300 env AMP_VAMP_GEMM=h2 python3 tools/trace_persist.py --config cfg4 ;;
    configs) run configs 600 python3 tools/configs_bench.py ;;
    cfg5) run cfg5 600 python3 tools/cfg5_bench.py ;;
    cfg3l) run cfg3l 300 python3 tools/configs_bench.py cfg3-launches ;;
    cfg3) run cfg3 300 python3 tools/configs_bench.py cfg3 cfg3-qpsk ;;
    cfg3w4) run cfg3w4 300 env AMP_SCAMP_X3_WAVES=4 python3 tools/configs_bench.py cfg3 cfg3-qpsk ;;
    tests_vamp) run tests_vamp 900 $PYT tests/test_gpu_vamp.py -m gpu ;;
    qprobe) run_nogate qprobe 300 env AMP_LIB_PATH=amp-sparc-spatialmodulation_amd/lib_diag/libampsparc_diag.so AMP_SHARD_ANY_STREAM=1 python3 tools/shard_queue_probe.py 8 ;;
    tests_shard) run tests_shard 600 $PYT tests/test_gpu_shard_trials.py tests/test_gpu_epochs.py -m gpu ;;
    acc) run acc 300 python3 tools/gemm_accuracy.py --variants launches,persistent,persistent-f32 ;;
    tests_q4) run_nogate tests_q4 600 python3 -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_vamp.py -m gpu -k "curve_point and cfg4 and persistent and not f32 and not h2 and not i8" ;;
    tests_epochs) run tests_epochs 600 $PYT tests/test_gpu_epochs.py -m gpu ;;
    tests_cfg5) run tests_cfg5 900 $PYT tests/test_gpu_cfg5.py -m gpu ;;
    tests_bs) run tests_bs 900 $PYT tests/test_gpu_bamp_scamp.py -m gpu ;;
    tests) run tests 1100 $PYT tests -m gpu ;;
    # occ2 needs the diagnostic libraries, built in the container first:
    #   make -C amp-sparc-spatialmodulation_amd/csrc SPILLCHECK=true OBJDIR=../build_diag2 \
    #     OUT=../lib_diag/libampsparc_pk_du2.so CXXFLAGS="<Makefile flags> -DAMP_OCC2_PK=1 -DAMP_KK4_DU=2" \
    #     ../lib_diag/libampsparc_pk_du2.so        (and the same with DU=4 -> _pk_du4)
    occ2) run occ2_prod 300 python3 tools/occ2_repro.py 10 &&
          run occ2_pk4 300 env AMP_LIB_PATH=amp-sparc-spatialmodulation_amd/lib_diag/libampsparc_pk_du4.so python3 tools/occ2_repro.py 10 &&
          run occ2_pk2 300 env AMP_LIB_PATH=amp-sparc-spatialmodulation_amd/lib_diag/libampsparc_pk_du2.so python3 tools/occ2_repro.py 10 ;;
    ttrace) run ttrace 600 python3 tools/t_trace.py --save 11,12 ;;
    pkocc2) run pkocc2 300 tools/ubench/bin/pk_occ2 20 ;;
    gemms) run gemm_x3 120 tools/ubench/bin/gemm_x3 && run gemm_h2 120 tools/ubench/bin/gemm_h2 &&
           run gemm_i8 120 tools/ubench/bin/gemm_i8 ;;
    pkdpp) run pkdpp 300 tools/ubench/bin/pk_dpp 3 ;;
    gi8) run gemm_i8 120 tools/ubench/bin/gemm_i8 ;;
    svd) run svd 300 python3 tools/svd_bench.py ;;
    simb) run simb 300 python3 tools/simulate_bench.py --epochs 8 ;;
    tests_model) run tests_model 600 $PYT tests/test_gpu_vamp.py -m gpu -k "device or random or model" ;;
    tprobe) run tprobe 300 python3 tools/t_probe.py ;;
    tests_vdef) run tests_vdef 900 $PYT tests/test_gpu_vamp.py -m gpu -k "persistent and not f32 and not h2" ;;
    isi) run isi 300 python3 tools/isi_bench.py 512 50 ;;
    isi_bn256) run isi_bn256 300 env AMP_SECTION_BN=256 python3 tools/isi_bench.py 512 50 ;;
    isiprofB) run isiprof256 300 rocprofv3 --kernel-trace --stats -d "$OUT/isiprof256" -o isi --output-format csv -- python3 tools/isi_bench.py 256 50 &&
              run isiprof1024 300 rocprofv3 --kernel-trace --stats -d "$OUT/isiprof1024" -o isi --output-format csv -- python3 tools/isi_bench.py 1024 50 ;;
    isipmc) run isipmc 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d "$OUT/isipmc" -o pmc --output-format csv -- python3 tools/isi_bench.py 512 10 ;;
    isitcc) run isitcc 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE -d "$OUT/isitcc" -o tcc --output-format csv -- python3 tools/isi_bench.py 512 10 ;;
    isi_ka4) run isi_ka4 300 env AMP_SCAMP_KA_WAVES=4 python3 tools/isi_bench.py 512 50 ;;
    isi_wnt) run isi_def 300 python3 tools/isi_bench.py 512 50 &&
             run isi_wnt 300 env AMP_LIB_PATH=amp-sparc-spatialmodulation_amd/lib_diag/libampsparc_wnt.so python3 tools/isi_bench.py 512 50 &&
             run isi_def2 300 python3 tools/isi_bench.py 512 50 ;;
    isi_bkc) run isi_bkc256 300 python3 tools/isi_bench.py 512 50 &&
             run isi_bkc512 300 env AMP_BAMP_KC=512 python3 tools/isi_bench.py 512 50 ;;
    isiprof) run isiprof 300 rocprofv3 --kernel-trace --stats -d "$OUT/isiprof" -o isi --output-format csv -- python3 tools/isi_bench.py 512 50 ;;
    tests_launch) run tests_launch 1100 $PYT tests/test_gpu_bamp_scamp.py tests/test_gpu_cfg5.py tests/test_gpu_published.py tests/test_gpu_shard_trials.py tests/test_gpu_rescue.py tests/test_gpu_isi_model.py tests/test_gpu_segmented.py tests/test_gpu_random.py -m gpu ;;
    smoke) run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()" ;;
    profile) run profile 900 bash tools/profile.sh ;;
    ubench) run ubench 300 bash tools/ubench/run.sh ;;
    # round 5: denoiser precision diagnostics (libraries built in the container: -DAMP_DEN_EXACT_EXP=1,
    # -DAMP_DEN_DIV=1, both; lib_diag/libampsparc_{exp,div,expdiv}.so) and the PKGRID A/B
    deniso) run deniso_def 600 python3 tools/den_isolate.py --oracle &&
            for v in ${DIAGS:-expdiv exp div}; do
                run deniso_$v 600 env AMP_LIB_PATH=amp-sparc-spatialmodulation_amd/lib_diag/libampsparc_$v.so python3 tools/den_isolate.py || exit 1
            done ;;
    tprobe_diag) for v in ${DIAGS:-expdiv}; do
                run tprobe_$v 600 env AMP_LIB_PATH=amp-sparc-spatialmodulation_amd/lib_diag/libampsparc_$v.so python3 tools/t_probe.py || exit 1
            done ;;
    ab_pkg0) run ab_def 300 python3 bench.py --no-cpu-baseline &&
             run ab_pkg0 300 env AMP_LIB_PATH=amp-sparc-spatialmodulation_amd/lib_diag/libampsparc_pkg0.so python3 bench.py --no-cpu-baseline &&
             run ab_def2 300 python3 bench.py --no-cpu-baseline &&
             run ab_pkg0_2 300 env AMP_LIB_PATH=amp-sparc-spatialmodulation_amd/lib_diag/libampsparc_pkg0.so python3 bench.py --no-cpu-baseline &&
             run ab_cfg3 300 python3 tools/configs_bench.py cfg3 cfg3-qpsk &&
             run ab_cfg3_pkg0 300 env AMP_LIB_PATH=amp-sparc-spatialmodulation_amd/lib_diag/libampsparc_pkg0.so python3 tools/configs_bench.py cfg3 cfg3-qpsk ;;
    ab_stg) run ab_stg_def 300 python3 bench.py --no-cpu-baseline &&
            run ab_stg0 300 env AMP_LIB_PATH=amp-sparc-spatialmodulation_amd/lib_diag/libampsparc_stg0.so python3 bench.py --no-cpu-baseline &&
            run ab_stg_def2 300 python3 bench.py --no-cpu-baseline &&
            run ab_stg0_2 300 env AMP_LIB_PATH=amp-sparc-spatialmodulation_amd/lib_diag/libampsparc_stg0.so python3 bench.py --no-cpu-baseline ;;
    # A/B of a diagnostic library (lib_diag/libampsparc_$DIAG.so) against the default on one box
    ab) D=amp-sparc-spatialmodulation_amd/lib_diag/libampsparc_${DIAG:-tgr}.so
        run ab_def 300 python3 bench.py --no-cpu-baseline &&
        run ab_${DIAG:-tgr} 300 env AMP_LIB_PATH=$D python3 bench.py --no-cpu-baseline &&
        run ab_def2 300 python3 bench.py --no-cpu-baseline &&
        run ab_${DIAG:-tgr}_2 300 env AMP_LIB_PATH=$D python3 bench.py --no-cpu-baseline ;;
    # A/B of an environment switch (ENVAB="NAME=value") against the default on one box
    ab_env) run abe_def 300 python3 bench.py --no-cpu-baseline &&
            run abe_env 300 env $ENVAB python3 bench.py --no-cpu-baseline &&
            run abe_def2 300 python3 bench.py --no-cpu-baseline &&
            run abe_env2 300 env $ENVAB python3 bench.py --no-cpu-baseline ;;
    tests_ytil) run tests_ytil 300 $PYT tests/test_gpu_vamp.py -m gpu -k "ytil or engines_agree or n256 or x3_gemm" ;;
    trace_diag) run trace_${DIAG:-tgr} 300 env AMP_LIB_PATH=amp-sparc-spatialmodulation_amd/lib_diag/libampsparc_${DIAG:-tgr}.so python3 tools/trace_persist.py --config cfg4 ;;
    configs_res1) run configs_res1 300 python3 tools/configs_bench.py cfg2 cfg2-epochs8 cfg2-res1 ;;
    ttrace1) run ttrace1 600 python3 tools/t_trace.py --point cfg4_vamp_qpsk:1/0 --save "" --variants persistent,launches ;;
    cfg5_kc) run cfg5_kc256 600 python3 tools/cfg5_bench.py &&
             run cfg5_kc512 600 env AMP_BAMP_KC=512 python3 tools/cfg5_bench.py ;;
    transpk) run transpk 300 tools/ubench/bin/trans_pk 3 ;;
    gemmacc) run gemmacc 600 python3 tools/gemm_accuracy.py --point cfg4_vamp_qpsk:1/0 &&
             run gemmacc0 600 python3 tools/gemm_accuracy.py --point cfg4_vamp_qpsk:0/0 ;;
    curves) run_nogate curves 900 python3 -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_vamp.py -m gpu -k curve_point -rf ;;
    tests_nocurve) run tests_nocurve 1100 $PYT tests -m gpu -k "not curve_point" ;;
    tests_repro) run tests_repro 600 $PYT tests/test_gpu_vamp.py tests/test_gpu_bamp_scamp.py tests/test_gpu_epochs.py -m gpu -k "reproducible or n256 or g2_denoiser or per_channel or res1" ;;
    *) echo "unknown step $s"; exit 2 ;;
    esac
done
echo "=== done"
