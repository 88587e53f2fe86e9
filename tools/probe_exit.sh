#!/usr/bin/env bash
# rocprofv3 exit-crash probe: one VAMP forward per engine under --kernel-trace (tools/exit_probe.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; O=gpurun_out/probe; mkdir -p $O
for m in ${PROBES:-"persistent x" "persistent profile"}; do
  set -- $m
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/$1$2 -o p --output-format csv -- python3 tools/exit_probe.py $1 $2 > $O/$1$2.log 2>&1
  rc=$?; echo "$m rc=$rc"; tail -2 $O/$1$2.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
