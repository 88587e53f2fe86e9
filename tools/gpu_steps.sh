#!/usr/bin/env bash
# Run GPU steps given as arguments "name|timeout_s|command" in order, each under its own time
# limit, logs under gpurun_out/$TAG/; any failure (non-zero exit, fault, abort, time limit) ends
# the script at once, so nothing more runs on the GPU after it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-steps}; mkdir -p "$O"
for spec in "$@"; do
    name=${spec%%|*}; rest=${spec#*|}; lim=${rest%%|*}; cmd=${rest#*|}
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$lim" bash -c "$cmd" > "$O/$name.log" 2>&1
    rc=$?
    echo "=== $name rc=$rc"; tail -4 "$O/$name.log"
    [ $rc -ne 0 ] && { echo "stopping after $name"; exit $rc; }
done
echo "=== done"
