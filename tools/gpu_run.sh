#!/bin/bash
# Generic GPU-box pass: run each step in STEPS (";"-separated shell commands) under its own time limit,
# output to gpurun_out/$TAG/step<i>.log.  A step that fails with exit 1 (test failures) lets the next step run;
# any other non-zero exit (timeout 124/137, abort 134, segfault 139, ...) ends the pass there.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-run}
mkdir -p $OUT
LIMIT=${LIMIT:-600}
i=0
IFS=';' read -ra CMDS <<< "$STEPS"
for c in "${CMDS[@]}"; do
  i=$((i+1))
  echo "== step $i: $c"
  timeout -k 10 $LIMIT bash -c "$c" > $OUT/step$i.log 2>&1
  rc=$?
  tail -${TAILN:-6} $OUT/step$i.log
  echo "== step $i rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
