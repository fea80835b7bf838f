#!/bin/bash
# rocprof kernel stats of one bench config: CONFIG=cfg3 TAG=x [EXTRA="--sampler device"] bash tools/prof_stats.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-ps}
mkdir -p $OUT
c=${CONFIG:-cfg3}
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_$c -o prof --output-format csv -- python3 bench.py --config $c --steps 50 --warmup 10 --cpu-baseline-seconds 0 $EXTRA > $OUT/rocprof_$c.log 2>&1 || { tail -20 $OUT/rocprof_$c.log; exit 1; }
f=$(find $OUT/prof_$c -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
steps = max(int(r["Calls"]) for r in rows if "adam_step" in r["Name"])
tot = sum(int(r["TotalDurationNs"]) for r in rows)
print(f"steps {steps}  per step {tot / steps / 1000:.1f} us")
for r in sorted(rows, key=lambda r: -int(r["TotalDurationNs"]))[:int(__import__('os').environ.get('TOP', 30))]:
    print(f"{int(r['TotalDurationNs']) / steps / 1000:8.1f} {int(r['Calls']) / steps:5.1f} {r['Name'][:110]}")
PY
