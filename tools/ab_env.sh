#!/bin/bash
# Interleaved A/B of one env knob on the bench's workloads (one GPU box).
# Usage: tools/ab_env.sh VAR "VAL_A VAL_B" ROUNDS WORKLOAD... (outputs gpurun_out/ab_env/)
set -o pipefail
cd "$(dirname "$0")/.."
VAR=$1; VALS=$2; ROUNDS=$3; shift 3
OUT=gpurun_out/ab_env
mkdir -p "$OUT"
for r in $(seq 1 "$ROUNDS"); do
  for wl in "$@"; do
    for v in $VALS; do
      env "$VAR=$v" timeout -k 10 200 python3 bench.py --workload "$wl" --steps 10 --warmup 3 --no-cpu-baseline \
        --no-variants --no-host-abi --no-legs > "$OUT/${wl}_${v}_$r.json" 2> "$OUT/${wl}_${v}_$r.err" || { echo "bench $wl $v failed"; tail -5 "$OUT/${wl}_${v}_$r.err"; exit 1; }
      python3 - "$OUT/${wl}_${v}_$r.json" "$VAR=$v" "$wl" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d.get("kernels", {})
print("%s %-22s %8.3f ms  %s" % (sys.argv[3], sys.argv[2], d["ms_per_step"],
      "  ".join("%s %.1fus x%d" % (n, v["avg_us"], v["launches"]) for n, v in k.items())))
PY
    done
  done
done
