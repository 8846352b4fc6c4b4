#!/bin/bash
# A/B of the speculation knob in one GPU call: C2 bench lines with TVL1_SPEC=1/0,
# alternating, plus the single-pair breakdown each bench line carries.
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for sp in 1 0; do
    TVL1_SPEC=$sp timeout -k 10 150 python bench.py --no-strips-line --no-fast-math-line --no-cpu-baseline \
      > gpurun_out/ab_spec_${sp}_$i.json 2> gpurun_out/ab_spec_${sp}_$i.err || exit $?
    python - "$sp" "$i" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/ab_spec_{sys.argv[1]}_{sys.argv[2]}.json").read().strip().splitlines()[-1])
print("spec", sys.argv[1], "run", sys.argv[2], "pairs/s", d["value"], "single_pair_ms", d.get("single_pair_ms"),
      "breakdown", d.get("pair_breakdown_ms"), flush=True)
PY
  done
done
