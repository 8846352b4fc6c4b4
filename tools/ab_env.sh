#!/bin/bash
# A/B of engine environment settings in one GPU call: C2 bench lines per setting, alternating.
# usage: tools/ab_env.sh ROUNDS "ENV=a ..." "ENV=b ..." ...   (extra bench flags in BENCH_FLAGS)
set -o pipefail
mkdir -p gpurun_out
rounds=$1; shift
for i in $(seq 1 "$rounds"); do
  j=0
  for setting in "$@"; do
    j=$((j + 1))
    out=gpurun_out/ab_env_${j}_$i
    env $setting timeout -k 10 150 python bench.py --no-strips-line --no-fast-math-line --no-cpu-baseline \
      $BENCH_FLAGS > $out.json 2> $out.err || exit $?
    python - "$out.json" "$setting" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{sys.argv[2]:40s} pairs/s {d['value']:.3f}  single_pair_ms {d.get('single_pair_ms')}", flush=True)
PY
  done
done
