#!/bin/bash
# A/B of bench.py flag sets in one GPU call: one bench line per flag set, alternating.
# usage: tools/ab_flags.sh ROUNDS OUT_PREFIX "--flags a" "--flags b" ...
# (flags common to every arm in BENCH_FLAGS; each line's value, unit and ms_per_step printed)
set -o pipefail
mkdir -p gpurun_out
rounds=$1; shift
prefix=$1; shift
for i in $(seq 1 "$rounds"); do
  j=0
  for flags in "$@"; do
    j=$((j + 1))
    out=gpurun_out/${prefix}_${j}_$i
    timeout -k 10 300 python bench.py --no-strips-line --no-fast-math-line --no-cpu-baseline \
      $BENCH_FLAGS $flags > $out.json 2> $out.err || exit $?
    python - "$out.json" "$flags" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{sys.argv[2]:40s} {d['value']:.3f} {d['unit']}  ms/step {d['ms_per_step']}", flush=True)
PY
  done
done
