#!/bin/bash
# r4 A/B: the 3/4-iteration rolling passes with their input rows staged in LDS by the buffer
# unit's LDS path (ab_r4q/LDS: <4,2> 164 VGPRs, 3 wavefronts per SIMD) against the in-tree
# register ring (189, 2 per SIMD).  Parity first (the variant must be bit-identical), then a
# kernel trace of one C2 pair each, then C2 and strips alternations.
set -o pipefail
out=gpurun_out/r4q
mkdir -p $out
export TVL1_ENGINE_SO=ab_r4q/LDS/libtvl1_hip.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch.py -x -q --timeout 200 --timeout-method thread > $out/t_lds.log 2>&1 || { echo "PARITY_FAIL"; tail -30 $out/t_lds.log; exit 1; }
echo "LDS parity: $(tail -1 $out/t_lds.log)"
unset TVL1_ENGINE_SO
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for d in . ab_r4q/LDS; do
  if [ "$d" = "." ]; then unset TVL1_ENGINE_SO; else export TVL1_ENGINE_SO=$d/libtvl1_hip.so; fi
  tag=$(echo "$d" | tr '/.' '__')
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/k$tag -o run -- python3 bench.py --steps 2 --warmup 1 --inflight 1 --no-cpu-baseline --no-fast-math-line --no-strips-line > $out/k$tag.log 2>&1 || { echo TRACE_FAIL; tail -5 $out/k$tag.log; exit 1; }
done
for i in 1 2 3; do
  for d in . ab_r4q/LDS; do
    if [ "$d" = "." ]; then unset TVL1_ENGINE_SO; else export TVL1_ENGINE_SO=$d/libtvl1_hip.so; fi
    tag=$(echo "$d" | tr '/.' '__')
    timeout -k 10 200 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-fast-math-line --no-strips-line > $out/c2$tag$i.log 2>&1 || { echo BENCH_FAIL $d; exit 1; }
    echo "$d c2 round $i $(tail -1 $out/c2$tag$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("pairs/s", d["value"], "single_pair_ms", d.get("single_pair_ms"))')"
    timeout -k 10 200 python bench.py --workload strips --steps 3 --warmup 1 --no-cpu-baseline > $out/s$tag$i.log 2>&1 || { echo STRIPS_FAIL $d; exit 1; }
    echo "$d strips round $i $(tail -1 $out/s$tag$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"])')"
  done
done | tee $out/ab.txt
echo ALL_DONE
