set -o pipefail
mkdir -p gpurun_out/r5_c1
O=gpurun_out/r5_c1
T="timeout -k 10 240"
$T python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-fast-math-line --no-strips-line > $O/pair_a.json 2> $O/pair_a.err &&
$T python bench.py --workload strips --width 6144 --height 4096 --nscales 5 --warps 30 --batch 3 --inflight 1 --steps 4 --warmup 1 --no-cpu-baseline > $O/batch3x1.json 2> $O/batch3x1.err &&
$T python bench.py --workload strips --width 6144 --height 4096 --nscales 5 --warps 30 --batch 3 --inflight 2 --steps 2 --warmup 1 --no-cpu-baseline > $O/batch3x2.json 2> $O/batch3x2.err &&
$T python bench.py --workload strips --width 6144 --height 4096 --nscales 5 --warps 30 --batch 1 --inflight 3 --steps 4 --warmup 1 --no-cpu-baseline > $O/batch1x3.json 2> $O/batch1x3.err &&
$T python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-fast-math-line --no-strips-line > $O/pair_b.json 2> $O/pair_b.err
