# Per-depth frame cost and region shares of one scene (diagnostics, one GPU call).
# Usage (via gpurun): bash tools/diag_depth.sh <outdir> <config> <depth>...
R=$PWD
O=$R/gpurun_out/${1:-diag_depth}
CFG=${2:-c5}
shift 2
mkdir -p $O
for d in "$@"; do
timeout -k 10 300 python -u bench.py --config $CFG --depth $d --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_${CFG}_d$d.json 2> $O/bench_${CFG}_d$d.err || exit 1
done
exit 0
