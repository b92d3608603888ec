# C5 diagnostics in one GPU call: region cycle shares + cull statistics, segment-loop lane use, and bench
# lines for C3 and C5.  Usage (via gpurun): bash tools/diag_c5.sh <outdir under gpurun_out>
R=$PWD
O=$R/gpurun_out/${1:-diag_c5}
mkdir -p $O
timeout -k 10 200 python -u tools/regionprof.py --scene stress4096 --depth 12 > $O/regionprof_c5.json 2>&1 || exit 1
timeout -k 10 200 python -u tools/regionprof.py > $O/regionprof_c3.json 2>&1 || exit 2
timeout -k 10 200 python -u tools/segstats.py stress4096 12 > $O/segstats_c5.txt 2>&1 || exit 3
timeout -k 10 300 python -u bench.py --config c5 --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err || exit 4
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err || exit 5
exit 0
