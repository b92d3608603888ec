R=$PWD
O=$R/gpurun_out/${1:-diag2}
mkdir -p $O
timeout -k 10 200 python -u tools/regionprof.py --scene stress4096 --depth 12 > $O/regionprof_c5.json 2>&1 || exit 1
timeout -k 10 200 python -u tools/regionprof.py --scene stress4096 --depth 1 > $O/regionprof_c5_d1.json 2>&1 || exit 1
for d in 1 2 3 12; do
timeout -k 10 300 python -u bench.py --config c5 --depth $d --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_c5_d$d.json 2> $O/bench_c5_d$d.err || exit 4
done
exit 0
