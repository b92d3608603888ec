# Final-library profiling, part 1: rocprofv3 kernel stats of the C3 and C5 bench runs, PMC records of C3, C5, C1, C2.
R=$PWD
O=$R/gpurun_out/${1:-r6f1}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-c4 > $O/bench_c3_under_rocprof.json 2> $O/prof_c3.err || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o run -- python3 $R/bench.py --config c5 --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_c5_under_rocprof.json 2> $O/prof_c5.err || exit 3
cd $R
PMC_ONLY="c3 c5 c1 c2" bash tools/pmc_configs.sh ${1:-r6f1}/pmc || exit 4
exit 0
