# Final-library profiling, part 2: PMC records of the C4 frame, the screenshot and shot128, and shot128's rocprofv3
# kernel stats.
R=$PWD
O=$R/gpurun_out/${1:-r6f2}
mkdir -p $O
PMC_ONLY="c4 shot shot128" bash tools/pmc_configs.sh ${1:-r6f2}/pmc || exit 4
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_shot128 -o run -- python3 $R/bench.py --config shot128 --steps 2 --warmup 1 --no-cpu-baseline --no-first-view > $O/bench_shot128_under_rocprof.json 2> $O/prof_shot128.err || exit 5
exit 0
