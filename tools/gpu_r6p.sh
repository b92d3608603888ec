# Round-6 GPU call on the final library (device a8853a24): smoke(), shot128's rocprofv3 kernel stats.
R=$PWD
O=$R/gpurun_out/${1:-r6p}
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_shot128 -o run -- python3 $R/bench.py --config shot128 --steps 2 --warmup 1 --no-cpu-baseline --no-first-view > $O/bench_shot128_under_rocprof.json 2> $O/prof_shot128.err || exit 2
exit 0
