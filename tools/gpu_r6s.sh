# Round-6 GPU call: kernel traces of the small configs (C1, C2 d1 / d4) on the final build, for per-frame gaps.
R=$PWD
O=$R/gpurun_out/${1:-r6s}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for c in "c1 --config c1" "c2d1 --config c2 --depth 1" "c2d4 --config c2"; do
  set -- $c; n=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$n -o run -- python3 $R/bench.py "$@" --steps 30 --warmup 3 --no-cpu-baseline --no-first-view > $O/bench_$n.json 2> $O/prof_$n.err || exit 2
done
exit 0
