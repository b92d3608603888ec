# Round-6 GPU call: kernel traces of the 4x4 screenshot and the C4 frame on the final build (per-frame gaps).
R=$PWD
O=$R/gpurun_out/${1:-r6w}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for c in "shot --config shot" "c4 --config c4"; do
  set -- $c; n=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$n -o run -- python3 $R/bench.py "$@" --steps 20 --warmup 3 --no-cpu-baseline --no-first-view > $O/bench_$n.json 2> $O/prof_$n.err || exit 2
done
exit 0
