# Ray-regrouping A/B in one GPU call: parity tests, then C3 and C5 frames by park depth (bench.py --regroup).
# Usage (via gpurun): bash tools/regroup_ab.sh <outdir under gpurun_out>
O=gpurun_out/${1:-regroup}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
for g in 0 2; do
timeout -k 10 200 python -u bench.py --regroup $g --steps 20 --warmup 3 --no-cpu-baseline > $O/c3_g$g.json 2>/dev/null || exit 2
done
for g in 0 2 3 4; do
timeout -k 10 200 python -u bench.py --config c5 --regroup $g --steps 5 --warmup 1 --no-cpu-baseline > $O/c5_g$g.json 2>/dev/null || exit 3
done
exit 0
