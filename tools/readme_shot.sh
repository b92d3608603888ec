# One GPU call: the split / screenshot tests, the C3 region profile, and the shot128 bench line.
# Usage: bash tools/readme_shot.sh <outdir under gpurun_out>
O=$PWD/gpurun_out/${1:-shot}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_split.py tests/test_dropin_pulse.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/regionprof.py > $O/regionprof_c3.json 2> $O/regionprof.err || exit 2
timeout -k 10 300 python -u bench.py --config shot128 > $O/shot128.json 2> $O/shot128.err || exit 3
exit 0
