# One GPU call: the parity tests of the trace paths, then an interleaved A/B of built variants and the C3
# region profile.  Usage: bash tools/ab_round.sh <outdir under gpurun_out> <variant,variant,..> [ab.py args]
R=$PWD
O=$R/gpurun_out/${1:-ab}
V=${2:-base}
shift 2
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kat.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab.py run --only $V --rounds 10 "$@" > $O/ab.json 2> $O/ab.err || exit 2
timeout -k 10 200 python -u tools/regionprof.py > $O/regionprof.json 2>&1 || exit 3
exit 0
