# One GPU call: the large-scene parity tests, then an interleaved A/B on C5 of the given variants.
# Usage: bash tools/ab_c5.sh <outdir under gpurun_out> <variant,variant,..>
O=$PWD/gpurun_out/${1:-abc5}
V=${2:-base}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "stress or 4096 or regroup or c5 or planes300 or large" --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/ab.py run --only $V --rounds 8 --scene stress4096 --width 3840 --height 2160 --depth 12 > $O/c5.jsonl 2> $O/c5.err || exit 2
exit 0
