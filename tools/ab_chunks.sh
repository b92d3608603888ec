# One GPU call: the SSAA parity tests (goldens, split frames, the drop-in screenshots), then an interleaved A/B of the
# given variants on chunk-mode frames (sampleNum > 8).  Usage: bash tools/ab_chunks.sh <outdir under gpurun_out> <variants>
O=$PWD/gpurun_out/${1:-abch}
V=${2:-base}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_parity.py tests/test_dropin_pulse.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
A="timeout -k 10 300 python -u tools/ab.py run --only $V --rounds 8"
$A --scene default --width 480 --height 270 --depth 20 --ss 64 --frames 4 > $O/ss64_480.jsonl 2> $O/ss64_480.err || exit 2
$A --scene default --width 960 --height 540 --depth 20 --ss 16 --frames 6 > $O/ss16_960.jsonl 2> $O/ss16_960.err || exit 3
$A --scene default --width 320 --height 180 --depth 20 --ss 128 --frames 3 --rounds 5 > $O/ss128_320.jsonl 2> $O/ss128_320.err || exit 4
exit 0
