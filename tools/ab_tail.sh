# One GPU call: the whole GPU suite, then an interleaved A/B of the given variants on C3, C2 (depth 1 and 4), C1 and C5.
# Usage: bash tools/ab_tail.sh <outdir under gpurun_out> <variants>
O=$PWD/gpurun_out/${1:-abtail}
V=${2:-base}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
A="timeout -k 10 300 python -u tools/ab.py run --only $V --rounds 10"
$A --scene synth16 --width 3840 --height 2160 --depth 8 > $O/c3.jsonl 2> $O/c3.err || exit 2
$A --scene default --width 1920 --height 1080 --depth 1 --frames 20 > $O/c2d1.jsonl 2> $O/c2d1.err || exit 3
$A --scene default --width 1920 --height 1080 --depth 4 --frames 20 > $O/c2d4.jsonl 2> $O/c2d4.err || exit 4
$A --scene default --width 640 --height 480 --depth 4 --frames 30 > $O/c1.jsonl 2> $O/c1.err || exit 5
$A --scene stress4096 --width 3840 --height 2160 --depth 12 --frames 4 --rounds 6 > $O/c5.jsonl 2> $O/c5.err || exit 6
exit 0
