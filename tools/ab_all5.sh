# One GPU call: interleaved A/B of the given variants on C1, C3, C2 depth 4, the screenshot and C5.
# Usage: bash tools/ab_all5.sh <outdir under gpurun_out> <variants>
O=$PWD/gpurun_out/${1:-ab5}
V=${2:-base}
mkdir -p $O
A="timeout -k 10 300 python -u tools/ab.py run --only $V --rounds 10"
$A --scene default --width 640 --height 480 --depth 4 --frames 30 > $O/c1.jsonl 2> $O/c1.err || exit 1
$A --scene synth16 --width 3840 --height 2160 --depth 8 > $O/c3.jsonl 2> $O/c3.err || exit 2
$A --scene default --width 1920 --height 1080 --depth 4 --frames 20 > $O/c2d4.jsonl 2> $O/c2d4.err || exit 3
$A --scene default --width 1920 --height 1080 --depth 20 --ss 4 > $O/shot.jsonl 2> $O/shot.err || exit 4
$A --scene stress4096 --width 3840 --height 2160 --depth 12 --frames 4 --rounds 6 > $O/c5.jsonl 2> $O/c5.err || exit 5
exit 0
