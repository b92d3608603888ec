# One GPU call: interleaved A/B of the given variants on the small-scene configs (C3, the screenshot, C2 depth 4).
# Usage: bash tools/ab_small.sh <outdir under gpurun_out> <variant,variant,..>
O=$PWD/gpurun_out/${1:-abs}
V=${2:-base}
mkdir -p $O
A="timeout -k 10 300 python -u tools/ab.py run --only $V --rounds 10"
$A --scene synth16 --width 3840 --height 2160 --depth 8 > $O/c3.jsonl 2> $O/c3.err || exit 1
$A --scene default --width 1920 --height 1080 --depth 20 --ss 4 > $O/shot.jsonl 2> $O/shot.err || exit 2
$A --scene default --width 1920 --height 1080 --depth 4 > $O/c2d4.jsonl 2> $O/c2d4.err || exit 3
exit 0
