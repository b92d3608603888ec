# One GPU call: interleaved A/B of the given variants on split frames (128x128 SSAA, depth 20): 480x270 (2 launches)
# and 640x360 (4 launches).  Usage: bash tools/ab_split.sh <outdir under gpurun_out> <variants>
O=$PWD/gpurun_out/${1:-absplit}
V=${2:-base}
mkdir -p $O
A="timeout -k 10 400 python -u tools/ab.py run --only $V"
$A --rounds 4 --scene default --width 480 --height 270 --depth 20 --ss 128 --frames 2 > $O/ss128_480.jsonl 2> $O/ss128_480.err || exit 1
$A --rounds 3 --scene default --width 640 --height 360 --depth 20 --ss 128 --frames 2 > $O/ss128_640.jsonl 2> $O/ss128_640.err || exit 2
exit 0
