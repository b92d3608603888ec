# One GPU call: interleaved A/B of the given variants on high-SSAA frames whose pre-pass has many blocks: 320x180 at
# 128x128 (one launch, 230K blocks) and 480x270 at 128x128 (two split launches).  Usage: bash tools/ab_bigss.sh <outdir> <variants>
O=$PWD/gpurun_out/${1:-abbig}
V=${2:-base}
mkdir -p $O
A="timeout -k 10 400 python -u tools/ab.py run --only $V"
$A --rounds 6 --scene default --width 320 --height 180 --depth 20 --ss 128 --frames 3 > $O/ss128_320.jsonl 2> $O/ss128_320.err || exit 1
$A --rounds 4 --scene default --width 480 --height 270 --depth 20 --ss 128 --frames 2 > $O/ss128_480.jsonl 2> $O/ss128_480.err || exit 2
exit 0
