# One GPU call: interleaved A/B of the given variants on the frames the lanes mode runs (the screenshot, 2x2 SSAA,
# jittered one-sample frames of C3's scene and of the default scene).  Usage: bash tools/ab_lanes.sh <outdir> <variants>
O=$PWD/gpurun_out/${1:-abl}
V=${2:-base}
mkdir -p $O
A="timeout -k 10 300 python -u tools/ab.py run --only $V --rounds 10"
$A --scene default --width 1920 --height 1080 --depth 20 --ss 4 > $O/shot.jsonl 2> $O/shot.err || exit 1
$A --scene default --width 1920 --height 1080 --depth 8 --ss 2 > $O/ss2.jsonl 2> $O/ss2.err || exit 2
$A --scene synth16 --width 3840 --height 2160 --depth 8 --additive 1 > $O/add1.jsonl 2> $O/add1.err || exit 3
$A --scene default --width 1920 --height 1080 --depth 15 --additive 1 > $O/add1d.jsonl 2> $O/add1d.err || exit 4
exit 0
