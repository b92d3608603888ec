# One GPU call: bench.py at every BASELINE.json config that fits one GPU (C1, C2 d1/d4, C3, C4 frame
# size on 1 GPU, C5), each with its CPU-reference sample.  Usage: bash tools/configs_round.sh <outdir>
O=$PWD/gpurun_out/${1:-configs}
mkdir -p $O
B="timeout -k 10 300 python -u bench.py"
$B --scene default --width 640 --height 480 --depth 4 --steps 50 --warmup 5 --cpu-stride 1 > $O/c1_default_640x480_d4.json 2> $O/c1.err || exit 1
$B --scene default --width 1920 --height 1080 --depth 1 --steps 30 --warmup 3 --cpu-stride 8 > $O/c2_default_1920x1080_d1.json 2> $O/c2a.err || exit 2
$B --scene default --width 1920 --height 1080 --depth 4 --steps 30 --warmup 3 --cpu-stride 4 > $O/c2_default_1920x1080_d4.json 2> $O/c2b.err || exit 3
$B --steps 20 --warmup 3 > $O/c3_synth16_3840x2160_d8.json 2> $O/c3.err || exit 4
$B --width 7680 --height 4320 --steps 10 --warmup 2 --cpu-stride 16 > $O/c4_synth16_7680x4320_d8_1gpu.json 2> $O/c4.err || exit 5
$B --scene stress4096 --depth 12 --steps 5 --warmup 1 --cpu-stride 270 > $O/c5_stress4096_3840x2160_d12.json 2> $O/c5.err || exit 6
exit 0
