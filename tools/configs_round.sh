# One GPU call: bench.py at every BASELINE.json config that fits one GPU (C1, C2 d1/d4, C3, C4 frame on
# 1 GPU, C5) and the screenshot workload, each with its CPU-reference sample (and all-core context row).
# Usage: bash tools/configs_round.sh <outdir under gpurun_out>
O=$PWD/gpurun_out/${1:-configs}
mkdir -p $O
B="timeout -k 10 300 python -u bench.py"
$B --config c1 --steps 50 --warmup 5 --cpu-stride 1 > $O/c1_default_640x480_d4.json 2> $O/c1.err || exit 1
$B --config c2 --depth 1 --steps 30 --warmup 3 --cpu-stride 8 > $O/c2_default_1920x1080_d1.json 2> $O/c2a.err || exit 2
$B --config c2 --steps 30 --warmup 3 --cpu-stride 4 > $O/c2_default_1920x1080_d4.json 2> $O/c2b.err || exit 3
$B --config c3 --steps 20 --warmup 3 > $O/c3_synth16_3840x2160_d8.json 2> $O/c3.err || exit 4
$B --config c4 --steps 10 --warmup 2 --cpu-stride 16 > $O/c4_synth16_7680x4320_d8_1gpu.json 2> $O/c4.err || exit 5
$B --config c5 --steps 5 --warmup 1 --cpu-stride 270 > $O/c5_stress4096_3840x2160_d12.json 2> $O/c5.err || exit 6
$B --config shot --steps 10 --warmup 2 > $O/shot_default_1920x1080_d20_ss4.json 2> $O/shot.err || exit 7
$B --config shot128 > $O/shot128_default_1920x1080_d20_ss128.json 2> $O/shot128.err || exit 8
exit 0
