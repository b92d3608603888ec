# One GPU call: the mask parity tests, then interleaved A/B of the lanes-mode masks on the screenshot frame, ss2 and
# jittered one-sample frames.  Usage: bash tools/ab_masks.sh <outdir under gpurun_out>
O=$PWD/gpurun_out/${1:-abm}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "primary_masks or golden or full_size_hash" --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
A="timeout -k 10 200 python -u tools/ab.py run --only base,noprimlanes --rounds 10"
$A --scene default --width 1920 --height 1080 --depth 20 --ss 4 > $O/shot.jsonl 2> $O/shot.err || exit 2
$A --scene default --width 1920 --height 1080 --depth 8 --ss 2 > $O/ss2.jsonl 2> $O/ss2.err || exit 3
$A --scene synth16 --width 3840 --height 2160 --depth 8 --additive 1 > $O/add1.jsonl 2> $O/add1.err || exit 4
$A --scene default --width 1920 --height 1080 --depth 15 --additive 1 > $O/add1d.jsonl 2> $O/add1d.err || exit 5
exit 0
