# Round-6 GPU call after the pre-pass block limit (host-only): the GPU suite, the default bench line and the lines of
# the configs whose pre-pass form changed (C1 keeps the one-pass kernel, C2 returns to the two-kernel form).
O=$PWD/gpurun_out/${1:-r6g}
mkdir -p $O/configs
B="timeout -k 10 300 python -u bench.py"
timeout -k 10 500 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
$B > $O/bench_c3.json 2> $O/bench_c3.err || exit 2
$B --config c1 --steps 50 --warmup 5 --cpu-stride 1 > $O/configs/c1_default_640x480_d4.json 2> $O/c1.err || exit 3
$B --config c2 --depth 1 --steps 30 --warmup 3 --cpu-stride 8 > $O/configs/c2_default_1920x1080_d1.json 2> $O/c2a.err || exit 4
$B --config c2 --steps 30 --warmup 3 --cpu-stride 4 > $O/configs/c2_default_1920x1080_d4.json 2> $O/c2b.err || exit 5
exit 0
