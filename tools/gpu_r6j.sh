# Round-6 GPU call: the RNG pre-pass's integer accept test (RFX_RNG_INT_ACCEPT) -- GPU suite, interleaved A/B of whole
# frames at C1 / C2 / C3, kernel stats of the C3 line (rng_count / rng_emit per launch).
O=gpurun_out/${1:-r6j}
R=$PWD
V=base,intacc0
bash tools/gpu_step.sh $O \
 "600 gpu_tests python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "200 ab_c3 python -u tools/ab.py run --only $V --rounds 10" \
 "120 ab_c1 python -u tools/ab.py run --only $V --rounds 12 --scene default --width 640 --height 480 --depth 4 --frames 30" \
 "120 ab_c2d1 python -u tools/ab.py run --only $V --rounds 12 --scene default --width 1920 --height 1080 --depth 1 --frames 30" \
 "300 prof_c3 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-c4"
