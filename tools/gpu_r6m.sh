# Round-6 GPU call: the count kernel as a grid-stride launch of RFX_COUNT_WGS workgroups (cw0: one per block) on top of
# the pre-pass rework -- GPU suite on the product build, interleaved A/B at C3, the C4 frame and C2, kernel stats.
O=gpurun_out/${1:-r6m}
R=$PWD
AB="python -u tools/ab.py run"
bash tools/gpu_step.sh $O \
 "600 gpu_tests python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "300 ab_c3 $AB --only head,base,cw0,cw1024,cw4096 --rounds 8" \
 "400 ab_c4 $AB --only head,base,cw0,cw4096 --rounds 6 --width 7680 --height 4320 --frames 5" \
 "200 ab_c2d1 $AB --only head,base,cw0 --rounds 10 --scene default --width 1920 --height 1080 --depth 1 --frames 30" \
 "300 prof_c3 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-c4"
