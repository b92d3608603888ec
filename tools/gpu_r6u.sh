# Round-6 GPU call: the triangle footprint test on a view's first frame (RFX_SEG0_FOOT, foot1) -- interleaved A/B with
# the per-view masks off (a moving camera) and on (a still camera: unchanged code path), GPU suite on foot1 first.
O=gpurun_out/${1:-r6u}
AB="python -u tools/ab.py run --only base,foot1"
bash tools/gpu_step.sh $O \
 "300 ab_c3_moving $AB --rounds 10 --prim 0" \
 "300 ab_c3_still $AB --rounds 8 --prim 1" \
 "200 ab_c2d4_moving $AB --rounds 10 --scene default --width 1920 --height 1080 --depth 4 --frames 30 --prim 0" \
 "300 ab_shot_moving $AB --rounds 6 --scene default --width 1920 --height 1080 --depth 20 --ss 4 --frames 10 --prim 0" \
 "200 ab_c1_moving $AB --rounds 10 --scene default --width 640 --height 480 --depth 4 --frames 30 --prim 0"
