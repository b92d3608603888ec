# Round-6 GPU call: the one-pass pre-pass's block limit (ticket contention grows with the block count).
O=gpurun_out/${1:-r6e}
V=base,fmax256,fmax512,fused0
bash tools/gpu_step.sh $O \
 "120 ab_c1 python -u tools/ab.py run --only $V --rounds 12 --scene default --width 640 --height 480 --depth 4 --frames 30" \
 "120 ab_960 python -u tools/ab.py run --only $V --rounds 12 --scene default --width 960 --height 540 --depth 4 --frames 30" \
 "120 ab_720 python -u tools/ab.py run --only $V --rounds 12 --scene default --width 1280 --height 720 --depth 4 --frames 30" \
 "120 ab_c2d1 python -u tools/ab.py run --only $V --rounds 12 --scene default --width 1920 --height 1080 --depth 1 --frames 30" \
 "120 ab_c2d4 python -u tools/ab.py run --only $V --rounds 12 --scene default --width 1920 --height 1080 --depth 4 --frames 20"
