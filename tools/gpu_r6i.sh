# Round-6 GPU call: the split frame's launch size at the ReadMe screenshot (host-side only).
O=gpurun_out/${1:-r6i}
bash tools/gpu_step.sh $O \
 "400 ab_shot128 python -u tools/ab.py run --only base,lt31,lt29 --scene default --width 1920 --height 1080 --depth 20 --ss 128 --frames 1 --rounds 4 --later-frame 2 --warmup 1"
