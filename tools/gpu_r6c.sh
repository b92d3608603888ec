# Round-6 GPU call: the GPU suite and interleaved A/B of the division guards, the large-scene default and the tile scan.
O=gpurun_out/${1:-r6c}
bash tools/gpu_step.sh $O \
 "420 gpu_tests python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 300 --timeout-method thread" \
 "150 ab_c3 python -u tools/ab.py run --only base,div0,divfast2,divall2 --rounds 10" \
 "100 ab_c2 python -u tools/ab.py run --only base,div0,divfast2,divall2 --scene default --width 1920 --height 1080 --depth 4 --frames 20 --rounds 10" \
 "150 ab_c5 python -u tools/ab.py run --only base,div0,divsel1,prefetch1 --scene stress4096 --depth 12 --frames 4 --rounds 6" \
 "120 ab_shot python -u tools/ab.py run --only base,div0 --scene default --width 1920 --height 1080 --depth 20 --ss 4 --frames 10 --rounds 8" \
 "200 ab_shot128 python -u tools/ab.py run --only base,tiles0 --scene default --width 1920 --height 1080 --depth 20 --ss 128 --frames 1 --rounds 3 --later-frame 2 --warmup 1"
