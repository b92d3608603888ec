O=gpurun_out/r6a
bash tools/gpu_step.sh $O \
 "420 gpu_tests python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 300 --timeout-method thread" \
 "200 ab_c3 python -u tools/ab.py run --only base,div0,divsingle,divall2 --rounds 10" \
 "150 ab_c1 python -u tools/ab.py run --only base,ticket0,fused0,lookback0 --rounds 10 --scene default --width 640 --height 480 --depth 4 --frames 30" \
 "200 ab_c5 python -u tools/ab.py run --only base,div0,divsingle --scene stress4096 --depth 12 --frames 4 --rounds 6" \
 "150 ab_c2 python -u tools/ab.py run --only base,div0,divsingle --scene default --width 1920 --height 1080 --depth 4 --frames 20 --rounds 10"
