# Round-6 GPU call: the GPU suite, interleaved A/B of the round's variants, the N=2 screenshot rehearsal.
O=gpurun_out/${1:-r6b}
bash tools/gpu_step.sh $O \
 "420 gpu_tests python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 300 --timeout-method thread" \
 "150 ab_c3 python -u tools/ab.py run --only base,div0,divsingle,divall2 --rounds 10" \
 "120 ab_c1 python -u tools/ab.py run --only base,ticket0,fused0,lookback0 --rounds 10 --scene default --width 640 --height 480 --depth 4 --frames 30" \
 "150 ab_c5 python -u tools/ab.py run --only base,div0,divsingle --scene stress4096 --depth 12 --frames 4 --rounds 6" \
 "100 ab_c2 python -u tools/ab.py run --only base,div0,divsingle --scene default --width 1920 --height 1080 --depth 4 --frames 20 --rounds 10" \
 "150 ab_split python -u tools/ab.py run --only base,tiles0 --scene default --width 480 --height 270 --depth 20 --ss 128 --frames 2 --rounds 5 --later-frame 2" \
 "300 shot128_n2 python -u bench.py --gpus 2 --one-device --backend gloo --config shot128"
