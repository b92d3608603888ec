O=gpurun_out/ab8
bash tools/gpu_step.sh $O \
 "300 rng python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py tests/test_gpu_steady.py tests/test_gpu_group.py tests/test_gpu_kat.py -m gpu -x -q --timeout 120 --timeout-method thread" \
 "400 c3 python -u tools/ab.py run --only base,rngchain --rounds 12" \
 "300 c1 python -u tools/ab.py run --only base,rngchain --scene default --width 640 --height 480 --depth 4 --rounds 12 --frames 50"
