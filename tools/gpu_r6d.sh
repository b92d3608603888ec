# Round-6 GPU call: interleaved A/B of the range tests as med3/min3 + one compare against compare pairs.
O=gpurun_out/${1:-r6d}
bash tools/gpu_step.sh $O \
 "200 gpu_kat python -u -m pytest tests/test_gpu_kat.py tests/test_gpu_parity.py -m gpu -v --timeout 300 --timeout-method thread -k 'kat or full_size or golden_bitexact'" \
 "150 ab_c3 python -u tools/ab.py run --only base,guardcmp,div0 --rounds 12" \
 "100 ab_c2 python -u tools/ab.py run --only base,guardcmp,div0 --scene default --width 1920 --height 1080 --depth 4 --frames 20 --rounds 12" \
 "120 ab_shot python -u tools/ab.py run --only base,guardcmp,div0 --scene default --width 1920 --height 1080 --depth 20 --ss 4 --frames 10 --rounds 8"
