O=gpurun_out/ab10
bash tools/gpu_step.sh $O \
 "600 c5 python -u tools/ab.py run --only base,bvhl2 --scene stress4096 --depth 12 --rounds 6 --frames 4" \
 "300 par python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k 'stress or planes or mesh'"
