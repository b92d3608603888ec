O=gpurun_out/ab9
bash tools/gpu_step.sh $O \
 "600 c5 python -u tools/ab.py run --only base,cr2,cr15 --scene stress4096 --depth 12 --rounds 5 --frames 4" \
 "400 c3 python -u tools/ab.py run --only base,cr2,cr15 --rounds 10"
