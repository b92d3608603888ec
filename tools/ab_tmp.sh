O=gpurun_out/ab16
bash tools/gpu_step.sh $O \
 "600 c3 python -u tools/ab.py run --only base,eifcvt,trackers,nounclust,bias100 --rounds 8" \
 "600 c5 python -u tools/ab.py run --only base,eifcvt,trackers,nounclust,bias100 --scene stress4096 --depth 12 --rounds 4 --frames 3"
