# Round-6 GPU call: where a moving camera's extra C3 time goes -- region profiles (RFX_DEBUG_PROF build) with and without
# the per-view masks, and the interleaved A/B of the product build's mask modes (0 never, 1 on a repeated view).
O=gpurun_out/${1:-r6t}
mkdir -p $O
bash tools/gpu_step.sh $O \
 "120 region_masks python -u tools/regionprof.py" \
 "120 region_nomasks python -u tools/regionprof.py --prim 0"
