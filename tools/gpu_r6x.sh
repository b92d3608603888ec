# Round-6 GPU call: one-device emits of more than RFX_SCAN_EMIT_BLOCKS blocks through the tile scan (rng_tile_sums +
# rng_tile_scan + rng_emit_band) instead of per-block prefix sums (rng_emit): the threshold at 16384 (base), 4096, 2048.
O=gpurun_out/${1:-r6x}
AB="python -u tools/ab.py run --only base,se4096,se2048"
bash tools/gpu_step.sh $O \
 "400 ab_c4 $AB --rounds 6 --width 7680 --height 4320 --frames 8" \
 "400 ab_shot $AB --rounds 6 --scene default --width 1920 --height 1080 --depth 20 --ss 4 --frames 10" \
 "300 ab_c3 $AB --rounds 8 --frames 20" \
 "200 ab_c2d4 $AB --rounds 8 --scene default --width 1920 --height 1080 --depth 4 --frames 30"
