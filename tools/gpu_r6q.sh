# Round-6 GPU call: the tile sort's cost -- lpt_scan as a wave-parallel scan (base vs the committed head), the sort on
# the trace's own stream (sortmain), and a sort every 16th / 32nd launch instead of every 4th.  GPU suite first.
O=gpurun_out/${1:-r6q}
R=$PWD
AB="python -u tools/ab.py run"
V=head,base,sortmain,sort16,sortmain16,sort32
bash tools/gpu_step.sh $O \
 "600 gpu_tests python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "400 ab_c3 $AB --only $V --rounds 8 --frames 32" \
 "300 ab_c2d4 $AB --only $V --rounds 8 --scene default --width 1920 --height 1080 --depth 4 --frames 64" \
 "400 ab_shot $AB --only $V --rounds 6 --scene default --width 1920 --height 1080 --depth 20 --ss 4 --frames 16" \
 "300 prof_c3 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-c4"
