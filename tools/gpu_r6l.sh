# Round-6 GPU call: the RNG pre-pass rework -- integer accept test, emit loads issued together, the one-pass kernel's
# block jump composed in scalar registers, a workgroup-wide look-back window (lb0: the one-wave window) and the
# one-pass kernel's block limit (fmaxN).  GPU suite on the product build, interleaved A/B against the committed
# pre-pass (head), and the RNG kernels' issue counters.
O=gpurun_out/${1:-r6l}
R=$PWD
P="python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-c4 --no-first-view"
AB="python -u tools/ab.py run"
bash tools/gpu_step.sh $O \
 "600 gpu_tests python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "300 ab_c3 $AB --only head,base,intacc0,lb0,fmax4096,fmax4096lb16 --rounds 8" \
 "200 ab_c2d1 $AB --only head,base,lb0,fmax1024,fmax1024lb0,fmax4096 --rounds 10 --scene default --width 1920 --height 1080 --depth 1 --frames 30" \
 "200 ab_c2d4 $AB --only head,base,fmax1024,fmax4096 --rounds 10 --scene default --width 1920 --height 1080 --depth 4 --frames 20" \
 "150 ab_c1 $AB --only head,base,intacc0,lb0 --rounds 12 --scene default --width 640 --height 480 --depth 4 --frames 30" \
 "150 ab_720 $AB --only head,base,fmax1024,fmax1024lb0 --rounds 10 --scene default --width 1280 --height 720 --depth 4 --frames 30" \
 "90 pmc_rng1 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY --kernel-include-regex rng_ --output-format csv -d $O/pmc_rng1 -o run -- $P"
