O=gpurun_out/t13
bash tools/gpu_step.sh $O \
 "600 tests python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread" \
 "300 bench python -u bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline"
