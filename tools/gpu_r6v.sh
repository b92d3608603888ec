# Round-6 GPU call: the count kernel's per-block parity test against the float test.
O=gpurun_out/${1:-r6v}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "rng_count_blocks or rng_stream_state" > $O/tests.log 2>&1 || exit 1
exit 0
