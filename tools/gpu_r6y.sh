# Round-6 final check of HEAD's library: the GPU suite, smoke() and the default bench line.
O=gpurun_out/${1:-r6y}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py > $O/bench_c3.json 2> $O/bench_c3.err || exit 3
exit 0
