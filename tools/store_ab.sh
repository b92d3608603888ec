# One GPU call: parity tests of the trace paths, interleaved A/B of the output-store and texture-block
# variants, and the WRITE_SIZE PMC pass of the C3 bench.  Usage: bash tools/store_ab.sh <outdir under gpurun_out>
R=$PWD
O=$R/gpurun_out/${1:-store_ab}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kat.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab.py run --only base,nostaged,texlds --rounds 10 > $O/ab.json 2> $O/ab.err || exit 2
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc3 -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/pmc3.log 2>&1 || exit 3
exit 0
