# One GPU call for a library build: the GPU tests, rocprofv3 kernel stats of the default bench (C3) and of C5, and the
# PMC records of every config (tools/pmc_configs.sh).  Copy gpurun_out/<outdir>/records/*.json into profiles/pmc/
# afterwards, then run tools/lines_round.sh for the bench lines that read them.
# Usage (repo root, via gpurun): bash tools/round_profile.sh <outdir under gpurun_out>
R=$PWD
O=$R/gpurun_out/${1:-round_profile}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-c4 > $O/bench_c3_under_rocprof.json 2> $O/prof_c3.err || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o run -- python3 $R/bench.py --config c5 --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_c5_under_rocprof.json 2> $O/prof_c5.err || exit 3
cd $R
bash tools/pmc_configs.sh ${1:-round_profile}/pmc || exit 4
exit 0
