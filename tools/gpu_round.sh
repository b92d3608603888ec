# One GPU call: parity tests, bench, region/segment diagnostics, rocprofv3 kernel stats and the PMC passes
# (one counter group per run) for C3 and C5.  Usage (from the repo root, via gpurun):
#   bash tools/gpu_round.sh <outdir under gpurun_out>
R=$PWD
O=$R/gpurun_out/${1:-round}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $O/bench.json 2> $O/bench.err || exit 2
timeout -k 10 200 python -u tools/regionprof.py > $O/regionprof.json 2>&1 || exit 3
timeout -k 10 200 python -u tools/segstats.py > $O/segstats.txt 2>&1 || exit 4
cd /tmp && export TMPDIR=/tmp
C3="$R/bench.py --steps 3 --warmup 1 --no-cpu-baseline"
C5="$R/bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_prof.json 2> $O/bench_prof.err || exit 5
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o run -- python3 $C5 > $O/bench_prof_c5.json 2> $O/bench_prof_c5.err || exit 6
for cfg in C3 C5; do
  args=${!cfg}
  timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU --output-format csv -d $O/pmc1_$cfg -o run -- python3 $args > $O/pmc1_$cfg.log 2>&1 || exit 7
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc2_$cfg -o run -- python3 $args > $O/pmc2_$cfg.log 2>&1 || exit 8
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc3_$cfg -o run -- python3 $args > $O/pmc3_$cfg.log 2>&1 || exit 9
  timeout -s KILL 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/pmc4_$cfg -o run -- python3 $args > $O/pmc4_$cfg.log 2>&1 || exit 10
done
exit 0
