# One GPU call: bench.py under rocprofv3 --kernel-trace --stats, then the PMC passes (one counter group per
# run) whose per-launch means feed roofline.traffic.  Usage: bash tools/prof_round.sh <outdir under gpurun_out>
R=$PWD
O=$R/gpurun_out/${1:-prof}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-c4 > $O/bench_prof.json 2> $O/bench_prof.err || exit 1
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU --output-format csv -d $O/pmc1 -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-c4 > $O/pmc1.log 2>&1 || exit 2
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc2 -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-c4 > $O/pmc2.log 2>&1 || exit 3
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc3 -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-c4 > $O/pmc3.log 2>&1 || exit 4
timeout -s KILL 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/pmc4 -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-c4 > $O/pmc4.log 2>&1 || exit 5
exit 0
