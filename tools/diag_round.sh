# Diagnostics in one GPU call: region cycle shares, segment-loop lane use, and two PMC passes over the bench.
# Usage (from the repo root, via gpurun): bash tools/diag_round.sh <outdir under gpurun_out>
R=$PWD
O=$R/gpurun_out/${1:-diag}
mkdir -p $O
timeout -k 10 200 python -u tools/regionprof.py > $O/regionprof.json 2>&1 || exit 1
timeout -k 10 200 python -u tools/segstats.py > $O/segstats.txt 2>&1 || exit 2
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU --output-format csv -d $O/pmc1 -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/pmc1.log 2>&1 || exit 3
timeout -s KILL 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE --output-format csv -d $O/pmc4 -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/pmc4.log 2>&1 || exit 4
exit 0
