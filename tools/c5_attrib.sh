# C5's HBM writes attributed per kernel (trace / bounce), with ray regrouping at its default (park after 3 segments)
# and off: separate rocprofv3 --pmc passes (WRITE_SIZE; FETCH_SIZE; memory-instruction counts), plus the segment
# histogram (how many traces park).  Usage (repo root, via gpurun): bash tools/c5_attrib.sh <outdir under gpurun_out>
R=$PWD
O=$R/gpurun_out/${1:-c5attrib}
mkdir -p $O
timeout -k 10 200 python -u tools/segstats.py stress4096 12 > $O/segstats_c5.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
for rg in 3 0; do
  C5="$R/bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline --prewarm-ms 0 --regroup $rg"
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w_rg$rg -o run -- python3 $C5 > $O/w_rg$rg.log 2>&1 || exit 2
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f_rg$rg -o run -- python3 $C5 > $O/f_rg$rg.log 2>&1 || exit 3
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_FLAT SQ_WAVES --output-format csv -d $O/i_rg$rg -o run -- python3 $C5 > $O/i_rg$rg.log 2>&1 || exit 4
done
exit 0
