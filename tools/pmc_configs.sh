# One GPU call: the PMC passes (one counter group per run) of the trace kernel (+ its bounce kernel) at every
# config bench.py reports -- C1, C2 depth 1 and 4, C3, the C4 frame on one GPU, C5, the screenshot -- summarised into
# profiles/pmc records keyed by the library's device-code hash.  Records land under gpurun_out/<outdir>/records
# (copy them into profiles/pmc/ afterwards); with --lines, every config's bench line again so each carries
# roofline.frac.  Any device-code change invalidates every record: re-run this after the last kernel change.
# Usage (repo root, via gpurun): bash tools/pmc_configs.sh <outdir under gpurun_out> [--lines]
R=$PWD
O=$R/gpurun_out/${1:-pmc_configs}
mkdir -p $O/records
cd /tmp && export TMPDIR=/tmp
run_cfg() {  # name  scene W H depth ss  bench args...   (PMC_ONLY="c3 c5 ..": only the configs whose name starts so)
  local name=$1 scene=$2 W=$3 H=$4 depth=$5 ss=$6
  if [ -n "$PMC_ONLY" ]; then
    local keep=0 p
    for p in $PMC_ONLY; do case $name in ${p}_*) keep=1 ;; esac; done
    [ $keep = 1 ] || return 0
  fi
  shift 6
  # steady-state frames only: no first-view frames and no same-run C4 frames in the per-dispatch means
  local args="$R/bench.py $* --no-cpu-baseline --no-first-view --no-c4"
  timeout -s KILL ${PMC_T:-120} rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU --output-format csv -d $O/pmc1_$name -o run -- python3 $args > $O/pmc1_$name.log 2>&1 || return 7
  timeout -s KILL ${PMC_T:-120} rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc2_$name -o run -- python3 $args > $O/pmc2_$name.log 2>&1 || return 8
  timeout -s KILL ${PMC_T:-120} rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc3_$name -o run -- python3 $args > $O/pmc3_$name.log 2>&1 || return 9
  timeout -s KILL ${PMC_T:-120} rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/pmc4_$name -o run -- python3 $args > $O/pmc4_$name.log 2>&1 || return 10
  python3 $R/tools/pmc_summary.py --kernel "trace_kernel<false,bounce_kernel" --out $O/records/$name.json --config $scene $W $H $depth 1 $ss \
    $(find $O/pmc1_$name $O/pmc2_$name $O/pmc3_$name $O/pmc4_$name -name '*counter_collection.csv') > $O/summary_$name.json || return 11
}
run_cfg c3_synth16_3840x2160_d8 synth16 3840 2160 8 1 --config c3 --steps 3 --warmup 1 || exit $?
run_cfg c5_stress4096_3840x2160_d12 stress4096 3840 2160 12 1 --config c5 --steps 2 --warmup 1 || exit $?
run_cfg c1_default_640x480_d4 default 640 480 4 1 --config c1 --steps 20 --warmup 3 || exit $?
run_cfg c2_default_1920x1080_d1 default 1920 1080 1 1 --config c2 --depth 1 --steps 10 --warmup 2 || exit $?
run_cfg c2_default_1920x1080_d4 default 1920 1080 4 1 --config c2 --steps 10 --warmup 2 || exit $?
run_cfg c4_synth16_7680x4320_d8 synth16 7680 4320 8 1 --config c4 --steps 3 --warmup 1 || exit $?
run_cfg shot_default_1920x1080_d20 default 1920 1080 20 4 --config shot --steps 3 --warmup 1 || exit $?
PMC_T=300 run_cfg shot128_default_1920x1080_d20 default 1920 1080 20 128 --config shot128 --steps 1 --warmup 0 || exit $?
if [ "$2" = "--lines" ]; then
  cp $O/records/*.json $R/profiles/pmc/ || exit 12
  cd $R
  bash tools/configs_round.sh ${1:-pmc_configs}/configs || exit 13
fi
exit 0
