# One GPU call (after the PMC records of this library are in profiles/pmc): the default bench line, every config's
# line, the drop-in's interactive cost through Pulse, the device group's band-copy cost, and gloo rehearsals of the
# N > 1 bench on one GPU (bands, with the f32-gather timing).
# Usage (repo root, via gpurun): bash tools/lines_round.sh <outdir under gpurun_out>
O=$PWD/gpurun_out/${1:-lines}
mkdir -p $O
timeout -k 10 300 python -u bench.py > $O/bench_c3.json 2> $O/bench_c3.err || exit 1
bash tools/configs_round.sh ${1:-lines}/configs || exit 2
timeout -k 10 300 python -u tools/pulse_session_time.py --reps 5 --out $O/pulse_session_640x480.json > $O/pulse.log 2>&1 || exit 3
timeout -k 10 200 python -u tools/group_copy_cost.py > $O/group_copy_cost_c4_8members_one_device.json 2> $O/group_copy.err || exit 4
for n in 2 4; do
  timeout -k 10 400 python bench.py --gpus $n --backend gloo --one-device --steps 20 --warmup 3 --no-cpu-baseline > $O/rehearsal_c4_n${n}_bands_gloo_one_device.json 2> $O/rehearsal_n$n.err || exit 5
done
# the ReadMe screenshot over 2 ranks: row-span passes (dist.BandFrame), hashed against the reference's frame
timeout -k 10 400 python bench.py --gpus 2 --backend gloo --one-device --config shot128 > $O/rehearsal_shot128_n2_bands_gloo_one_device.json 2> $O/rehearsal_shot128_n2.err || exit 6
exit 0
