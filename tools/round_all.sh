# One GPU call for a library build, end to end: tools/round_profile.sh (GPU tests, rocprof kernel stats, PMC records),
# the records copied into the box's profiles/pmc so the lines read them, then tools/lines_round.sh.  Copy
# gpurun_out/<outdir>/prof/pmc/records/*.json into profiles/pmc/ afterwards, and the lines into profiles/<round>/.
# Usage (repo root, via gpurun): bash tools/round_all.sh <outdir under gpurun_out>
N=${1:-round_all}
bash tools/round_profile.sh $N/prof || exit $?
cp gpurun_out/$N/prof/pmc/records/*.json profiles/pmc/ || exit 20
bash tools/lines_round.sh $N/lines || exit $((30 + $?))
exit 0
