# Round-6 GPU call for the final build (device 81d6096c: + the tile sort on the launch's stream, every 16th launch):
# GPU suite, kernel stats, every config's PMC record (copied into profiles/pmc on the box so the lines carry them), then
# every bench line.
O=${1:-r6r}
bash tools/round_profile.sh $O || exit $?
cp gpurun_out/$O/pmc/records/*.json profiles/pmc/ || exit 20
bash tools/lines_round.sh $O/lines || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$O/smoke.log 2>&1 || exit 21
exit 0
