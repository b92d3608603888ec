# Round-6 GPU call: every bench line of the final build (device a8853a24), its PMC records in profiles/pmc.
bash tools/lines_round.sh ${1:-r6o}
