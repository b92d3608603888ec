# Round-6 GPU call for the final pre-pass build (device a8853a24): GPU suite, kernel stats, every config's PMC record.
bash tools/round_profile.sh ${1:-r6n}
