# Round-6 GPU call: the C3 and C5 region profiles of the final kernels (RFX_DEBUG_PROF build).
O=gpurun_out/${1:-r6h}
mkdir -p $O
timeout -k 10 200 python -u tools/regionprof.py > $O/regionprof_c3.json 2> $O/regionprof_c3.err || exit 1
timeout -k 10 300 python -u tools/regionprof.py --scene stress4096 --depth 12 --regroup 0 > $O/regionprof_c5_noregroup.json 2> $O/regionprof_c5.err || exit 2
exit 0
