export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/bootprof -o run -- python tools/boot_prof.py > $O/bootprof.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INST_CYCLES_SALU SQ_BUSY_CU_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS --kernel-include-regex "k_sift|k_blur|k_extrema|k_upsample" --output-format csv -d $O/bootsq -o run -- python tools/boot_prof.py > $O/bootsq.log 2>&1 || exit $?
find $O/bootprof -name "*kernel_trace.csv" -delete
