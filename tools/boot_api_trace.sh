#!/bin/bash
# kernel + HIP API trace of tools/boot_prof.py (first-call costs of the bootstrap)
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --output-format csv -d $O/bootapi -o run -- python tools/boot_prof.py > $O/bootapi.log 2>&1 || exit $?
python3 tools/boot_api_summary.py $O/bootapi > $O/bootapi_summary.txt && rm -f $O/bootapi/*trace.csv
grep -v hipMemcpyWithStream $O/bootapi_summary.txt | tail -30
