#!/bin/bash
# round-5: every step kernel alone (one group of 384 chains, all stages on one stream): kernel-trace stats
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
VO_ONE_STREAM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/solo -o run -- python bench.py --groups 1 --chains 384 --no-sequence --no-single --no-match --no-cpu --steps 10 --warmup 3 > gpurun_out/solo.log 2>&1 || { tail -5 gpurun_out/solo.log; exit 1; }
python tools/trace_by_grid.py gpurun_out/solo gpurun_out/solo/by_grid.csv && rm -f gpurun_out/solo/*kernel_trace.csv
head -30 gpurun_out/solo/by_grid.csv
tail -1 gpurun_out/solo.log | cut -c1-300
