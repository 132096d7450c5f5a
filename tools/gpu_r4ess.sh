#!/bin/bash
# E-RANSAC five-point solve in registers: bootstrap GPU tests, kernel trace of a 64-chain
# bootstrap, the 768-chain bootstrap time and the sequence leg
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bootstrap.py tests/test_gpu_parity.py -k "essential or bootstrap or five" -m gpu > gpurun_out/r4ess_tests.log 2>&1 || { tail -20 gpurun_out/r4ess_tests.log; exit 1; }
tail -1 gpurun_out/r4ess_tests.log
rm -rf gpurun_out/ess
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ess -o ess -- python -u tools/boot_prof.py 64 > gpurun_out/ess_boot64.log 2>&1 || { tail -5 gpurun_out/ess_boot64.log; exit 1; }
cat gpurun_out/ess_boot64.log | tail -3
f=$(find gpurun_out/ess -name "*kernel_stats.csv" | head -1); grep -i "essential\|recover\|desc_w\|KERNEL" "$f" | cut -c1-160
find gpurun_out/ess -name "*kernel_trace.csv" -delete
timeout -k 10 300 python -u tools/boot_prof.py 768 > gpurun_out/ess_boot768.log 2>&1 || { tail -5 gpurun_out/ess_boot768.log; exit 1; }
tail -3 gpurun_out/ess_boot768.log
timeout -k 10 300 python -u tools/seq_sweep.py --groups 2 --reps 2 64 > gpurun_out/ess_seq.jsonl 2> gpurun_out/ess_seq.err || { tail -5 gpurun_out/ess_seq.err; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/ess_seq.jsonl'):
    d=json.loads(l); print({k: d.get(k) for k in ('chains_per_gpu','groups','sequence_frames_per_s','wall_s','bootstrap_s','step_s','ms_per_step')})"
