#!/bin/bash
# round-5: sequence plan sweep at overlap 15 with the row-streaming pyramid (rank slices, 3 runs each)
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 900 python -u tools/slice_sweep.py ${SPECS:-1:48:15 1:64:15} --reps ${REPS:-3} > gpurun_out/r5l_slice_sweep.jsonl 2> gpurun_out/r5l_slice_sweep.err || { tail -5 gpurun_out/r5l_slice_sweep.err; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/r5l_slice_sweep.jsonl'):
    d=json.loads(l); print(d['world'], d['per_gpu'], d['overlap'], d['groups'], d['wall_s_runs'], d['predicted_frames_per_s'], d['shards_compared'], d['shards_identical'])"
