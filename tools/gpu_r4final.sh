#!/bin/bash
# round-4 final verification: smoke(), the whole GPU suite, the default bench line
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final_smoke.log 2>&1 || { tail -20 gpurun_out/final_smoke.log; exit 1; }
tail -1 gpurun_out/final_smoke.log
bash tools/gpu_r4tests.sh || exit 1
bash tools/gpu_r4bench.sh final
