#!/bin/bash
# late round-3 verification: GPU tests, smoke, the default bench line, single-chain latency and
# the PnP phase profile.  usage: bash tools/gpu_final_r3d.sh <tag>
tag=${1:-r3d}
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_$tag.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_$tag.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$tag.log 2>&1 || { tail -5 gpurun_out/smoke_$tag.log; exit 1; }
tail -1 gpurun_out/smoke_$tag.log
timeout -k 10 400 python bench.py > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err || { tail -5 gpurun_out/bench_$tag.err; exit 1; }
tail -1 gpurun_out/bench_$tag.json | cut -c1-300
for v in 1 2; do timeout -k 10 200 python -u tools/single_prof.py 200 2>&1 | grep frames; done
timeout -k 10 120 python -u tools/pnp_prof.py 80 > gpurun_out/pnp_$tag.log 2>&1 && tail -1 gpurun_out/pnp_$tag.log
