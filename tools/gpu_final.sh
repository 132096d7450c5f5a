#!/bin/bash
# Round-end verification in one GPU call: the full -m gpu suite, smoke(), the default bench
# line.  usage: bash tools/gpu_final.sh <tag>
tag=${1:-f}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_$tag.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_$tag.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$tag.log 2>&1 || { tail -5 gpurun_out/smoke_$tag.log; exit 1; }
tail -1 gpurun_out/smoke_$tag.log
timeout -k 10 400 python bench.py > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err || { tail -5 gpurun_out/bench_$tag.err; exit 1; }
tail -1 gpurun_out/bench_$tag.json
