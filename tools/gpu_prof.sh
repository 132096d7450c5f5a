#!/bin/bash
# rocprofv3 kernel stats + HBM counters (separate --pmc passes) for the bench workload,
# restricted to this repo's kernels (k_*).  usage: bash tools/gpu_prof.sh <tag> [bench args...]
# The stats pass runs the given bench command; the PMC passes add --no-match so that the
# per-kernel counter averages are those of the headline workload only.
tag=$1; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
R="--output-format csv"
timeout -k 10 600 rocprofv3 --kernel-trace --stats $R -d gpurun_out/prof_$tag -o run -- python bench.py "$@" > gpurun_out/prof_$tag.log 2>&1 || exit $?
ls -la gpurun_out/prof_$tag/*
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "::k_" $R -d gpurun_out/pmc_fetch_$tag -o run -- python bench.py --no-cpu --no-single --no-match "$@" > gpurun_out/pmc_fetch_$tag.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "::k_" $R -d gpurun_out/pmc_write_$tag -o run -- python bench.py --no-cpu --no-single --no-match "$@" > gpurun_out/pmc_write_$tag.log 2>&1 || exit $?
du -sh gpurun_out/*
python3 tools/trace_by_grid.py gpurun_out/prof_$tag gpurun_out/prof_${tag}_by_grid.csv
rm -f gpurun_out/prof_$tag/*kernel_trace.csv
