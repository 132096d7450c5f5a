#!/bin/bash
# per-dispatch kernel trace of the single-group one-stream bench for kernels matching a regex
# usage: bash tools/gpu_ktrace.sh <tag> <regex>
tag=${1:-t}; rx=${2:-k_pyr_level}
mkdir -p gpurun_out
export TMPDIR=/tmp VO_ONE_STREAM=1
A="--no-cpu --no-single --no-match --groups 1 --chains 192 --steps 4 --warmup 2"
timeout -k 10 300 rocprofv3 --kernel-trace --kernel-include-regex "$rx" --output-format csv -d gpurun_out/kt_$tag -o run -- python bench.py $A > gpurun_out/kt_$tag.log 2>&1 || exit $?
python3 - "$tag" <<'PY'
import csv, glob, sys, collections
f = glob.glob(f"gpurun_out/kt_{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    import re; m = re.search(r"(k_\w+(<[^>]*>)?)", r["Kernel_Name"]); n = m.group(1) if m else r["Kernel_Name"][:40]
    acc[(n, r["Grid_Size_X"], r["Grid_Size_Y"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
for k, v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
    print(f"{k[0]:40s} grid {k[1]:>7s} x {k[2]:>4s}  n={len(v):3d}  mean {sum(v)/len(v):8.1f} us")
PY
